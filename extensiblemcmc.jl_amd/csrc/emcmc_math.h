// emcmc_math.h — bit-reproducible fp64 math shared by the host side of
// libemcmc.so and its gfx950 kernels.
//
// Why this exists: parity with the CPU oracle is defined bit-for-bit on the
// accept/reject stream (BASELINE.json north_star).  Device libm (ocml) and
// host glibc disagree in the last ulp for log/exp, so every transcendental is
// built here from IEEE basic operations (+ − × ÷, fma, sqrt, rint — all
// correctly rounded on both sides) and compiled with -ffp-contract=off.
// Normal and exponential variates come from a 256-layer ziggurat whose fast
// path is integer work plus one multiply (see below).  The variate stream itself is counter-based
// (Philox4x32-10), keyed by the master seed and indexed by
// (global chain id, mcmciter, block, pidx/attempt), so any chain on any shard
// can be replayed independently.
//
// Reference semantics replaced (src/ paths under /root/reference):
//   randn via rand(MvNormal(θ,Σ))      transition_kernels/random_walk.jl:147
//   rand(Exponential(1.0))             run.jl:278
//   rand(Uniform(-ϵ,ϵ))                transition_kernels/random_walk.jl:71
// Julia's GLOBAL_RNG/ziggurat stream cannot be reproduced offline (SURVEY §7
// "Hard parts" 1), so the stream is defined here and shared with oracle/.
#pragma once

#ifndef __HIPCC_RTC__  // hiprtc (user targets, emcmc_user.cpp) provides its own builtins
#include <stddef.h>
#include <stdint.h>
#include <math.h>
#else
typedef unsigned char uint8_t;
typedef unsigned short uint16_t;
typedef unsigned int uint32_t;
typedef unsigned long uint64_t;
typedef int int32_t;
typedef long int64_t;
typedef __SIZE_TYPE__ size_t;
#define offsetof(t, m) __builtin_offsetof(t, m)
#endif

#include "emcmc_tables.h"

#if defined(__HIPCC__)
#define EMCMC_HD __host__ __device__ __forceinline__
#else
#define EMCMC_HD static inline
#endif

namespace emcmc {

// ---- bit casts --------------------------------------------------------------
EMCMC_HD uint64_t d2u(double x) { return __builtin_bit_cast(uint64_t, x); }
EMCMC_HD double u2d(uint64_t u) { return __builtin_bit_cast(double, u); }

// ---- Philox4x32-10 (Salmon, Moraes, Dror, Shaw, SC'11) ----------------------
struct u32x4 {
    uint32_t x, y, z, w;
};

#if defined(__HIP_DEVICE_COMPILE__)
// a ^ b ^ k in one VALU op (gfx950 v_bitop3_b32, truth table 0x96); k is a
// round key derived from the seed, wave-uniform, so it sits in an SGPR
// (the builtin, not inline asm: the compiler must otherwise assume the worst
// hazard after every asm block and pads each following v_mad_u64_u32 with an
// s_nop — ≈ 75 wasted issue slots per wave-step of the step kernel)
__device__ __forceinline__ uint32_t xor3_key(uint32_t a, uint32_t b, uint32_t k) {
    return __builtin_amdgcn_bitop3_b32(a, b, k, 0x96);
}
#else
static inline uint32_t xor3_key(uint32_t a, uint32_t b, uint32_t k) { return a ^ b ^ k; }
#endif

#if defined(__HIP_DEVICE_COMPILE__)
// The key words re-materialised through an opaque SALU move: the ten round
// keys of each Philox call are then derived inside the call (s_add per round)
// instead of being hoisted out of the step loop as 20 live SGPRs (which the
// register allocator spills into VGPR lanes and reloads with v_readlane).
__device__ __forceinline__ uint32_t key_local(uint32_t k) {
    uint32_t r;
    asm volatile("s_mov_b32 %0, %1" : "=s"(r) : "s"(k));
    return r;
}
#else
static inline uint32_t key_local(uint32_t k) { return k; }
#endif

EMCMC_HD u32x4 philox4x32_10(u32x4 c, uint32_t k0, uint32_t k1) {
    k0 = key_local(k0);
    k1 = key_local(k1);
    const uint32_t M0 = 0xD2511F53u, M1 = 0xCD9E8D57u;
    const uint32_t W0 = 0x9E3779B9u, W1 = 0xBB67AE85u;
#pragma unroll
    for (int r = 0; r < 10; ++r) {
        // full 32×32→64 products: one v_mad_u64_u32 each on gfx950
        const uint64_t p0 = (uint64_t)M0 * (uint64_t)c.x;
        const uint64_t p1 = (uint64_t)M1 * (uint64_t)c.z;
        u32x4 n;
        n.x = xor3_key((uint32_t)(p1 >> 32), c.y, k0);
        n.y = (uint32_t)p1;
        n.z = xor3_key((uint32_t)(p0 >> 32), c.w, k1);
        n.w = (uint32_t)p0;
        c = n;
        k0 += W0;
        k1 += W1;
    }
    return c;
}

// The 20 round keys of Philox4x32-10 (k0 + r·W0, k1 + r·W1, r = 0..9) held in
// VGPRs for a whole kernel: the step loop's Philox calls then spend no SALU on
// key derivation (≈ 20 scalar adds per call, 8.5 calls per step), and a wave
// issues one instruction per quad-cycle whatever its type.
struct PhiloxVKeys {
    uint32_t k0[10], k1[10];
};
EMCMC_HD PhiloxVKeys philox_vkeys(uint32_t k0, uint32_t k1) {
    PhiloxVKeys K;
#pragma unroll
    for (int r = 0; r < 10; ++r) {
        const uint32_t a = k0 + (uint32_t)r * 0x9E3779B9u, b = k1 + (uint32_t)r * 0xBB67AE85u;
#if defined(__HIP_DEVICE_COMPILE__)
        asm volatile("v_mov_b32 %0, %1" : "=v"(K.k0[r]) : "s"(a));
        asm volatile("v_mov_b32 %0, %1" : "=v"(K.k1[r]) : "s"(b));
#else
        K.k0[r] = a;
        K.k1[r] = b;
#endif
    }
    return K;
}
EMCMC_HD uint32_t xor3_vkey(uint32_t a, uint32_t b, uint32_t k) {
#if defined(__HIP_DEVICE_COMPILE__)
    return __builtin_amdgcn_bitop3_b32(a, b, k, 0x96);
#else
    return a ^ b ^ k;
#endif
}
// philox4x32_10 with the keys from VGPRs (the same bits)
EMCMC_HD u32x4 philox4x32_10_vk(u32x4 c, const PhiloxVKeys &K) {
    const uint32_t M0 = 0xD2511F53u, M1 = 0xCD9E8D57u;
#pragma unroll
    for (int r = 0; r < 10; ++r) {
        const uint64_t p0 = (uint64_t)M0 * (uint64_t)c.x;
        const uint64_t p1 = (uint64_t)M1 * (uint64_t)c.z;
        u32x4 n;
        n.x = xor3_vkey((uint32_t)(p1 >> 32), c.y, K.k0[r]);
        n.y = (uint32_t)p1;
        n.z = xor3_vkey((uint32_t)(p0 >> 32), c.w, K.k1[r]);
        n.w = (uint32_t)p0;
        c = n;
    }
    return c;
}
EMCMC_HD u32x4 draw_vk(const PhiloxVKeys &K, uint32_t chain, uint32_t iter, uint32_t block, uint32_t pidx0) {
    return philox4x32_10_vk(u32x4{chain, iter, block, pidx0 << 16}, K);
}

// Counter layout of the shared stream:
//   x = global chain id, y = mcmciter (1-based), z = block, w = (pidx << 16) | attempt
// Blocks: normal pair j → z = j; accept draws → z = kBlockAccept.  The fast
// (attempt 0) accept draws of iterations 2m and 2m+1 share one block, indexed
// by y = m: words (x,y) serve the even iteration, (z,w) the odd one.  Their
// rare-path blocks use y = mcmciter and attempt ≥ 1, so they never collide.
constexpr uint32_t kBlockAccept = 0xFFFFFFFFu;

EMCMC_HD u32x4 draw(uint32_t k0, uint32_t k1, uint32_t chain, uint32_t iter, uint32_t block,
                    uint32_t pidx0, uint32_t attempt) {
    u32x4 c;
    c.x = chain;
    c.y = iter;
    c.z = block;
    c.w = (pidx0 << 16) | (attempt & 0xFFFFu);
    return philox4x32_10(c, k0, k1);
}

// 53 random bits from two words: hi word fully, top 21 bits of lo word.
EMCMC_HD uint64_t bits53(uint32_t hi, uint32_t lo) {
    return ((uint64_t)hi << 21) | (uint64_t)(lo >> 11);
}
// u ∈ (0, 1]  (never 0, so log(u) is finite)
EMCMC_HD double u01_open0(uint32_t hi, uint32_t lo) {
    return (double)(bits53(hi, lo) + 1ull) * 0x1p-53;
}
// u ∈ [0, 1)  (Julia rand() convention, for Uniform(a,b) = a + (b−a)·u)
EMCMC_HD double u01_closed0(uint32_t hi, uint32_t lo) {
    return (double)bits53(hi, lo) * 0x1p-53;
}

// ---- natural log (fdlibm e_log.c reduction; Lg1..Lg7 polynomial by fma Horner)
// Valid for finite normal x > 0, which covers u ∈ [2^-53, 1] and every
// positive normal argument used on the hot path.  ≤ 1 ulp (tests/).
EMCMC_HD double log_pos(double x) {
    const double ln2_hi = 6.93147180369123816490e-01;
    const double ln2_lo = 1.90821492927058770002e-10;
    const double Lg1 = 6.666666666666735130e-01, Lg2 = 3.999999999940941908e-01,
                 Lg3 = 2.857142874366239149e-01, Lg4 = 2.222219843214978396e-01,
                 Lg5 = 1.818357216161805012e-01, Lg6 = 1.531383769920937332e-01,
                 Lg7 = 1.479819860511658591e-01;
    const uint64_t b = d2u(x);
    int32_t hx = (int32_t)(b >> 32);
    const uint32_t lx = (uint32_t)b;
    int32_t k = (hx >> 20) - 1023;
    hx &= 0x000fffff;
    const int32_t i = (hx + 0x95f64) & 0x100000;
    // mantissa scaled into [sqrt(2)/2, sqrt(2))
    const double xn = u2d(((uint64_t)(uint32_t)(hx | (i ^ 0x3ff00000)) << 32) | lx);
    k += (i >> 20);
    const double f = xn - 1.0;
    const double s = f / (2.0 + f);
    const double dk = (double)k;
    const double z = s * s;
    const double w = z * z;
    const double t1 = w * fma(w, fma(w, Lg6, Lg4), Lg2);
    const double t2 = z * fma(w, fma(w, fma(w, Lg7, Lg5), Lg3), Lg1);
    const double R = t2 + t1;
    const double hfsq = 0.5 * f * f;
    return dk * ln2_hi - ((hfsq - fma(s, hfsq + R, dk * ln2_lo)) - f);
}

// ---- exp on [−700, 0] (rare paths and table construction) ------------------
// x = k·ln2 + r, |r| ≤ ln2/2, e^r by its degree-13 Taylor polynomial in fma
// Horner form (truncation < 5e-18), 2^k applied through the exponent bits.
EMCMC_HD double exp_nonpos(double x) {
    const double invln2 = 1.44269504088896338700e+00;
    const double ln2_hi = 6.93147180369123816490e-01, ln2_lo = 1.90821492927058770002e-10;
    const double kd = rint(x * invln2);
    double r = fma(-kd, ln2_hi, x);
    r = fma(-kd, ln2_lo, r);
    double p = 1.0 / 6227020800.0;  // 1/13!
    p = fma(p, r, 1.0 / 479001600.0);
    p = fma(p, r, 1.0 / 39916800.0);
    p = fma(p, r, 1.0 / 3628800.0);
    p = fma(p, r, 1.0 / 362880.0);
    p = fma(p, r, 1.0 / 40320.0);
    p = fma(p, r, 1.0 / 5040.0);
    p = fma(p, r, 1.0 / 720.0);
    p = fma(p, r, 1.0 / 120.0);
    p = fma(p, r, 1.0 / 24.0);
    p = fma(p, r, 1.0 / 6.0);
    p = fma(p, r, 0.5);
    p = fma(p, r, 1.0);
    p = fma(p, r, 1.0);
    const int k = (int)kd;
    return p * u2d((uint64_t)(1023 + k) << 52);
}

// ---- exp and log over the whole range (GaussianRandomWalkMix density) ------
// log((1−λ)·e^{lp_A} + λ·e^{lp_B}) (random_walk.jl:229-232) exponentiates
// log-densities of either sign.  exp_any: the exp_nonpos reduction and
// polynomial; 2^k in two exact steps for subnormal results (one rounding) and
// k = 1024; 0 below −745.13, +Inf above 709.78.  log_any: 0 → −Inf, +Inf →
// +Inf, NaN → NaN, subnormals scaled by 2^54 first.
EMCMC_HD double exp_any(double x) {
    // branch-free: the range cases are selects at the end; the scaling is the
    // two-step form of oracle_math.h orc_exp_any (one rounding for subnormal
    // results, exact otherwise)
    const double invln2 = 1.44269504088896338700e+00;
    const double ln2_hi = 6.93147180369123816490e-01, ln2_lo = 1.90821492927058770002e-10;
    const double xc = fmin(fmax(x, -746.0), 710.0);  // keeps k in int range (NaN → −746, selected away)
    const double kd = rint(xc * invln2);
    double r = fma(-kd, ln2_hi, xc);
    r = fma(-kd, ln2_lo, r);
    double p = 1.0 / 6227020800.0;
    p = fma(p, r, 1.0 / 479001600.0);
    p = fma(p, r, 1.0 / 39916800.0);
    p = fma(p, r, 1.0 / 3628800.0);
    p = fma(p, r, 1.0 / 362880.0);
    p = fma(p, r, 1.0 / 40320.0);
    p = fma(p, r, 1.0 / 5040.0);
    p = fma(p, r, 1.0 / 720.0);
    p = fma(p, r, 1.0 / 120.0);
    p = fma(p, r, 1.0 / 24.0);
    p = fma(p, r, 1.0 / 6.0);
    p = fma(p, r, 0.5);
    p = fma(p, r, 1.0);
    p = fma(p, r, 1.0);
    const int k = (int)kd;
    const bool lo = k < -1022, hi = k > 1023;
    double e = p * u2d((uint64_t)(1023 + (lo ? k + 64 : hi ? k - 1 : k)) << 52);
    e = lo ? e * 0x1p-64 : hi ? e * 2.0 : e;
    e = (x < -745.1332191019412) ? 0.0 : e;
    e = (x > 709.782712893384) ? __builtin_inf() : e;
    return (x != x) ? x : e;
}

EMCMC_HD double log_any(double x) {
    if (x != x) return x;
    if (x == 0.0) return -__builtin_inf();
    if (x == __builtin_inf()) return x;
    if (x < 0x1p-1022) return log_pos(x * 0x1p54) - 37.42994775023705;
    return log_pos(x);
}

// ---- log(1 + y) (prior densities: Beta, Cauchy, TDist) -------------------------
// u = 1 + y rounded, then log u corrected by that rounding: log(1 + y) =
// log u + log((1 + y)/u) ≈ log u − ((u − 1) − y)/u.  −Inf at y = −1, NaN below
// (and for NaN), +Inf at +Inf.  Restated as orc_log1p_any in oracle/oracle_math.h.
EMCMC_HD double log1p_any(double y) {
    const double u = 1.0 + y;
    if (!(u >= 0.0)) return __builtin_nan("");
    if (u == 0.0) return -__builtin_inf();
    if (u == __builtin_inf()) return u;
    return log_any(u) - ((u - 1.0) - y) / u;
}

// ---- table-driven exp (x ≤ 0) and log (1 ≤ u ≤ 2): the MALA logistic terms --
// e^{−|η|} and log(1 + e^{−|η|}) run once per observation and chain (4·10⁹ times
// per cfg 3 step), so they get shorter forms than exp_any / log_pos; the
// correctly rounded tables come from scripts/gen_math_tables.py
// (emcmc_tables.h; the oracle holds its own copy).
//
// exp_le0: x = k·ln2/64 + r, |r| ≤ ln2/128 (Cody–Waite, ln2/64 split so k·hi is
// exact), e^x = 2^⌊k/64⌋ · 2^{(k mod 64)/64} · e^r with e^r − 1 by a degree-6
// polynomial (truncation < 3e-20); the table entry times (1 + p) in one fma,
// the power of two by ldexp (IEEE: subnormal results rounded once, 0 below
// −745.13).  ≤ 1 ulp (tests/test_oracle.py).  NaN → NaN.
template <bool NANSEL = true>
EMCMC_HD double exp_le0(double x, const double *exp2_64) {
    const double ln2_64_hi = 6.93147180369123816490e-01 / 64.0, ln2_64_lo = 1.90821492927058770002e-10 / 64.0;
    const double xc = fmax(x, -746.0);  // keeps k in int range (NaN → −746, selected away)
    const double kd = rint(xc * 92.332482616893656);  // 64/ln2
    double r = fma(-kd, ln2_64_hi, xc);
    r = fma(-kd, ln2_64_lo, r);
    const int k = (int)kd;
    const int j = k & 63, m = k >> 6;  // floor(k/64) (arithmetic shift)
    double q = 1.0 / 720.0;
    q = fma(q, r, 1.0 / 120.0);
    q = fma(q, r, 1.0 / 24.0);
    q = fma(q, r, 1.0 / 6.0);
    q = fma(q, r, 0.5);
    const double pm1 = fma(q * r, r, r);  // e^r − 1
    const double tj = exp2_64[j];
    const double e = ldexp(fma(tj, pm1, tj), m);
    if constexpr (!NANSEL) return e;  // x must be a number (NaN gives ≈ 0, not NaN)
    return (x != x) ? x : e;
}
// log_1_2: u ∈ [1, 2]; u = 2^e·w, w ∈ [1, 2), w in interval j of 128 with
// centre c_j: log u = e·ln2 − log(RN(1/c_j)) + log1p(r), r = w·RN(1/c_j) − 1
// (|r| < 2^-8, one fma) by a degree-7 series (truncation < 5e-21).  The error
// is absolute, ≤ 2^-60 for u near 1 (relative ≤ 1.5 ulp away from 1): what
// the log-likelihood sum needs, where log1p(t) is added to terms of order 1.
EMCMC_HD double log_1_2(double u, const double *invc, const double *logc) {
    const double ln2_hi = 6.93147180369123816490e-01, ln2_lo = 1.90821492927058770002e-10;
    const uint64_t b = d2u(u);
    const double e = (double)((int)(b >> 52) - 1023);  // 0, or 1 at u = 2
    const double w = u2d((b & 0x000FFFFFFFFFFFFFull) | 0x3FF0000000000000ull);
    const int j = (int)((b >> 45) & 127u);
    const double r = fma(w, invc[j], -1.0);
    double q = 1.0 / 7.0;
    q = fma(q, r, -1.0 / 6.0);
    q = fma(q, r, 1.0 / 5.0);
    q = fma(q, r, -0.25);
    q = fma(q, r, 1.0 / 3.0);
    q = fma(q, r, -0.5);
    const double l1 = fma(q * r, r, r);  // log1p(r)
    return fma(e, ln2_hi, logc[j]) + fma(e, ln2_lo, l1);
}
// log_1_2 and 1/u from the same reduction (the MALA logistic terms need both):
// 1/u = 2^−e · RN(1/c_j) / (1 + r), 1/(1 + r) = Σ_{k≤6} (−r)^k (|r|^7 < 2^-56),
// ≤ 2 ulp (tests/test_oracle_mala.py) with no division: 6 fma, a product and an
// ldexp instead of the IEEE quotient's scale/reciprocal/refine/fixup sequence.
EMCMC_HD double log_rcp_1_2(double u, const double *invc, const double *logc, double &rcp) {
    const double ln2_hi = 6.93147180369123816490e-01, ln2_lo = 1.90821492927058770002e-10;
    const uint64_t b = d2u(u);
    const int ei = (int)(b >> 52) - 1023;  // 0, or 1 at u = 2
    const double e = (double)ei;
    const double w = u2d((b & 0x000FFFFFFFFFFFFFull) | 0x3FF0000000000000ull);
    const int j = (int)((b >> 45) & 127u);
    const double ic = invc[j];
    const double r = fma(w, ic, -1.0);
    double q = 1.0 / 7.0;
    q = fma(q, r, -1.0 / 6.0);
    q = fma(q, r, 1.0 / 5.0);
    q = fma(q, r, -0.25);
    q = fma(q, r, 1.0 / 3.0);
    q = fma(q, r, -0.5);
    const double l1 = fma(q * r, r, r);  // log1p(r)
    double p = 1.0 - r;
    p = fma(-r, p, 1.0);
    p = fma(-r, p, 1.0);
    p = fma(-r, p, 1.0);
    p = fma(-r, p, 1.0);
    p = fma(-r, p, 1.0);  // Σ_{k≤6} (−r)^k
    rcp = ldexp(ic * p, -ei);
    return fma(e, ln2_hi, logc[j]) + fma(e, ln2_lo, l1);
}

// ---- Marsaglia–Tsang ziggurat (J. Stat. Softw. 5(8), 2000) ---------------
// The same sampler family as Julia's randn/randexp (Random stdlib), fed by the
// Philox stream: 8192 layers for N(0,1), 256 for Exp(1).  One 64-bit draw
// (hi:lo) per variate.
//   N(0,1): layer ℓ = lo[12:0], magnitude = (hi:lo)[63:12] (52 bits), sign = lo[13]
//           (layer and sign share the magnitude's last two bits, as Julia's
//           randn shares its 8 layer bits with the magnitude: Random/src/normal.jl)
//   Exp(1): layer = lo[11:4], magnitude = (hi:lo)[63:12] (52 bits), lo[3:0] unused
// v = 1 + u (u = magnitude / 2^52) is built directly as a double from two
// v_alignbit_b32, and x = fma(v, W, −W) = u·W is one rounding (the bits of
// (double)mag · W/2^52).
// N(0,1) table: 8-byte entries n[0..L] — n[0] = 0, n[j] = x_j (strip j's
// width, x_1 < … < x_{L−1} = r), n[L] = q (the base strip's width).  Layer ℓ
// reads the pair (n[ℓ], n[ℓ+1]) = (bound, width) of strip j = ℓ + 1 at byte
// address ℓ·8 (one ds_read2_b64): accepted iff |x| < bound, i.e. the point
// lies inside the strip's rectangle (layer L − 1 is the base strip, bound r;
// layer 0 the top strip, bound 0: never).  8192 layers in the LDS footprint
// 4096 16-byte entries took: 99.94 % of normals take the fast path (4096:
// 99.88 %), so a wave drawing 1024 normals needs a rare-path pass on ≈ 45 %
// of its steps instead of ≈ 70 %.
// Exp(1) table: 16-byte entries (kv, w), accepted iff v < kv = 1 + k/2^52 (the
// integer test mag < k, exactly).  Wedge/tail draws use the portable log/exp
// above with fresh counter blocks.  Tables are built on the host by
// build_ziggurat() (oracle/ restates the same construction).
constexpr int kZigNL = 8192;                        // normal layers
constexpr double kZigNR = 4.548600609949139;        // normal: rightmost strip edge r (8192 layers)
constexpr double kZigNV = 1.5303723494629906e-4;    // normal: area per strip v
constexpr double kZigNInvR = 1.0 / 4.548600609949139;
constexpr double kZigER = 7.69711747013104972;      // exponential: r (256 layers)
constexpr double kZigEV = 3.949659822581572e-3;     // exponential: v

struct ZigEntry {
    double kv;  // 1 + k/2^bits: fast-accept bound on v = 1 + u
    double w;   // layer width x_i (base layer: q = v/f(r))
};
// Layout: the prefix [n, e, ef] is what the step kernels stage into LDS
// (70 KiB; n first, at LDS address 0, so both reads of a layer's pair fold
// into one ds_read2_b64 on the layer's byte offset); nf is read from global
// memory on the rare path only.
struct Ziggurat {
    double n[kZigNL + 2];  // n[0] = 0, n[j] = x_j (1 ≤ j < L), n[L] = q, n[L+1] = 0 (pad)
    ZigEntry e[256];
    double ef[256];          // exp(−x_i)
    double nf[kZigNL + 2];   // nf[j] = f(x_j) = exp(−x_j²/2), nf[0] = 1 (x_0 = 0)
};
constexpr size_t kZigLdsBytes = offsetof(Ziggurat, nf);

// Where a kernel finds the tables (LDS prefix + global nf, or all global).
struct ZigTabs {
    const double *n;
    const double *nf;
    const ZigEntry *e;
    const double *ef;
};
EMCMC_HD ZigTabs zig_tabs(const Ziggurat &z) { return ZigTabs{z.n, z.nf, z.e, z.ef}; }
#ifndef __HIPCC_RTC__  // host-side table construction
inline void build_ziggurat(Ziggurat &z) {
    {  // N(0,1), f(x) = exp(−x²/2): strips x_{L−1} = r down to x_1, then x_0 = 0
        constexpr int L = kZigNL;
        double dn = kZigNR;
        const double q = kZigNV / exp_nonpos(-0.5 * (dn * dn));
        z.n[0] = 0.0;
        z.n[L - 1] = dn;
        z.n[L] = q;
        z.n[L + 1] = 0.0;
        z.nf[0] = 1.0;
        z.nf[L - 1] = exp_nonpos(-0.5 * (dn * dn));
        z.nf[L] = z.nf[L - 1];
        z.nf[L + 1] = 0.0;
        for (int i = L - 2; i >= 1; --i) {
            dn = sqrt(-2.0 * log_pos(kZigNV / dn + exp_nonpos(-0.5 * (dn * dn))));
            z.nf[i] = exp_nonpos(-0.5 * (dn * dn));
            z.n[i] = dn;
        }
    }
    {  // Exp(1), f(x) = exp(−x), 52-bit magnitudes
        const double m = 0x1p52;
        auto kv = [](uint64_t k) { return u2d(0x3FF0000000000000ull | k); };
        double de = kZigER, te = de;
        const double q = kZigEV / exp_nonpos(-de);
        z.e[0].kv = kv((uint64_t)((de / q) * m));
        z.e[1].kv = kv(0);
        z.e[0].w = q;
        z.e[255].w = de;
        z.ef[0] = 1.0;
        z.ef[255] = exp_nonpos(-de);
        for (int i = 254; i >= 1; --i) {
            de = -log_pos(kZigEV / de + exp_nonpos(-de));
            z.e[i + 1].kv = kv((uint64_t)((de / te) * m));
            te = de;
            z.ef[i] = exp_nonpos(-de);
            z.e[i].w = de;
        }
    }
}
#endif

struct ZigDraw {
    uint32_t off;   // byte offset of the layer's ZigEntry (layer · 16)
    uint32_t sbit;  // sign in bit 31 (normals)
    double v;       // 1 + u
};
// N(0,1) draw: layer lo[12:0] (off = ℓ·8), magnitude (hi:lo)[63:12], sign lo[13]
EMCMC_HD ZigDraw zig_split_n(uint32_t hi, uint32_t lo) {
    ZigDraw d;
    d.off = (lo << 3) & 0xFFF8u;
    d.sbit = (lo << 18) & 0x80000000u;
#if defined(__HIP_DEVICE_COMPILE__)
    const uint32_t vlo = __builtin_amdgcn_alignbit(hi, lo, 12);
    const uint32_t vhi = __builtin_amdgcn_alignbit(0x3FFu, hi, 12);
#else
    const uint32_t vlo = (hi << 20) | (lo >> 12);
    const uint32_t vhi = 0x3FF00000u | (hi >> 12);
#endif
    d.v = u2d(((uint64_t)vhi << 32) | vlo);
    return d;
}
// Exp(1) draw: layer lo[11:4], magnitude (hi:lo)[63:12]
EMCMC_HD ZigDraw zig_split_e(uint32_t hi, uint32_t lo) {
    ZigDraw d;
    d.off = lo & 0xFF0u;
    d.sbit = 0;
#if defined(__HIP_DEVICE_COMPILE__)
    const uint32_t vlo = __builtin_amdgcn_alignbit(hi, lo, 12);
    const uint32_t vhi = __builtin_amdgcn_alignbit(0x3FFu, hi, 12);
#else
    const uint32_t vlo = (hi << 20) | (lo >> 12);
    const uint32_t vhi = 0x3FF00000u | (hi >> 12);
#endif
    d.v = u2d(((uint64_t)vhi << 32) | vlo);
    return d;
}
EMCMC_HD uint32_t zig_layer(const ZigDraw &d) { return d.off >> 4; }    // Exp(1) draws
EMCMC_HD uint32_t zig_layer_n(const ZigDraw &d) { return d.off >> 3; }  // N(0,1) draws: ℓ
EMCMC_HD const ZigEntry &zig_entry(const ZigEntry *tab, const ZigDraw &d) {
    return *reinterpret_cast<const ZigEntry *>(reinterpret_cast<const char *>(tab) + d.off);
}
// (bound, width) of the strip of N(0,1) layer ℓ: (n[ℓ], n[ℓ+1])
struct ZigNPair {
    double b, w;
};
EMCMC_HD ZigNPair zig_npair(const double *tab, const ZigDraw &d) {
    const double *p = reinterpret_cast<const double *>(reinterpret_cast<const char *>(tab) + d.off);
    return ZigNPair{p[0], p[1]};
}
EMCMC_HD double with_sign(double x, uint32_t sbit) { return u2d(d2u(x) | ((uint64_t)sbit << 32)); }
// u·W with one rounding (v = 1 + u exactly)
EMCMC_HD double zig_scale(double v, double w) { return fma(v, w, -w); }

constexpr uint32_t kFaultRngRetries = 2u;  // EMCMC_FAULT_RNG_RETRIES
constexpr uint32_t kMaxAttempt = 0xFFFFu;

EMCMC_HD bool zig_normal_fast(ZigDraw d, const double *tab, double &z) {
    const ZigNPair t = zig_npair(tab, d);
    z = zig_scale(d.v, with_sign(t.w, d.sbit));
    return fabs(z) < t.b;
}

// Rare path of normal number `gj` of (chain, iter, pidx0) whose attempt-0
// draw `d` failed the fast test.  Slow step k uses the counter block
// (pair = gj/2, attempt = 1 + 2k + gj%2), so the two normals of a pair never
// share a block.
EMCMC_HD double zig_normal_slow(ZigDraw d, const double *tab, const double *f, uint32_t key0, uint32_t key1,
                                uint32_t chain, uint32_t iter, uint32_t pidx0, uint32_t gj, uint32_t &faults) {
    const uint32_t pair = gj >> 1, h = gj & 1u;
    for (uint32_t k = 0;; ++k) {
        const uint32_t attempt = 1u + 2u * k + h;
        if (attempt > kMaxAttempt) {
            faults |= kFaultRngRetries;
            return 0.0;
        }
        const u32x4 b = draw(key0, key1, chain, iter, pair, pidx0, attempt);
        const uint32_t j = zig_layer_n(d) + 1u;  // strip
        if (j == (uint32_t)kZigNL) {  // base strip beyond the rectangle: tail x > r
            const double xx = -log_pos(u01_open0(b.x, b.y)) * kZigNInvR;
            const double yy = -log_pos(u01_open0(b.z, b.w));
            if (yy + yy > xx * xx) return with_sign(kZigNR + xx, d.sbit);
        } else {  // wedge test, else a fresh draw
            const double x = zig_scale(d.v, tab[j]);
            const double u = u01_closed0(b.x, b.y);
            if (fma(u, f[j - 1] - f[j], f[j]) < exp_nonpos(-0.5 * (x * x))) return with_sign(x, d.sbit);
            d = zig_split_n(b.z, b.w);
            double z;
            if (zig_normal_fast(d, tab, z)) return z;
        }
    }
}

EMCMC_HD bool zig_exp_fast(ZigDraw d, const ZigEntry *tab, double &e) {
    const ZigEntry t = zig_entry(tab, d);
    e = zig_scale(d.v, t.w);
    return d.v < t.kv;
}

// Rare path of an Exp(1) draw: slow step k uses the block (mcmciter, attempt 1 + k).
EMCMC_HD double zig_exp_slow(ZigDraw d, const ZigEntry *tab, const double *f, uint32_t key0, uint32_t key1,
                             uint32_t chain, uint32_t iter, uint32_t block, uint32_t pidx0, uint32_t &faults) {
    for (uint32_t k = 0;; ++k) {
        const uint32_t attempt = 1u + k;
        if (attempt > kMaxAttempt) {
            faults |= kFaultRngRetries;
            return 0.0;
        }
        const u32x4 b = draw(key0, key1, chain, iter, block, pidx0, attempt);
        const uint32_t L = zig_layer(d);
        if (L == 0) return kZigER - log_pos(u01_open0(b.x, b.y));
        const double x = zig_scale(d.v, tab[L].w);
        const double u = u01_closed0(b.x, b.y);
        if (fma(u, f[L - 1] - f[L], f[L]) < exp_nonpos(-x)) return x;
        d = zig_split_e(b.z, b.w);
        double e;
        if (zig_exp_fast(d, tab, e)) return e;
    }
}

// The attempt-0 draw of the accept exponential of `iter` (shared block, see
// kBlockAccept).
EMCMC_HD ZigDraw accept_split(const u32x4 &r, uint32_t iter) {
    return (iter & 1u) ? zig_split_e(r.z, r.w) : zig_split_e(r.x, r.y);
}

// Scalar reference forms (probes, host code): the full draw of normal gj and
// of the accept exponential.
EMCMC_HD double normal_draw(const ZigTabs &zt, uint32_t key0, uint32_t key1, uint32_t chain, uint32_t iter,
                            uint32_t pidx0, uint32_t gj, uint32_t &faults) {
    const u32x4 r = draw(key0, key1, chain, iter, gj >> 1, pidx0, 0);
    const ZigDraw d = (gj & 1u) ? zig_split_n(r.z, r.w) : zig_split_n(r.x, r.y);
    double z;
    if (zig_normal_fast(d, zt.n, z)) return z;
    return zig_normal_slow(d, zt.n, zt.nf, key0, key1, chain, iter, pidx0, gj, faults);
}
EMCMC_HD double exp_draw(const ZigTabs &zt, uint32_t key0, uint32_t key1, uint32_t chain, uint32_t iter,
                         uint32_t pidx0, uint32_t &faults) {
    const u32x4 r = draw(key0, key1, chain, iter >> 1, kBlockAccept, pidx0, 0);
    const ZigDraw d = accept_split(r, iter);
    double e;
    if (zig_exp_fast(d, zt.e, e)) return e;
    return zig_exp_slow(d, zt.e, zt.ef, key0, key1, chain, iter, kBlockAccept, pidx0, faults);
}

// log(2π) rounded to double, Float64(log2π) in Distributions' mvnormal_c0.
constexpr double kLog2Pi = 1.8378770664093454835606594728112;

}  // namespace emcmc
