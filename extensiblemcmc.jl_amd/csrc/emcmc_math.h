// emcmc_math.h — bit-reproducible fp64 math shared by the host side of
// libemcmc.so and its gfx950 kernels.
//
// Why this exists: parity with the CPU oracle is defined bit-for-bit on the
// accept/reject stream (BASELINE.json north_star).  Device libm (ocml) and
// host glibc disagree in the last ulp for log/sin/cos, so every
// transcendental on the hot path is built here from IEEE basic operations
// (+ − × ÷ and sqrt, all correctly rounded on both sides) and compiled with
// -ffp-contract=off.  The variate stream itself is counter-based
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

#include <stdint.h>
#include <math.h>

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

EMCMC_HD u32x4 philox4x32_10(u32x4 c, uint32_t k0, uint32_t k1) {
    const uint32_t M0 = 0xD2511F53u, M1 = 0xCD9E8D57u;
    const uint32_t W0 = 0x9E3779B9u, W1 = 0xBB67AE85u;
#pragma unroll
    for (int r = 0; r < 10; ++r) {
        // full 32×32→64 products: one v_mad_u64_u32 each on gfx950
        const uint64_t p0 = (uint64_t)M0 * (uint64_t)c.x;
        const uint64_t p1 = (uint64_t)M1 * (uint64_t)c.z;
        u32x4 n;
        n.x = (uint32_t)(p1 >> 32) ^ c.y ^ k0;
        n.y = (uint32_t)p1;
        n.z = (uint32_t)(p0 >> 32) ^ c.w ^ k1;
        n.w = (uint32_t)p0;
        c = n;
        k0 += W0;
        k1 += W1;
    }
    return c;
}

// Counter layout of the shared stream:
//   x = global chain id, y = mcmciter (1-based), z = block, w = (pidx << 16) | attempt
// Blocks: normal pair j → z = j; accept uniform → z = kBlockAccept.
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

// ---- sin/cos kernels on [0, π/4] (FreeBSD msun k_sin.c / k_cos.c
// coefficients, y = 0, fma Horner) ---------------------------------------------
EMCMC_HD double ksin(double x) {
    const double S1 = -1.66666666666666324348e-01, S2 = 8.33333333332248946124e-03,
                 S3 = -1.98412698298579493134e-04, S4 = 2.75573137070700676789e-06,
                 S5 = -2.50507602534068634195e-08, S6 = 1.58969099521155010221e-10;
    const double z = x * x;
    double p = fma(z, S6, S5);
    p = fma(z, p, S4);
    p = fma(z, p, S3);
    p = fma(z, p, S2);
    p = fma(z, p, S1);
    return fma(z * x, p, x);
}
EMCMC_HD double kcos(double x) {
    const double C1 = 4.16666666666666019037e-02, C2 = -1.38888888888741095749e-03,
                 C3 = 2.48015872894767294178e-05, C4 = -2.75573143513906633035e-07,
                 C5 = 2.08757232129817482790e-09, C6 = -1.13596475577881948265e-11;
    const double z = x * x;
    double p = fma(z, C6, C5);
    p = fma(z, p, C4);
    p = fma(z, p, C3);
    p = fma(z, p, C2);
    p = fma(z, p, C1);
    const double r = z * p;
    const double hz = 0.5 * z;
    const double w = 1.0 - hz;
    return w + fma(z, r, (1.0 - w) - hz);
}

// ---- Box–Muller pair from one Philox block ----------------------------------
// radius from (x,y): r = sqrt(-2 log u), u ∈ (0,1]
// angle from (z,w): a 53-bit turn fraction; quadrant = top 2 bits, the
// remaining 51 bits are folded to [0, π/4] exactly in integer arithmetic.
EMCMC_HD void box_muller(u32x4 r, double &z0, double &z1) {
    const double u = u01_open0(r.x, r.y);
    const double rad = sqrt(-2.0 * log_pos(u));
    const uint64_t b = bits53(r.z, r.w);
    const uint32_t q = (uint32_t)(b >> 51);
    const uint64_t rem = b & ((1ull << 51) - 1ull);
    const bool fold = rem >= (1ull << 50);
    const uint64_t rr = fold ? ((1ull << 51) - rem) : rem;
    const double x = (double)rr * 0x1.921fb54442d18p-51;  // rr · (π/2)·2^-51 ∈ [0, π/4]
    const double s = ksin(x), c = kcos(x);
    // angle = q·π/2 + φ, φ = fold ? π/2 − x : x.  Branch-free: pick magnitudes,
    // then flip sign bits (exact negation).
    const bool t = ((q & 1u) != 0) != fold;
    const double mc = t ? s : c;
    const double ms = t ? c : s;
    const uint64_t negc = (uint64_t)(((q >> 1) ^ q) & 1u) << 63;
    const uint64_t negs = (uint64_t)((q >> 1) & 1u) << 63;
    z0 = rad * u2d(d2u(mc) ^ negc);
    z1 = rad * u2d(d2u(ms) ^ negs);
}

// Exponential(1) draw for accept_reject! (run.jl:278): E = −log(u), u ∈ (0,1].
EMCMC_HD double exp1(u32x4 r) { return -log_pos(u01_open0(r.x, r.y)); }

// log(2π) rounded to double, Float64(log2π) in Distributions' mvnormal_c0.
constexpr double kLog2Pi = 1.8378770664093454835606594728112;

}  // namespace emcmc
