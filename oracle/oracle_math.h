/*
 * oracle_math.h — TEST INFRASTRUCTURE ONLY (see oracle/README.md).
 *
 * Plain-C restatement of the variate stream and the fp64 kernels that the
 * engine defines for the MH hot path.  It is written independently of the
 * product header (extensiblemcmc.jl_amd/csrc/emcmc_math.h); bitwise agreement
 * between the two is what tests/ check.
 *
 * Published algorithms restated here:
 *  - Philox4x32-10: Salmon, Moraes, Dror & Shaw, "Parallel random numbers: as
 *    easy as 1, 2, 3", SC'11 (Random123).  Pinned by the Random123 known-answer
 *    vectors in tests/golden/philox_kat.json.
 *  - natural log: fdlibm e_log.c argument reduction + Lg1..Lg7 polynomial,
 *    evaluated with the single formula of its main branch.
 *  - sin/cos on [0, π/4]: FreeBSD msun k_sin.c / k_cos.c (y = 0).
 *  - Box–Muller transform (radius from one 53-bit uniform in (0,1], angle from
 *    a 53-bit turn fraction folded to [0, π/4] in integer arithmetic).
 *
 * The reference (Julia) draws from Random.GLOBAL_RNG via Distributions
 * (src/transition_kernels/random_walk.jl:147, src/run.jl:278); that stream
 * cannot be reproduced without Julia, so "identical seeds" is defined on this
 * counter-based stream (SURVEY.md §7 "Hard parts" 1).
 */
#ifndef ORACLE_MATH_H
#define ORACLE_MATH_H

#include <math.h>
#include <stdint.h>
#include <string.h>

typedef struct {
    uint32_t v[4];
} orc_u32x4;

static inline uint64_t orc_d2u(double x) {
    uint64_t u;
    memcpy(&u, &x, 8);
    return u;
}
static inline double orc_u2d(uint64_t u) {
    double x;
    memcpy(&x, &u, 8);
    return x;
}

static inline orc_u32x4 orc_philox4x32_10(orc_u32x4 ctr, uint32_t key0, uint32_t key1) {
    uint32_t k[2] = {key0, key1};
    uint32_t c[4] = {ctr.v[0], ctr.v[1], ctr.v[2], ctr.v[3]};
    for (int round = 0; round < 10; ++round) {
        if (round > 0) {
            k[0] += 0x9E3779B9u; /* golden ratio */
            k[1] += 0xBB67AE85u; /* sqrt(3) - 1 */
        }
        uint64_t p0 = (uint64_t)0xD2511F53u * (uint64_t)c[0];
        uint64_t p1 = (uint64_t)0xCD9E8D57u * (uint64_t)c[2];
        uint32_t n0 = (uint32_t)(p1 >> 32) ^ c[1] ^ k[0];
        uint32_t n1 = (uint32_t)p1;
        uint32_t n2 = (uint32_t)(p0 >> 32) ^ c[3] ^ k[1];
        uint32_t n3 = (uint32_t)p0;
        c[0] = n0;
        c[1] = n1;
        c[2] = n2;
        c[3] = n3;
    }
    orc_u32x4 out = {{c[0], c[1], c[2], c[3]}};
    return out;
}

/* Counter layout: (chain id, mcmciter, block, (pidx0 << 16) | attempt). */
#define ORC_BLOCK_ACCEPT 0xFFFFFFFFu

static inline orc_u32x4 orc_draw(uint32_t key0, uint32_t key1, uint32_t chain, uint32_t iter,
                                 uint32_t block, uint32_t pidx0, uint32_t attempt) {
    orc_u32x4 c = {{chain, iter, block, (pidx0 << 16) | (attempt & 0xFFFFu)}};
    return orc_philox4x32_10(c, key0, key1);
}

static inline uint64_t orc_bits53(uint32_t hi, uint32_t lo) {
    return ((uint64_t)hi << 21) | (uint64_t)(lo >> 11);
}
static inline double orc_u01_open0(uint32_t hi, uint32_t lo) {
    return (double)(orc_bits53(hi, lo) + 1u) * 0x1p-53;
}
static inline double orc_u01_closed0(uint32_t hi, uint32_t lo) {
    return (double)orc_bits53(hi, lo) * 0x1p-53;
}

/* log for finite normal x > 0: fdlibm e_log.c reduction, main-branch formula,
 * Lg polynomial in fma Horner form. */
static inline double orc_log(double x) {
    static const double ln2_hi = 6.93147180369123816490e-01, ln2_lo = 1.90821492927058770002e-10,
                        Lg1 = 6.666666666666735130e-01, Lg2 = 3.999999999940941908e-01,
                        Lg3 = 2.857142874366239149e-01, Lg4 = 2.222219843214978396e-01,
                        Lg5 = 1.818357216161805012e-01, Lg6 = 1.531383769920937332e-01,
                        Lg7 = 1.479819860511658591e-01;
    uint64_t bits = orc_d2u(x);
    int32_t hx = (int32_t)(bits >> 32);
    uint32_t lx = (uint32_t)bits;
    int32_t k = (hx >> 20) - 1023;
    hx &= 0x000fffff;
    int32_t i = (hx + 0x95f64) & 0x100000;
    double m = orc_u2d(((uint64_t)(uint32_t)(hx | (i ^ 0x3ff00000)) << 32) | lx);
    k += (i >> 20);
    double f = m - 1.0;
    double s = f / (2.0 + f);
    double dk = (double)k;
    double z = s * s;
    double w = z * z;
    double t1 = w * fma(w, fma(w, Lg6, Lg4), Lg2);
    double t2 = z * fma(w, fma(w, fma(w, Lg7, Lg5), Lg3), Lg1);
    double R = t2 + t1;
    double hfsq = 0.5 * f * f;
    return dk * ln2_hi - ((hfsq - fma(s, hfsq + R, dk * ln2_lo)) - f);
}

/* sin on [0, π/4]: x + x³·P(x²), FreeBSD k_sin.c coefficients S1..S6. */
static inline double orc_sin_k(double x) {
    static const double S[6] = {-1.66666666666666324348e-01, 8.33333333332248946124e-03,
                                -1.98412698298579493134e-04, 2.75573137070700676789e-06,
                                -2.50507602534068634195e-08, 1.58969099521155010221e-10};
    double z = x * x;
    double p = fma(z, S[5], S[4]);
    for (int j = 3; j >= 0; --j) p = fma(z, p, S[j]);
    return fma(z * x, p, x);
}

/* cos on [0, π/4]: 1 − z/2 + z²·P(z), FreeBSD k_cos.c coefficients C1..C6,
 * with the compensated 1 − z/2 step. */
static inline double orc_cos_k(double x) {
    static const double Cc[6] = {4.16666666666666019037e-02, -1.38888888888741095749e-03,
                                 2.48015872894767294178e-05, -2.75573143513906633035e-07,
                                 2.08757232129817482790e-09, -1.13596475577881948265e-11};
    double z = x * x;
    double p = fma(z, Cc[5], Cc[4]);
    for (int j = 3; j >= 0; --j) p = fma(z, p, Cc[j]);
    double r = z * p;
    double hz = 0.5 * z;
    double one_minus = 1.0 - hz;
    return one_minus + fma(z, r, (1.0 - one_minus) - hz);
}

/* cos and sin of a 53-bit turn fraction (angle = 2π·turn/2^53). */
static inline void orc_sincos_turn(uint64_t turn, double *cz, double *sz) {
    uint32_t quadrant = (uint32_t)(turn >> 51);
    uint64_t rem = turn & ((1ull << 51) - 1u);
    int folded = rem >= (1ull << 50);
    uint64_t rr = folded ? ((1ull << 51) - rem) : rem;
    double x = (double)rr * 0x1.921fb54442d18p-51;
    double s = orc_sin_k(x), c = orc_cos_k(x);
    double sin_phi = folded ? c : s;
    double cos_phi = folded ? s : c;
    switch (quadrant) {
    case 0: *cz = cos_phi; *sz = sin_phi; break;
    case 1: *cz = -sin_phi; *sz = cos_phi; break;
    case 2: *cz = -cos_phi; *sz = -sin_phi; break;
    default: *cz = sin_phi; *sz = -cos_phi; break;
    }
}

/* Two independent N(0,1) variates from one Philox block. */
static inline void orc_box_muller(orc_u32x4 r, double *z0, double *z1) {
    double u = orc_u01_open0(r.v[0], r.v[1]);
    double radius = sqrt(-2.0 * orc_log(u));
    double cz, sz;
    orc_sincos_turn(orc_bits53(r.v[2], r.v[3]), &cz, &sz);
    *z0 = radius * cz;
    *z1 = radius * sz;
}

/* rand(Exponential(1.0)) of run.jl:278 restated as −log(u), u ∈ (0,1]. */
static inline double orc_exp1(orc_u32x4 r) { return -orc_log(orc_u01_open0(r.v[0], r.v[1])); }

#define ORC_LOG2PI 1.8378770664093454835606594728112

#endif
