// emcmc_kernels.h — fused many-chain Metropolis–Hastings step kernels (gfx950).
//
// One launch runs `nsteps` consecutive schedule steps of ONE update for all
// chains; θ, ll and the rolling-acceptance state stay in VGPRs across those
// steps and only the per-step history streams leave the CU.  The step loop
// issues no vector-memory loads: on gfx950 loads and stores share vmcnt, so a
// load inside the loop would make every step wait for the previous step's
// history stores to drain.  Each chain is
// owned by LPC ∈ {1,2,4} adjacent lanes of a wave (a "quad" for LPC=4), each
// lane holding D/LPC coordinates; per-chain sums combine across those lanes
// with DPP quad permutes.
//
// Per step and chain this fuses (reference src/ paths):
//   update_workspaces!        run.jl:101-112    (register carry of θ and ll)
//   proposal!/rand!           updates.jl:191-196, random_walk.jl:145-159
//   set_proposal!             run.jl:221-240    (state_proposal_history write)
//   compute_ll!/loglikelihood run.jl:251-260, gsn_target.jl:23-29
//   accept_reject!            run.jl:268-281    (llr order, Exponential draw)
//   log_transition_density    run.jl:344-367, random_walk.jl:161-171
//   log_prior                 run.jl:374-385, priors.jl:18-19
//   register_accept_reject_results!/set_chain_param!  run.jl:299-335
//   update_stats! rolling acceptance  chain_statistics.jl:51-65
//
// Summation order (defines the bits, shared with oracle/): a length-D sum is
// split into blocks of 8 consecutive coordinates when D % 8 == 0 and D ≥ 16
// (else one block); each block sums left to right; blocks combine by a
// pairwise tree over adjacent blocks (odd tail carried up).  See DESIGN.md.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include "emcmc_math.h"

namespace emcmc {

struct StepParams {
    // carried chain state (SoA over chains, row-major [C][D] for θ)
    double *theta;     // [C][D]
    double *ll;        // [C]
    double *ra;        // [C] rolling acceptance (current value)
    uint64_t *ring;    // [C][2] acceptance bits of the last 128 iterations
    uint32_t *nacc;    // [C] accepted proposals
    uint32_t *faults;  // [C]
    // history streams (FULL mode), slot = (mcmciter-1)*P + pidx0
    double *hist_theta;  // [M*P][C][D]
    double *hist_prop;   // [M*P][C][D]
    double *hist_ll;     // [M*P][C]
    uint8_t *hist_acc;   // [M*P][Cw*8] bytes, bit c of row = chain c
    // device constants (see DeviceConsts layout in emcmc.hip)
    const Ziggurat *zig;  // N(0,1) / Exp(1) ziggurat tables (host-built)
    const double *consts;
    const double *obs;    // [nobs][D]
    uint64_t C;
    uint64_t row_bytes;   // bytes per accept-bit row (= Cw*8)
    uint32_t chain0;      // global id of local chain 0
    uint32_t key0, key1;  // seed
    uint32_t iter0;
    uint32_t nsteps;
    uint32_t pidx0;       // 0-based update index
    uint32_t P;           // number of updates
    uint32_t W;           // roll window (≤ 128)
    uint32_t nobs;
    uint32_t _pad;
    uint64_t N0;          // GenericChainStats.N before the first step of this launch
    double rw_c0;         // −(D·log2π + logdet Σ_rw)/2
    double t_c0;          // −(D·log2π + logdet Σ_t)/2
    double n_tc0;         // nobs · t_c0     (SUFFSTAT)
    double S_c;           // Σ_k ‖L_t⁻¹(x_k − x̄)‖²  (SUFFSTAT)
    double nobs_d;        // (double) nobs
};

// constants layout (offsets in doubles), D = dimension
//   diag kernels : [0,D) L_rw diag | [D,2D) 1/L_rw | [2D,3D) 1/L_t | [3D,4D) x̄
//   dense kernels: [0,D²) L_rw (row-major lower) | [D²,D²+D) 1/diag(L_rw)
//                  | [D²+D, 2D²+D) L_t | [2D²+D, 2D²+2D) 1/diag(L_t) | [2D²+2D, 2D²+3D) x̄
constexpr int LL_PER_OBS = 0;
constexpr int LL_SUFFSTAT = 1;

// HBM layout of θ state and θ/θ° histories (per history slot): pair-interleaved
// SoA, element (d, c) at ((d/2)·C + c)·2 + d%2 when D is even, so lane c stores
// the Box–Muller pair (2j, 2j+1) as one 16-byte word and a wave's store covers
// contiguous 1 KiB (LPC = 1) or 4 × 256 B (LPC = 4).  Odd D: plain SoA d·C + c.
__host__ __device__ __forceinline__ uint64_t state_pos(uint64_t d, uint64_t c, uint64_t C, uint32_t D) {
    return (D % 2 == 0) ? (((d >> 1) * C + c) << 1) + (d & 1) : d * C + c;
}

typedef double d2v __attribute__((ext_vector_type(2)));

// Stage the ziggurat tables (12 KiB, 16-byte aligned at LDS offset 0) and then
// `nconst` constants and `nobs_d` observation doubles behind them.
constexpr int kZigLdsDoubles = (int)(sizeof(Ziggurat) / sizeof(double));
__device__ __forceinline__ void stage_lds(double *lds, const Ziggurat *zig, const double *consts, int nconst,
                                          const double *obs, int nobs_d) {
    const double *zsrc = reinterpret_cast<const double *>(zig);
    const int total = kZigLdsDoubles + nconst + nobs_d;
    for (int i = threadIdx.x; i < total; i += blockDim.x) {
        double v;
        if (i < kZigLdsDoubles) v = zsrc[i];
        else if (i < kZigLdsDoubles + nconst) v = consts[i - kZigLdsDoubles];
        else v = obs[i - kZigLdsDoubles - nconst];
        lds[i] = v;
    }
    __syncthreads();
}

#ifndef EMCMC_SERIAL_PAIRS
#define EMCMC_SERIAL_PAIRS 1
#endif
// 1: keep the scheduler from interleaving the Philox blocks of different
// pairs (register pressure → occupancy; the waves of a SIMD supply the ILP)
constexpr bool kSerialPairs = EMCMC_SERIAL_PAIRS != 0;

// N normals of (chain, iter, pidx0) with lane-local index i ↔ global normal
// index g0 + i, written as out[i] = base[i] + scale[i]·z (the diagonal
// proposal θ° = θ + L z, random_walk.jl:147).  Fast pass over all pairs, then
// a wave-uniform loop resolves the ≈1% wedge/tail draws one per lane per trip.
template <int N>
__device__ __forceinline__ void propose_diag(const Ziggurat &zt, uint32_t key0, uint32_t key1, uint32_t chain,
                                             uint32_t iter, uint32_t pidx0, uint32_t g0, const double (&base)[N],
                                             const double *scale, double (&out)[N], uint32_t &faults) {
    constexpr int NP = (N + 1) / 2;
    uint64_t pend = 0;
#pragma unroll
    for (int j = 0; j < NP; ++j) {
        if constexpr (kSerialPairs) __builtin_amdgcn_sched_barrier(0);
        const u32x4 r = draw(key0, key1, chain, iter, (g0 >> 1) + j, pidx0, 0);
        double z0, z1;
        const bool ok0 = zig_normal_fast(zig_split(r.x, r.y), zt.n, z0);
        out[2 * j] = base[2 * j] + scale[2 * j] * z0;
        if (!ok0) pend |= 1ull << (2 * j);
        if (2 * j + 1 < N) {
            const bool ok1 = zig_normal_fast(zig_split(r.z, r.w), zt.n, z1);
            out[2 * j + 1] = base[2 * j + 1] + scale[2 * j + 1] * z1;
            if (!ok1) pend |= 1ull << (2 * j + 1);
        }
    }
    while (__ballot(pend != 0) != 0) {
        if (pend != 0) {
            const int i = __builtin_ctzll(pend);
            pend &= pend - 1;
            const double z = normal_draw(zt, key0, key1, chain, iter, pidx0, g0 + (uint32_t)i, faults);
#pragma unroll
            for (int q = 0; q < N; ++q)
                if (q == i) out[q] = base[q] + scale[q] * z;
        }
    }
}

// The N standard normals themselves (dense-L proposals).
template <int N>
__device__ __forceinline__ void normals(const Ziggurat &zt, uint32_t key0, uint32_t key1, uint32_t chain,
                                        uint32_t iter, uint32_t pidx0, double (&z)[N], uint32_t &faults) {
    constexpr int NP = (N + 1) / 2;
    uint64_t pend = 0;
#pragma unroll
    for (int j = 0; j < NP; ++j) {
        const u32x4 r = draw(key0, key1, chain, iter, j, pidx0, 0);
        if (!zig_normal_fast(zig_split(r.x, r.y), zt.n, z[2 * j])) pend |= 1ull << (2 * j);
        if (2 * j + 1 < N)
            if (!zig_normal_fast(zig_split(r.z, r.w), zt.n, z[2 * j + 1])) pend |= 1ull << (2 * j + 1);
    }
    while (__ballot(pend != 0) != 0) {
        if (pend != 0) {
            const int i = __builtin_ctzll(pend);
            pend &= pend - 1;
            const double v = normal_draw(zt, key0, key1, chain, iter, pidx0, (uint32_t)i, faults);
#pragma unroll
            for (int q = 0; q < N; ++q)
                if (q == i) z[q] = v;
        }
    }
}

// Exp(1) draw of the accept test (run.jl:278).
__device__ __forceinline__ double accept_exp(const Ziggurat &zt, uint32_t key0, uint32_t key1, uint32_t chain,
                                             uint32_t iter, uint32_t pidx0, uint32_t &faults) {
    const u32x4 r = draw(key0, key1, chain, iter, kBlockAccept, pidx0, 0);
    const ZigDraw d = zig_split(r.x, r.y);
    double e;
    if (!zig_exp_fast(d, zt.e, e))
        e = zig_exp_slow(d, zt.e, zt.ef, key0, key1, chain, iter, kBlockAccept, pidx0, faults);
    return e;
}

// ---------------------------------------------------------------------------
// cross-lane helpers (DPP quad permutes; 64-bit values move as two dwords)
template <int CTRL>
__device__ __forceinline__ double dpp_perm(double v) {
    const uint64_t b = __builtin_bit_cast(uint64_t, v);
    const int lo = __builtin_amdgcn_update_dpp(0, (int)(uint32_t)b, CTRL, 0xF, 0xF, false);
    const int hi = __builtin_amdgcn_update_dpp(0, (int)(uint32_t)(b >> 32), CTRL, 0xF, 0xF, false);
    return __builtin_bit_cast(double, ((uint64_t)(uint32_t)hi << 32) | (uint32_t)lo);
}
// quad_perm [1,0,3,2] = 0xB1 (xor 1), [2,3,0,1] = 0x4E (xor 2)
template <int LPC>
__device__ __forceinline__ double lane_tree(double s) {
    if constexpr (LPC >= 2) s = s + dpp_perm<0xB1>(s);
    if constexpr (LPC >= 4) s = s + dpp_perm<0x4E>(s);
    return s;
}

// canonical blocked-8 pairwise sum of the lane's NV values, then across lanes
template <int D>
struct SumShape {
    static constexpr int BLK = (D % 8 == 0 && D >= 16) ? 8 : D;
    static constexpr int NB = D / BLK;
};

template <int N>
__device__ __forceinline__ double tree_inplace(double (&b)[N]) {
    int n = N;
#pragma unroll
    for (int lvl = 0; lvl < 8; ++lvl) {
        if (n <= 1) break;
#pragma unroll
        for (int i = 0; i < N / 2; ++i)
            if (i < n / 2) b[i] = b[2 * i] + b[2 * i + 1];
        if (n & 1) b[n / 2] = b[n - 1];
        n = (n + 1) / 2;
    }
    return b[0];
}

// Σ y_i² over the chain's D coordinates in the canonical order: blocks of BLK
// accumulated s = y0·y0, s = fma(y_i, y_i, s); blocks combine pairwise, first
// inside the lane, then across the chain's LPC lanes.
template <int D, int LPC, int NV>
__device__ __forceinline__ double canon_sumsq(const double (&y)[NV]) {
    constexpr int BLK = SumShape<D>::BLK;
    constexpr int BPL = NV / BLK;
    double b[BPL];
#pragma unroll
    for (int k = 0; k < BPL; ++k) {
        double s = y[k * BLK] * y[k * BLK];
#pragma unroll
        for (int i = 1; i < BLK; ++i) s = fma(y[k * BLK + i], y[k * BLK + i], s);
        b[k] = s;
    }
    double s = tree_inplace<BPL>(b);
    return lane_tree<LPC>(s);
}

// compact one accept bit per chain out of a 64-lane ballot (LPC lanes/chain)
template <int LPC>
__device__ __forceinline__ uint64_t compact_ballot(uint64_t m) {
    if constexpr (LPC == 1) {
        return m;
    } else if constexpr (LPC == 2) {
        m &= 0x5555555555555555ull;
        m = (m | (m >> 1)) & 0x3333333333333333ull;
        m = (m | (m >> 2)) & 0x0F0F0F0F0F0F0F0Full;
        m = (m | (m >> 4)) & 0x00FF00FF00FF00FFull;
        m = (m | (m >> 8)) & 0x0000FFFF0000FFFFull;
        m = (m | (m >> 16)) & 0x00000000FFFFFFFFull;
        return m;
    } else {
        m &= 0x1111111111111111ull;
        m = (m | (m >> 3)) & 0x0303030303030303ull;
        m = (m | (m >> 6)) & 0x000F000F000F000Full;
        m = (m | (m >> 12)) & 0x000000FF000000FFull;
        m = (m | (m >> 24)) & 0x000000000000FFFFull;
        return m;
    }
}

template <int LPC>
__device__ __forceinline__ void store_acc_bits(uint8_t *row, uint64_t chain_first, uint64_t bits) {
    // chain_first is a multiple of 64/LPC: the wave's bits are one aligned word
    uint8_t *p = row + (chain_first >> 3);
    if constexpr (LPC == 1) *reinterpret_cast<uint64_t *>(p) = bits;
    else if constexpr (LPC == 2) *reinterpret_cast<uint32_t *>(p) = (uint32_t)bits;
    else *reinterpret_cast<uint16_t *>(p) = (uint16_t)bits;
}

// rolling acceptance, chain_statistics.jl:53-65 (N = cs.N before increment)
__device__ __forceinline__ double rolling_update(double ra, uint64_t &r0, uint64_t &r1, uint32_t iter,
                                                 uint32_t W, uint64_t N, bool acc) {
    int out = 0;
    if (iter > W) {
        const uint32_t j = (iter - W) & 127u;
        const uint64_t w = (j & 64u) ? r1 : r0;
        out = (int)((w >> (j & 63u)) & 1ull);
    }
    const uint64_t mn = (N < (uint64_t)W) ? N : (uint64_t)W;
    const double nra = (ra * (double)W + (double)((int)acc - out)) / (double)mn;
    const uint32_t jw = iter & 127u;
    const uint64_t bit = 1ull << (jw & 63u);
    if (jw & 64u) r1 = acc ? (r1 | bit) : (r1 & ~bit);
    else r0 = acc ? (r0 | bit) : (r0 & ~bit);
    return nra;
}

// ---------------------------------------------------------------------------
// Diagonal Gaussian RW proposal + diagonal Gaussian target (cfg 2 fast path).
// GaussianRandomWalk(Σ_rw) with Σ_rw diagonal, GsnTargetLaw(μ, Σ_t) with Σ_t
// diagonal, coords = 1:D, ImproperPrior, P = 1 schedule slot per step.
// UNIT_T: Σ_t = I, so L_t⁻¹ = I and the solve y = (x − μ)·1 is skipped (the
// product by 1.0 is exact: same bits).
// Store / load the lane's N coordinates [d0, d0+N) of chain c in state_pos
// layout; base points at the slot start.  Even D: 16-byte words.
template <int D, int N>
__device__ __forceinline__ void store_state(double *base, uint64_t C, uint64_t c, int d0, const double (&v)[N],
                                            bool nt) {
    if constexpr (D % 2 == 0) {
        static_assert(N % 2 == 0, "pairs");
#pragma unroll
        for (int j = 0; j < N / 2; ++j) {
            d2v x = {v[2 * j], v[2 * j + 1]};
            d2v *p = reinterpret_cast<d2v *>(base) + ((uint64_t)(d0 / 2 + j) * C + c);
            if (nt) __builtin_nontemporal_store(x, p);
            else *p = x;
        }
    } else {
#pragma unroll
        for (int i = 0; i < N; ++i) {
            double *p = base + (uint64_t)(d0 + i) * C + c;
            if (nt) __builtin_nontemporal_store(v[i], p);
            else *p = v[i];
        }
    }
}
template <int D, int N>
__device__ __forceinline__ void load_state(const double *base, uint64_t C, uint64_t c, int d0, double (&v)[N]) {
    if constexpr (D % 2 == 0) {
#pragma unroll
        for (int j = 0; j < N / 2; ++j) {
            const d2v x = reinterpret_cast<const d2v *>(base)[(uint64_t)(d0 / 2 + j) * C + c];
            v[2 * j] = x.x;
            v[2 * j + 1] = x.y;
        }
    } else {
#pragma unroll
        for (int i = 0; i < N; ++i) v[i] = base[(uint64_t)(d0 + i) * C + c];
    }
}

// MINW = minimum waves per SIMD the register allocation must allow
// (__launch_bounds__ second argument; 4 ⇒ ≤ 128 VGPRs).
template <int D, int LPC, bool FULL, int LLMODE, bool UNIT_T, int MINW = 1>
__global__ void __launch_bounds__(256, MINW) rwm_gsn_diag_kernel(const StepParams a) {
    static_assert(D % LPC == 0, "D must split evenly over the chain's lanes");
    constexpr int DPL = D / LPC;  // coordinates per lane
    static_assert(LPC == 1 || DPL % 8 == 0, "multi-lane chains need whole 8-blocks");
    static_assert(LPC == 1 || DPL % 2 == 0, "normal pairs must not straddle lanes");

    extern __shared__ __attribute__((aligned(16))) double lds[];
    const uint32_t nobs = a.nobs;
    const int nconst = 4 * D;
    stage_lds(lds, a.zig, a.consts, nconst, a.obs, (LLMODE == LL_PER_OBS) ? (int)nobs * D : 0);
    const Ziggurat &zt = *reinterpret_cast<const Ziggurat *>(lds);
    const double *cst = lds + kZigLdsDoubles;
    const double *Lrw = cst;
    const double *iLrw = cst + D;
    const double *iLt = cst + 2 * D;
    const double *xbar = cst + 3 * D;
    const double *X = cst + 4 * D;

    const uint64_t tid = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const uint64_t chain = tid / LPC;
    const int sub = (int)(tid % LPC);
    if (chain >= a.C) return;
    const int d0 = sub * DPL;
    const uint32_t gid = a.chain0 + (uint32_t)chain;

    const uint64_t C = a.C;
    double th[DPL];
    load_state<D>(a.theta, C, chain, d0, th);
    double ll = a.ll[chain];
    double ra = a.ra[chain];
    uint64_t r0 = a.ring[2 * chain], r1 = a.ring[2 * chain + 1];
    uint32_t nacc = a.nacc[chain];
    uint32_t faults = a.faults[chain];

    for (uint32_t s = 0; s < a.nsteps; ++s) {
        const uint32_t iter = a.iter0 + s;  // consecutive (host splits gaps)
        const uint64_t slot = (uint64_t)(iter - 1) * a.P + a.pidx0;
        // ---- proposal!: θ° = θ + L z, z ~ N(0, I) (random_walk.jl:145-151)
        double thp[DPL];
        propose_diag<DPL>(zt, a.key0, a.key1, gid, iter, a.pidx0, (uint32_t)d0, th, Lrw + d0, thp, faults);
        // ---- log_transition_density both ways (random_walk.jl:161-171):
        // sqmahal(θ°−θ) == sqmahal(θ−θ°) bitwise, so one evaluation serves both
        double ltd;
        {
            double y[DPL];
#pragma unroll
            for (int i = 0; i < DPL; ++i) y[i] = (thp[i] - th[i]) * iLrw[d0 + i];
            ltd = a.rw_c0 - canon_sumsq<D, LPC>(y) / 2.0;
        }
        // ---- compute_ll!: Σ_k logpdf(N(θ°, Σ_t), x_k) (gsn_target.jl:23-29)
        double llp;
        if constexpr (LLMODE == LL_PER_OBS) {
            llp = 0.0;
            for (uint32_t k = 0; k < nobs; ++k) {
                const double *xk = X + (size_t)k * D + d0;
                double y[DPL];
#pragma unroll
                for (int i = 0; i < DPL; ++i) {
                    y[i] = xk[i] - thp[i];
                    if constexpr (!UNIT_T) y[i] = y[i] * iLt[d0 + i];
                }
                llp = llp + (a.t_c0 - canon_sumsq<D, LPC>(y) / 2.0);
            }
        } else {
            double y[DPL];
#pragma unroll
            for (int i = 0; i < DPL; ++i) {
                y[i] = xbar[d0 + i] - thp[i];
                if constexpr (!UNIT_T) y[i] = y[i] * iLt[d0 + i];
            }
            const double qv = canon_sumsq<D, LPC>(y);
            llp = a.n_tc0 - (a.S_c + a.nobs_d * qv) * 0.5;
        }
        if (!(llp - llp == 0.0)) faults |= 1u;  // NaN or ±Inf
        // ---- accept_reject! (run.jl:271-278), left-associative as written
        const double llr = ((((llp - ll) + ltd) - ltd) + 0.0) - 0.0;
        const double E = accept_exp(zt, a.key0, a.key1, gid, iter, a.pidx0, faults);
        const bool acc = E > -llr;
        // ---- set_proposal! history: θ° with coords replaced (run.jl:237-239)
        if constexpr (FULL) store_state<D>(a.hist_prop + slot * D * C, C, chain, d0, thp, true);
        // ---- register_accept_reject_results! / set_chain_param! (run.jl:312-335)
#pragma unroll
        for (int i = 0; i < DPL; ++i) th[i] = acc ? thp[i] : th[i];
        ll = acc ? llp : ll;
        nacc += acc ? 1u : 0u;
        if constexpr (FULL) {
            store_state<D>(a.hist_theta + slot * D * C, C, chain, d0, th, true);
            if (sub == 0) __builtin_nontemporal_store(ll, a.hist_ll + slot * a.C + chain);
        }
        {
            const uint64_t m = compact_ballot<LPC>(__ballot(acc));
            if ((threadIdx.x & 63) == 0)
                store_acc_bits<LPC>(a.hist_acc + slot * a.row_bytes, chain, m);
        }
        // ---- update_stats! rolling acceptance (chain_statistics.jl:53-65)
        ra = rolling_update(ra, r0, r1, iter, a.W, a.N0 + s, acc);
    }

    if (sub == 0) {
        a.ll[chain] = ll;
        a.ra[chain] = ra;
        a.ring[2 * chain] = r0;
        a.ring[2 * chain + 1] = r1;
        a.nacc[chain] = nacc;
        a.faults[chain] = faults;
    }
    store_state<D>(a.theta, C, chain, d0, th, false);
}

// ---------------------------------------------------------------------------
// Dense Gaussian RW proposal (lower Cholesky factor of Σ_rw) + dense Gaussian
// target (lower Cholesky factor of Σ_t): the general GsnTargetLaw case
// (cfg 1: GsnTargetLaw([1,2], [1 .5; .5 1])).  One lane per chain.
template <int D, bool FULL, int LLMODE>
__global__ void __launch_bounds__(256) rwm_gsn_dense_kernel(const StepParams a) {
    extern __shared__ __attribute__((aligned(16))) double lds[];
    const uint32_t nobs = a.nobs;
    const int nconst = 2 * D * D + 3 * D;
    stage_lds(lds, a.zig, a.consts, nconst, a.obs, (LLMODE == LL_PER_OBS) ? (int)nobs * D : 0);
    const Ziggurat &zt = *reinterpret_cast<const Ziggurat *>(lds);
    const double *cst = lds + kZigLdsDoubles;
    const double *Lrw = cst;
    const double *iLrw = cst + D * D;
    const double *Lt = cst + D * D + D;
    const double *iLt = cst + 2 * D * D + D;
    const double *xbar = cst + 2 * D * D + 2 * D;
    const double *X = cst + 2 * D * D + 3 * D;

    const uint64_t chain = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (chain >= a.C) return;
    const uint32_t gid = a.chain0 + (uint32_t)chain;

    const uint64_t C = a.C;
    double th[D];
    load_state<D>(a.theta, C, chain, 0, th);
    double ll = a.ll[chain];
    double ra = a.ra[chain];
    uint64_t r0 = a.ring[2 * chain], r1 = a.ring[2 * chain + 1];
    uint32_t nacc = a.nacc[chain];
    uint32_t faults = a.faults[chain];

    for (uint32_t s = 0; s < a.nsteps; ++s) {
        const uint32_t iter = a.iter0 + s;  // consecutive (host splits gaps)
        const uint64_t slot = (uint64_t)(iter - 1) * a.P + a.pidx0;
        double z[D];
        normals<D>(zt, a.key0, a.key1, gid, iter, a.pidx0, z, faults);
        double thp[D];
#pragma unroll
        for (int i = 0; i < D; ++i) {
            double acc = Lrw[i * D] * z[0];
#pragma unroll
            for (int j = 1; j <= i; ++j) acc = fma(Lrw[i * D + j], z[j], acc);
            thp[i] = th[i] + acc;
        }
        double ltd;
        {
            double y[D];
#pragma unroll
            for (int i = 0; i < D; ++i) {
                double acc = thp[i] - th[i];
#pragma unroll
                for (int j = 0; j < i; ++j) acc = fma(-Lrw[i * D + j], y[j], acc);
                y[i] = acc * iLrw[i];
            }
            ltd = a.rw_c0 - canon_sumsq<D, 1>(y) / 2.0;
        }
        double llp;
        if constexpr (LLMODE == LL_PER_OBS) {
            llp = 0.0;
            for (uint32_t k = 0; k < nobs; ++k) {
                const double *xk = X + (size_t)k * D;
                double y[D];
#pragma unroll
                for (int i = 0; i < D; ++i) {
                    double acc = xk[i] - thp[i];
#pragma unroll
                    for (int j = 0; j < i; ++j) acc = fma(-Lt[i * D + j], y[j], acc);
                    y[i] = acc * iLt[i];
                }
                llp = llp + (a.t_c0 - canon_sumsq<D, 1>(y) / 2.0);
            }
        } else {
            double y[D];
#pragma unroll
            for (int i = 0; i < D; ++i) {
                double acc = xbar[i] - thp[i];
#pragma unroll
                for (int j = 0; j < i; ++j) acc = fma(-Lt[i * D + j], y[j], acc);
                y[i] = acc * iLt[i];
            }
            const double qv = canon_sumsq<D, 1>(y);
            llp = a.n_tc0 - (a.S_c + a.nobs_d * qv) * 0.5;
        }
        if (!(llp - llp == 0.0)) faults |= 1u;
        const double llr = ((((llp - ll) + ltd) - ltd) + 0.0) - 0.0;
        const double E = accept_exp(zt, a.key0, a.key1, gid, iter, a.pidx0, faults);
        const bool acc = E > -llr;
        if constexpr (FULL) store_state<D>(a.hist_prop + slot * D * C, C, chain, 0, thp, true);
#pragma unroll
        for (int i = 0; i < D; ++i) th[i] = acc ? thp[i] : th[i];
        ll = acc ? llp : ll;
        nacc += acc ? 1u : 0u;
        if constexpr (FULL) {
            store_state<D>(a.hist_theta + slot * D * C, C, chain, 0, th, true);
            __builtin_nontemporal_store(ll, a.hist_ll + slot * C + chain);
        }
        {
            const uint64_t m = __ballot(acc);
            if ((threadIdx.x & 63) == 0) store_acc_bits<1>(a.hist_acc + slot * a.row_bytes, chain, m);
        }
        ra = rolling_update(ra, r0, r1, iter, a.W, a.N0 + s, acc);
    }
    a.ll[chain] = ll;
    a.ra[chain] = ra;
    a.ring[2 * chain] = r0;
    a.ring[2 * chain + 1] = r1;
    a.nacc[chain] = nacc;
    a.faults[chain] = faults;
    store_state<D>(a.theta, C, chain, 0, th, false);
}

// ---------------------------------------------------------------------------
// Diagnostics: per-(half-)chain mean and unbiased variance of θ over a window
// of history slots, then a deterministic tree reduction over chains.
__global__ void __launch_bounds__(256)
chain_moments_kernel(const double *__restrict__ hist, uint64_t C, uint32_t D, uint64_t slot0,
                     uint32_t slot_stride, uint32_t n, uint32_t halves, double *__restrict__ mean_out,
                     double *__restrict__ var_out) {
    // one thread per (half, element position within a slot): consecutive
    // threads read consecutive addresses; the reduce step maps (d, c) → position
    const uint64_t t = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const uint64_t total = C * D * halves;
    if (t >= total) return;
    const uint32_t h = (uint32_t)(t / (C * D));
    const uint64_t cd = t % (C * D);
    const uint32_t len = n / halves;
    const uint64_t first = slot0 + (uint64_t)h * len * slot_stride;
    double s = 0.0;
    for (uint32_t i = 0; i < len; ++i) s = s + hist[(first + (uint64_t)i * slot_stride) * C * D + cd];
    const double m = s / (double)len;
    double q = 0.0;
    for (uint32_t i = 0; i < len; ++i) {
        const double e = hist[(first + (uint64_t)i * slot_stride) * C * D + cd] - m;
        q = q + e * e;
    }
    mean_out[t] = m;
    var_out[t] = (len > 1) ? q / (double)(len - 1) : 0.0;
}

// out[d] = Σ over (half-)chains of f(x), f ∈ {x, x², y}: one block per d,
// fixed chunking → deterministic for a given (C, halves).
__global__ void __launch_bounds__(256)
moments_reduce_kernel(const double *__restrict__ mean_in, const double *__restrict__ var_in, uint64_t C,
                      uint32_t D, uint32_t halves, double *__restrict__ out3d) {
    const uint32_t d = blockIdx.x;
    __shared__ double sm[3][256];
    double a = 0.0, b = 0.0, c = 0.0;
    const uint64_t rows = C * halves;
    for (uint64_t r = threadIdx.x; r < rows; r += blockDim.x) {
        const uint64_t h = r / C, ch = r % C;
        const uint64_t idx = h * C * D + state_pos(d, ch, C, D);
        const double m = mean_in[idx];
        a = a + m;
        b = b + m * m;
        c = c + var_in[idx];
    }
    sm[0][threadIdx.x] = a;
    sm[1][threadIdx.x] = b;
    sm[2][threadIdx.x] = c;
    __syncthreads();
    for (int w = 128; w > 0; w >>= 1) {
        if ((int)threadIdx.x < w) {
            sm[0][threadIdx.x] = sm[0][threadIdx.x] + sm[0][threadIdx.x + w];
            sm[1][threadIdx.x] = sm[1][threadIdx.x] + sm[1][threadIdx.x + w];
            sm[2][threadIdx.x] = sm[2][threadIdx.x] + sm[2][threadIdx.x + w];
        }
        __syncthreads();
    }
    if (threadIdx.x == 0) {
        out3d[d] = sm[0][0];
        out3d[D + d] = sm[1][0];
        out3d[2 * D + d] = sm[2][0];
    }
}

// accepted proposals in a window of accept-bit rows (integer → deterministic)
__global__ void __launch_bounds__(256)
popcount_kernel(const uint64_t *__restrict__ bits, uint64_t words, unsigned long long *__restrict__ out) {
    uint64_t acc = 0;
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < words;
         i += (uint64_t)gridDim.x * blockDim.x)
        acc += (uint64_t)__popcll(bits[i]);
    if (acc) atomicAdd(out, (unsigned long long)acc);
}

// device state_pos layout → [slot][nc][D] (host layout) for chains [c0, c0+nc)
__global__ void __launch_bounds__(256)
gather_hist_kernel(const double *__restrict__ src, uint64_t C, uint32_t D, uint64_t slot0, uint64_t nslots,
                   uint64_t c0, uint64_t nc, double *__restrict__ dst) {
    const uint64_t t = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= nslots * nc * D) return;
    const uint64_t s = t / (nc * D), r = t % (nc * D);
    const uint64_t c = r / D, d = r % D;
    dst[t] = src[(slot0 + s) * D * C + state_pos(d, c0 + c, C, D)];
}

// self-test probes
__global__ void __launch_bounds__(256)
probe_variates_kernel(const Ziggurat *__restrict__ zig, uint32_t key0, uint32_t key1, uint32_t pidx0, uint32_t D,
                      uint64_t n, const uint32_t *__restrict__ chains, const uint32_t *__restrict__ iters,
                      double *__restrict__ z, double *__restrict__ E) {
    const uint64_t t = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= n) return;
    uint32_t faults = 0;
    for (uint32_t j = 0; j < D; ++j) z[t * D + j] = normal_draw(*zig, key0, key1, chains[t], iters[t], pidx0, j, faults);
    E[t] = exp_draw(*zig, key0, key1, chains[t], iters[t], pidx0, faults);
}

__global__ void __launch_bounds__(256) probe_log_kernel(const double *__restrict__ x, double *__restrict__ y,
                                                        uint64_t n) {
    const uint64_t t = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (t < n) y[t] = log_pos(x[t]);
}

}  // namespace emcmc
