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

#ifndef __HIPCC_RTC__
#include <hip/hip_runtime.h>
#include <stdint.h>
#endif

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
    uint32_t *fault_flag;  // set to 1 by any lane that ends a launch with a fault bit (emcmc_synchronize)
    double *ll_prop;       // [C] sub_ws°.ll: log-likelihood of the launch's last proposal (update pidx0)
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
    uint32_t xcd;         // 1: XCD-aware block order (xcd_block), 0: blockIdx order
    uint64_t N0;          // GenericChainStats.N before the first step of this launch
    double rw_c0;         // −(D·log2π + logdet Σ_rw)/2
    double t_c0;          // −(D·log2π + logdet Σ_t)/2
    double n_tc0;         // nobs · t_c0     (SUFFSTAT)
    double S_c;           // Σ_k ‖L_t⁻¹(x_k − x̄)‖²  (SUFFSTAT)
    double nobs_d;        // (double) nobs
    double rcp_W;         // RN(1/W) for the rolling-acceptance quotient
    // rwm_gsn_diag_kernel only: θ is loaded from theta_in when set (the previous launch's
    // last θ history slot), and not stored back when theta is null (this launch's last
    // history slot then holds it: emcmc.hip, theta_live)
    const double *theta_in;
};

// constants layout (offsets in doubles), D = dimension
//   diag kernels : [0,D) L_rw diag | [D,2D) 1/L_rw | [2D,3D) 1/L_t | [3D,4D) x̄
//   dense kernels: [0,D²) L_rw (row-major lower) | [D²,D²+D) 1/diag(L_rw)
//                  | [D²+D, 2D²+D) L_t | [2D²+D, 2D²+2D) 1/diag(L_t) | [2D²+2D, 2D²+3D) x̄
constexpr int LL_PER_OBS = 0;
constexpr int LL_SUFFSTAT = 1;

// HBM layout of θ state and θ/θ° histories (per history slot), and of every
// per-chain vector kept "in state_pos layout": tiled, pair-interleaved SoA.
// The chains are cut into tiles of T = 32 (when C is a multiple of 32; else one
// tile of all C chains).  A tile holds its chains' R "rows" one after another
// (R = D/2 pairs (2j, 2j+1) as 16-byte words when D is even, R = D single
// doubles when odd), each row T consecutive chains: row k of chain c is word
// c0·R + k·T + (c − c0), c0 = c's tile start.  A wave of 32 chains (LPC = 2)
// then writes one contiguous 8 KiB run per history and step (its tile), which
// HBM takes at +3% over the untiled layout (T = C, where one wave's words lay
// 16·C bytes apart; scripts/ubench/write_layout.hip, profiles/r4_store_ab/).
#ifndef EMCMC_SOA_TILE
#define EMCMC_SOA_TILE 32  // chains per tile (a power of two); 0: the untiled round-3 layout (A/B builds)
#endif
__host__ __device__ __forceinline__ uint64_t soa_tile(uint64_t C) {
    return (EMCMC_SOA_TILE && (C & (uint64_t)(EMCMC_SOA_TILE - 1)) == 0) ? (uint64_t)EMCMC_SOA_TILE : C;
}
__host__ __device__ __forceinline__ uint64_t soa_tile0(uint64_t c, uint64_t C) {
    return (EMCMC_SOA_TILE && (C & (uint64_t)(EMCMC_SOA_TILE - 1)) == 0) ? (c & ~(uint64_t)(EMCMC_SOA_TILE - 1)) : 0u;
}
// word index of row k of chain c, R rows per chain
__host__ __device__ __forceinline__ uint64_t soa_row(uint64_t k, uint64_t c, uint64_t C, uint64_t R) {
    const uint64_t c0 = soa_tile0(c, C);
    return c0 * R + k * soa_tile(C) + (c - c0);
}
__host__ __device__ __forceinline__ uint64_t state_pos(uint64_t d, uint64_t c, uint64_t C, uint32_t D) {
    return (D % 2 == 0) ? (soa_row(d >> 1, c, C, D >> 1) << 1) + (d & 1) : soa_row(d, c, C, D);
}

typedef double d2v __attribute__((ext_vector_type(2)));

// Stage the LDS part of the ziggurat tables (N(0,1) 8192 + Exp(1) 256 layers,
// 70 KiB) into the kernel's STATIC LDS — their addresses are then link-time
// constants that fold into the ds_read offset field — and `nconst` constants
// followed by `nobs_d` observation doubles into the dynamic LDS at offset 0
// (offsets below 64 KiB: a row's reads share one address register).
struct ZigLds {
    double n[kZigNL + 2];
    ZigEntry e[256];
    double ef[256];
};
static_assert(sizeof(ZigLds) == kZigLdsBytes, "LDS prefix of Ziggurat");
__device__ __forceinline__ ZigTabs stage_lds(double *lds, const Ziggurat *zig, const double *consts, int nconst,
                                             const double *obs, int nobs_d) {
    __shared__ ZigLds tabs;
    const d2v *zsrc = reinterpret_cast<const d2v *>(zig);
    d2v *zdst = reinterpret_cast<d2v *>(&tabs);
    for (int i = threadIdx.x; i < (int)(kZigLdsBytes / 16); i += blockDim.x) zdst[i] = zsrc[i];
    for (int i = threadIdx.x; i < nconst + nobs_d; i += blockDim.x) lds[i] = (i < nconst) ? consts[i] : obs[i - nconst];
    __syncthreads();
    return ZigTabs{tabs.n, zig->nf, tabs.e, tabs.ef};
}


// N normals of (chain, iter, pidx0) with lane-local index i ↔ global normal
// index g0 + i, written as out[i] = base[i] + scale[i]·z (the diagonal
// proposal θ° = θ + L z, random_walk.jl:147).  Fast pass over all pairs, then
// a wave-uniform loop resolves the ≈1% wedge/tail draws one per lane per trip
// (with 64 lanes × N draws per wave most steps take one trip, so the trip only
// fixes z[i]; the proposal arithmetic runs once, after it).
template <int N, bool VK = false>
__device__ __forceinline__ void propose_diag(const ZigTabs &zt, uint32_t key0, uint32_t key1, uint32_t chain,
                                             uint32_t iter, uint32_t pidx0, uint32_t g0, const double (&base)[N],
                                             const double *scale, double (&out)[N], uint32_t &faults,
                                             const PhiloxVKeys &vk = PhiloxVKeys{}) {
    constexpr int NP = (N + 1) / 2;
    uint32_t pend = 0;
#pragma unroll
    for (int j = 0; j < NP; ++j) {
        // one Philox block at a time: interleaving the pairs' blocks costs registers
        // (occupancy), and the waves of a SIMD supply the ILP
        __builtin_amdgcn_sched_barrier(0);
        u32x4 r;
        if constexpr (VK) r = draw_vk(vk, chain, iter, (g0 >> 1) + j, pidx0);
        else r = draw(key0, key1, chain, iter, (g0 >> 1) + j, pidx0, 0);
        if (!zig_normal_fast(zig_split_n(r.x, r.y), zt.n, out[2 * j])) pend |= 1u << (2 * j);
        if (2 * j + 1 < N)
            if (!zig_normal_fast(zig_split_n(r.z, r.w), zt.n, out[2 * j + 1])) pend |= 1u << (2 * j + 1);
    }
    // wave-uniform loop, one pending draw per lane per trip (with 8192 normal
    // layers a wave of 1024 draws has ≈ 0.6 pending, usually on one lane); the
    // result is written with selects OUTSIDE the divergent region, so the
    // per-element update stays branch-free v_cndmask code
    while (__ballot(pend != 0) != 0) {
        const bool act = pend != 0;
        const uint32_t i = act ? (uint32_t)__builtin_ctz(pend) : 0xFFu;
        pend &= pend - 1;
        double z = 0.0;
        if (act) z = normal_draw(zt, key0, key1, chain, iter, pidx0, g0 + i, faults);
#pragma unroll
        for (int q = 0; q < N; ++q) out[q] = (i == (uint32_t)q) ? z : out[q];
    }
#pragma unroll
    for (int i = 0; i < N; ++i) out[i] = base[i] + scale[i] * out[i];
}

__host__ __device__ constexpr size_t lds_align16(size_t b) { return (b + 15) & ~(size_t)15; }

__device__ __forceinline__ void wave_lds_sync() {
    // LDS ops of one wave execute in order; this only stops the compiler from
    // moving LDS accesses across the phase boundary
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// The N standard normals themselves (dense-L proposals).
template <int N, bool VK = false>
__device__ __forceinline__ void normals(const ZigTabs &zt, uint32_t key0, uint32_t key1, uint32_t chain,
                                        uint32_t iter, uint32_t pidx0, double (&z)[N], uint32_t &faults,
                                        const PhiloxVKeys &vk = PhiloxVKeys{}) {
    constexpr int NP = (N + 1) / 2;
    uint64_t pend = 0;
#pragma unroll
    for (int j = 0; j < NP; ++j) {
        if constexpr (N > 8) __builtin_amdgcn_sched_barrier(0);  // one Philox block at a time
        u32x4 r;
        if constexpr (VK) r = draw_vk(vk, chain, iter, j, pidx0);
        else r = draw(key0, key1, chain, iter, j, pidx0, 0);
        if (!zig_normal_fast(zig_split_n(r.x, r.y), zt.n, z[2 * j])) pend |= 1ull << (2 * j);
        if (2 * j + 1 < N)
            if (!zig_normal_fast(zig_split_n(r.z, r.w), zt.n, z[2 * j + 1])) pend |= 1ull << (2 * j + 1);
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

// Exp(1) draws of the accept test (run.jl:278) for consecutive iterations: one
// Philox block serves iterations 2m and 2m+1 (kBlockAccept), so a launch pays
// half a block per step.  `first` forces the block at the launch's first step.
struct AcceptStream {
    u32x4 r;
    template <bool VK = false>
    __device__ __forceinline__ double next(const ZigTabs &zt, uint32_t key0, uint32_t key1, uint32_t chain,
                                           uint32_t iter, uint32_t pidx0, bool first, uint32_t &faults,
                                           const PhiloxVKeys &vk = PhiloxVKeys{}) {
        if (first || (iter & 1u) == 0) {
            if constexpr (VK) r = draw_vk(vk, chain, iter >> 1, kBlockAccept, pidx0);
            else r = draw(key0, key1, chain, iter >> 1, kBlockAccept, pidx0, 0);
        }
        const ZigDraw d = accept_split(r, iter);
        double e;
        if (!zig_exp_fast(d, zt.e, e)) e = zig_exp_slow(d, zt.e, zt.ef, key0, key1, chain, iter, kBlockAccept, pidx0, faults);
        return e;
    }
};

// ---------------------------------------------------------------------------
// cross-lane helpers (DPP quad permutes; 64-bit values move as two dwords)
template <int CTRL>
__device__ __forceinline__ double dpp_perm(double v) {
    const uint64_t b = __builtin_bit_cast(uint64_t, v);
    // mov_dpp: every lane of a quad permute has a source, so no "old" value is
    // needed (update_dpp(0, …) materialises one with an extra v_mov per dword)
    const int lo = __builtin_amdgcn_mov_dpp((int)(uint32_t)b, CTRL, 0xF, 0xF, true);
    const int hi = __builtin_amdgcn_mov_dpp((int)(uint32_t)(b >> 32), CTRL, 0xF, 0xF, true);
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

// Σ y_i² in the canonical order with y_i = yf(i) produced on the fly, one
// block at a time (sched barriers keep the scheduler from materialising all
// NV values — e.g. a whole observation row — at once).
template <int D, int LPC, int NV, typename YF>
__device__ __forceinline__ double canon_sumsq_f(YF yf) {
    constexpr int BLK = SumShape<D>::BLK;
    constexpr int BPL = NV / BLK;
    double b[BPL];
#pragma unroll
    for (int k = 0; k < BPL; ++k) {
        if constexpr (BPL > 1) __builtin_amdgcn_sched_barrier(0);
        const double y0 = yf(k * BLK);
        double s = y0 * y0;
#pragma unroll
        for (int i = 1; i < BLK; ++i) {
            const double yi = yf(k * BLK + i);
            s = fma(yi, yi, s);
        }
        b[k] = s;
    }
    double s = tree_inplace<BPL>(b);
    return lane_tree<LPC>(s);
}

// Σ y_i² over the chain's D coordinates in the canonical order: blocks of BLK
// accumulated s = y0·y0, s = fma(y_i, y_i, s); blocks combine pairwise, first
// inside the lane, then across the chain's LPC lanes.
template <int D, int LPC, int NV>
__device__ __forceinline__ double canon_sumsq(const double (&y)[NV]) {
    return canon_sumsq_f<D, LPC, NV>([&](int i) { return y[i]; });
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

// x / b for b = W with q = RN(x·y), y = RN(1/b): Markstein's correction
// q + (x − b·q)·y rounds to the IEEE quotient (tests/test_oracle.py checks it)
__device__ __forceinline__ double div_markstein(double x, double b, double y) {
    const double q = x * y;
    const double r = fma(-q, b, x);
    return fma(r, y, q);
}

// rolling acceptance, chain_statistics.jl:53-65 (N = cs.N before increment;
// N is the same for every chain, so the divisor branch is wave-uniform)
__device__ __forceinline__ double rolling_update(double ra, uint64_t &r0, uint64_t &r1, uint32_t iter,
                                                 uint32_t W, uint64_t N, double rcpW, bool acc) {
    int out = 0;
    if (iter > W) {
        const uint32_t j = (iter - W) & 127u;
        const uint64_t w = (j & 64u) ? r1 : r0;
        out = (int)((w >> (j & 63u)) & 1ull);
    }
    const double num = ra * (double)W + (double)((int)acc - out);
    double nra;
    if (N >= (uint64_t)W) nra = div_markstein(num, (double)W, rcpW);
    else nra = num / (double)N;
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
            d2v *p = reinterpret_cast<d2v *>(base) + soa_row((uint64_t)(d0 / 2 + j), c, C, D / 2);
            if (nt) __builtin_nontemporal_store(x, p);
            else *p = x;
        }
    } else {
#pragma unroll
        for (int i = 0; i < N; ++i) {
            double *p = base + soa_row((uint64_t)(d0 + i), c, C, D);
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
            const d2v x = reinterpret_cast<const d2v *>(base)[soa_row((uint64_t)(d0 / 2 + j), c, C, D / 2)];
            v[2 * j] = x.x;
            v[2 * j + 1] = x.y;
        }
    } else {
#pragma unroll
        for (int i = 0; i < N; ++i) v[i] = base[soa_row((uint64_t)(d0 + i), c, C, D)];
    }
}

// A history slot is written as (wave-uniform slot base + j·stride) + one
// per-lane 32-bit byte offset: the base and the per-word stride live in
// SGPRs, so a store needs no per-step VALU address math (global_store with
// saddr).  The host guarantees a slot is < 4 GiB (EMCMC_INVALID_ARG otherwise).
template <int D>
struct SlotOffset {
    uint32_t o;       // lane's first word: pair d0/2 (even D) or coordinate d0 (odd D) of chain c
    uint64_t stride;  // bytes between consecutive words of one chain (uniform: the tile width)
    __device__ __forceinline__ SlotOffset(uint64_t C, uint64_t c, int d0) {
        if constexpr (D % 2 == 0) {
            o = (uint32_t)(soa_row((uint64_t)(d0 / 2), c, C, D / 2) * 16u);
            stride = soa_tile(C) * 16u;
        } else {
            o = (uint32_t)(soa_row((uint64_t)d0, c, C, D) * 8u);
            stride = soa_tile(C) * 8u;
        }
    }
};
template <int D, int N>
__device__ __forceinline__ void store_slot(double *slot_base, const SlotOffset<D> &off, const double (&v)[N]) {
    char *b = reinterpret_cast<char *>(slot_base);
    if constexpr (D % 2 == 0) {
#pragma unroll
        for (int j = 0; j < N / 2; ++j) {
            d2v x = {v[2 * j], v[2 * j + 1]};
            __builtin_nontemporal_store(x, reinterpret_cast<d2v *>(b + (uint64_t)j * off.stride + off.o));
        }
    } else {
#pragma unroll
        for (int i = 0; i < N; ++i)
            __builtin_nontemporal_store(v[i], reinterpret_cast<double *>(b + (uint64_t)i * off.stride + off.o));
    }
}

template <int D, int N>
__device__ __forceinline__ void load_slot(const double *slot_base, const SlotOffset<D> &off, double (&v)[N]) {
    const char *b = reinterpret_cast<const char *>(slot_base);
    if constexpr (D % 2 == 0) {
#pragma unroll
        for (int j = 0; j < N / 2; ++j) {
            const d2v x = *reinterpret_cast<const d2v *>(b + (uint64_t)j * off.stride + off.o);
            v[2 * j] = x.x;
            v[2 * j + 1] = x.y;
        }
    } else {
#pragma unroll
        for (int i = 0; i < N; ++i) v[i] = *reinterpret_cast<const double *>(b + (uint64_t)i * off.stride + off.o);
    }
}
template <int D, int N>
__device__ __forceinline__ void store_slot_cached(double *slot_base, const SlotOffset<D> &off, const double (&v)[N]) {
    char *b = reinterpret_cast<char *>(slot_base);
    if constexpr (D % 2 == 0) {
#pragma unroll
        for (int j = 0; j < N / 2; ++j)
            *reinterpret_cast<d2v *>(b + (uint64_t)j * off.stride + off.o) = d2v{v[2 * j], v[2 * j + 1]};
    } else {
#pragma unroll
        for (int i = 0; i < N; ++i) *reinterpret_cast<double *>(b + (uint64_t)i * off.stride + off.o) = v[i];
    }
}
// element `c` of a per-chain array through a 32-bit byte offset (saddr form)
template <typename T>
__device__ __forceinline__ T &chain_elem(T *base, uint32_t c) {
    return *reinterpret_cast<T *>(reinterpret_cast<char *>(base) + c * (uint32_t)sizeof(T));
}

// XCD-aware block order (cdna_hip_programming.md §5 T1).  Blocks are dealt
// round-robin over the 8 XCDs (block b on the XCD of b mod 8); block b runs the
// work of block x·q + min(x, r) + b/8 (x = b mod 8, q = nwg/8, r = nwg mod 8),
// so each XCD sweeps one contiguous eighth of the chains.  A step's history
// stores then touch each slot's pages from one XCD instead of all eight: each
// XCD's L2 TLB translates 1/8 of the ≈34 MB a step writes.  Bijective for any
// nwg; speed only (every chain's results are keyed by its id).
__device__ __forceinline__ uint32_t xcd_block(uint32_t b, uint32_t nwg, uint32_t enable) {
    if (!enable) return b;
    const uint32_t q = nwg >> 3, r = nwg & 7u, x = b & 7u;
    return x * q + (x < r ? x : r) + (b >> 3);
}

// ---------------------------------------------------------------------------
// Correlated Σ at D ≥ 16 (rows a5/a10 at the headline D): the same proposal,
// transition densities and per-observation solves as rwm_gsn_dense_kernel, one
// lane per chain, but the factors are read through the SCALAR cache: Σ_rw and
// Σ_t are the same for every chain, so every factor element is wave-uniform and
// enters v_fma_f64 as an SGPR operand (no per-lane LDS traffic: an LDS
// broadcast would still return 8 B per lane per fma).  The sweeps run column by
// column (forward substitution as column updates acc_i −= L_ij·y_j, i > j, and
// the proposal L·z as acc_i += L_ij·z_j, i ≥ j): every row still accumulates
// over j = 0, 1, … in ascending order, i.e. the oracle's row sums bit for bit,
// and the D − j updates of a column are independent (ILP at 1 wave per SIMD).
// Σ y_j² is accumulated as y_j leaves the sweep, in the canonical blocked order.
//
// Factor tables are packed column-major lower triangles (P = D(D+1)/2 doubles;
// column j starts at chol_col(D, j) and holds rows j..D−1).  A "propose" table
// keeps L_jj; a "solve" table stores 1/L_jj in its place, so a sweep is ONE flat
// stream of scalar loads.  Constants (address space 4, in doubles):
//   [0,P) L_rw propose | [P,2P) L_rw solve | [2P,3P) L_t solve | [3P,3P+D) x̄
//   | [3P+D, 3P+D+nobs·D) observations, row-major
typedef const __attribute__((address_space(4))) double cdouble;
__host__ __device__ constexpr int chol_col(int D, int j) { return j * D - j * (j - 1) / 2; }
__host__ __device__ constexpr int chol_col_of(int D, int e) {
    int j = 0;
    while (j + 1 < D && chol_col(D, j + 1) <= e) ++j;
    return j;
}

// the opaque copy keeps the compiler from hoisting loop-invariant scalar loads
// of the factors out of the step / observation loops (hundreds of SGPRs)
__device__ __forceinline__ cdouble *opaque_cptr(const double *q) {
    cdouble *p = (cdouble *)q;
    asm volatile("" : "+s"(p));
    return p;
}
__device__ __forceinline__ void sbar() { __builtin_amdgcn_sched_barrier(0); }
// pins a value's computation between the surrounding volatile asm statements
// (the IR moves pure arithmetic freely across sched_barrier)
__device__ __forceinline__ void vpin(double &v) { asm volatile("" : "+v"(v)); }

// compile-time loop (guaranteed full unrolling: the sweeps index register
// arrays by the column, and a partially rolled loop would put them in scratch)
template <int V>
struct IntC {
    static constexpr int value = V;
};
template <int I, int N, typename F>
__device__ __forceinline__ void static_for(F &&f) {
    if constexpr (I < N) {
        f(IntC<I>{});
        static_for<I + 1, N>(f);
    }
}

// One flat stream of NA prefix doubles (X, e.g. an observation row) followed by
// a packed factor table T, in chunks of CH doubles.  The next chunk's scalar
// loads are issued right after the FIRST use of this chunk's values (SMEM
// returns out of order, so every wait is lgkmcnt(0): loads issued earlier would
// be waited for too) and stay in flight during the chunk's other CH − 1 fmas.
// Before each chunk's loads the base pointer (X or T) goes through an empty asm,
// in place (loads from constant memory alias nothing, so the IR would otherwise
// hoist and merge a whole sweep's loads into SGPRs), and the chunk's offset from it
// is a compile-time constant folded into the s_load's immediate: no scalar address
// arithmetic per chunk.  Every result is pinned with vpin, so the stream keeps its order.
// fpre(IntC<i>, x_i) for the prefix, ftab(IntC<j>, IntC<i>, T_ij) for the table.
// Chunks are 16 doubles at any D: the prefix takes ⌈NA/16⌉ chunks (the last one
// partial) and the table starts on a chunk of its own, so an odd D streams the
// same ≤ 134 chunks per sweep as an even one (SMEM needs 4-byte alignment only).
constexpr int kCholChunk = 16;
constexpr int kCholTouchD = 64;  // D from which the stream batches its scalar-cache touches
template <int D, int NA>
struct CholChunks {
    static constexpr int NCA = (NA + kCholChunk - 1) / kCholChunk;  // prefix chunks
    static constexpr int P = D * (D + 1) / 2;
    static constexpr int NCH = NCA + (P + kCholChunk - 1) / kCholChunk;
    // first element (stream index: prefix 0..NA−1, table NA..) and length of chunk t
    static constexpr int first(int t) { return t < NCA ? t * kCholChunk : NA + (t - NCA) * kCholChunk; }
    static constexpr int len(int t) {
        return t < NCA ? ((NA - t * kCholChunk) < kCholChunk ? NA - t * kCholChunk : kCholChunk)
                       : ((P - (t - NCA) * kCholChunk) < kCholChunk ? P - (t - NCA) * kCholChunk : kCholChunk);
    }
};
template <int D, int NA, typename FP, typename FT>
__device__ __forceinline__ void chol_stream(cdouble *X, cdouble *T, FP &&fpre, FT &&ftab) {
    constexpr int CH = kCholChunk;
    using S = CholChunks<D, NA>;
    constexpr int NCH = S::NCH;
    auto load = [&](auto TC, double(&buf)[CH]) {
        constexpr int t = decltype(TC)::value, e0 = S::first(t), n = S::len(t);
        cdouble *p;
        if constexpr (e0 < NA) {
            asm volatile("" : "+s"(X));
            p = X + e0;
        } else {
            asm volatile("" : "+s"(T));
            p = T + (e0 - NA);
        }
#pragma unroll
        for (int r = 0; r < CH; ++r)
            if (r < n) buf[r] = p[r];
    };
    auto elem = [&](auto EC, double v) {
        constexpr int e = decltype(EC)::value;
        if constexpr (e < NA) {
            fpre(IntC<e>{}, v);
        } else {
            constexpr int j = chol_col_of(D, e - NA);
            ftab(IntC<j>{}, IntC<j + (e - NA) - chol_col(D, j)>{}, v);
        }
    };
    double cur[CH], nxt[CH];
    // D = 64: every fourth chunk, one batch of scalar loads of one dword per 64-byte line
    // of the next four chunks ("touches", results never read) so that their scalar-cache
    // misses overlap in one wait instead of stalling the stream one by one (+7% at D = 64;
    // at D = 48 / 56 the same batches cost 2–3%: DESIGN.md §6)
    constexpr int G = D >= kCholTouchD ? 4 : 0;
    uint32_t pf = 0u;  // destination of the touches (never read)
    auto touch = [&pf, &X, &T](auto CC) {  // the two 64-byte lines at the start of chunk c
        constexpr int c = decltype(CC)::value, e0 = S::first(c);
        if constexpr (e0 < NA)
            asm volatile("s_load_dword %0, %1, %2\n\ts_load_dword %0, %1, %3" : "+s"(pf) : "s"(X), "n"(8 * e0),
                         "n"(8 * e0 + 64));
        else
            asm volatile("s_load_dword %0, %1, %2\n\ts_load_dword %0, %1, %3" : "+s"(pf) : "s"(T), "n"(8 * (e0 - NA)),
                         "n"(8 * (e0 - NA) + 64));
    };
    load(IntC<0>{}, cur);
    static_for<0, NCH>([&](auto TC) {
        constexpr int t = decltype(TC)::value, e0 = S::first(t), n = S::len(t);
        elem(IntC<e0>{}, cur[0]);
        if constexpr (G > 0 && t > 0 && (t - 1) % G == 0) {
            uint32_t &pfr = pf;
            asm volatile("" ::"s"(pfr));  // landed: waited with cur
        }
        sbar();
        if constexpr (t + 1 < NCH) load(IntC<t + 1>{}, nxt);
        if constexpr (G > 0 && t % G == 0) {
            // one batch of touches for the chunks t + 2 … t + G + 1: their misses overlap in
            // one wait (the next chunk's) instead of stalling the stream one by one
            static_for<t + 2, (t + G + 2 < NCH ? t + G + 2 : NCH)>([&](auto CC) { touch(CC); });
        }
        sbar();
        static_for<1, n>([&](auto RC) {
            constexpr int r = decltype(RC)::value;
            elem(IntC<e0 + r>{}, cur[r]);
        });
        sbar();
#pragma unroll
        for (int r = 0; r < CH; ++r) cur[r] = nxt[r];
    });
}

// ‖L⁻¹ r‖² by forward substitution as column updates, r given by the prefix
// (NA = D: acc_i = x_i − θ°_i) or already in acc (NA = 0); canonical order.  y_j's
// square joins the blocked sum one column late, right after y_{j+1} is formed: the
// column's first update reads y_{j+1} at once, and the square fills the fp64
// result-to-use wait that an s_nop took (same operations in the same order).
template <int D, int NA>
__device__ __forceinline__ double chol_sqmahal(cdouble *X, cdouble *Ts, const double (&thp)[D], double (&acc)[D]) {
    constexpr int BLK = SumShape<D>::BLK, NB = D / BLK;
    double b[NB];
    double s = 0.0, y = 0.0, yl = 0.0;
    auto square = [&](auto JC, double v) {
        constexpr int j = decltype(JC)::value;
        s = (j % BLK == 0) ? v * v : fma(v, v, s);
        if constexpr (j % BLK == BLK - 1) b[j / BLK] = s;
    };
    chol_stream<D, NA>(
        X, Ts,
        [&](auto IC, double x) {
            constexpr int i = decltype(IC)::value;
            acc[i] = x - thp[i];
            vpin(acc[i]);
        },
        [&](auto JC, auto IC, double v) {
            constexpr int j = decltype(JC)::value, i = decltype(IC)::value;
            if constexpr (i == j) {  // v = 1/L_jj
                y = acc[j] * v;
                vpin(y);
                if constexpr (j > 0) square(IntC<j - 1>{}, yl);
                yl = y;
            } else {
                acc[i] = fma(-v, y, acc[i]);
                vpin(acc[i]);
            }
        });
    square(IntC<D - 1>{}, yl);
    return tree_inplace<NB>(b);
}

// θ° = θ + L z with row sums over j ascending (rand(MvNormal(θ, Σ))): column
// sweep acc_i += L_ij z_j for i ≥ j; row j is complete after column j
template <int D>
__device__ __forceinline__ void chol_propose(cdouble *Tp, const double (&z)[D], const double (&th)[D],
                                             double (&thp)[D]) {
    chol_stream<D, 0>(
        Tp, Tp, [&](auto, double) {},
        [&](auto JC, auto IC, double v) {
            constexpr int j = decltype(JC)::value, i = decltype(IC)::value;
            thp[i] = (j == 0) ? v * z[0] : fma(v, z[j], thp[i]);
            if constexpr (i == j) thp[j] = th[j] + thp[j];
            vpin(thp[i]);
        });
}

// store_slot with the word stride made opaque at the store site: otherwise the
// D/2 loop-invariant products j·stride are hoisted out of the step loop and
// held in SGPRs across the sweeps
template <int D, int N>
__device__ __forceinline__ void store_slot_late(double *slot_base, const SlotOffset<D> &off, const double (&v)[N]) {
    uint64_t stride = off.stride;
    asm volatile("" : "+s"(stride));
    char *b = reinterpret_cast<char *>(slot_base);
    if constexpr (D % 2 == 0) {
#pragma unroll
        for (int j = 0; j < N / 2; ++j) {
            d2v x = {v[2 * j], v[2 * j + 1]};
            __builtin_nontemporal_store(x, reinterpret_cast<d2v *>(b + off.o));
            b += stride;
        }
    } else {
#pragma unroll
        for (int i = 0; i < N; ++i) {
            __builtin_nontemporal_store(v[i], reinterpret_cast<double *>(b + off.o));
            b += stride;
        }
    }
}

// 16 doubles through the scalar cache (pointer opaque: see chol_stream)
__device__ __forceinline__ void sload16(double (&buf)[16], cdouble *p) {
    asm volatile("" : "+s"(p));
#pragma unroll
    for (int r = 0; r < 16; ++r) buf[r] = p[r];
}
// one 16-coordinate chunk of Σ_i ((x_i − θ°_i)/L_ii)² in the canonical blocked
// order; the next chunk is requested right after the first use of this one
template <int D, int BLK, bool UNIT_T, int c>
__device__ __forceinline__ void sobs_chunk(const double (&cur)[16], double (&nxt)[16], cdouble *pn,
                                           const double (&thp)[D], const double *iLt, double &sblk,
                                           double (&b)[D / BLK]) {
#pragma unroll
    for (int r = 0; r < 16; ++r) {
        const int i = c * 16 + r;
        double y = cur[r] - thp[i];
        if constexpr (!UNIT_T) y = y * iLt[i];
        sblk = (i % BLK == 0) ? y * y : fma(y, y, sblk);
        vpin(sblk);
        if (i % BLK == BLK - 1) b[i / BLK] = sblk;
        if (r == 0) {
            sbar();
            sload16(nxt, pn);
            sbar();
        }
    }
}

// ---------------------------------------------------------------------------
// rwm_gsn_diag_kernel with one lane per chain and the OBSERVATIONS through the
// scalar cache (EMCMC_VARIANT_SCALAR_OBS): with all D coordinates of a chain in
// one lane, observation x_k,i is the same for every lane of the wave, so it
// enters v_add_f64 as an SGPR operand instead of a ds_read (the LPC = 2 kernel
// issues 80 ds_read_b128 per wave-step and waits on them for ≈ 30% of its
// time).  The rows stream through two 16-double SGPR buffers: chunk t + 1 is
// requested right after the first use of chunk t.  Same arithmetic, same order
// and same bits as rwm_gsn_diag_kernel<D, 1, …>.
template <int D, bool FULL, int LLMODE, bool UNIT_T>
__global__ void __launch_bounds__(256) rwm_gsn_diag_s_kernel(const StepParams a) {
    static_assert(D % 16 == 0, "rows stream in 16-double chunks");
    constexpr int BLK = SumShape<D>::BLK, NB = D / BLK, NCK = D / 16;
    extern __shared__ __attribute__((aligned(16))) double lds[];
    const uint32_t nobs = a.nobs;
    const ZigTabs zt = stage_lds(lds, a.zig, a.consts, 4 * D, nullptr, 0);
    const double *cst0 = lds;

    const uint64_t chain = (uint64_t)xcd_block(blockIdx.x, gridDim.x, a.xcd) * blockDim.x + threadIdx.x;
    if (chain >= a.C) return;
    const uint32_t gid = a.chain0 + (uint32_t)chain;
    const uint64_t C = a.C;
    const SlotOffset<D> soff(C, chain, 0);
    const uint32_t c32 = (uint32_t)chain;
    double th[D];
    load_slot<D>(a.theta, soff, th);
    double ll = chain_elem(a.ll, c32);
    double ra = chain_elem(a.ra, c32);
    uint64_t r0 = chain_elem(a.ring, 2 * c32), r1 = chain_elem(a.ring, 2 * c32 + 1);
    uint32_t nacc = chain_elem(a.nacc, c32);
    uint32_t faults = chain_elem(a.faults, c32);
    AcceptStream accs;
    const PhiloxVKeys vkeys = philox_vkeys(a.key0, a.key1);

    for (uint32_t s = 0; s < a.nsteps; ++s) {
        const uint32_t iter = a.iter0 + s;
        const uint64_t slot = (uint64_t)(iter - 1) * a.P + a.pidx0;
        const double *cst = cst0;
        const double *Lrw = cst, *iLrw = cst + D, *iLt = cst + 2 * D, *xbar = cst + 3 * D;
        double thp[D];
        propose_diag<D, true>(zt, a.key0, a.key1, gid, iter, a.pidx0, 0u, th, Lrw, thp, faults, vkeys);
        const double ltd =
            fma(-0.5, canon_sumsq_f<D, 1, D>([&](int i) { return (thp[i] - th[i]) * iLrw[i]; }), a.rw_c0);
        double llp;
        if constexpr (LLMODE == LL_PER_OBS) {
            llp = 0.0;
            cdouble *X = opaque_cptr(a.obs);
            double bufA[16], bufB[16];
            sload16(bufA, X);
            for (uint32_t k = 0; k < nobs; ++k) {
                // chunk c of row k is in bufA (c even) / bufB (c odd); NCK chunks per row
                double b[NB];
                double sblk = 0.0;
                cdouble *xnext = X + (size_t)((k + 1 < nobs) ? k + 1 : 0u) * D;  // past the last row: row 0 again
                static_for<0, NCK>([&](auto CC) {
                    constexpr int c = decltype(CC)::value;
                    cdouble *pn = (c + 1 < NCK) ? X + (size_t)k * D + (c + 1) * 16 : xnext;
                    if constexpr (c % 2 == 0)
                        sobs_chunk<D, BLK, UNIT_T, c>(bufA, bufB, pn, thp, iLt, sblk, b);
                    else
                        sobs_chunk<D, BLK, UNIT_T, c>(bufB, bufA, pn, thp, iLt, sblk, b);
                });
                if constexpr (NCK % 2 == 1) {  // keep row k+1's first chunk in bufA
#pragma unroll
                    for (int r = 0; r < 16; ++r) bufA[r] = bufB[r];
                }
                const double q = tree_inplace<NB>(b);
                llp = llp + fma(-0.5, q, a.t_c0);
            }
        } else {
            const double qv = canon_sumsq_f<D, 1, D>([&](int i) {
                const double y = xbar[i] - thp[i];
                return UNIT_T ? y : y * iLt[i];
            });
            llp = a.n_tc0 - (a.S_c + a.nobs_d * qv) * 0.5;
        }
        if (!(llp - llp == 0.0)) faults |= 1u;
        const double llr = ((((llp - ll) + ltd) - ltd) + 0.0) - 0.0;
        const double E = accs.next<true>(zt, a.key0, a.key1, gid, iter, a.pidx0, s == 0, faults, vkeys);
        const bool acc = E > -llr;
        if constexpr (FULL) store_slot<D>(a.hist_prop + slot * D * C, soff, thp);
#pragma unroll
        for (int i = 0; i < D; ++i) th[i] = acc ? thp[i] : th[i];
        if (s + 1 == a.nsteps) chain_elem(a.ll_prop, c32) = llp;
        ll = acc ? llp : ll;
        nacc += acc ? 1u : 0u;
        if constexpr (FULL) {
            store_slot<D>(a.hist_theta + slot * D * C, soff, th);
            __builtin_nontemporal_store(ll, &chain_elem(a.hist_ll + slot * a.C, c32));
        }
        {
            const uint64_t m = __ballot(acc);
            if ((threadIdx.x & 63) == 0) store_acc_bits<1>(a.hist_acc + slot * a.row_bytes, chain, m);
        }
        ra = rolling_update(ra, r0, r1, iter, a.W, a.N0 + s, a.rcp_W, acc);
    }
    chain_elem(a.ll, c32) = ll;
    chain_elem(a.ra, c32) = ra;
    chain_elem(a.ring, 2 * c32) = r0;
    chain_elem(a.ring, 2 * c32 + 1) = r1;
    chain_elem(a.nacc, c32) = nacc;
    chain_elem(a.faults, c32) = faults;
    if (faults) *a.fault_flag = 1u;
    store_slot_cached<D>(a.theta, soff, th);
}

// Host-unit kernels (diagnostics, gathers, probes): compiled once, in emcmc.hip.
#ifdef EMCMC_HOST_UNIT
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

// out = [mean of the (half-)chain means | M2 = Σ (m_c − m̄)² | Σ var_c], per d:
// one block per d.  Each thread runs Welford over its strided rows; the block
// combines them by Chan's pairwise merge in a fixed tree, so the result is
// deterministic for a given (C, halves) and M2 does not cancel at 1M chains the
// way Σm² − (Σm)²/m does.  Shards merge the same way (diagnostics.py).
__device__ __forceinline__ void chan_merge(double &na, double &ma, double &qa, double nb, double mb, double qb) {
    const double n = na + nb;
    if (nb == 0.0) return;
    if (na == 0.0) {
        na = nb;
        ma = mb;
        qa = qb;
        return;
    }
    const double dl = mb - ma;
    ma = ma + dl * (nb / n);
    qa = (qa + qb) + dl * dl * (na * nb / n);
    na = n;
}

__global__ void __launch_bounds__(256)
moments_reduce_kernel(const double *__restrict__ mean_in, const double *__restrict__ var_in, uint64_t C,
                      uint32_t D, uint32_t halves, double *__restrict__ out3d) {
    const uint32_t d = blockIdx.x;
    __shared__ double sm[4][256];
    double n = 0.0, mu = 0.0, q = 0.0, c = 0.0;
    const uint64_t rows = C * halves;
    for (uint64_t r = threadIdx.x; r < rows; r += blockDim.x) {
        const uint64_t h = r / C, ch = r % C;
        const uint64_t idx = h * C * D + state_pos(d, ch, C, D);
        const double m = mean_in[idx];
        n = n + 1.0;
        const double dl = m - mu;
        mu = mu + dl / n;
        q = q + dl * (m - mu);
        c = c + var_in[idx];
    }
    sm[0][threadIdx.x] = n;
    sm[1][threadIdx.x] = mu;
    sm[2][threadIdx.x] = q;
    sm[3][threadIdx.x] = c;
    __syncthreads();
    for (int w = 128; w > 0; w >>= 1) {
        if ((int)threadIdx.x < w) {
            double na = sm[0][threadIdx.x], ma = sm[1][threadIdx.x], qa = sm[2][threadIdx.x];
            chan_merge(na, ma, qa, sm[0][threadIdx.x + w], sm[1][threadIdx.x + w], sm[2][threadIdx.x + w]);
            sm[0][threadIdx.x] = na;
            sm[1][threadIdx.x] = ma;
            sm[2][threadIdx.x] = qa;
            sm[3][threadIdx.x] = sm[3][threadIdx.x] + sm[3][threadIdx.x + w];
        }
        __syncthreads();
    }
    if (threadIdx.x == 0) {
        out3d[d] = sm[1][0];
        out3d[D + d] = sm[2][0];
        out3d[2 * D + d] = sm[3][0];
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
    for (uint32_t j = 0; j < D; ++j) z[t * D + j] = normal_draw(zig_tabs(*zig), key0, key1, chains[t], iters[t], pidx0, j, faults);
    E[t] = exp_draw(zig_tabs(*zig), key0, key1, chains[t], iters[t], pidx0, faults);
}

__global__ void __launch_bounds__(256) probe_log_kernel(const double *__restrict__ x, double *__restrict__ y,
                                                        uint64_t n) {
    const uint64_t t = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (t < n) y[t] = log_pos(x[t]);
}

#endif  // EMCMC_HOST_UNIT

}  // namespace emcmc
