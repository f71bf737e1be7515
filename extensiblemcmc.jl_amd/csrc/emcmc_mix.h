// emcmc_mix.h — GaussianRandomWalkMix + HaarioTypeAdaptation + on-device
// GenericChainStats mean/cov (BASELINE cfg 4), one lane per chain (gfx950).
//
// One joint update (P = 1) on coords 1:D.  Reference semantics (src/ under
// /root/reference), restated in oracle/emcmc_oracle.c (orc_run_mix) and
// oracle/literal.py (run_mix_chain):
//   pick_kernel        B iff rand() ≤ λ (Bernoulli(λ))          random_walk.jl:225-227
//   rand(gsn_X, θ)     θ° = θ + L_X z                           random_walk.jl:145-151
//   logpdf(mix)        log((1−λ)·e^{lp_A} + λ·e^{lp_B}); lp_X = MvNormal logpdf
//                      + logJ (−0.0: identity)                  random_walk.jl:161-171,229-232
//   update_stats!      running mean/cov of θ after the step (phantom zero
//                      sample: N = 1, mean 0, cov 0) and rolling acceptance
//                                                          chain_statistics.jl:41-66
//   HaarioTypeAdaptation  registers θ with the same recurrence (P = 1: equal to
//                      the chain-stats mean/cov, kept once); M += 1 per step;
//                      readjust at M ≥ k: Σ_B = 2.38²/D·cov     adaptation.jl:399-426
// The readjust runs as its own kernel between step launches (M is the same for
// every chain, so the host splits launches at readjust steps): a per-chain
// canonical Cholesky of Σ_B; a non-positive pivot sets EMCMC_FAULT_POSDEF and
// keeps the previous factor (the reference throws PosDefException at the next
// MvNormal(θ, Σ_B)).
//
// HBM layout (all SoA over chains, state_pos pair-interleaving):
//   mean  [D]        state_pos(d, c, C, D)
//   cov   [DP]       packed upper, row-major: (i, j ≥ i) ↦ i·D − i(i−1)/2 + j − i
//   L_B   [DP]       packed lower, row-major: (i, j ≤ i) ↦ i(i+1)/2 + j
//   1/L_B,ii [D][C], c0_B [C]
// DP = D(D+1)/2.  Per chain-step the kernel reads and writes cov and mean and
// reads L_B: the step is HBM-bound.
#pragma once

#include "emcmc_kernels.h"
#include "emcmc_fused.h"  // SiblingPace

namespace emcmc {

// Philox block of the mixture pick uniform (block ids 0..D/2 are normals,
// kBlockAccept the accept exponentials).
constexpr uint32_t kBlockMixPick = 0xFFFFFFFEu;

__host__ __device__ constexpr int packed_n(int D) { return D * (D + 1) / 2; }
__host__ __device__ constexpr int up_idx(int D, int i, int j) { return i * D - i * (i - 1) / 2 + (j - i); }
__host__ __device__ constexpr int lo_idx(int i, int j) { return i * (i + 1) / 2 + j; }

struct MixParams {
    double *theta;   // [D] state_pos
    double *ll;      // [C]
    double *ra;      // [C]
    uint64_t *ring;  // [C][2]
    uint32_t *nacc;  // [C]
    uint32_t *faults;
    uint32_t *fault_flag;
    double *ll_prop;  // [C] sub_ws°.ll after the launch
    double *mom_theta;  // ACCEPT_ONLY: θ after each step of the launch, [nsteps] slots (state_pos)
    const double *LB;   // [DP] packed lower, state_pos(q, c, C, DP)
    const double *iLB;  // [D][C]
    const double *c0B;  // [C]
    double *hist_theta, *hist_prop, *hist_ll;
    uint8_t *hist_acc;
    const Ziggurat *zig;
    const double *consts;  // L_A (D×D row-major lower) | 1/L_A,ii | L_t | 1/L_t,ii | x̄
    const double *obs;     // [nobs][D]
    const double *sconsts;  // mix_chol_kernel: the scalar-cache constants (layout there)
    uint64_t C;
    uint64_t row_bytes;
    uint64_t N0;  // GenericChainStats.N before the first step of the launch
    uint32_t chain0, key0, key1, iter0, nsteps, W, nobs, tdiag;
    double lam, oml;  // λ and 1 − λ
    double c0A, t_c0, n_tc0, S_c, nobs_d, rcp_W;
};

// Canonical Σ y_i² accumulated as y_i is produced (blocks of 8 when D % 8 == 0
// and D ≥ 16, then a pairwise tree over the blocks — canon_sumsq's order).
template <int D>
struct SumSqAcc {
    static constexpr int BLK = SumShape<D>::BLK;
    static constexpr int NB = SumShape<D>::NB;
    double b[NB];
    __device__ __forceinline__ void add(int i, double y) {
        if (i % BLK == 0) b[i / BLK] = y * y;
        else b[i / BLK] = fma(y, y, b[i / BLK]);
    }
    __device__ __forceinline__ double finish() { return tree_inplace(b); }
};

// Per-chain SoA arrays addressed as (wave-uniform row base) + (32-bit lane
// offset): the row base is SALU arithmetic on an opaque per-step stride, so the
// compiler neither hoists hundreds of 64-bit per-element addresses out of the
// step loop (they would not fit in registers) nor spends VALU on them; loads
// and stores use the global saddr form.
struct LaneSoA {
    uint64_t stride;  // bytes between consecutive words of one chain (uniform)
    uint64_t off;     // lane's byte offset of its first word (tile start included)
};
// tiled pair-interleaved layout (state_pos) of an n-element per-chain vector
__device__ __forceinline__ LaneSoA lane_soa(uint64_t C, uint64_t chain, int n) {
    const uint64_t w = (n % 2 == 0) ? 16u : 8u;
    uint64_t stride = soa_tile(C) * w;
    asm volatile("" : "+s"(stride));  // opaque: recomputed per step, never hoisted
    return LaneSoA{stride, soa_row(0, chain, C, (uint64_t)((n % 2 == 0) ? n / 2 : n)) * w};
}
template <int NP>
__device__ __forceinline__ double *soa_ptr(double *base, const LaneSoA &l, int q) {
    if constexpr (NP % 2 == 0)
        return reinterpret_cast<double *>(reinterpret_cast<char *>(base) + (uint64_t)(q >> 1) * l.stride + l.off) +
               (q & 1);
    else
        return reinterpret_cast<double *>(reinterpret_cast<char *>(base) + (uint64_t)q * l.stride + l.off);
}
template <int NP>
__device__ __forceinline__ const double *soa_ptr(const double *base, const LaneSoA &l, int q) {
    return soa_ptr<NP>(const_cast<double *>(base), l, q);
}
// element q (lane-dependent) of a packed per-chain vector in state_pos layout
template <int NP>
__device__ __forceinline__ double *soa_ptr_dyn(double *base, const LaneSoA &l, int q) {
    const uint32_t row = (NP % 2 == 0) ? (uint32_t)q >> 1 : (uint32_t)q;
    return reinterpret_cast<double *>(reinterpret_cast<char *>(base) + (uint64_t)row * l.stride + l.off) +
           ((NP % 2 == 0) ? (q & 1) : 0);
}
template <int NP>
__device__ __forceinline__ const double *soa_ptr_dyn(const double *base, const LaneSoA &l, int q) {
    return soa_ptr_dyn<NP>(const_cast<double *>(base), l, q);
}
// plain [n][C] layout (element q of chain c at q·C + c)
__device__ __forceinline__ LaneSoA lane_plain(uint64_t C, uint64_t chain) {
    uint64_t stride = C * 8u;
    asm volatile("" : "+s"(stride));
    return LaneSoA{stride, (uint32_t)(chain * 8u)};
}
__device__ __forceinline__ const double *plain_ptr(const double *base, const LaneSoA &l, int q) {
    return reinterpret_cast<const double *>(reinterpret_cast<const char *>(base) + (uint64_t)q * l.stride + l.off);
}

// Keeps a value's computation where it is written: without it LLVM sinks the
// whole y_B substitution (used only after exp_any's branches) past the row loop,
// and every L_B element loaded there stays live until then.
__device__ __forceinline__ void pin(double &x) { asm volatile("" : "+v"(x)); }

// ‖L_t⁻¹ (x − θ°)‖² of the target (factor in LDS).  DIAG: y_i = r_i/L_ii,
// summed as produced; dense: forward substitution (the dense formulas give the
// diagonal formulas' bits on a diagonal factor, tests/test_oracle.py).
template <int D, bool DIAG>
__device__ __forceinline__ double target_sqmahal(const double *Lt, const double *iLt, const double *x,
                                                 const double (&thp)[D]) {
    if constexpr (DIAG) {
        SumSqAcc<D> q;
#pragma unroll
        for (int i = 0; i < D; ++i) q.add(i, (x[i] - thp[i]) * iLt[i]);
        return q.finish();
    } else {
        double y[D];
#pragma unroll
        for (int i = 0; i < D; ++i) {
            double acc = x[i] - thp[i];
#pragma unroll
            for (int j = 0; j < i; ++j) acc = fma(-Lt[i * D + j], y[j], acc);
            y[i] = acc * iLt[i];
        }
        return canon_sumsq<D, 1>(y);
    }
}

// DIAG: Σ_A and Σ_t both diagonal (diagonal formulas); otherwise the dense
// formulas for both.
template <int D, bool FULL, int LLMODE, bool MIX, bool DIAG>
__global__ void __launch_bounds__(256) mix_gsn_kernel(const MixParams a) {
    constexpr bool ADIAG = DIAG;
    constexpr int DP = packed_n(D);
    extern __shared__ __attribute__((aligned(16))) double lds[];
    const uint32_t nobs = a.nobs;
    const ZigTabs zt =
        stage_lds(lds, a.zig, a.consts, 2 * D * D + 3 * D, a.obs, (LLMODE == LL_PER_OBS) ? (int)nobs * D : 0);

    const uint64_t chain = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (chain >= a.C) return;
    const uint64_t C = a.C;
    const uint32_t gid = a.chain0 + (uint32_t)chain;

    double th[D];
    load_state<D>(a.theta, C, chain, 0, th);
    double ll = a.ll[chain];
    double ra = a.ra[chain];
    uint64_t r0 = a.ring[2 * chain], r1 = a.ring[2 * chain + 1];
    uint32_t nacc = a.nacc[chain];
    uint32_t faults = a.faults[chain];
    const double c0B = MIX ? a.c0B[chain] : 0.0;
    const SlotOffset<D> soff(C, chain, 0);

    for (uint32_t s = 0; s < a.nsteps; ++s) {
        const uint32_t iter = a.iter0 + s;  // consecutive (host splits gaps)
        const uint64_t N = a.N0 + s;
        const uint64_t slot = (uint64_t)(iter - 1);
        // LDS constants through an opaque per-step offset: loop-invariant LDS
        // loads (up to 2·D² of them) must not be hoisted out of the step loop
        uint32_t o = 0;
        asm volatile("" : "+s"(o));
        const double *LA = lds + o;
        const double *iLA = LA + D * D;
        const double *Lt = LA + D * D + D;
        const double *iLt = LA + 2 * D * D + D;
        const double *xbar = LA + 2 * D * D + 2 * D;
        const double *X = LA + 2 * D * D + 3 * D;
        // ---- proposal!: pick the kernel, θ° = θ + L z
        bool useB = false;
        if constexpr (MIX) {
            const u32x4 pr = draw(a.key0, a.key1, gid, iter, kBlockMixPick, 0, 0);
            useB = u01_closed0(pr.x, pr.y) <= a.lam;
        }
        double z[D];
        normals<D>(zt, a.key0, a.key1, gid, iter, 0, z, faults);
        // One pass over the rows of L_B: the proposal row (θ°_i) and the forward
        // substitutions y_A = L_A⁻¹(θ° − θ), y_B = L_B⁻¹(θ° − θ) share each load.
        // logpdf(θ → θ°) and logpdf(θ° → θ) see ±(θ° − θ): bitwise equal
        // sqmahal values, so the mixture density is evaluated once.
        double thp[D];
        double yA[ADIAG ? 1 : D];
        double yB[MIX ? D : 1];
        SumSqAcc<D> qa, qb;
#pragma unroll
        for (int i = 0; i < D; ++i) {
            // one row at a time: without the barrier the scheduler hoists all
            // DP loads of L_B and spills
            __builtin_amdgcn_sched_barrier(0);
            const LaneSoA lb = lane_soa(C, chain, DP);
            const LaneSoA il = lane_plain(C, chain);
            double lzA;
            if constexpr (ADIAG) {
                lzA = LA[i * D + i] * z[i];
            } else {
                lzA = LA[i * D] * z[0];
#pragma unroll
                for (int j = 1; j <= i; ++j) lzA = fma(LA[i * D + j], z[j], lzA);
            }
            double lz = lzA;
            double Lr[MIX ? D : 1];
            if constexpr (MIX) {
#pragma unroll
                for (int j = 0; j <= i; ++j) Lr[j] = *soa_ptr<DP>(a.LB, lb, lo_idx(i, j));
                double lzB = Lr[0] * z[0];
#pragma unroll
                for (int j = 1; j <= i; ++j) lzB = fma(Lr[j], z[j], lzB);
                lz = useB ? lzB : lzA;
            }
            thp[i] = th[i] + lz;
            const double r = thp[i] - th[i];
            if constexpr (ADIAG) {
                qa.add(i, r * iLA[i]);
            } else {
                double acc = r;
#pragma unroll
                for (int j = 0; j < i; ++j) acc = fma(-LA[i * D + j], yA[j], acc);
                yA[i] = acc * iLA[i];
                qa.add(i, yA[i]);
            }
            if constexpr (MIX) {
                double acc = r;
#pragma unroll
                for (int j = 0; j < i; ++j) acc = fma(-Lr[j], yB[j], acc);
                yB[i] = acc * *plain_ptr(a.iLB, il, i);
                pin(yB[i]);
                qb.add(i, yB[i]);
            }
        }
        const double lpA = fma(-0.5, qa.finish(), a.c0A);  // = c0 − q/2 (q/2 exact)
        double ltd = lpA;
        if constexpr (MIX) {
            const double lpB = fma(-0.5, qb.finish(), c0B);
            ltd = log_any(a.oml * exp_any(lpA) + a.lam * exp_any(lpB));
        }
        // ---- compute_ll!
        double llp;
        if constexpr (LLMODE == LL_PER_OBS) {
            llp = 0.0;
            for (uint32_t k = 0; k < nobs; ++k)
                llp = llp + fma(-0.5, target_sqmahal<D, DIAG>(Lt, iLt, X + (size_t)k * D, thp), a.t_c0);
        } else {
            const double qv = target_sqmahal<D, DIAG>(Lt, iLt, xbar, thp);
            llp = a.n_tc0 - (a.S_c + a.nobs_d * qv) * 0.5;
        }
        if (!(llp - llp == 0.0)) faults |= 1u;
        // ---- accept_reject!
        const double llr = ((((llp - ll) + ltd) - ltd) + 0.0) - 0.0;
        const double E = exp_draw(zt, a.key0, a.key1, gid, iter, 0, faults);
        const bool acc = E > -llr;
        if constexpr (FULL) store_slot<D>(a.hist_prop + slot * D * C, soff, thp);
#pragma unroll
        for (int i = 0; i < D; ++i) th[i] = acc ? thp[i] : th[i];
        if (s + 1 == a.nsteps) a.ll_prop[chain] = llp;
        ll = acc ? llp : ll;
        nacc += acc ? 1u : 0u;
        if constexpr (FULL) {
            store_slot<D>(a.hist_theta + slot * D * C, soff, th);
            __builtin_nontemporal_store(ll, a.hist_ll + slot * C + chain);
        }
        {
            const uint64_t m = __ballot(acc);
            if ((threadIdx.x & 63) == 0) store_acc_bits<1>(a.hist_acc + slot * a.row_bytes, chain, m);
        }
        ra = rolling_update(ra, r0, r1, iter, a.W, N, a.rcp_W, acc);
        // update_stats!' mean/cov recurrence runs batched over the launch in
        // mix_moments_kernel; it reads θ from the θ history (FULL) or here:
        if constexpr (!FULL) store_slot<D>(a.mom_theta + (uint64_t)s * D * C, soff, th);
    }
    a.ll[chain] = ll;
    a.ra[chain] = ra;
    a.ring[2 * chain] = r0;
    a.ring[2 * chain + 1] = r1;
    a.nacc[chain] = nacc;
    a.faults[chain] = faults;
    if (faults) *a.fault_flag = 1u;
    store_state<D>(a.theta, C, chain, 0, th, false);
}

// ---- correlated Σ_A / Σ_t at the headline D: mix_chol_kernel -------------------
// The same step as mix_gsn_kernel<D, …, DIAG = false> (the same formulas, so the
// same bits as orc_run_mix and the general kernel's kind 3), for a dense Σ_A and
// a dense target Σ_t at D ≥ 16, where the LDS route of mix_gsn_kernel would read
// one broadcast LDS word per fma (4× the LDS bandwidth the fp64 VALU consumes)
// and D×D factors per lane.  L_A and L_t are the same for every chain, so they
// come through the SCALAR cache and enter v_fma_f64 as SGPR operands, as in
// rwm_gsn_chol_kernel; each chain's own L_B streams from HBM once per step, row
// by row, as in mix_gsn_kernel (that stream, 4.2 KB per chain-step at D = 32, is
// what bounds the kernel).  Scalar constants (a.sconsts, doubles):
//   [0, DP)      L_A packed lower, row-major, with its diagonal (the proposal rows)
//   [DP, 2DP)    L_A packed lower, column-major, 1/L_jj on the diagonal (solve)
//   [2DP, 3DP)   L_t the same (solve)
//   [3DP, 3DP+D) x̄   |   [3DP+D, …) the observations, row-major
// Order of each quantity (as mix_gsn_kernel): the proposal row i over j
// ascending for both factors, then the pick; y_B by rows (the L_B row loaded
// once serves the proposal and the substitution); y_A = L_A⁻¹(θ° − θ) and the
// target's L_t⁻¹(x_k − θ°) as column sweeps (each row still accumulates over
// j ascending: the bits of the row forms, DESIGN.md §6 rwm_gsn_chol_kernel).
template <int D, bool FULL, int LLMODE, bool MIX>
__global__ void __launch_bounds__(256) mix_chol_kernel(const MixParams a) {
    constexpr int DP = packed_n(D);
    const ZigTabs zt = stage_lds(nullptr, a.zig, nullptr, 0, nullptr, 0);

    const uint64_t chain = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (chain >= a.C) return;
    const uint64_t C = a.C;
    const uint32_t gid = a.chain0 + (uint32_t)chain;
    const uint32_t nobs = a.nobs;

    double th[D];
    load_state<D>(a.theta, C, chain, 0, th);
    double ll = a.ll[chain];
    double ra = a.ra[chain];
    uint64_t r0 = a.ring[2 * chain], r1 = a.ring[2 * chain + 1];
    uint32_t nacc = a.nacc[chain];
    uint32_t faults = a.faults[chain];
    const double c0B = MIX ? a.c0B[chain] : 0.0;
    const SlotOffset<D> soff(C, chain, 0);

    for (uint32_t s = 0; s < a.nsteps; ++s) {
        const uint32_t iter = a.iter0 + s;  // consecutive (host splits gaps)
        const uint64_t N = a.N0 + s;
        const uint64_t slot = (uint64_t)(iter - 1);
        // ---- proposal!: pick the kernel, θ° = θ + L z
        bool useB = false;
        if constexpr (MIX) {
            const u32x4 pr = draw(a.key0, a.key1, gid, iter, kBlockMixPick, 0, 0);
            useB = u01_closed0(pr.x, pr.y) <= a.lam;
        }
        double thp[D];
        double qb = 0.0;
        {
            double z[D];
            normals<D>(zt, a.key0, a.key1, gid, iter, 0, z, faults);
            double yB[MIX ? D : 1];
            SumSqAcc<D> sb;
#pragma unroll
            for (int i = 0; i < D; ++i) {
                // one row at a time (bounded live L_B loads; the opaque pointer keeps
                // the row's scalar loads of L_A here, not hoisted out of the loops)
                __builtin_amdgcn_sched_barrier(0);
                cdouble *la = opaque_cptr(a.sconsts) + lo_idx(i, 0);
                double lzA = la[0] * z[0];
#pragma unroll
                for (int j = 1; j <= i; ++j) lzA = fma(la[j], z[j], lzA);
                double lz = lzA;
                if constexpr (MIX) {
                    const LaneSoA lb = lane_soa(C, chain, DP);
                    const LaneSoA il = lane_plain(C, chain);
                    double Lr[D];
#pragma unroll
                    for (int j = 0; j <= i; ++j) Lr[j] = *soa_ptr<DP>(a.LB, lb, lo_idx(i, j));
                    double lzB = Lr[0] * z[0];
#pragma unroll
                    for (int j = 1; j <= i; ++j) lzB = fma(Lr[j], z[j], lzB);
                    lz = useB ? lzB : lzA;
                    thp[i] = th[i] + lz;
                    double acc = thp[i] - th[i];
#pragma unroll
                    for (int j = 0; j < i; ++j) acc = fma(-Lr[j], yB[j], acc);
                    yB[i] = acc * *plain_ptr(a.iLB, il, i);
                    pin(yB[i]);
                    sb.add(i, yB[i]);
                } else {
                    thp[i] = th[i] + lz;
                }
                pin(thp[i]);
            }
            if constexpr (MIX) qb = sb.finish();
        }
        // logpdf(gsn_A, θ, θ°): y_A = L_A⁻¹(θ° − θ) as a column sweep over the solve table
        double ltd;
        {
            double acc[D];
#pragma unroll
            for (int i = 0; i < D; ++i) acc[i] = thp[i] - th[i];
            cdouble *c = opaque_cptr(a.sconsts);
            const double lpA = fma(-0.5, chol_sqmahal<D, 0>(c, c + DP, thp, acc), a.c0A);  // = c0 − q/2
            ltd = lpA;
            if constexpr (MIX) {
                const double lpB = fma(-0.5, qb, c0B);
                ltd = log_any(a.oml * exp_any(lpA) + a.lam * exp_any(lpB));
            }
        }
        // ---- compute_ll!: Σ_k logpdf(N(θ°, Σ_t), x_k) (gsn_target.jl:23-29)
        double llp;
        if constexpr (LLMODE == LL_PER_OBS) {
            llp = 0.0;
            for (uint32_t k = 0; k < nobs; ++k) {
                cdouble *c = opaque_cptr(a.sconsts);
                double acc[D];
                llp = llp + fma(-0.5, chol_sqmahal<D, D>(c + 3 * DP + D + (size_t)k * D, c + 2 * DP, thp, acc),
                                a.t_c0);
            }
        } else {
            cdouble *c = opaque_cptr(a.sconsts);
            double acc[D];
            const double qv = chol_sqmahal<D, D>(c + 3 * DP, c + 2 * DP, thp, acc);
            llp = a.n_tc0 - (a.S_c + a.nobs_d * qv) * 0.5;
        }
        if (!(llp - llp == 0.0)) faults |= 1u;
        // ---- accept_reject!
        const double llr = ((((llp - ll) + ltd) - ltd) + 0.0) - 0.0;
        const double E = exp_draw(zt, a.key0, a.key1, gid, iter, 0, faults);
        const bool acc = E > -llr;
        if constexpr (FULL) store_slot_late<D>(a.hist_prop + slot * D * C, soff, thp);
#pragma unroll
        for (int i = 0; i < D; ++i) th[i] = acc ? thp[i] : th[i];
        if (s + 1 == a.nsteps) a.ll_prop[chain] = llp;
        ll = acc ? llp : ll;
        nacc += acc ? 1u : 0u;
        if constexpr (FULL) {
            store_slot_late<D>(a.hist_theta + slot * D * C, soff, th);
            __builtin_nontemporal_store(ll, a.hist_ll + slot * C + chain);
        }
        {
            const uint64_t m = __ballot(acc);
            if ((threadIdx.x & 63) == 0) store_acc_bits<1>(a.hist_acc + slot * a.row_bytes, chain, m);
        }
        ra = rolling_update(ra, r0, r1, iter, a.W, N, a.rcp_W, acc);
        if constexpr (!FULL) store_slot_late<D>(a.mom_theta + (uint64_t)s * D * C, soff, th);
    }
    a.ll[chain] = ll;
    a.ra[chain] = ra;
    a.ring[2 * chain] = r0;
    a.ring[2 * chain + 1] = r1;
    a.nacc[chain] = nacc;
    a.faults[chain] = faults;
    if (faults) *a.fault_flag = 1u;
    store_state<D>(a.theta, C, chain, 0, th, false);
}

// ---- GenericChainStats mean/cov (chain_statistics.jl:46-49), batched ----------
// Nothing reads the running cov between readjusts (the proposals use L_B), so
// the recurrence of every step of a launch runs here, after the step kernel,
// from the θ history of the launch.  Each cov element follows exactly the
// per-step recurrence (elements are independent):
//   old = (N−1)/N·c + m_i m_j;  new = old + (θ_i θ_j)/N;  c = new − (N+1)/N·(m'_i m'_j)
//   m' = m·(N/(N+1)) + θ/(N+1)
// One block = 64 consecutive chains; one wave = one "unit" of the packed
// triangle held in registers for the whole launch: a TB×TB diagonal block
// (upper part) or half (TB×TB/2) of an off-diagonal block.  The chains' θ of a
// step is staged once per block into LDS (double-buffered, the next step's
// global load in flight while this step computes) and read by every unit, so
// HBM sees θ once and the cov once per launch.  The means are double-buffered
// across launches (`mean` in, `mean_out` out); every unit advances its own
// copy of the means it needs (the same formula, the same bits).
struct MixMomentsParams {
    const double *theta;  // θ after step s of the launch at theta + s·D·C (state_pos layout)
    const double *mean;   // [D] state_pos, before the launch
    double *mean_out;     // [D] state_pos, after the launch (written by the diagonal units)
    double *cov;          // [DP] packed upper
    const double *kst;    // [nsteps][8] per-step scalars (moments_consts_kernel)
    uint64_t C;
    uint64_t N0;          // GenericChainStats.N at the launch's first step
    uint32_t nsteps;
};

#ifdef EMCMC_HOST_UNIT
// The step-dependent scalars of the recurrence, (N, N+1, (N−1)/N, N/(N+1),
// (N+1)/N, 1/N, 1/(N+1)) for the launch's steps, computed once per launch
// (the same IEEE divisions, so the same bits) instead of by every lane of
// every wave; the moments kernel reads them with scalar loads.
__global__ void __launch_bounds__(64) moments_consts_kernel(uint64_t N0, uint32_t nsteps, double *kst) {
    const uint32_t s = blockIdx.x * 64u + threadIdx.x;
    if (s >= nsteps) return;
    const uint64_t N = N0 + s;
    const double Nd = (double)N, N1d = (double)(N + 1);
    double *k = kst + 8 * (uint64_t)s;
    k[0] = Nd;
    k[1] = N1d;
    k[2] = (double)(N - 1) / Nd;
    k[3] = Nd / N1d;
    k[4] = N1d / Nd;
    k[5] = 1.0 / Nd;
    k[6] = 1.0 / N1d;
    k[7] = 0.0;
}

#endif  // EMCMC_HOST_UNIT

template <int D>
struct MomentTiles {
    static constexpr int TB = D <= 8 ? D : 8;                 // block edge
    static constexpr int NB = D / TB;                         // blocks per edge
    static constexpr int HALF = TB == 8 ? 4 : TB;             // columns per off-diagonal unit
    static constexpr int NOFF = NB * (NB - 1) / 2 * (TB / HALF);
    static constexpr int NU = NB + NOFF;                      // units of the packed triangle
    static constexpr int WPB = NU < 8 ? NU : 8;               // waves per block
    static constexpr int UPW = NU / WPB;                      // units per wave (1 or 2)
    static constexpr int BLOCK = 64 * WPB;
    static constexpr int PR = (D % 2 == 0) ? D / 2 : D;       // LDS rows: coordinate pairs (even D) or coordinates
    static constexpr int EW = (D % 2 == 0) ? 2 : 1;           // doubles per row element
    static constexpr int NPF = (PR * 64 + BLOCK - 1) / BLOCK; // staged row elements per thread
    static_assert(NU % WPB == 0, "units per wave");
};

// unit U → its block of the packed triangle (compile time)
template <int D, int U>
struct MomentUnit {
    using MT = MomentTiles<D>;
    static constexpr bool DIAG = U < MT::NB;
    static constexpr int O = DIAG ? 0 : U - MT::NB, PER = MT::TB / MT::HALF;
    static constexpr int bi_of(int p, int bi) { return p < MT::NB - 1 - bi ? bi : bi_of(p - (MT::NB - 1 - bi), bi + 1); }
    static constexpr int p_of(int p, int bi) { return p < MT::NB - 1 - bi ? p : p_of(p - (MT::NB - 1 - bi), bi + 1); }
    static constexpr int BI = DIAG ? U : bi_of(O / PER, 0);
    static constexpr int I0 = BI * MT::TB;
    static constexpr int J0 = DIAG ? I0 : (BI + 1 + p_of(O / PER, 0)) * MT::TB + (O % PER) * MT::HALF;
    static constexpr int NJ = DIAG ? MT::TB : MT::HALF;
    static constexpr int NC = DIAG ? MT::TB * (MT::TB + 1) / 2 : MT::TB * NJ;
    // register slot of element (u, v): diagonal units u ≤ v (row-major upper),
    // off-diagonal units u·NJ + v
    static constexpr int slot(int u, int v) { return DIAG ? u * MT::TB - u * (u - 1) / 2 + (v - u) : u * NJ + v; }
};

// One unit's registers for the whole launch: its cov block and the means of
// its rows / columns (each unit advances its own copy of the means: the same
// formula, the same bits).
template <int D, int U>
struct MomentUnitState {
    using MT = MomentTiles<D>;
    using UT = MomentUnit<D, U>;
    static constexpr int TB = MT::TB, NJ = UT::NJ, I0 = UT::I0, J0 = UT::J0, DP = packed_n(D);
    static constexpr bool DIAG = UT::DIAG;
    double c[UT::NC], mi[TB], mj[DIAG ? 1 : NJ];

    __device__ __forceinline__ void load(const MixMomentsParams &a, uint64_t chain) {
        const LaneSoA lm = lane_soa(a.C, chain, D), lc = lane_soa(a.C, chain, DP);
#pragma unroll
        for (int u = 0; u < TB; ++u) mi[u] = *soa_ptr<D>(a.mean, lm, I0 + u);
        if constexpr (!DIAG) {
#pragma unroll
            for (int v = 0; v < NJ; ++v) mj[v] = *soa_ptr<D>(a.mean, lm, J0 + v);
        }
#pragma unroll
        for (int u = 0; u < TB; ++u)
#pragma unroll
            for (int v = DIAG ? u : 0; v < NJ; ++v) c[UT::slot(u, v)] = *soa_ptr<DP>(a.cov, lc, up_idx(D, I0 + u, J0 + v));
    }
    // one step of chain_statistics.jl:46-49 with θ from the staged rows
    // ROWS_NEW: the new row means of another unit of the same wave with the same
    // row block, already advanced this step (the same formula, so the same bits):
    // taken instead of recomputed; nullptr: advance them here
    template <typename TH>
    __device__ __forceinline__ void step(TH theta_at, double Nd, double N1d, double ca, double cb, double cc, double rN,
                                         double rN1, const double *rows_new) {
        double ti[TB], tj[NJ];
#pragma unroll
        for (int u = 0; u < TB; ++u) ti[u] = theta_at(I0 + u);
#pragma unroll
        for (int v = 0; v < NJ; ++v) tj[v] = DIAG ? ti[v] : theta_at(J0 + v);
        // old_sq + (θ_i θ_j)/N with the means before the step, then the means
        // (m' = m·cb + θ/(N+1)) and the subtraction
#pragma unroll
        for (int u = 0; u < TB; ++u) {
            __builtin_amdgcn_sched_barrier(0);  // one row at a time: bounded live temporaries
#pragma unroll
            for (int v = DIAG ? u : 0; v < NJ; ++v) {
                const double old_sq = ca * c[UT::slot(u, v)] + mi[u] * (DIAG ? mi[v] : mj[v]);
                c[UT::slot(u, v)] = old_sq + div_markstein(ti[u] * tj[v], Nd, rN);
            }
        }
        if (rows_new) {
#pragma unroll
            for (int u = 0; u < TB; ++u) mi[u] = rows_new[u];
        } else {
#pragma unroll
            for (int u = 0; u < TB; ++u) mi[u] = mi[u] * cb + div_markstein(ti[u], N1d, rN1);
        }
        if constexpr (!DIAG) {
#pragma unroll
            for (int v = 0; v < NJ; ++v) mj[v] = mj[v] * cb + div_markstein(tj[v], N1d, rN1);
        }
#pragma unroll
        for (int u = 0; u < TB; ++u) {
            __builtin_amdgcn_sched_barrier(0);
#pragma unroll
            for (int v = DIAG ? u : 0; v < NJ; ++v)
                c[UT::slot(u, v)] = c[UT::slot(u, v)] - cc * (mi[u] * (DIAG ? mi[v] : mj[v]));
        }
    }
    __device__ __forceinline__ void store(const MixMomentsParams &a, uint64_t chain) const {
        // fresh opaque strides: the load addresses are not kept live across the sweep
        const LaneSoA lm = lane_soa(a.C, chain, D), lc = lane_soa(a.C, chain, DP);
#pragma unroll
        for (int u = 0; u < TB; ++u)
#pragma unroll
            for (int v = DIAG ? u : 0; v < NJ; ++v) *soa_ptr<DP>(a.cov, lc, up_idx(D, I0 + u, J0 + v)) = c[UT::slot(u, v)];
        if constexpr (DIAG) {
#pragma unroll
            for (int u = 0; u < TB; ++u) *soa_ptr<D>(a.mean_out, lm, I0 + u) = mi[u];
        }
    }
};

// Units of wave W: W and W + WPB, except at D = 32 (16 units, 2 per wave), where
// the pairs are chosen so that 6 of the 8 waves hold two units of one row block
// and advance its 8 row means once: (0,4) (5,6) (7,8) (9,13) (1,10) (11,12)
// (2,14) (15,3) — the diagonal unit of each row block first, so it stores them.
template <int D>
struct MomentPairs {
    static constexpr int WPB = MomentTiles<D>::WPB;
    static constexpr int a(int W) {
        constexpr int t[8] = {0, 5, 7, 9, 1, 11, 2, 15};
        return (MomentTiles<D>::NU == 16 && WPB == 8) ? t[W] : W;
    }
    static constexpr int b(int W) {
        constexpr int t[8] = {4, 6, 8, 13, 10, 12, 14, 3};
        return (MomentTiles<D>::NU == 16 && WPB == 8) ? t[W] : W + WPB;
    }
};

// The whole launch sweep of wave W (units a(W) and b(W)); every wave runs the
// same number of block barriers.
template <int D, int W>
__device__ __forceinline__ void moments_wave(const MixMomentsParams &a, double *stage0, double *stage1) {
    using MT = MomentTiles<D>;
    constexpr int PR = MT::PR, EW = MT::EW, NPF = MT::NPF;
    constexpr bool TWO = MT::UPW == 2;
    typedef double rowv __attribute__((ext_vector_type(EW)));
    const int lane = threadIdx.x & 63;
    const uint64_t C = a.C;
    const uint64_t c0 = (uint64_t)blockIdx.x * 64u;
    const uint64_t chain = c0 + (uint64_t)lane;
    const bool live = chain < C;
    const uint64_t cl = live ? chain : c0;  // chains past C read chain c0's values and store nothing
    auto fetch = [&](uint32_t s, rowv (&pf)[NPF]) {
        const rowv *src = reinterpret_cast<const rowv *>(a.theta + (uint64_t)s * D * C);
#pragma unroll
        for (int q = 0; q < NPF; ++q) {
            const int e = (int)threadIdx.x + q * MT::BLOCK;
            const int k = e >> 6, l = e & 63;
            const uint64_t cc = (c0 + (uint64_t)l < C) ? c0 + (uint64_t)l : c0;
            pf[q] = (e < PR * 64) ? __builtin_nontemporal_load(src + soa_row((uint64_t)k, cc, C, (uint64_t)PR)) : rowv{};
        }
    };
    auto put = [&](double *st, const rowv (&pf)[NPF]) {
        rowv *dst = reinterpret_cast<rowv *>(st);
#pragma unroll
        for (int q = 0; q < NPF; ++q) {
            const int e = (int)threadIdx.x + q * MT::BLOCK;
            if (e < PR * 64) dst[e] = pf[q];
        }
    };
    constexpr int UA = MomentPairs<D>::a(W), UB = TWO ? MomentPairs<D>::b(W) : UA;
    constexpr bool SHARE_ROWS = TWO && MomentUnit<D, UA>::I0 == MomentUnit<D, UB>::I0;
    MomentUnitState<D, UA> ua;
    MomentUnitState<D, UB> ub;
    ua.load(a, cl);
    if constexpr (TWO) ub.load(a, cl);
    {
        rowv pf[NPF];
        fetch(0, pf);
        put(stage0, pf);
    }
    __syncthreads();
    for (uint32_t s = 0; s < a.nsteps; ++s) {
        const double *st = (s & 1u) ? stage1 : stage0;
        rowv pf[NPF];
        if (s + 1 < a.nsteps) fetch(s + 1, pf);  // in flight during this step
        auto theta_at = [&](int d) -> double {
            const rowv v = reinterpret_cast<const rowv *>(st)[(EW == 2 ? d >> 1 : d) * 64 + lane];
            if constexpr (EW == 2) return (d & 1) ? v[1] : v[0];
            else return v[0];
        };
        const double *k = a.kst + 8 * (uint64_t)s;  // wave-uniform: scalar loads
        const double Nd = k[0], N1d = k[1], ca = k[2], cb = k[3], cc = k[4], rN = k[5], rN1 = k[6];
        ua.step(theta_at, Nd, N1d, ca, cb, cc, rN, rN1, nullptr);
        if constexpr (TWO) ub.step(theta_at, Nd, N1d, ca, cb, cc, rN, rN1, SHARE_ROWS ? ua.mi : nullptr);
        if (s + 1 < a.nsteps) put((s & 1u) ? stage0 : stage1, pf);
        __syncthreads();
    }
    if (!live) return;
    ua.store(a, chain);
    if constexpr (TWO) ub.store(a, chain);
}

template <int D, int W>
__device__ __forceinline__ void moments_dispatch(int wave, const MixMomentsParams &a, double *stage0, double *stage1) {
    if constexpr (W < MomentTiles<D>::WPB) {
        if (wave == W) moments_wave<D, W>(a, stage0, stage1);
        else moments_dispatch<D, W + 1>(wave, a, stage0, stage1);
    }
}

template <int D>
__global__ void __launch_bounds__(MomentTiles<D>::BLOCK) mix_moments_kernel(const MixMomentsParams a) {
    using MT = MomentTiles<D>;
    __shared__ __attribute__((aligned(16))) double stage[2][MT::PR * 64 * MT::EW];
    const int wave = __builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6));  // wave-uniform
    moments_dispatch<D, 0>(wave, a, stage[0], stage[1]);
}

// ---- HaarioTypeAdaptation readjust! (adaptation.jl:422-426) -----------------
struct MixReadjustParams {
    const double *cov;  // [DP] packed upper
    double *LB;         // [DP] packed lower
    double *iLB;        // [D][C]
    double *c0B;        // [C]
    uint32_t *faults;
    uint32_t *fault_flag;
    uint64_t C;
    double sB;  // 2.38²/D
};

// R lanes per chain (R = D rounded up to a power of two), 64/R chains per wave,
// 4 waves per block.
template <int D>
struct ReadjustShape {
    static constexpr int R = D <= 1 ? 1 : D <= 2 ? 2 : D <= 4 ? 4 : D <= 8 ? 8 : D <= 16 ? 16 : 32;
    static constexpr int CPW = 64 / R;
    static constexpr int CPB = 4 * CPW;
};

// Σ_B = sB·cov; L_B = cholesky(Symmetric(Σ_B)).L in the canonical order of
// oracle/emcmc_oracle.c orc_cholesky (each element's sum over k ascending, the
// products rounded before the subtraction).  Lane i of a chain's R lanes owns
// row i; a sweep over the columns j = 0..D−1: lane j takes the square root of
// its finished diagonal sum and publishes it, then every lane i > j forms
// L_ij = (Σ_B,ij − Σ_{k<j} L_ik L_jk) / L_jj with row j read from LDS
// (broadcast), publishes L_ij and subtracts L_ij² from its own diagonal sum.
template <int D>
__global__ void __launch_bounds__(256) mix_readjust_kernel(const MixReadjustParams a) {
    using RS = ReadjustShape<D>;
    constexpr int R = RS::R, CPW = RS::CPW, DP = packed_n(D);
    __shared__ double Ls[4 * CPW][DP];  // each chain's factor, packed lower (row-major)
    __shared__ double dgs[4 * CPW][D];
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const int g = lane / R, i = lane % R;
    const int lc = w * CPW + g;
    const uint64_t C = a.C;
    const uint64_t chain = (uint64_t)blockIdx.x * RS::CPB + (uint64_t)lc;
    const bool live = chain < C && i < D;
    const uint64_t cl = chain < C ? chain : 0;  // tail lanes read chain 0 and write nothing
    const int ic = i < D ? i : D - 1;
    // column i of the upper triangle: Σ_B[j][i] = sB·cov(j, i), j ≤ i
    double col[D], row[D];
    {
        const LaneSoA lp = lane_soa(C, cl, DP);
#pragma unroll
        for (int j = 0; j < D; ++j) {
            // up_idx(D, j, i) for j ≤ i (lanes with j > i read their own diagonal: unused)
            const int jj = j <= ic ? j : ic;
            col[j] = a.sB * *soa_ptr_dyn<DP>(a.cov, lp, up_idx(D, jj, ic));
        }
    }
    double s = col[D - 1];  // replaced below by the diagonal once j reaches i
#pragma unroll
    for (int j = 0; j < D; ++j)
        if (j == ic) s = col[j];  // Σ_B[i][i]
    bool ok = true;
#pragma unroll
    for (int j = 0; j < D; ++j) {
        if (live && i == j) {
            ok = s > 0.0;
            const double d = sqrt(s);
            row[j] = d;
            dgs[lc][j] = d;
            Ls[lc][lo_idx(j, j)] = d;
        }
        wave_lds_sync();
        if (live && i > j) {
            double t = col[j];
#pragma unroll
            for (int k = 0; k < j; ++k) t = t - row[k] * Ls[lc][lo_idx(j, k)];
            row[j] = t / dgs[lc][j];
            Ls[lc][lo_idx(i, j)] = row[j];
            s = s - row[j] * row[j];
        }
        wave_lds_sync();
    }
    // every row of the chain must have had a positive diagonal (NaN fails)
    const uint64_t okm = __ballot(!live || ok);
    const uint64_t gm = (R == 64 ? ~0ull : ((1ull << R) - 1)) << (g * R);
    const bool chain_ok = (okm & gm) == gm;
    if (chain >= C) return;
    if (!chain_ok) {
        if (i == 0) {
            a.faults[chain] |= 4u;  // EMCMC_FAULT_POSDEF
            *a.fault_flag = 1u;
        }
        return;
    }
    if (i >= D) return;
    {
        const LaneSoA lp = lane_soa(C, chain, DP);
#pragma unroll
        for (int j = 0; j < D; ++j)
            if (j <= i) *soa_ptr_dyn<DP>(a.LB, lp, lo_idx(i, j)) = row[j];
    }
    double dgi = 0.0;
#pragma unroll
    for (int j = 0; j < D; ++j)
        if (j == i) dgi = row[j];
    a.iLB[(uint64_t)i * C + chain] = 1.0 / dgi;
    dgs[lc][i] = log_pos(dgi);
    wave_lds_sync();
    if (i == 0) {
        double dd = 0.0;
#pragma unroll
        for (int k = 0; k < D; ++k) dd = dd + dgs[lc][k];
        a.c0B[chain] = -((double)D * kLog2Pi + (dd + dd)) / 2.0;
    }
}

}  // namespace emcmc
