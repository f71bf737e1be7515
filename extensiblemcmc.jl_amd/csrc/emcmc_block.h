// emcmc_block.h — one update over all D coordinates at 17 ≤ D ≤ 64: MALA and
// user-defined updates with every per-chain vector in registers (gfx950).
//
// The general kernel (emcmc_mwg.h mwg_wide_kernel) handles any schedule, but an
// update of NU > 16 coordinates keeps its local vectors in rolled loops, and
// their dynamic indexing puts them in scratch (2.3 KB per lane at NU = 32): the
// D² triangular solves of the likelihood then run out of scratch memory.  This
// kernel serves the drop-in shapes the plugin surface is for — one MALA update
// or one user update (updates.jl:42-93, 129-133; run.jl:110, 259) over θ with
// coords = 1:D, ImproperPrior, P = 1 — with the schedule loop of mwg_wide_kernel
// and the same arithmetic, bit for bit:
//   - every per-chain vector (θ, ∇ℓ(θ), θ°, ∇ℓ(θ°), the solve accumulators) is a
//     register array indexed only by compile-time constants (static_for);
//   - the target's factor, x̄ and the observations stream through the scalar
//     cache as in rwm_gsn_chol_kernel (chol_stream): the forward substitution
//     of loglikelihood(P°, obs) per observation, and for ∇ℓ the forward sweep
//     followed by the backward one over a reversed row table (same row sums in
//     the same order as GsnTarget::grad);
//   - ∇ℓ(θ) is carried in registers across the launch's steps (mala_carry's
//     argument: with one update over all coordinates it is the previous step's
//     proposal gradient if accepted, else its own) and computed at the launch's
//     first step;
//   - a user update's proposal!/log_transition_density and a user law run on
//     copies of the vectors, so only those copies can end up in scratch when the
//     user's loops are not unrolled; the kernel's own vectors stay in registers.
// Oracle: orc_run_mwg (kinds 4 and 5), exactly as for mwg_wide_kernel.
#pragma once

#include "emcmc_mwg.h"

namespace emcmc {

constexpr int kBlockMinD = 17;  // D ≤ 16: mwg_gsn_kernel holds everything in registers already

// Constant table of the block kernel (address space 4, doubles), P = D(D+1)/2:
//   [0, P)       L_t forward-solve table: packed column-major lower, 1/L_jj on the diagonal
//   [P, 2P)      L_t backward-solve table: rows j = D−1 … 0, each [1/L_jj, L_j0, …, L_j,j−1]
//   [2P, 2P+D)   x̄
//   [2P+D, 2P+2D) 1/L_t,ii
//   [2P+2D, …)   observations, row-major (per-observation likelihood)
template <int D>
struct BlockConsts {
    static constexpr int P = D * (D + 1) / 2;
    static constexpr int kFwd = 0, kBwd = P, kXbar = 2 * P, kInvDiag = 2 * P + D, kObs = 2 * P + 2 * D;
};

// The built-in GsnTargetLaw through the scalar cache: GsnTarget's loglik / grad
// (emcmc_mwg.h) with the same operations in the same order.  TDENSE = false: a
// diagonal Σ_t (GsnTarget's tdiag branch, no substitution).
template <bool TDENSE>
struct GsnSweep {
    // ‖L_t⁻¹(x − m)‖², x from the table at xoff (forward substitution as column updates)
    template <int D>
    __device__ __forceinline__ static double sqmahal(const MwgParams &a, int xoff, const double (&m)[D]) {
        using K = BlockConsts<D>;
        cdouble *c = opaque_cptr(a.consts);
        if constexpr (TDENSE) {
            double acc[D];
            return chol_sqmahal<D, D>(c + xoff, c + K::kFwd, m, acc);
        } else {
            cdouble *x = c + xoff;
            cdouble *il = c + K::kInvDiag;
            return canon_sumsq_f<D, 1, D>([&](int i) { return (x[i] - m[i]) * il[i]; });
        }
    }
    template <int D, int LLMODE, bool ROLL = false>
    __device__ __forceinline__ static double loglik(const MwgParams &a, const double (&mp)[D]) {
        using K = BlockConsts<D>;
        if constexpr (LLMODE == LL_PER_OBS) {
            double llp = 0.0;
            for (uint32_t k = 0; k < a.nobs; ++k)
                llp = llp + fma(-0.5, sqmahal<D>(a, K::kObs + (int)k * D, mp), a.t_c0);  // t_c0 − q/2
            return llp;
        } else {
            const double qv = sqmahal<D>(a, K::kXbar, mp);
            return a.n_tc0 - (a.S_c + a.nobs_d * qv) * 0.5;
        }
    }
    // ∇_μ loglikelihood = n·L_t⁻ᵀ L_t⁻¹ (x̄ − μ): GsnTarget::grad's forward and backward
    // substitutions (row sums over j ascending, then over j descending)
    template <int D, int LLMODE, bool ROLL = false>
    __device__ __forceinline__ static void grad(const MwgParams &a, const double (&mp)[D], double (&g)[D]) {
        using K = BlockConsts<D>;
        cdouble *c = opaque_cptr(a.consts);
        if constexpr (TDENSE) {
            double acc[D];
            // forward: acc_i = x̄_i − μ_i, y_j = acc_j / L_jj kept in acc[j]
            chol_stream<D, D>(
                c + K::kXbar, c + K::kFwd,
                [&](auto IC, double x) {
                    constexpr int i = decltype(IC)::value;
                    acc[i] = x - mp[i];
                    vpin(acc[i]);
                },
                [&](auto JC, auto IC, double v) {
                    constexpr int j = decltype(JC)::value, i = decltype(IC)::value;
                    if constexpr (i == j) acc[j] = acc[j] * v;
                    else acc[i] = fma(-v, acc[j], acc[i]);
                    vpin(acc[i]);
                });
            // backward: step t handles row j = D−1−t: g_j = acc_j / L_jj, then acc_i −= L_ji g_j (i < j)
            chol_stream<D, 0>(
                c + K::kBwd, c + K::kBwd, [&](auto, double) {},
                [&](auto TC, auto IC, double v) {
                    constexpr int t = decltype(TC)::value, off = decltype(IC)::value - t, j = D - 1 - t;
                    if constexpr (off == 0) {
                        g[j] = acc[j] * v;
                        vpin(g[j]);
                    } else {
                        acc[off - 1] = fma(-v, g[j], acc[off - 1]);
                        vpin(acc[off - 1]);
                    }
                });
        } else {
            cdouble *x = c + K::kXbar;
            cdouble *il = c + K::kInvDiag;
#pragma unroll
            for (int i = 0; i < D; ++i) {
                const double y = (x[i] - mp[i]) * il[i];
                g[i] = y * il[i];
            }
        }
#pragma unroll
        for (int i = 0; i < D; ++i) g[i] = a.nobs_d * g[i];
    }
};

template <class T>
struct IsGsnSweep {
    static constexpr bool value = false;
};
template <bool B>
struct IsGsnSweep<GsnSweep<B>> {
    static constexpr bool value = true;
};

// normals g0 … g0+N−1 of (chain, iter, update 0): normals() from normal index g0 (even)
template <int N>
__device__ __forceinline__ void normals_from(const ZigTabs &zt, uint32_t key0, uint32_t key1, uint32_t chain,
                                             uint32_t iter, uint32_t g0, double (&z)[N], uint32_t &faults,
                                             const PhiloxVKeys &vk) {
    constexpr int NP = (N + 1) / 2;
    uint64_t pend = 0;
#pragma unroll
    for (int j = 0; j < NP; ++j) {
        __builtin_amdgcn_sched_barrier(0);  // one Philox block at a time
        const u32x4 r = draw_vk(vk, chain, iter, (g0 >> 1) + j, 0u);
        if (!zig_normal_fast(zig_split_n(r.x, r.y), zt.n, z[2 * j])) pend |= 1ull << (2 * j);
        if (2 * j + 1 < N)
            if (!zig_normal_fast(zig_split_n(r.z, r.w), zt.n, z[2 * j + 1])) pend |= 1ull << (2 * j + 1);
    }
    while (__ballot(pend != 0) != 0) {
        if (pend != 0) {
            const int i = __builtin_ctzll(pend);
            pend &= pend - 1;
            const double v = normal_draw(zt, key0, key1, chain, iter, 0u, g0 + (uint32_t)i, faults);
#pragma unroll
            for (int q = 0; q < N; ++q)
                if (q == i) z[q] = v;
        }
    }
}

template <int D, bool FULL, int LLMODE, class TGT, class UPD>
__global__ void __launch_bounds__(256) mwg_block_kernel(const MwgParams a) {
    static_assert(D >= kBlockMinD && D <= kMwgMaxD, "one update over 17 ≤ D ≤ 64 coordinates");
    static_assert(UPD::kEnabled || UPD::kMala, "a user update or MALA");
    constexpr int BLK = SumShape<D>::BLK, NB = D / BLK;
    const ZigTabs zt = stage_lds(nullptr, a.zig, nullptr, 0, nullptr, 0);
    const uint64_t chain = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (chain >= a.C) return;
    const uint64_t C = a.C;
    const uint32_t gid = a.chain0 + (uint32_t)chain;
    const uint32_t c32 = (uint32_t)chain;
    const SlotOffset<D> soff(C, chain, 0);
    const MwgUpdate &u = a.updates[0];
    double th[D];
    load_slot<D>(a.theta, soff, th);
    double ll = chain_elem(a.ll, c32);
    uint32_t faults = chain_elem(a.faults, c32);
    AcceptStream accs;
    const PhiloxVKeys vkeys = philox_vkeys(a.key0, a.key1);
    uint32_t prev_iter = 0;

    for (uint32_t s = 0; s < a.nsteps; ++s) {
        const uint32_t iter = a.steps[4 * s], flags = a.steps[4 * s + 2];
        // the accept draws of iterations 2m, 2m+1 share one Philox block: it is reused only
        // when this step directly follows the previous one (a schedule may skip iterations)
        const bool fresh = (s == 0) || iter != prev_iter + 1;
        prev_iter = iter;
        const uint64_t slot = (uint64_t)(iter - 1);
        double tp[D];
        double ltd_fwd, ltd_rev;
        if constexpr (UPD::kEnabled) {
            // proposal!(updt, …) and log_transition_density both ways of the user's update
            // (updates.jl:42-93), on copies: the user's loops may index them dynamically
            UserRng rng{zt, a.key0, a.key1, gid, iter, 0u, 0u};
            double ux[D], uy[D];
#pragma unroll
            for (int j = 0; j < D; ++j) {
                ux[j] = th[j];
                uy[j] = 0.0;
            }
            UPD::propose(rng, ux, uy, D, u.L);
            faults |= rng.faults;
            ltd_fwd = UPD::ltd(ux, uy, D, u.L);  // log_transition_density(__PREVIOUS): (θ, θ°)
            ltd_rev = UPD::ltd(uy, ux, D, u.L);  // (__PROPOSAL): (θ°, θ)
#pragma unroll
            for (int j = 0; j < D; ++j) tp[j] = uy[j];
        } else {
            // compute_gradients_and_momenta!(__PREVIOUS) (run.jl:110): ∇ℓ(θ) at the launch's
            // first step, afterwards the carried value (gcache: ∇ℓ(θ°) of an accepted step,
            // else unchanged) — HBM/L2, so it holds no registers through the sweeps
            double g[D];
            if (s == 0) {
                TGT::template grad<D, LLMODE>(a, th, g);
                store_slot_cached<D>(a.gcache, soff, g);
            } else {
                load_slot<D>(a.gcache, soff, g);
            }
            // θ° = m + ϵz, m = θ + h·∇ℓ(θ), and log_transition_density(θ → θ°) =
            // logpdf(MvNormal(m, ϵ²I), θ°), one canonical block of normals at a time.  MALA's
            // factor is ϵI: every 1/L_jj is the same 1/ϵ (emcmc_add_update)
            const double eps = u.eps0[0], h = u.eps0[1], il = u.iL[0];
            double bq[NB];
            static_for<0, NB>([&](auto BC) {
                constexpr int b = decltype(BC)::value;
                double z[BLK];
                normals_from<BLK>(zt, a.key0, a.key1, gid, iter, (uint32_t)(b * BLK), z, faults, vkeys);
                double sb = 0.0;
#pragma unroll
                for (int i = 0; i < BLK; ++i) {
                    const int j = b * BLK + i;
                    const double m = th[j] + h * g[j];
                    tp[j] = m + eps * z[i];
                    const double y = (tp[j] - m) * il;
                    sb = (i == 0) ? y * y : fma(y, y, sb);
                }
                bq[b] = sb;
            });
            ltd_fwd = u.c0 - tree_inplace<NB>(bq) / 2.0;
        }
        // ---- set_proposal!: P°.θ ← θ° (every coordinate); compute_ll! at P°
        double llp;
        if constexpr (IsGsnSweep<TGT>::value) {
            llp = TGT::template loglik<D, LLMODE>(a, tp);
        } else {  // a user law: on a copy (see above)
            double um[D];
#pragma unroll
            for (int j = 0; j < D; ++j) um[j] = tp[j];
            llp = TGT::template loglik<D, LLMODE>(a, um);
        }
        double gp[UPD::kEnabled ? 1 : D];  // ∇ℓ(θ°): the next step's ∇ℓ(θ) if accepted
        if constexpr (!UPD::kEnabled) {
            // compute_gradients_and_momenta!(__PROPOSAL) (run.jl:259); the reverse density
            // logpdf(MvNormal(θ° + h·∇ℓ(θ°), ϵ²I), θ)
            TGT::template grad<D, LLMODE>(a, tp, gp);
            const double h = u.eps0[1], il = u.iL[0];
            ltd_rev = u.c0 - canon_sumsq_f<D, 1, D>([&](int j) { return (th[j] - (tp[j] + h * gp[j])) * il; }) / 2.0;
        }
        if (!(llp - llp == 0.0)) faults |= 1u;
        // ---- accept_reject! (run.jl:268-281): ImproperPrior contributes +0.0 − 0.0
        const double llr = ((((llp - ll) + ltd_rev) - ltd_fwd) + 0.0) - 0.0;
        const double E = accs.next<true>(zt, a.key0, a.key1, gid, iter, 0u, fresh, faults, vkeys);
        const bool acc = E > -llr;
        if constexpr (FULL) store_slot_late<D>(a.hist_prop + slot * D * C, soff, tp);  // run.jl:237-239
#pragma unroll
        for (int j = 0; j < D; ++j) th[j] = acc ? tp[j] : th[j];  // set_chain_param! (run.jl:312-318)
        if constexpr (!UPD::kEnabled)
            if (acc) store_slot_cached<D>(a.gcache, soff, gp);
        ll = acc ? llp : ll;
        if constexpr (FULL) {
            store_slot_late<D>(a.hist_theta + slot * D * C, soff, th);
            __builtin_nontemporal_store(ll, &chain_elem(a.hist_ll + slot * C, c32));
        }
        mwg_register_step(a, u, (uint32_t)D, chain, iter, 0u, s, flags, slot, acc);
        if (s + 1 == a.nsteps) {
            chain_elem(a.ll_prop, c32) = llp;        // sub_ws°.ll: the last proposal's
            store_slot_cached<D>(a.mu_p, soff, tp);  // P°.θ = the last θ° (every coordinate)
        }
    }
    chain_elem(a.ll, c32) = ll;
    chain_elem(a.faults, c32) = faults;
    if (faults) *a.fault_flag = 1u;
    store_slot_cached<D>(a.theta, soff, th);
}

}  // namespace emcmc
