// emcmc_fused.h — the fused single-update step kernels on LDS constants:
// rwm_gsn_diag_kernel (diagonal Σ_rw and Σ_t, LPC lanes per chain: the cfg 2
// hot kernel) and rwm_gsn_dense_kernel (dense factors, D ≤ 8).  Kept out of
// emcmc_kernels.h, whose text the run-time compiler embeds (emcmc_rtc.hip): a
// change here does not invalidate the on-disk code-object cache.
#pragma once

#include "emcmc_kernels.h"

namespace emcmc {

// threads per block of the diag kernel: one block per CU holds 256·MINW
// threads when MINW ≥ 3, so a single copy of the 70 KiB of tables serves
// MINW waves per SIMD (two 256-thread blocks, each with its own copy, are
// all the LDS allows)
// MINW = 2 with sibling pacing (below): one 512-thread block per CU, whose two
// waves on each SIMD keep pace with each other; 256 threads otherwise
constexpr int diag_block(int MINW) { return MINW >= 3 ? 256 * MINW : MINW == 2 ? 512 : 256; }

// Sibling pacing.  Two waves share a SIMD at MINW = 2, and the SIMD issues for the
// older one whenever it is ready (age order), so it runs ahead: on MI355X the older
// wave of a pair finished its 100 steps at ≈ 0.78 of the pair's time and the younger
// one ran the rest alone, at 0.21 steps/µs per SIMD instead of the pair's 0.33
// (scripts/trace_diag.py, profiles/r4_pace/).  With both waves in one workgroup each
// finds its sibling (the other wave on its SIMD, from HW_ID) and, at every step,
// publishes its step count in LDS and lowers its issue priority when it is ahead of
// the sibling, raises it when behind: the pair stays within a step of each other and
// the SIMD keeps two waves' worth of overlap to the end.  No result depends on it.
struct SiblingPace {
    uint32_t *prog;  // [waves per block] steps done, in LDS
    int me, sib;     // wave in block; sibling wave (−1: none)
    __device__ __forceinline__ void publish(uint32_t steps_done) const {
        if ((threadIdx.x & 63) == 0) __hip_atomic_store(prog + me, steps_done, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
        if (sib < 0) return;
        const uint32_t o = __hip_atomic_load(prog + sib, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
        const uint32_t other = (uint32_t)__builtin_amdgcn_readfirstlane((int)o);
        if (steps_done > other) __builtin_amdgcn_s_setprio(0);
        else if (steps_done < other) __builtin_amdgcn_s_setprio(2);
        else __builtin_amdgcn_s_setprio(1);
    }
};

// The update's separable terms in the fused step.  NoFusedPrior: GaussianRandomWalk with
// ImproperPrior (the cfg 2 kernel, whose ratio adds + 0.0 − 0.0).  emcmc_fprior.h FusedUpdate<S>
// (compiled at run time) supplies kOn (a prior term), kUniform (UniformRandomWalk's proposal and
// transition densities, propose_uniform), the prior's constants per coordinate (kConsts doubles
// per coordinate, staged in LDS after the kernel's own), eval<D, LPC, DPL>(consts, d0, x) =
// logpdf(prior, θ) of the chain (every lane of the chain gets the same double), the proposal!
// redraw cap and its fault bit.
struct NoFusedPrior {
    static constexpr bool kOn = false;
    static constexpr bool kUniform = false;
    static constexpr bool kRoundTrip = false;  // GaussianRandomWalk's positivity round trips
    static constexpr int kConsts = 0;
};

// MINW = minimum waves per SIMD the register allocation must allow
// (__launch_bounds__ second argument; 4 ⇒ ≤ 128 VGPRs).
// PR: the update's separable terms (NoFusedPrior: GaussianRandomWalk, ImproperPrior; emcmc_fprior.h
// FusedUpdate<S>, compiled at run time for the structure).
template <int D, int LPC, bool FULL, int LLMODE, bool UNIT_T, int MINW = 1, class PR = NoFusedPrior>
__global__ void __launch_bounds__(diag_block(MINW), MINW) rwm_gsn_diag_kernel(const StepParams a) {
    static_assert(D % LPC == 0, "D must split evenly over the chain's lanes");
    constexpr int DPL = D / LPC;  // coordinates per lane
    static_assert(LPC == 1 || DPL % 8 == 0, "multi-lane chains need whole 8-blocks");
    static_assert(LPC == 1 || DPL % 2 == 0, "normal pairs must not straddle lanes");

    extern __shared__ __attribute__((aligned(16))) double lds[];
    const uint32_t nobs = a.nobs;
    constexpr int kPrc = PR::kConsts;  // prior constants per coordinate, after the kernel's own 4
    const int nconst = (4 + kPrc) * D;
    constexpr bool kPace = MINW == 2;
    constexpr int kWavesPerBlock = diag_block(MINW) / 64;
    __shared__ uint32_t pace_prog[kWavesPerBlock], pace_simd[kWavesPerBlock];
    if constexpr (kPace) {
        if ((threadIdx.x & 63) == 0) {
            pace_simd[threadIdx.x >> 6] = (__builtin_amdgcn_s_getreg((31 << 11) | 4) >> 4) & 3u;  // HW_ID.simd_id
            pace_prog[threadIdx.x >> 6] = 0u;
        }
    }  // (stage_lds's barrier orders these before the sibling search)
    const ZigTabs zt = stage_lds(lds, a.zig, a.consts, nconst, a.obs, (LLMODE == LL_PER_OBS) ? (int)nobs * D : 0);
    const double *cst0 = lds;

    const uint64_t tid = (uint64_t)xcd_block(blockIdx.x, gridDim.x, a.xcd) * blockDim.x + threadIdx.x;
    const uint64_t chain = tid / LPC;
    const int sub = (int)(tid % LPC);
    if (chain >= a.C) {
        if (kPace && (threadIdx.x & 63) == 0) pace_prog[threadIdx.x >> 6] = ~0u;  // no steps to pace
        return;
    }
    const int d0 = sub * DPL;
    const uint32_t gid = a.chain0 + (uint32_t)chain;

    const uint64_t C = a.C;
    const SlotOffset<D> soff(C, chain, d0);
    const SlotOffset<D> &hoff = soff;
    const uint32_t c32 = (uint32_t)chain;  // C < 2^32 (emcmc_create)
    double th[DPL];
    load_slot<D>(a.theta_in ? a.theta_in : a.theta, soff, th);
    double ll = chain_elem(a.ll, c32);
    double ra = chain_elem(a.ra, c32);
    uint64_t r0 = chain_elem(a.ring, 2 * c32), r1 = chain_elem(a.ring, 2 * c32 + 1);
    uint32_t nacc = chain_elem(a.nacc, c32);
    uint32_t faults = chain_elem(a.faults, c32);
    SiblingPace pace{pace_prog, (int)(threadIdx.x >> 6), -1};
    if constexpr (kPace) {
        const int nw = (int)(blockDim.x >> 6);
        for (int w = 0; w < nw; ++w)
            if (w != pace.me && pace.sib < 0 && pace_simd[w] == pace_simd[pace.me]) pace.sib = w;
    }
    AcceptStream accs;
    const PhiloxVKeys vkeys = philox_vkeys(a.key0, a.key1);
    // log_prior(::Previous) carried: logpdf(prior, θ) at the launch's start, then the accepted
    // step's log_prior(::Proposal) (the same doubles)
    double lpc = 0.0;
    if constexpr (PR::kOn && !PR::kRoundTrip) lpc = PR::template eval<D, LPC, DPL>(cst0 + 4 * D, a.consts + 4 * D, d0, th);
    // UniformRandomWalk with positivity flags: logpdf(rw, θ°, θ) carried the same way
    double ltd_rev_c = 0.0;
    if constexpr (PR::kUniform)
        if constexpr (PR::kPos) ltd_rev_c = PR::template rev_terms<D, LPC, DPL>(d0, cst0 + D, th);

    for (uint32_t s = 0; s < a.nsteps; ++s) {
        const uint32_t iter = a.iter0 + s;  // consecutive (host splits gaps)
        const uint64_t slot = (uint64_t)(iter - 1) * a.P + a.pidx0;
        const double *cst = cst0;
        const double *Lrw = cst;
        const double *iLrw = cst + D;
        const double *iLt = cst + 2 * D;
        const double *xbar = cst + 3 * D;
        const double *X = cst + (4 + kPrc) * D;
        // ---- proposal!: θ° = θ + L z, z ~ N(0, I) (random_walk.jl:145-151); with a prior, drawn
        // again while logpdf(prior, θ°) === −Inf (updates.jl:191-196), redraw r from normals
        // (r << 17) | j
        // (UniformRandomWalk, PR::kUniform: θ° from ϵ and the positivity flags, emcmc_fprior.h, with the
        // two transition-density sums formed as θ° is; the Lrw / iLrw slots hold ϵ and −log 2ϵ)
        double thp[DPL];
        double lpp = 0.0, ltd_fwd = 0.0;
        // PR::kRoundTrip: the step's local θ, which a redraw's round trip changes (θ itself does not)
        double tl[PR::kRoundTrip ? DPL : 1];
        if constexpr (PR::kRoundTrip) {
#pragma unroll
            for (int i = 0; i < DPL; ++i) tl[i] = th[i];
        }
        auto propose = [&](uint32_t rs) {
            if constexpr (PR::kRoundTrip)
                PR::template propose_round_trip<D, LPC, DPL>(zt, a.key0, a.key1, vkeys, gid, iter, a.pidx0, rs, d0, Lrw,
                                                             tl, thp, faults);
            else if constexpr (PR::kUniform)
                PR::template propose_uniform<D, LPC, DPL>(vkeys, gid, iter, a.pidx0, rs, d0, Lrw, iLrw, th, thp,
                                                          ltd_fwd);
            else
                propose_diag<DPL, true>(zt, a.key0, a.key1, gid, iter, a.pidx0, (rs << 17) + (uint32_t)d0, th,
                                        Lrw + d0, thp, faults, vkeys);
        };
        if constexpr (PR::kOn) {
            for (uint32_t rs = 0;; ++rs) {
                propose(rs);
                lpp = PR::template eval<D, LPC, DPL>(cst + 4 * D, a.consts + 4 * D, d0, thp);
                if (!(lpp == -__builtin_inf())) break;
                if (rs >= PR::kCap) {
                    faults |= PR::kFault;
                    break;
                }
            }
        } else if constexpr (PR::kUniform || PR::kRoundTrip) {
            propose(0u);
        } else {
            propose_diag<DPL, true>(zt, a.key0, a.key1, gid, iter, a.pidx0, (uint32_t)d0, th, Lrw + d0, thp, faults,
                                    vkeys);
        }
        // ---- log_transition_density both ways (random_walk.jl:161-171):
        // sqmahal(θ°−θ) == sqmahal(θ−θ°) bitwise, so one evaluation serves both
        double ltd = 0.0;
        if constexpr (!PR::kUniform && !PR::kRoundTrip)
            ltd = fma(-0.5, canon_sumsq_f<D, LPC, DPL>([&](int i) { return (thp[i] - th[i]) * iLrw[d0 + i]; }),
                      a.rw_c0);  // = c0 − q/2 (q/2 exact)
        // ---- compute_ll!: Σ_k logpdf(N(θ°, Σ_t), x_k) (gsn_target.jl:23-29)
        double llp;
        if constexpr (LLMODE == LL_PER_OBS) {
            llp = 0.0;
            // observation rows are read one canonical block ahead of use
          constexpr int BLK = SumShape<D>::BLK, BPL = DPL / BLK;
          if constexpr (BLK % 2 == 0) {
            d2v cur[BLK / 2];
            const d2v *xrow = reinterpret_cast<const d2v *>(X + d0);
#pragma unroll
            for (int i = 0; i < BLK / 2; ++i) cur[i] = xrow[i];
            for (uint32_t k = 0; k < nobs; ++k) {
                double b[BPL];
#pragma unroll
                for (int blk = 0; blk < BPL; ++blk) {
                    // next block: same row's next block, else the next row's first
                    // (past the last row: row 0 again, a harmless read)
                    const uint32_t nk = (blk + 1 < BPL) ? k : ((k + 1 < nobs) ? k + 1 : 0u);
                    const int nb = (blk + 1 < BPL) ? blk + 1 : 0;
                    const d2v *xn = reinterpret_cast<const d2v *>(X + (size_t)nk * D + d0 + nb * BLK);
                    d2v nxt[BLK / 2];
                    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
                    for (int i = 0; i < BLK / 2; ++i) nxt[i] = xn[i];
                    __builtin_amdgcn_sched_barrier(0);
                    const int c0 = blk * BLK;
                    auto y = [&](int i) {
                        const double xv = (i & 1) ? cur[i >> 1].y : cur[i >> 1].x;
                        const double yv = xv - thp[c0 + i];
                        return UNIT_T ? yv : yv * iLt[d0 + c0 + i];
                    };
                    double acc = y(0) * y(0);
#pragma unroll
                    for (int i = 1; i < BLK; ++i) acc = fma(y(i), y(i), acc);
                    b[blk] = acc;
#pragma unroll
                    for (int i = 0; i < BLK / 2; ++i) cur[i] = nxt[i];
                }
                const double q = lane_tree<LPC>(tree_inplace<BPL>(b));
                llp = llp + fma(-0.5, q, a.t_c0);
            }
          } else {
            for (uint32_t k = 0; k < nobs; ++k) {
                const double *xk = X + (size_t)k * D + d0;
                const double q = canon_sumsq_f<D, LPC, DPL>([&](int i) {
                    const double y = xk[i] - thp[i];
                    return UNIT_T ? y : y * iLt[d0 + i];
                });
                llp = llp + fma(-0.5, q, a.t_c0);
            }
          }
        } else {
            const double qv = canon_sumsq_f<D, LPC, DPL>([&](int i) {
                const double y = xbar[d0 + i] - thp[i];
                return UNIT_T ? y : y * iLt[d0 + i];
            });
            llp = a.n_tc0 - (a.S_c + a.nobs_d * qv) * 0.5;
        }
        if (!(llp - llp == 0.0)) faults |= 1u;  // NaN or ±Inf
        // PR::kRoundTrip: θ° is stored before its round trips; then both densities, θ°₃ / θ₃ and
        // the prior at each (no carry: θ₃ is not the θ the previous step's prior saw)
        double ta[PR::kRoundTrip ? DPL : 1];
        double ltd_rev_rt = 0.0;
        if constexpr (PR::kRoundTrip) {
            if constexpr (FULL) store_slot<D>(a.hist_prop + slot * D * C, hoff, thp);
            double t3[DPL];
            PR::template ltd_round_trip<D, LPC, DPL>(d0, iLrw, a.rw_c0, tl, thp, ta, t3, ltd_rev_rt, ltd_fwd);
            if constexpr (PR::kOn) {
                lpp = PR::template eval<D, LPC, DPL>(cst + 4 * D, a.consts + 4 * D, d0, ta);
                lpc = PR::template eval<D, LPC, DPL>(cst + 4 * D, a.consts + 4 * D, d0, t3);
            }
        }
        // ---- accept_reject! (run.jl:271-278), left-associative as written
        double llr;
        if constexpr (PR::kRoundTrip) llr = ((((llp - ll) + ltd_rev_rt) - ltd_fwd) + lpp) - lpc;
        else if constexpr (PR::kUniform) llr = ((((llp - ll) + ltd_rev_c) - ltd_fwd) + lpp) - lpc;
        else llr = ((((llp - ll) + ltd) - ltd) + lpp) - lpc;
        const double E = accs.next<true>(zt, a.key0, a.key1, gid, iter, a.pidx0, s == 0, faults, vkeys);
        const bool acc = E > -llr;
        if constexpr (PR::kOn && !PR::kRoundTrip) lpc = acc ? lpp : lpc;
        if constexpr (PR::kUniform) ltd_rev_c = acc ? ltd_fwd : ltd_rev_c;
        // ---- set_proposal! history: θ° with coords replaced (run.jl:237-239)
        if constexpr (FULL && !PR::kRoundTrip) store_slot<D>(a.hist_prop + slot * D * C, hoff, thp);
        // ---- register_accept_reject_results! / set_chain_param! (run.jl:312-335)
        if constexpr (PR::kRoundTrip) {
#pragma unroll
            for (int i = 0; i < DPL; ++i) th[i] = acc ? ta[i] : th[i];
        } else {
#pragma unroll
            for (int i = 0; i < DPL; ++i) th[i] = acc ? thp[i] : th[i];
        }
        if (s + 1 == a.nsteps && sub == 0) chain_elem(a.ll_prop, c32) = llp;  // sub_ws°.ll after the launch
        ll = acc ? llp : ll;
        nacc += acc ? 1u : 0u;
        if constexpr (FULL) {
            store_slot<D>(a.hist_theta + slot * D * C, hoff, th);
            if (sub == 0) __builtin_nontemporal_store(ll, &chain_elem(a.hist_ll + slot * a.C, c32));
        }
        {
            const uint64_t m = compact_ballot<LPC>(__ballot(acc));
            if ((threadIdx.x & 63) == 0)
                store_acc_bits<LPC>(a.hist_acc + slot * a.row_bytes, chain, m);
        }
        // ---- update_stats! rolling acceptance (chain_statistics.jl:53-65)
        ra = rolling_update(ra, r0, r1, iter, a.W, a.N0 + s, a.rcp_W, acc);
        if constexpr (kPace) pace.publish(s + 1);
    }
    if constexpr (kPace) {
        pace.publish(~0u);  // done: the sibling, alone now, stops lowering itself
        __builtin_amdgcn_s_setprio(0);
    }

    // the chain's lanes may hold different rare-path fault bits (each draws its own normals)
    if constexpr (LPC >= 2) faults |= (uint32_t)__builtin_amdgcn_update_dpp(0, (int)faults, 0xB1, 0xF, 0xF, false);
    if constexpr (LPC >= 4) faults |= (uint32_t)__builtin_amdgcn_update_dpp(0, (int)faults, 0x4E, 0xF, 0xF, false);
    if (sub == 0) {
        chain_elem(a.ll, c32) = ll;
        chain_elem(a.ra, c32) = ra;
        chain_elem(a.ring, 2 * c32) = r0;
        chain_elem(a.ring, 2 * c32 + 1) = r1;
        chain_elem(a.nacc, c32) = nacc;
        chain_elem(a.faults, c32) = faults;
        if (faults) *a.fault_flag = 1u;
    }
    if (a.theta) store_slot_cached<D>(a.theta, soff, th);  // else: the last θ history slot holds it
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
    const ZigTabs zt = stage_lds(lds, a.zig, a.consts, nconst, a.obs, (LLMODE == LL_PER_OBS) ? (int)nobs * D : 0);
    const double *cst = lds;
    const double *Lrw = cst;
    const double *iLrw = cst + D * D;
    const double *Lt = cst + D * D + D;
    const double *iLt = cst + 2 * D * D + D;
    const double *xbar = cst + 2 * D * D + 2 * D;
    const double *X = cst + 2 * D * D + 3 * D;

    const uint64_t chain = (uint64_t)xcd_block(blockIdx.x, gridDim.x, a.xcd) * blockDim.x + threadIdx.x;
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
    const SlotOffset<D> soff(C, chain, 0);
    AcceptStream accs;

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
            ltd = fma(-0.5, canon_sumsq<D, 1>(y), a.rw_c0);  // = c0 − q/2 (q/2 exact)
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
                llp = llp + fma(-0.5, canon_sumsq<D, 1>(y), a.t_c0);
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
        const double E = accs.next(zt, a.key0, a.key1, gid, iter, a.pidx0, s == 0, faults);
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
        ra = rolling_update(ra, r0, r1, iter, a.W, a.N0 + s, a.rcp_W, acc);
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

}  // namespace emcmc
