// emcmc_chol.h — rwm_gsn_chol_kernel: one GaussianRandomWalk update over all D coordinates
// with a correlated Σ_rw and/or Σ_t (rows a5, a6, a10 at D ≥ 9), the factors streamed
// through the scalar cache (chol_stream, emcmc_kernels.h).  Kept in its own header: the
// run-time compiler embeds it (emcmc_rtc.hip), and only the chol programs include it, so
// a change here leaves the other cached run-time kernels valid.
#pragma once

#include "emcmc_kernels.h"

namespace emcmc {

constexpr int kCholSharedD = 52;  // D from which ltd and the likelihood share one sweep
template <int D, bool FULL, int LLMODE>
__global__ void __launch_bounds__(256) rwm_gsn_chol_kernel(const StepParams a) {
    constexpr bool kCholShared = D >= kCholSharedD;
    const ZigTabs zt = stage_lds(nullptr, a.zig, nullptr, 0, nullptr, 0);
    constexpr int P = D * (D + 1) / 2;

    const uint64_t chain = (uint64_t)xcd_block(blockIdx.x, gridDim.x, a.xcd) * blockDim.x + threadIdx.x;
    if (chain >= a.C) return;
    const uint32_t gid = a.chain0 + (uint32_t)chain;
    const uint64_t C = a.C;
    const uint32_t c32 = (uint32_t)chain;
    const SlotOffset<D> soff(C, chain, 0);
    double th[D];
    load_slot<D>(a.theta, soff, th);
    double ll = chain_elem(a.ll, c32);
    double ra = chain_elem(a.ra, c32);
    uint64_t r0 = chain_elem(a.ring, 2 * c32), r1 = chain_elem(a.ring, 2 * c32 + 1);
    uint32_t nacc = chain_elem(a.nacc, c32);
    uint32_t faults = chain_elem(a.faults, c32);
    AcceptStream accs;
    const PhiloxVKeys vkeys = philox_vkeys(a.key0, a.key1);
    const uint32_t nobs = a.nobs;

    for (uint32_t s = 0; s < a.nsteps; ++s) {
        const uint32_t iter = a.iter0 + s;  // consecutive (host splits gaps)
        const uint64_t slot = (uint64_t)(iter - 1) * a.P + a.pidx0;
        cdouble *cst = opaque_cptr(a.consts);
        // ---- proposal!: θ° = θ + L z (random_walk.jl:145-151), row sums over j ascending
        double thp[D];
        {
            double z[D];
            normals<D, true>(zt, a.key0, a.key1, gid, iter, a.pidx0, z, faults, vkeys);
            chol_propose<D>(cst, z, th, thp);
        }
        // ---- log_transition_density both ways (random_walk.jl:161-171): one evaluation
        double ltd;
        double llp;
        if constexpr (kCholShared) {
        // One copy of the substitution sweep serves log_transition_density (‖L_rw⁻¹(θ° − θ)‖²)
        // and compute_ll! (‖L_t⁻¹(x_k − θ°)‖² per observation, or the x̄ term once): the sweep
        // is the kernel's largest code, and with three unrolled copies (propose, ltd, ll) the
        // kernel outgrew the instruction cache at D ≥ 48 (66 KB of code at D = 48, 105 KB at
        // D = 64).  Same operations, same order.
        ltd = 0.0;
        llp = 0.0;
        {
            const int kn = (LLMODE == LL_PER_OBS) ? (int)nobs : 1;
            for (int k = -1; k < kn; ++k) {
                cdouble *c = opaque_cptr(a.consts);
                double acc[D];
                if (k < 0) {
#pragma unroll
                    for (int i = 0; i < D; ++i) acc[i] = thp[i] - th[i];
                } else {
                    cdouble *x = (LLMODE == LL_PER_OBS) ? c + 3 * P + D + (size_t)k * D : c + 3 * P;
#pragma unroll
                    for (int i = 0; i < D; ++i) {
                        acc[i] = x[i] - thp[i];
                        vpin(acc[i]);
                    }
                }
                cdouble *T = (k < 0) ? c + P : c + 2 * P;
                const double q = chol_sqmahal<D, 0>(T, T, thp, acc);
                if (k < 0) ltd = fma(-0.5, q, a.rw_c0);  // = c0 − q/2 (q/2 exact)
                else if constexpr (LLMODE == LL_PER_OBS) llp = llp + fma(-0.5, q, a.t_c0);
                else llp = a.n_tc0 - (a.S_c + a.nobs_d * q) * 0.5;
            }
        }
        } else {
        {
            double acc[D];
#pragma unroll
            for (int i = 0; i < D; ++i) acc[i] = thp[i] - th[i];
            ltd = fma(-0.5, chol_sqmahal<D, 0>(cst, cst + P, thp, acc), a.rw_c0);
        }
        // ---- compute_ll!: Σ_k logpdf(N(θ°, Σ_t), x_k) (gsn_target.jl:23-29)
        if constexpr (LLMODE == LL_PER_OBS) {
            llp = 0.0;
            for (uint32_t k = 0; k < nobs; ++k) {
                cdouble *c = opaque_cptr(a.consts);
                double acc[D];
                llp = llp + fma(-0.5, chol_sqmahal<D, D>(c + 3 * P + D + (size_t)k * D, c + 2 * P, thp, acc), a.t_c0);
            }
        } else {
            cdouble *c = opaque_cptr(a.consts);
            double acc[D];
            const double qv = chol_sqmahal<D, D>(c + 3 * P, c + 2 * P, thp, acc);
            llp = a.n_tc0 - (a.S_c + a.nobs_d * qv) * 0.5;
        }
        }
        if (!(llp - llp == 0.0)) faults |= 1u;
        // ---- accept_reject! (run.jl:271-278), left-associative as written
        const double llr = ((((llp - ll) + ltd) - ltd) + 0.0) - 0.0;
        const double E = accs.next<true>(zt, a.key0, a.key1, gid, iter, a.pidx0, s == 0, faults, vkeys);
        const bool acc = E > -llr;
        if constexpr (FULL) store_slot_late<D>(a.hist_prop + slot * D * C, soff, thp);
#pragma unroll
        for (int i = 0; i < D; ++i) th[i] = acc ? thp[i] : th[i];
        if (s + 1 == a.nsteps) chain_elem(a.ll_prop, c32) = llp;
        ll = acc ? llp : ll;
        nacc += acc ? 1u : 0u;
        if constexpr (FULL) {
            store_slot_late<D>(a.hist_theta + slot * D * C, soff, th);
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

}  // namespace emcmc
