// emcmc_fprior.h — a separable prior on the fused diagonal step kernel (gfx950).
//
// rwm_gsn_diag_kernel (emcmc_fused.h) runs the joint GaussianRandomWalk with a diagonal Σ on a
// diagonal GsnTargetLaw with LPC lanes per chain and two waves per SIMD: the cfg 2 kernel.  With
// ImproperPrior its ratio adds + 0.0 − 0.0.  FusedPrior<S> gives it the log-prior of one
// ProductPrior([Product(u_1 … u_D)]) or StandardPrior(Product(u_1 … u_D)) over coords 1:D
// (priors.jl:18-88) — D univariate factors, lane-symmetric families (the family of coordinate i
// equals that of i + k·D/LPC, so every lane of a chain runs the same code on its own
// coordinates) — compiled at run time for the families (hiprtc, emcmc_rtc.hip), its parameters
// per coordinate in LDS after the kernel's own constants.
//
// logpdf(prior, θ) = 0.0 + (((v_1 + v_2) + v_3) + … + v_D) (ProductPrior; StandardPrior without
// the 0.0 +), v_i the component's logpdf (univariate_logpdf, the oracle's and the schedule
// kernels' formulas).  Each lane forms the v_i of its D/LPC coordinates at once; the left fold
// runs segment by segment, each lane continuing from the previous lane's partial sum (a DPP
// move), and the last lane's total is broadcast to the chain's lanes: the same additions in the
// same order as one lane folding all D.
#pragma once

#include "emcmc_fused.h"
#include "emcmc_mwg.h"

namespace emcmc {

template <class S>
struct FusedPrior {
    using U = typename S::template U<0>;
    static constexpr bool kOn = true;
    static constexpr int kConsts = 3;  // a, b, c of univariate_logpdf, [3][D] in LDS
    static constexpr uint32_t kCap = kMaxResampleGsn;
    static constexpr uint32_t kFault = kFaultPriorResample;
    static_assert(U::prior == kPriorProduct || U::prior == kPriorStandard, "ProductPrior or StandardPrior");

    // lane k of an LPC group takes lane k−1's value (quad_perm [0,0,2,2] / [0,0,1,2])
    template <int LPC>
    __device__ __forceinline__ static double from_previous_lane(double v) {
        if constexpr (LPC == 2) return dpp_perm<0xA0>(v);
        else return dpp_perm<0x90>(v);
    }
    // every lane of an LPC group takes the group's last lane's value ([1,1,3,3] / [3,3,3,3])
    template <int LPC>
    __device__ __forceinline__ static double from_last_lane(double v) {
        if constexpr (LPC == 2) return dpp_perm<0xF5>(v);
        else return dpp_perm<0xFF>(v);
    }

    template <int D, int LPC, int DPL>
    __device__ __forceinline__ static double eval(const double *pc, int d0, const double (&x)[DPL]) {
        static_assert(LPC == 1 || LPC == 2 || LPC == 4, "lanes per chain: 1, 2 or 4 (one quad)");
        if constexpr (LPC == 1) {  // one lane folds as it goes: no vector of logpdfs stays live
            double s = 0.0;
            static_for<0, DPL>([&](auto IC) {
                constexpr int i = decltype(IC)::value;
                const double v = univariate_logpdf(U::fam[i], pc[d0 + i], pc[D + d0 + i], pc[2 * D + d0 + i], x[i]);
                s = (i == 0) ? v : s + v;
            });
            return (U::prior == kPriorProduct) ? 0.0 + s : s;
        } else {
            double v[DPL];
            static_for<0, DPL>([&](auto IC) {
                constexpr int i = decltype(IC)::value;
                v[i] = univariate_logpdf(U::fam[i], pc[d0 + i], pc[D + d0 + i], pc[2 * D + d0 + i], x[i]);
            });
            double s = 0.0, carry = 0.0;
            static_for<0, LPC>([&](auto KC) {
                constexpr int k = decltype(KC)::value;  // the lane whose segment this pass folds
                s = (k == 0) ? v[0] : carry + v[0];
#pragma unroll
                for (int i = 1; i < DPL; ++i) s = s + v[i];
                if constexpr (k + 1 < LPC) carry = from_previous_lane<LPC>(s);
            });
            s = from_last_lane<LPC>(s);
            return (U::prior == kPriorProduct) ? 0.0 + s : s;
        }
    }
};

}  // namespace emcmc
