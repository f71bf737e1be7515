// emcmc_fprior.h — separable random-walk updates on the fused diagonal step kernel (gfx950).
//
// rwm_gsn_diag_kernel (emcmc_fused.h) runs the joint GaussianRandomWalk with a diagonal Σ on a
// diagonal GsnTargetLaw with LPC lanes per chain and two waves per SIMD: the cfg 2 kernel.  With
// ImproperPrior its ratio adds + 0.0 − 0.0.  FusedUpdate<S> widens it to the joint updates over
// coords 1:D whose every term separates over coordinates:
//   - the proposal: GaussianRandomWalk with a diagonal Σ — with positivity flags, the reference's
//     exp/log round trips of θ and θ° (random_walk.jl:136-171) — or UniformRandomWalk(ϵ) with
//     positivity flags (random_walk.jl:45-94: θ° = θ·e^U + copysign(0, U) where pos, θ + U
//     elsewhere; logpdf terms −log 2ϵ_j − log θ°_j folded left over j);
//   - the prior: ImproperPrior, ImproperPosPrior (−Σ log θ_j), or ONE ProductPrior /
//     StandardPrior factor that is a Product of D univariates (priors.jl:18-88);
// compiled at run time for the structure (hiprtc, emcmc_rtc.hip) from the schedule struct S of
// mwg_rw_block_kernel (S::U<0>: kind, pos mask, families).  The families and pos flags repeat
// across the chain's lanes (those of coordinate i are those of i mod D/LPC), so every lane of a
// chain runs the same code on its own coordinates; ϵ, −log 2ϵ and the prior's parameters per
// coordinate sit in LDS with the kernel's constants.
//
// Every left fold over the D coordinates (the prior, the two transition-density sums) runs
// segment by segment: lane 0 folds its coordinates, lane k continues from lane k−1's partial sum
// (a DPP move), the last lane's total is broadcast to the chain's lanes — the same additions in
// the same order as one lane folding all D (the oracle's orc_run_mwg and rw_step's order).
#pragma once

#include "emcmc_fused.h"
#include "emcmc_mwg.h"

namespace emcmc {

template <class S>
struct FusedUpdate {
    using U = typename S::template U<0>;
    static constexpr bool kUniform = U::kind == 1u;  // else GaussianRandomWalk
    static constexpr bool kOn = U::prior != kPriorImproper;  // a prior term (and proposal! redraws)
    static constexpr bool kSlots = U::prior == kPriorProduct || U::prior == kPriorStandard;
    static constexpr bool kMvn = kSlots && U::pmvn != 0ull;  // one MvNormal factor over all D
    // univariates: a, b, c of univariate_logpdf, [3][D] staged in LDS; an MvNormal factor reads its
    // μ, 1/L_jj, packed lower factor and c0 from global memory through the scalar cache
    static constexpr int kConsts = (kSlots && !kMvn) ? 3 : 0;
    static constexpr uint32_t kCap = kUniform ? kMaxResample : kMaxResampleGsn;
    static constexpr uint32_t kFault = kFaultPriorResample;
    static constexpr bool kPos = kUniform && U::pos != 0ull;
    // GaussianRandomWalk with positivity flags: the reference's in-place exp/log round trips
    // (random_walk.jl:136-171), as mwg_rw_block_kernel's RT branch; no log-prior carry
    static constexpr bool kRoundTrip = !kUniform && U::pos != 0ull;
    template <int q>
    __device__ static constexpr bool pos_at() { return ((U::pos >> q) & 1ull) != 0ull; }
    __host__ __device__ static constexpr int first_pos() {
        int q = 0;
        while (q < 64 && ((U::pos >> q) & 1ull) == 0ull) ++q;
        return q;
    }

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

    // (((v_1 + v_2) + v_3) + … + v_D) over the chain's D values, DPL per lane
    template <int LPC, int DPL>
    __device__ __forceinline__ static double fold(const double (&v)[DPL]) {
        static_assert(LPC == 1 || LPC == 2 || LPC == 4, "lanes per chain: 1, 2 or 4 (one quad)");
        double s = 0.0, carry = 0.0;
        static_for<0, LPC>([&](auto KC) {
            constexpr int k = decltype(KC)::value;  // the lane whose segment this pass folds
            s = (k == 0) ? v[0] : carry + v[0];
#pragma unroll
            for (int i = 1; i < DPL; ++i) s = s + v[i];
            if constexpr (k + 1 < LPC) carry = from_previous_lane<LPC>(s);
        });
        if constexpr (LPC > 1) s = from_last_lane<LPC>(s);
        return s;
    }

    // logpdf(MvNormal(μ, LLᵀ), x) − as rw_log_prior's MvNormal rows: y = L⁻¹(x − μ) row by row
    // (row j: x_j − μ_j, then −L_jm·y_m for m ascending, times 1/L_jj), its squares folded left,
    // c0 − s/2.  Pass k solves lane k's rows: every lane runs it with the same (scalar-loaded) rows,
    // lane k's results are the ones kept; lane k−1's y's and running sum reach lane k by DPP.
    // gc: μ[D] | 1/L_jj[D] | L packed lower row-major [D(D+1)/2] | c0.
    template <int D, int LPC, int DPL>
    __device__ __forceinline__ static double eval_mvn(const double *gc, int d0, const double (&x)[DPL]) {
        if constexpr (LPC == 4) {
            return eval_mvn_quad<D, DPL>(gc, d0 / DPL, x);
        } else {
            return eval_mvn_pair<D, LPC, DPL>(gc, x);
        }
    }

    // every lane of the quad takes lane K's value (quad_perm [K,K,K,K])
    template <int K>
    __device__ __forceinline__ static double from_quad_lane(double v) {
        return dpp_perm<K * 0x55>(v);
    }

    // Four lanes per chain: pass k forms lane k's rows in accumulators — x − μ, then the columns of
    // lanes 0 … k−1 (each of their y's broadcast across the quad once, used by the DPL rows), then
    // the lane's own columns — so every row still takes its terms m ascending; lane k keeps the
    // pass's y's, the running sum moves on from lane k−1 by DPP.  Live: y and the accumulators
    // (2·DPL), where carrying the earlier lanes' y's would take D.
    template <int D, int DPL>
    __device__ __forceinline__ static double eval_mvn_quad(const double *gc, int kl, const double (&x)[DPL]) {
        constexpr int kL = 2 * D, kC = 2 * D + D * (D + 1) / 2;
        double y[DPL];
        double s = 0.0, carry = 0.0;
        static_for<0, 4>([&](auto KC) {
            constexpr int k = decltype(KC)::value;
            double acc[DPL];
            {
                cdouble *t = opaque_cptr(gc);
                static_for<0, DPL>([&](auto IC) {
                    constexpr int i = decltype(IC)::value;
                    acc[i] = x[i] - t[k * DPL + i];
                });
            }
            static_for<0, k>([&](auto SC) {  // the earlier lanes' columns, ascending
                constexpr int sl = decltype(SC)::value;
                static_for<0, DPL>([&](auto MC) {
                    constexpr int m = sl * DPL + decltype(MC)::value;
                    const double b = from_quad_lane<sl>(y[decltype(MC)::value]);
                    cdouble *t = opaque_cptr(gc);  // per column: one column's loads in flight
                    static_for<0, DPL>([&](auto IC) {
                        constexpr int i = decltype(IC)::value, r = k * DPL + i;
                        acc[i] = fma(-t[kL + r * (r + 1) / 2 + m], b, acc[i]);
                    });
                });
            });
            static_for<0, DPL>([&](auto IC) {  // the lane's own rows: forward substitution
                constexpr int i = decltype(IC)::value, r = k * DPL + i;
                cdouble *t = opaque_cptr(gc);
                static_for<0, i>([&](auto MC) {
                    constexpr int m = decltype(MC)::value;
                    acc[i] = fma(-t[kL + r * (r + 1) / 2 + k * DPL + m], acc[m], acc[i]);
                });
                acc[i] = acc[i] * t[D + r];
                if constexpr (k == 0 && i == 0) s = acc[i] * acc[i];
                else if constexpr (i == 0) s = fma(acc[i], acc[i], carry);
                else s = fma(acc[i], acc[i], s);
            });
#pragma unroll
            for (int i = 0; i < DPL; ++i) y[i] = (kl == k) ? acc[i] : y[i];
            if constexpr (k < 3) carry = from_previous_lane<4>(s);
        });
        s = from_last_lane<4>(s);
        const double fv = opaque_cptr(gc)[kC] - s / 2.0;
        return (U::prior == kPriorProduct) ? 0.0 + fv : fv;
    }

    template <int D, int LPC, int DPL>
    __device__ __forceinline__ static double eval_mvn_pair(const double *gc, const double (&x)[DPL]) {
        static_assert(LPC == 1 || LPC == 2, "an MvNormal prior on one or two lanes per chain");
        constexpr int kL = 2 * D, kC = 2 * D + D * (D + 1) / 2;
        double y[DPL];
        double s = 0.0;
        static_for<0, DPL>([&](auto IC) {  // lane 0's rows 0 … DPL−1
            constexpr int i = decltype(IC)::value;
            cdouble *t = opaque_cptr(gc);  // per row: one row's loads in flight
            double acc = x[i] - t[i];
            static_for<0, i>([&](auto MC) {
                constexpr int m = decltype(MC)::value;
                acc = fma(-t[kL + i * (i + 1) / 2 + m], y[m], acc);
            });
            y[i] = acc * t[D + i];
            s = (i == 0) ? y[i] * y[i] : fma(y[i], y[i], s);
        });
        if constexpr (LPC == 2) {  // lane 1's rows DPL … D−1, after lane 0's y's in ascending m
            double y0[DPL];
#pragma unroll
            for (int m = 0; m < DPL; ++m) y0[m] = from_previous_lane<2>(y[m]);
            const double s0 = from_previous_lane<2>(s);
            static_for<0, DPL>([&](auto IC) {
                constexpr int i = decltype(IC)::value, r = DPL + i;
                cdouble *t = opaque_cptr(gc);
                double acc = x[i] - t[r];
                static_for<0, DPL>([&](auto MC) {
                    constexpr int m = decltype(MC)::value;
                    acc = fma(-t[kL + r * (r + 1) / 2 + m], y0[m], acc);
                });
                static_for<0, i>([&](auto MC) {
                    constexpr int m = decltype(MC)::value;
                    acc = fma(-t[kL + r * (r + 1) / 2 + DPL + m], y[m], acc);
                });
                y[i] = acc * t[D + r];
                s = (i == 0) ? fma(y[i], y[i], s0) : fma(y[i], y[i], s);
            });
            s = from_last_lane<2>(s);
        }
        const double fv = opaque_cptr(gc)[kC] - s / 2.0;
        return (U::prior == kPriorProduct) ? 0.0 + fv : fv;
    }

    // logpdf(prior, x) of the chain (every lane gets the same double); pc: the LDS constants of the
    // univariate factors, gc: the MvNormal factor's tables in global memory
    template <int D, int LPC, int DPL>
    __device__ __forceinline__ static double eval(const double *pc, const double *gc, int d0, const double (&x)[DPL]) {
        if constexpr (kMvn) {
            return eval_mvn<D, LPC, DPL>(gc, d0, x);
        } else if constexpr (U::prior == kPriorImproperPos) {  // −sum(log.(θ))
            double v[DPL];
#pragma unroll
            for (int i = 0; i < DPL; ++i) v[i] = log_real(x[i]);
            return -fold<LPC, DPL>(v);
        } else if constexpr (LPC == 1) {  // one lane folds as it goes: no vector of logpdfs stays live
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
            const double s = fold<LPC, DPL>(v);
            return (U::prior == kPriorProduct) ? 0.0 + s : s;
        }
    }

    // (((v_p1 + v_p2) + …) over the flagged coordinates only, ascending, continued lane to lane (the
    // flags repeat across the lanes, so every lane holds flagged coordinates at the same offsets)
    template <int LPC, int DPL>
    __device__ __forceinline__ static double fold_pos(const double (&v)[DPL]) {
        double s = 0.0, carry = 0.0;
        static_for<0, LPC>([&](auto KC) {
            constexpr int k = decltype(KC)::value;
            static_for<0, DPL>([&](auto QC) {
                constexpr int q = decltype(QC)::value;
                if constexpr (q == first_pos()) s = (k == 0) ? v[q] : carry + v[q];
                else if constexpr (pos_at<q>()) s = s + v[q];
            });
            if constexpr (k + 1 < LPC) carry = from_previous_lane<LPC>(s);
        });
        if constexpr (LPC > 1) s = from_last_lane<LPC>(s);
        return s;
    }

    // GaussianRandomWalk's proposal draw rs with positivity flags (random_walk.jl:136-151): a redraw
    // first leaves θ ← exp(log θ) where flagged (the previous rand!'s round trip, cumulative over
    // redraws, on the step's local copy tl); θ° = exp(log θ + L z) where flagged, θ + L z elsewhere.
    // The normals are propose_diag's ((r << 17) | j); a flagged coordinate takes 0.0 + L z from it,
    // which enters log θ + · as L z does (x + ±0 differ only at x = −0, and exp(±0) = 1).
    template <int D, int LPC, int DPL>
    __device__ __forceinline__ static void propose_round_trip(const ZigTabs &zt, uint32_t key0, uint32_t key1,
                                                              const PhiloxVKeys &vk, uint32_t gid, uint32_t iter,
                                                              uint32_t pidx0, uint32_t rs, int d0, const double *Lrw,
                                                              double (&tl)[DPL], double (&tp)[DPL],
                                                              uint32_t &faults) {
        if (rs > 0) {
            static_for<0, DPL>([&](auto QC) {
                constexpr int q = decltype(QC)::value;
                if constexpr (pos_at<q>()) tl[q] = exp_any(log_any(tl[q]));
            });
        }
        double base[DPL];
        static_for<0, DPL>([&](auto QC) {
            constexpr int q = decltype(QC)::value;
            base[q] = pos_at<q>() ? 0.0 : tl[q];
        });
        propose_diag<DPL, true>(zt, key0, key1, gid, iter, pidx0, (rs << 17) + (uint32_t)d0, base, Lrw + d0, tp,
                                faults, vk);
        static_for<0, DPL>([&](auto QC) {
            constexpr int q = decltype(QC)::value;
            if constexpr (pos_at<q>()) tp[q] = exp_any(log_any(tl[q]) + tp[q]);
        });
    }

    // Both transition densities with the reference's round trips (mwg_rw_block_kernel's RT branch):
    // logpdf(rw, θ°, θ) logs θ₁ = exp(log θ) and θ°, adds −Σ log θ₁ over the flags; logpdf(rw, θ, θ°)
    // exponentiates both back and logs them again.  ta = θ°₃ (what an accept stores), t3 = θ₃
    // (log_prior(::Previous)).  The squared norms in the canonical order, split across the lanes.
    template <int D, int LPC, int DPL>
    __device__ __forceinline__ static void ltd_round_trip(int d0, const double *iLrw, double c0,
                                                          const double (&tl)[DPL], const double (&tp)[DPL],
                                                          double (&ta)[DPL], double (&t3)[DPL], double &ltd_rev,
                                                          double &ltd_fwd) {
        double a1[DPL], b1[DPL], lv[DPL];
        static_for<0, DPL>([&](auto QC) {
            constexpr int q = decltype(QC)::value;
            if constexpr (pos_at<q>()) {
                const double v = log_any(exp_any(log_any(tl[q])));  // log θ₁
                lv[q] = v;
                a1[q] = log_any(tp[q]);  // μ = log θ°₁
                b1[q] = v;               // x = log θ₁
            } else {
                lv[q] = 0.0;
                a1[q] = tp[q];
                b1[q] = tl[q];
            }
        });
        const double lj1 = fold_pos<LPC, DPL>(lv);
        const double q1 = canon_sumsq_f<D, LPC, DPL>([&](int i) { return (b1[i] - a1[i]) * iLrw[d0 + i]; });
        ltd_rev = (c0 - q1 / 2.0) + (-lj1);
        double r[DPL];
        static_for<0, DPL>([&](auto QC) {
            constexpr int q = decltype(QC)::value;
            if constexpr (pos_at<q>()) {
                const double v = log_any(exp_any(a1[q]));   // log θ°₂
                const double a2 = log_any(exp_any(b1[q]));  // μ = log θ₂
                lv[q] = v;
                r[q] = v - a2;
                ta[q] = exp_any(v);   // θ°₃
                t3[q] = exp_any(a2);  // θ₃
            } else {
                r[q] = a1[q] - b1[q];
                ta[q] = a1[q];
                t3[q] = b1[q];
            }
        });
        const double lj2 = fold_pos<LPC, DPL>(lv);
        const double q2 = canon_sumsq_f<D, LPC, DPL>([&](int i) { return r[i] * iLrw[d0 + i]; });
        ltd_fwd = (c0 - q2 / 2.0) + (-lj2);
    }

    // The reverse sum logpdf(rw, θ°, θ) = fold of −log 2ϵ_j − log θ_j depends on θ alone, so the
    // kernel carries it: rev_terms(θ) at the launch's start, then the accepted step's forward sum
    // (the same operations on the same doubles: θ_next = θ°).
    template <int D, int LPC, int DPL>
    __device__ __forceinline__ static double rev_terms(int d0, const double *uc, const double (&th)[DPL]) {
        double g[DPL];
        static_for<0, DPL>([&](auto QC) {
            constexpr int q = decltype(QC)::value;
            if constexpr (((U::pos >> q) & 1ull) != 0ull) g[q] = uc[d0 + q] - log_any(th[q]);
            else g[q] = 0.0;
        });
        return fold<LPC, DPL>(g);
    }

    // UniformRandomWalk's proposal draw rs (random_walk.jl:63-80) for this lane's coordinates
    // d0 … d0+DPL−1: θ° and, with positivity flags, logpdf(rw, θ, θ°) (random_walk.jl:81-94; 0.0
    // for the coordinates without the flag, 0.0 without any).  eps / uc: ϵ_j and −log(2ϵ_j) per
    // coordinate (LDS).
    template <int D, int LPC, int DPL>
    __device__ __forceinline__ static void propose_uniform(const PhiloxVKeys &vk, uint32_t gid, uint32_t iter,
                                                           uint32_t pidx0, uint32_t rs, int d0, const double *eps,
                                                           const double *uc, const double (&th)[DPL],
                                                           double (&tp)[DPL], double &ltd_fwd) {
        double f[DPL];
        static_for<0, DPL / 2>([&](auto PC) {
            constexpr int j = 2 * decltype(PC)::value;
            sbar();  // one Philox block at a time
            const u32x4 r = draw_vk(vk, gid, iter, (rs << 16) | ((uint32_t)(d0 + j) >> 1), pidx0);
            auto one = [&](auto QC, uint32_t hi, uint32_t lo) {
                constexpr int q = decltype(QC)::value;
                const double e = eps[d0 + q];
                const double Uq = (-e) + (e - (-e)) * u01_closed0(hi, lo);
                if constexpr (((U::pos >> q) & 1ull) != 0ull) {
                    tp[q] = th[q] * exp_any(Uq) + copysign(0.0, Uq);
                    f[q] = uc[d0 + q] - log_any(tp[q]);
                } else {
                    tp[q] = th[q] * 1.0 + Uq;
                    f[q] = 0.0;
                }
            };
            one(IntC<j>{}, r.x, r.y);
            one(IntC<j + 1>{}, r.z, r.w);
        });
        if constexpr (kPos) ltd_fwd = fold<LPC, DPL>(f);
        else ltd_fwd = 0.0;
    }
};

}  // namespace emcmc
