// emcmc_mwg.h — general schedule step kernel (gfx950): P ≥ 1 RandomWalkUpdates
// over coordinate subsets (Metropolis-within-Gibbs), one lane per chain.
//
// Covers what the fused single-update kernels do not: several updates per
// iteration (single-site or block), UniformRandomWalk, AdaptationUnifRW, and
// schedules with exclusions.  One launch runs an arbitrary slice of the
// MCMCSchedule (the (mcmciter, pidx) list, read with wave-uniform scalar loads).
//
// Reference semantics (src/ under /root/reference), restated in oracle/
// (orc_run_mwg) and oracle/literal.py (run_mwg_chain):
//   update_workspaces!  θ_local ← θ[coords]; ll carried from the previous step
//                       (−Inf before the first)                       run.jl:101-112
//   UniformRandomWalk   U = a + (b − a)·u (a = −ϵ, b = ϵ), θ° = θ·(e^U·pos + 1·!pos)
//                       + U·!pos, i.e. θ·1 + U, or θ·e^U + copysign(0, U) where
//                       pos; logpdf(θ, θ°) = Σ_i (pos_i ? −log(2ϵ_i) − log θ°_i
//                       : 0.0) folded left over the update's coordinates
//                                                                random_walk.jl:63-94
//   GaussianRandomWalk  θ°_local = θ_local + L z over the update's coordinates; with
//                       pos, on the log scale with the reference's in-place
//                       exp/log round trips (see the kernel)   random_walk.jl:136-171
//   set_parameters!(::Proposal)  P°.θ[coords] ← θ°; P° persists across updates
//                       and starts at the target's μ          updates.jl:198-205,
//                                                             workspaces.jl:225-233
//   compute_ll!         loglikelihood(P°, obs)                    workspaces.jl:236
//   accept_reject!      left-associative llr, E > −llr               run.jl:268-281
//   histories           θ° history = θ with coords ← θ°; θ after   run.jl:231-240,312
//   update_stats!       N over all update steps; ra_prev = rolling_ar[iter−1][p]
//                       (0.0 when (iter−1, p) did not run)   chain_statistics.jl:42-66
//   AdaptationUnifRW    register on own turn, readjust at k proposals
//                                                   run.jl:136-178, adaptation.jl:273-329
#pragma once

#include "emcmc_kernels.h"

namespace emcmc {

constexpr int kMwgMaxD = 16;

// One RandomWalkUpdate, host-built; read with scalar (uniform) loads.
struct MwgUpdate {
    uint32_t kind;    // EMCMC_RW_UNIFORM (1) / EMCMC_RW_GAUSSIAN (2)
    uint32_t nc;      // number of coordinates
    uint32_t adapt;   // EMCMC_ADPT_NONE (0) / EMCMC_ADPT_UNIF_RW (1)
    uint32_t k;       // adapt_every_k_steps
    uint32_t coords[kMwgMaxD];
    double eps0[kMwgMaxD];          // UniformRandomWalk ϵ (initial for adaptive updates)
    double L[kMwgMaxD * kMwgMaxD];  // GaussianRandomWalk: lower Cholesky factor, row-major, local indices
    double iL[kMwgMaxD];            // 1 / L_ii
    double c0;                      // −(nc·log2π + logdet Σ)/2
    uint32_t diag, posmask;          // posmask bit j: coordinate j positivity-restricted
    double target, scale, amin, amax, offset;  // AdaptationUnifRW (scalar form)
};

struct MwgParams {
    double *theta;     // [D][C] state_pos layout
    double *mu_p;      // [D][C] P°.θ[1:d] (state_pos layout)
    double *ll;        // [C]
    double *ra;        // [P][C]
    uint64_t *ring;    // [P][C][2]
    uint32_t *nacc;    // [P][C]
    uint32_t *aprop;   // [P][C]  AdaptationUnifRW counters
    uint32_t *aacc;    // [P][C]
    double *eps;       // [P][kMwgMaxD][C]  per-chain ϵ of adaptive updates
    uint32_t *faults;  // [C]
    uint32_t *fault_flag;
    double *hist_theta, *hist_prop, *hist_ll;
    uint8_t *hist_acc;
    const Ziggurat *zig;
    const MwgUpdate *updates;  // [P]
    const uint32_t *steps;     // [nsteps][4]: mcmciter, pidx (1-based), flags (bit 0: ra_prev valid), 0
    const double *Lt;          // target: lower Cholesky, row-major D×D
    const double *iLt;         // 1 / Lt_ii
    const double *xbar;        // [D]
    const double *obs;         // [nobs][D]
    uint64_t C;
    uint64_t row_bytes;
    uint64_t N0;
    uint32_t chain0, key0, key1, nsteps, P, W, nobs, tdiag;
    double t_c0, n_tc0, S_c, nobs_d;
};

// ‖L⁻¹ r‖² for a D-vector (target Σ; dense forward substitution unless
// diagonal), canonical order (SumShape<D>).
template <int D>
__device__ __forceinline__ double mwg_sqmahal_t(const MwgParams &a, const double (&r)[D]) {
    double y[D];
#pragma unroll
    for (int i = 0; i < D; ++i) {
        double acc = r[i];
        if (!a.tdiag) {
#pragma unroll
            for (int j = 0; j < i; ++j) acc = fma(-a.Lt[i * D + j], y[j], acc);
        }
        y[i] = acc * a.iLt[i];
    }
    return canon_sumsq<D, 1>(y);
}

// ‖L⁻¹ r‖² over the first n of D local entries (the update's Σ), canonical
// order of an n-vector: blocks of 8 when n % 8 == 0 and n ≥ 16, else one block.
template <int D>
__device__ __forceinline__ double mwg_sqmahal_u(const MwgUpdate &u, uint32_t n, const double (&r)[D]) {
    double y[D];
#pragma unroll
    for (int i = 0; i < D; ++i) {
        if ((uint32_t)i < n) {
            double acc = r[i];
            if (!u.diag) {
#pragma unroll
                for (int j = 0; j < i; ++j) acc = fma(-u.L[i * kMwgMaxD + j], y[j], acc);
            }
            y[i] = acc * u.iL[i];
        } else {
            y[i] = 0.0;
        }
    }
    const bool blocks = (n % 8 == 0 && n >= 16);
    if (!blocks) {
        double s = y[0] * y[0];
#pragma unroll
        for (int i = 1; i < D; ++i)
            if ((uint32_t)i < n) s = fma(y[i], y[i], s);
        return s;
    }
    // n = 16 (D = 16): two blocks of 8, one pairwise add
    double b0 = y[0] * y[0], b1 = y[8 % D] * y[8 % D];
#pragma unroll
    for (int i = 1; i < 8 && i < D; ++i) b0 = fma(y[i], y[i], b0);
#pragma unroll
    for (int i = 9; i < 16 && i < D; ++i) b1 = fma(y[i], y[i], b1);
    return b0 + b1;
}

template <int D, bool FULL, int LLMODE>
__global__ void __launch_bounds__(256) mwg_gsn_kernel(const MwgParams a) {
    static_assert(D <= kMwgMaxD, "MWG kernel supports D ≤ 16");
    // ziggurat tables → static LDS (the only lane-indexed constants)
    const ZigTabs zt = stage_lds(nullptr, a.zig, nullptr, 0, nullptr, 0);
    const uint64_t chain = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (chain >= a.C) return;
    const uint64_t C = a.C;
    const uint32_t gid = a.chain0 + (uint32_t)chain;

    double th[D], mp[D];
#pragma unroll
    for (int d = 0; d < D; ++d) {
        th[d] = a.theta[state_pos(d, chain, C, D)];
        mp[d] = a.mu_p[state_pos(d, chain, C, D)];
    }
    double ll = a.ll[chain];
    uint32_t faults = a.faults[chain];

    for (uint32_t s = 0; s < a.nsteps; ++s) {
        const uint32_t iter = a.steps[4 * s], pidx = a.steps[4 * s + 1], flags = a.steps[4 * s + 2];
        const uint32_t p = pidx - 1;
        const MwgUpdate &u = a.updates[p];
        const uint32_t n = u.nc;
        const uint64_t slot = (uint64_t)(iter - 1) * a.P + p;
        const uint64_t pc = (uint64_t)p * C + chain;
        // ---- update_workspaces!: θ_local ← θ[coords] (uniform coordinate indices)
        double tl[D], tp[D], ta[D];  // local θ, θ° (history / P°), θ° as stored on accept
#pragma unroll
        for (int j = 0; j < D; ++j) {
            double v = 0.0;
            if ((uint32_t)j < n) {
                const uint32_t cj = u.coords[j];
#pragma unroll
                for (int d = 0; d < D; ++d) v = (cj == (uint32_t)d) ? th[d] : v;
            }
            tl[j] = v;
        }
        // ---- proposal!
        double ltd_fwd = 0.0, ltd_rev = 0.0;
        if (u.kind == 1) {  // UniformRandomWalk: θ° = θ·1 + U, or θ·e^U where pos
            double ev[D];
#pragma unroll
            for (int j = 0; j < D; j += 2) {
                if ((uint32_t)j < n) {
                    const u32x4 r = draw(a.key0, a.key1, gid, iter, (uint32_t)j >> 1, p, 0);
                    const double e0 = u.adapt ? a.eps[((uint64_t)p * kMwgMaxD + j) * C + chain] : u.eps0[j];
                    const double U0 = (-e0) + (e0 - (-e0)) * u01_closed0(r.x, r.y);
                    tp[j] = ((u.posmask >> j) & 1u) ? tl[j] * exp_any(U0) + copysign(0.0, U0) : tl[j] * 1.0 + U0;
                    ev[j] = e0;
                    if (j + 1 < D && (uint32_t)(j + 1) < n) {
                        const double e1 = u.adapt ? a.eps[((uint64_t)p * kMwgMaxD + j + 1) * C + chain] : u.eps0[j + 1];
                        const double U1 = (-e1) + (e1 - (-e1)) * u01_closed0(r.z, r.w);
                        tp[j + 1] = ((u.posmask >> (j + 1)) & 1u) ? tl[j + 1] * exp_any(U1) + copysign(0.0, U1)
                                                                  : tl[j + 1] * 1.0 + U1;
                        ev[j + 1] = e1;
                    }
                }
            }
            if (u.posmask) {  // uniform branch: the mask is the update's
#pragma unroll
                for (int j = 0; j < D; ++j) {
                    if ((uint32_t)j < n) {
                        const bool pj = (u.posmask >> j) & 1u;
                        const double c = pj ? -log_any(2.0 * ev[j]) : 0.0;
                        const double f = pj ? c - log_any(tp[j]) : 0.0;  // logpdf(rw, θ, θ°) term
                        const double g = pj ? c - log_any(tl[j]) : 0.0;  // logpdf(rw, θ°, θ) term
                        ltd_fwd = (j == 0) ? f : ltd_fwd + f;
                        ltd_rev = (j == 0) ? g : ltd_rev + g;
                    }
                }
            }
        } else {  // GaussianRandomWalk over the update's coordinates
            const uint32_t pm = u.posmask;  // positivity-restricted coordinates (log scale)
            auto isp = [&](int i) { return ((pm >> i) & 1u) != 0u; };
            double z[D];
#pragma unroll
            for (int j = 0; j < D; ++j)
                z[j] = ((uint32_t)j < n) ? normal_draw(zt, a.key0, a.key1, gid, iter, p, (uint32_t)j, faults) : 0.0;
#pragma unroll
            for (int i = 0; i < D; ++i) {
                if ((uint32_t)i < n) {
                    double lz;
                    if (u.diag) {
                        lz = u.L[i * kMwgMaxD + i] * z[i];
                    } else {
                        lz = u.L[i * kMwgMaxD] * z[0];
#pragma unroll
                        for (int j = 1; j <= i; ++j) lz = fma(u.L[i * kMwgMaxD + j], z[j], lz);
                    }
                    // remove_constraints!: θ_i ← log θ_i where pos (random_walk.jl:136, 145-147)
                    tp[i] = (isp(i) ? log_any(tl[i]) : tl[i]) + lz;
                } else {
                    tp[i] = 0.0;
                }
            }
            double r[D];
            if (pm == 0u) {
#pragma unroll
                for (int i = 0; i < D; ++i) r[i] = tp[i] - tl[i];
                ltd_fwd = u.c0 - mwg_sqmahal_u<D>(u, n, r) / 2.0;
#pragma unroll
                for (int i = 0; i < D; ++i) r[i] = tl[i] - tp[i];
                ltd_rev = u.c0 - mwg_sqmahal_u<D>(u, n, r) / 2.0;
            } else {
                // The reference's in-place round trips, step by step (random_walk.jl:136-171):
                //   rand:   θ° ← exp(log θ + Lz), θ ← exp(log θ)               (θ°₁, θ₁)
                //   logpdf(θ°₁, θ₁): logJ = −Σ_pos log θ₁; MvNormal(log θ°₁) at log θ₁;
                //           then θ°₂ = exp(log θ°₁), θ₂ = exp(log θ₁)
                //   logpdf(θ₂, θ°₂): logJ = −Σ_pos log θ°₂; MvNormal(log θ₂) at log θ°₂;
                //           then θ°₃ = exp(log θ°₂) — the value an accept stores
                double t1[D], a1[D], b1[D];
                double lj = 0.0;
                bool first = true;
#pragma unroll
                for (int i = 0; i < D; ++i) {
                    if ((uint32_t)i < n) {
                        tp[i] = isp(i) ? exp_any(tp[i]) : tp[i];              // θ°₁
                        t1[i] = isp(i) ? exp_any(log_any(tl[i])) : tl[i];     // θ₁
                        if (isp(i)) {
                            const double v = log_any(t1[i]);
                            lj = first ? v : lj + v;
                            first = false;
                        }
                        a1[i] = isp(i) ? log_any(tp[i]) : tp[i];             // μ = log θ°₁
                        b1[i] = isp(i) ? log_any(t1[i]) : t1[i];             // x = log θ₁
                        r[i] = b1[i] - a1[i];
                    } else {
                        t1[i] = a1[i] = b1[i] = r[i] = 0.0;
                    }
                }
                ltd_rev = (u.c0 - mwg_sqmahal_u<D>(u, n, r) / 2.0) + (-lj);
                lj = 0.0;
                first = true;
#pragma unroll
                for (int i = 0; i < D; ++i) {
                    if ((uint32_t)i < n) {
                        const double p2 = isp(i) ? exp_any(a1[i]) : a1[i];  // θ°₂
                        const double l2 = isp(i) ? exp_any(b1[i]) : b1[i];  // θ₂
                        if (isp(i)) {
                            const double v = log_any(p2);
                            lj = first ? v : lj + v;
                            first = false;
                        }
                        const double a2 = isp(i) ? log_any(l2) : l2;        // μ = log θ₂
                        const double b2 = isp(i) ? log_any(p2) : p2;        // x = log θ°₂
                        r[i] = b2 - a2;
                        ta[i] = isp(i) ? exp_any(b2) : p2;                  // θ°₃
                    } else {
                        r[i] = 0.0;
                    }
                }
                ltd_fwd = (u.c0 - mwg_sqmahal_u<D>(u, n, r) / 2.0) + (-lj);
            }
        }
        if (!(u.kind == 2 && u.posmask != 0u)) {
#pragma unroll
            for (int j = 0; j < D; ++j) ta[j] = tp[j];
        }
        // ---- set_proposal!: proposal history and P°.θ[coords] ← θ°
        double prop[D], nst[D];
#pragma unroll
        for (int d = 0; d < D; ++d) prop[d] = nst[d] = th[d];
#pragma unroll
        for (int j = 0; j < D; ++j) {
            if ((uint32_t)j < n) {
                const uint32_t cj = u.coords[j];
#pragma unroll
                for (int d = 0; d < D; ++d) {
                    prop[d] = (cj == (uint32_t)d) ? tp[j] : prop[d];
                    mp[d] = (cj == (uint32_t)d) ? tp[j] : mp[d];
                    nst[d] = (cj == (uint32_t)d) ? ta[j] : nst[d];
                }
            }
        }
        // ---- compute_ll!: loglikelihood(P°, obs)
        double llp;
        if constexpr (LLMODE == LL_PER_OBS) {
            llp = 0.0;
            for (uint32_t k = 0; k < a.nobs; ++k) {
                double r[D];
#pragma unroll
                for (int i = 0; i < D; ++i) r[i] = a.obs[(size_t)k * D + i] - mp[i];
                llp = llp + (a.t_c0 - mwg_sqmahal_t<D>(a, r) / 2.0);
            }
        } else {
            double r[D];
#pragma unroll
            for (int i = 0; i < D; ++i) r[i] = a.xbar[i] - mp[i];
            const double qv = mwg_sqmahal_t<D>(a, r);
            llp = a.n_tc0 - (a.S_c + a.nobs_d * qv) * 0.5;
        }
        if (!(llp - llp == 0.0)) faults |= 1u;
        // ---- accept_reject!
        const double llr = ((((llp - ll) + ltd_rev) - ltd_fwd) + 0.0) - 0.0;
        const double E = exp_draw(zt, a.key0, a.key1, gid, iter, p, faults);
        const bool acc = E > -llr;
        if constexpr (FULL) {
#pragma unroll
            for (int d = 0; d < D; ++d) __builtin_nontemporal_store(prop[d], a.hist_prop + slot * D * C + state_pos(d, chain, C, D));
        }
        if (acc) {  // set_chain_param!: θ[coords] ← θ° (run.jl:312-318)
#pragma unroll
            for (int d = 0; d < D; ++d) th[d] = nst[d];
            ll = llp;
        }
        if constexpr (FULL) {
#pragma unroll
            for (int d = 0; d < D; ++d) __builtin_nontemporal_store(th[d], a.hist_theta + slot * D * C + state_pos(d, chain, C, D));
            __builtin_nontemporal_store(ll, a.hist_ll + slot * C + chain);
        }
        {
            const uint64_t m = __ballot(acc);
            if ((threadIdx.x & 63) == 0) store_acc_bits<1>(a.hist_acc + slot * a.row_bytes, chain, m);
        }
        a.nacc[pc] += acc ? 1u : 0u;
        // ---- update_stats!: rolling acceptance of update p
        {
            const uint64_t N = a.N0 + s;
            uint64_t r0 = a.ring[2 * pc], r1 = a.ring[2 * pc + 1];
            const double ra_prev = (flags & 1u) ? a.ra[pc] : 0.0;
            int out = 0;
            if (iter > a.W) {
                const uint32_t j = (iter - a.W) & 127u;
                out = (int)((((j & 64u) ? r1 : r0) >> (j & 63u)) & 1ull);
            }
            const uint64_t mn = (N < (uint64_t)a.W) ? N : (uint64_t)a.W;
            a.ra[pc] = (ra_prev * (double)a.W + (double)((int)acc - out)) / (double)mn;
            const uint32_t jw = iter & 127u;
            const uint64_t bit = 1ull << (jw & 63u);
            if (jw & 64u) r1 = acc ? (r1 | bit) : (r1 & ~bit);
            else r0 = acc ? (r0 | bit) : (r0 & ~bit);
            a.ring[2 * pc] = r0;
            a.ring[2 * pc + 1] = r1;
        }
        // ---- update_adaptation!: AdaptationUnifRW on its own turn
        if (u.adapt == 1) {
            const uint32_t pr = a.aprop[pc] + 1, ac = a.aacc[pc] + (acc ? 1u : 0u);
            if (pr >= u.k) {  // proposed counts are equal across chains: uniform branch
                const double delta = u.scale / sqrt(fmax(1.0, (double)iter / (double)u.k - u.offset));
                const double a_r = (double)ac / (double)pr;
                const double stp = (a_r > u.target) ? delta : -delta;
#pragma unroll
                for (int j = 0; j < D; ++j) {
                    if ((uint32_t)j < n) {
                        double *ep = a.eps + ((uint64_t)p * kMwgMaxD + j) * C + chain;
                        double e = *ep + stp;
                        e = (e < u.amax) ? e : u.amax;
                        *ep = (e > u.amin) ? e : u.amin;
                    }
                }
                a.aprop[pc] = 0;
                a.aacc[pc] = 0;
            } else {
                a.aprop[pc] = pr;
                a.aacc[pc] = ac;
            }
        }
    }
#pragma unroll
    for (int d = 0; d < D; ++d) {
        a.theta[state_pos(d, chain, C, D)] = th[d];
        a.mu_p[state_pos(d, chain, C, D)] = mp[d];
    }
    a.ll[chain] = ll;
    a.faults[chain] = faults;
    if (faults) *a.fault_flag = 1u;
}

}  // namespace emcmc
