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
//   proposal! resample  θ° is drawn again while logpdf(prior, θ°) === −Inf
//                       (resample r uses counter blocks (r << 16) | j/2, Gaussian normal
//                       indices (r << 17) | j; capped at kMaxResample / kMaxResampleGsn
//                       with fault bit 8)                               updates.jl:191-196
//   log_prior           logpdf(prior, θ_local) of ImproperPrior, ImproperPosPrior,
//                       ProductPrior (the constructor's index list: a dims-1 factor
//                       reads θ[1], a dims-k factor θ[last:last+k−1]) and StandardPrior
//                       of univariate, Product and MvNormal factors; llr adds
//                       lp(θ°) − lp(θ)                 priors.jl:18-88, run.jl:374-385
//   loglikelihood       a target policy: GsnTargetLaw (gsn_target.jl:23-29) or a
//                       user device function compiled at run time (emcmc_rtc.h)
//   user updates        an update policy: a user's proposal! and log_transition_density
//                       (updates.jl:42-93) compiled at run time; draws come from the
//                       engine's stream by index (UserRng)
#pragma once

#include "emcmc_kernels.h"

namespace emcmc {

constexpr int kMwgMaxD = 64;  // largest D of the general kernel (D ≤ 32 instantiated ahead of time, the rest at run time)
constexpr uint32_t kMaxResample = 0xFFFEu;          // proposal! resamples before fault bit 8 (UniformRandomWalk:
                                                    // counter block (r << 16) | j/2)
constexpr uint32_t kMaxResampleGsn = 0x7FFEu;       // GaussianRandomWalk: normal index (r << 17) | j stays below
                                                    // 2^32, so no redraw repeats an earlier one's variates
constexpr uint32_t kFaultPriorResample = 8u;       // EMCMC_FAULT_PRIOR_RESAMPLES

// prior kinds / univariate families (include/emcmc.h EMCMC_PRIOR_*, EMCMC_DIST_*)
constexpr uint32_t kPriorImproper = 0u, kPriorImproperPos = 1u, kPriorProduct = 2u, kPriorStandard = 3u;
constexpr uint32_t kDistNormal = 1u, kDistUniform = 2u, kDistExponential = 3u, kDistGamma = 4u, kDistLogNormal = 5u,
                   kDistBeta = 6u, kDistInverseGamma = 7u, kDistCauchy = 8u, kDistLaplace = 9u, kDistTDist = 10u;

// update kinds (include/emcmc.h): EMCMC_RW_UNIFORM 1, EMCMC_RW_GAUSSIAN 2, a user update 5,
// MALA 4 (with the target's gradient: the built-in GsnTargetLaw or a user law's EMCMC_USER_GRAD)
constexpr uint32_t kKindUser = 5u, kKindMix = 3u, kKindMala = 4u;
constexpr uint32_t kFaultPosdefMwg = 4u;  // EMCMC_FAULT_POSDEF

// One RandomWalkUpdate (or user update), host-built; read with scalar (uniform) loads.
struct MwgUpdate {
    uint32_t kind;    // EMCMC_RW_UNIFORM (1) / EMCMC_RW_GAUSSIAN (2)
    uint32_t nc;      // number of coordinates
    uint32_t adapt;   // EMCMC_ADPT_NONE (0) / AdaptationUnifRW (1, scalar or per-coordinate form)
    uint32_t k;       // adapt_every_k_steps
    uint32_t coords[kMwgMaxD];
    double eps0[kMwgMaxD];          // UniformRandomWalk ϵ (initial for adaptive updates)
    double uc[kMwgMaxD];            // UniformRandomWalk: −log(2ϵ_j) of eps0 by the device's log_any
                                    // (mwg_rw_block_kernel's logpdf constant; host-computed)
    double L[kMwgMaxD * kMwgMaxD];  // GaussianRandomWalk: lower Cholesky factor, row-major, local indices;
                                    // a user update: its parameters (≤ 4096 doubles)
    double iL[kMwgMaxD];            // 1 / L_ii
    double c0;                      // −(nc·log2π + logdet Σ)/2
    uint32_t diag, reserved0;
    uint64_t posmask;                // bit j: coordinate j positivity-restricted
    double target;                  // AdaptationUnifRW target_accpt_rate
    double ascale[kMwgMaxD], amin[kMwgMaxD], amax[kMwgMaxD], aoff[kMwgMaxD];  // per coordinate (the scalar
                                    // form repeats its values)
    // prior over the update's local coordinates (priors.jl), host-built from the
    // factors as a list of nslot term slots.  The constructor's index list makes
    // every factor take as many slots as its dims advance `last` (priors.jl:64-79),
    // so slot j reads θ_local[j] — or θ_local[1] (bit j of psrc0) for a dims-1
    // factor — and the slots of one factor are contiguous: bit j of pstart / pend
    // marks a factor's first / last slot.  Univariate and Product-component slots
    // hold a family and its parameters; MvNormal slots (bit j of pmvn) a row of the
    // forward substitution: μ_j, L_j· (lower factor, block-diagonal over the
    // factors, row-major by slot), 1/L_jj, the factor's first slot pmvs[j]; the
    // factor's c0 sits in pc of its last slot.
    uint32_t prior, nslot;
    uint64_t psrc0, pstart, pend, pmvn;
    uint32_t pfam[kMwgMaxD];
    uint32_t pmvs[kMwgMaxD];
    double pa[kMwgMaxD], pb[kMwgMaxD], pc[kMwgMaxD];  // family parameters + host-computed constants
    double pmu[kMwgMaxD], piL[kMwgMaxD];
    double pL[kMwgMaxD * kMwgMaxD];
    // GaussianRandomWalkMix (kind 3): Σ_A in L / iL / c0 / diag, λ, and per-chain
    // state in MwgParams::mixpool, SoA over chains: L_B packed lower row-major
    // [n(n+1)/2][C] at lb_off, 1/L_B,ii [n][C] at lbi_off, c0_B [C] at lbc_off,
    // a readjust scratch factor [n(n+1)/2][C] at lbs_off.  HaarioTypeAdaptation
    // (hk = adapt_every_k_steps > 0): mean [n][C] at hm_off, cov packed lower
    // [n(n+1)/2][C] at hc_off.
    double lam;
    uint32_t hk, reserved2;
    uint64_t lb_off, lbi_off, lbc_off, lbs_off, hm_off, hc_off;
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
    double *ll_prop;   // [P][C] sub_ws°.ll: log-likelihood of the update's latest proposal
    const double *user_params;  // user target: opaque parameters (emcmc_target_desc.user_params)
    double *hist_theta, *hist_prop, *hist_ll;
    uint8_t *hist_acc;
    const Ziggurat *zig;
    const MwgUpdate *updates;  // [P]
    const uint32_t *steps;     // [nsteps][4]: mcmciter, pidx (1-based), flags (bit 0: ra_prev valid), 0
    const double *Lt;          // target: lower Cholesky, row-major D×D
    const double *iLt;         // 1 / Lt_ii
    const double *xbar;        // [D]
    const double *obs;         // [nobs][D]
    double *mixpool;           // GaussianRandomWalkMix / Haario per-chain state (MwgUpdate offsets)
    double *smean, *scov;      // GenericChainStats mean [D][C] and cov packed lower [D(D+1)/2][C]
    double *gcache;            // [D][C] ∇ℓ at the current θ (state_pos layout), or null: the MALA carry below
    const double *consts;      // mwg_block_kernel's constant table (emcmc_block.h BlockConsts), else null
    uint64_t C;
    uint64_t row_bytes;
    uint64_t N0;
    uint32_t chain0, key0, key1, nsteps, P, W, nobs, tdiag;
    uint32_t chain_moments, nhaario;  // update_stats! mean/cov on; number of Haario updates
    double t_c0, n_tc0, S_c, nobs_d;
};

// MALA gradient carry.  The reference calls compute_gradients_and_momenta! twice per
// step: at P°.θ with coords ← θ (__PREVIOUS) and at P°.θ after set_parameters! (the
// proposal, __PROPOSAL; run.jl:110, 259).  With ONE update over all D coordinates the
// first point is θ itself, which is the previous step's proposal point when it was
// accepted and the previous step's first point when it was rejected: the same doubles,
// so the same gradient bits.  Within a launch the kernel therefore keeps ∇ℓ(θ) per chain
// in gcache and evaluates the gradient once per step (the first step of a launch
// computes it).  Anything else (P > 1, a partial update) evaluates both.
__device__ __forceinline__ bool mala_carry(const MwgParams &a, uint32_t n, uint32_t D) {
    return a.gcache != nullptr && a.P == 1u && n == D;
}

// log of any real: NaN below 0 (Julia's log throws DomainError there), −Inf at 0
__device__ __forceinline__ double log_real(double x) { return (x < 0.0) ? __builtin_nan("") : log_any(x); }

// logpdf of one univariate prior factor at x (Distributions.jl / StatsFuns
// forms; a, b the parameters, c a constant computed once on the
// host; restated in oracle/emcmc_oracle.c orc_univariate_logpdf):
//   Normal(μ=a, σ=b), c = log σ:      −(z² + log2π)/2 − c, z = (x − μ)/σ
//   Uniform(a, b), c = −log(b − a):   c on [a, b], else −Inf
//   Exponential(θ), b = 1/θ, c = log(1/θ):   x < 0 ? −Inf : c − b·x
//   Gamma(α=a, θ=b), c = −lgamma(α) − α·log θ:  x < 0 ? −Inf : (c + (α − 1)·log x) − x/θ
//   LogNormal(μ=a, σ=b), c = log σ:   x ≤ 0 ? −Inf : (−(z² + log2π)/2 − c) − log x, z = (log x − μ)/σ
//   Beta(α=a, β=b), c = logbeta(α, β): x ∉ [0, 1] ? −Inf : (xlogy(α−1, x) + xlog1py(β−1, −x)) − c
//   InverseGamma(α=a, θ=b), c = α·log θ − lgamma(α): x ≤ 0 ? −Inf : (c − (α + 1)·log x) − θ/x
//   Cauchy(μ=a, σ=b), c = log σ:  −((log1psq(z) + log π) + c), z = (x − μ)/σ (Distributions.jl's
//     −(log1psq(z) + logπ + log(σ)), left to right; log1psq(z) = |z| < 2^53 ? log1p(z²) : 2·log|z|)
//   Laplace(μ=a, θ=b), c = log(2θ):   −(|x − μ|/θ + c)
//   TDist(ν=a), b = (ν + 1)/2, c = (lgamma((ν+1)/2) − lgamma(ν/2)) − log(νπ)/2:  c − b·log1p(x²/ν)
__device__ __forceinline__ double univariate_logpdf(uint32_t fam, double a, double b, double c, double x) {
    const double ninf = -__builtin_inf();
    switch (fam) {
    case kDistNormal: {
        const double z = (x - a) / b;
        return -(z * z + kLog2Pi) / 2.0 - c;
    }
    case kDistUniform: return (x >= a && x <= b) ? c : ninf;
    case kDistExponential: return (x < 0.0) ? ninf : c - b * x;
    case kDistGamma: return (x < 0.0) ? ninf : (c + (a - 1.0) * log_real(x)) - x / b;
    case kDistLogNormal: {
        if (!(x > 0.0)) return (x != x) ? x : ninf;
        const double lx = log_any(x);
        const double z = (lx - a) / b;
        return (-(z * z + kLog2Pi) / 2.0 - c) - lx;
    }
    case kDistBeta: {
        if (x < 0.0 || x > 1.0) return ninf;
        const double t1 = (a - 1.0 == 0.0) ? 0.0 : (a - 1.0) * log_real(x);
        const double t2 = (b - 1.0 == 0.0) ? 0.0 : (b - 1.0) * log1p_any(-x);
        return (t1 + t2) - c;
    }
    case kDistInverseGamma:
        if (!(x > 0.0)) return (x != x) ? x : ninf;
        return (c - (a + 1.0) * log_any(x)) - b / x;
    case kDistCauchy: {  // log1psq(z): log1p(z²) below maxintfloat = 2^53, else 2·log|z|
        const double z = (x - a) / b, az = fabs(z);
        const double l = (az < 0x1p53) ? log1p_any(az * az) : 2.0 * log_any(az);
        return -((l + 1.1447298858494002) + c);  // log π
    }
    case kDistLaplace: return -(fabs(x - a) / b + c);
    default:  // kDistTDist
        return c - b * log1p_any((x * x) / a);
    }
}

// logpdf(prior, θ_local) (priors.jl:18-88) over the first n of D local entries.
//   ImproperPrior: 0.0.  ImproperPosPrior: −sum(log.(θ)), the sum folded left
//   from θ_1.  ProductPrior: lp = 0.0; lp += logpdf(dist_k, θ[idx_k]) in factor
//   order over the constructor's index list (MwgUpdate slots).  StandardPrior:
//   logpdf(dist, θ) of its one multivariate factor.  A factor's value: a
//   univariate's logpdf; a Product's component logpdfs folded left; an MvNormal's
//   c0 − ‖L⁻¹(θ − μ)‖²/2 with the squares folded left (s = y₁², s = fma(y_j, y_j, s)).
template <int D, bool ROLL = false>
__device__ __forceinline__ double mwg_log_prior(const MwgUpdate &u, uint32_t n, const double (&x)[D]) {
    constexpr int UJ = ROLL ? 1 : D;
    if (u.prior == kPriorImproper) return 0.0;
    if (u.prior == kPriorImproperPos) {
        double s = 0.0;
#pragma unroll UJ
        for (int j = 0; j < D; ++j) {
            if ((uint32_t)j < n) {
                const double v = log_real(x[j]);
                s = (j == 0) ? v : s + v;
            }
        }
        return -s;
    }
    const bool mvn = u.pmvn != 0ull;  // wave-uniform: the MvNormal rows only when a factor needs them
    double lp = 0.0, s = 0.0;
    double y[D];  // MvNormal factors: L⁻¹(θ − μ) by slot
#pragma unroll UJ
    for (int j = 0; j < D; ++j) {
        y[j] = 0.0;
        if ((uint32_t)j < u.nslot) {
            const double xv = ((u.psrc0 >> j) & 1ull) ? x[0] : x[j];
            const bool first = ((u.pstart >> j) & 1ull) != 0ull;
            const bool mj = ((u.pmvn >> j) & 1ull) != 0ull;
            if (mvn && mj) {
                double acc = xv - u.pmu[j];
                const uint32_t m0 = u.pmvs[j];
#pragma unroll UJ
                for (int m = 0; m < j; ++m)
                    if ((uint32_t)m >= m0) acc = fma(-u.pL[j * kMwgMaxD + m], y[m], acc);
                y[j] = acc * u.piL[j];
                s = first ? y[j] * y[j] : fma(y[j], y[j], s);
            } else {
                const double v = univariate_logpdf(u.pfam[j], u.pa[j], u.pb[j], u.pc[j], xv);
                s = first ? v : s + v;
            }
            if ((u.pend >> j) & 1ull) {
                const double fv = mj ? u.pc[j] - s / 2.0 : s;
                lp = (u.prior == kPriorProduct) ? lp + fv : fv;
            }
        }
    }
    return lp;
}

// ‖L⁻¹ r‖² for a D-vector (target Σ; dense forward substitution unless
// diagonal), canonical order (SumShape<D>).
template <int D, bool ROLL = false>
__device__ __forceinline__ double mwg_sqmahal_t(const MwgParams &a, const double (&r)[D]) {
    constexpr int UJ = ROLL ? 1 : D;
    double y[D];
#pragma unroll UJ
    for (int i = 0; i < D; ++i) {
        double acc = r[i];
        if (!a.tdiag) {
#pragma unroll UJ
            for (int j = 0; j < i; ++j) acc = fma(-a.Lt[i * D + j], y[j], acc);
        }
        y[i] = acc * a.iLt[i];
    }
    return canon_sumsq<D, 1>(y);
}

template <int D, bool ROLL>
__device__ __forceinline__ double mwg_sumsq_n(const double (&y)[D], uint32_t n);

// ‖L⁻¹ r‖² over the first n of D local entries (the update's Σ), canonical
// order of an n-vector: blocks of 8 when n % 8 == 0 and n ≥ 16, else one block.
template <int D, bool ROLL = false>
__device__ __forceinline__ double mwg_sqmahal_u(const MwgUpdate &u, uint32_t n, const double (&r)[D]) {
    constexpr int UJ = ROLL ? 1 : D;
    double y[D];
#pragma unroll UJ
    for (int i = 0; i < D; ++i) {
        if ((uint32_t)i < n) {
            double acc = r[i];
            if (!u.diag) {
#pragma unroll UJ
                for (int j = 0; j < i; ++j) acc = fma(-u.L[i * kMwgMaxD + j], y[j], acc);
            }
            y[i] = acc * u.iL[i];
        } else {
            y[i] = 0.0;
        }
    }
    return mwg_sumsq_n<D, ROLL>(y, n);
}

// Σ y_i² over the first n of D entries in the canonical order of an n-vector:
// blocks of 8 when n % 8 == 0 and n ≥ 16, else one block (s = y₀², s = fma(y_i, y_i, s)).
template <int D, bool ROLL>
__device__ __forceinline__ double mwg_sumsq_n(const double (&y)[D], uint32_t n) {
    constexpr int UJ = ROLL ? 1 : D;
    const bool blocks = (n % 8 == 0 && n >= 16);
    if (!blocks) {
        double s = y[0] * y[0];
#pragma unroll UJ
        for (int i = 1; i < D; ++i)
            if ((uint32_t)i < n) s = fma(y[i], y[i], s);
        return s;
    }
    // n ∈ {16, 24, …, 64}: blocks of 8, then the pairwise tree over the n/8
    // blocks (tree_inplace's order with a run-time block count)
    constexpr int NBMAX = D / 8 > 0 ? D / 8 : 1;
    double b[NBMAX];
#pragma unroll UJ
    for (int k = 0; k < NBMAX; ++k) {
        b[k] = y[8 * k] * y[8 * k];
#pragma unroll UJ
        for (int i = 1; i < 8; ++i) b[k] = fma(y[8 * k + i], y[8 * k + i], b[k]);
    }
    uint32_t nb = n / 8;
#pragma unroll
    for (int lvl = 0; lvl < 3; ++lvl) {  // NBMAX ≤ 8
        if (nb <= 1) break;
        double last = b[0];
#pragma unroll
        for (int q = 1; q < NBMAX; ++q) last = ((uint32_t)q == nb - 1) ? b[q] : last;
#pragma unroll
        for (int i = 0; i < NBMAX / 2; ++i)
            if ((uint32_t)i < nb / 2) b[i] = b[2 * i] + b[2 * i + 1];
        if (nb & 1u) {
#pragma unroll
            for (int q = 0; q < NBMAX; ++q) b[q] = ((uint32_t)q == nb / 2) ? last : b[q];
        }
        nb = (nb + 1) / 2;
    }
    return b[0];
}

// ---- GaussianRandomWalkMix on the general kernel -----------------------------
__device__ __forceinline__ uint32_t tri_idx(uint32_t i, uint32_t j) { return i * (i + 1) / 2 + j; }

// The chain's own L_B (packed lower, SoA over chains in MwgParams::mixpool).
struct MixB {
    const double *lb, *lbi;
    uint64_t C, chain;
    __device__ __forceinline__ double L(uint32_t i, uint32_t j) const { return lb[(uint64_t)tri_idx(i, j) * C + chain]; }
    __device__ __forceinline__ double iL(uint32_t i) const { return lbi[(uint64_t)i * C + chain]; }
};

// ‖L_B⁻¹ r‖², the same substitution and canonical sum as mwg_sqmahal_u
template <int D, bool ROLL>
__device__ __forceinline__ double mwg_sqmahal_b(const MixB &B, uint32_t n, const double (&r)[D]) {
    constexpr int UJ = ROLL ? 1 : D;
    double y[D];
#pragma unroll UJ
    for (int i = 0; i < D; ++i) {
        if ((uint32_t)i < n) {
            double acc = r[i];
#pragma unroll UJ
            for (int j = 0; j < i; ++j) acc = fma(-B.L((uint32_t)i, (uint32_t)j), y[j], acc);
            y[i] = acc * B.iL((uint32_t)i);
        } else {
            y[i] = 0.0;
        }
    }
    return mwg_sumsq_n<D, ROLL>(y, n);
}

// logpdf(rw::GaussianRandomWalk, a, b) (random_walk.jl:161-171) with its in-place
// round trips (oracle orc_gsn_rw_lp): logJ = −sum(log b[pos]) folded left,
// logpdf(MvNormal(log a, Σ), log b) + logJ, then a, b ← exp(log ·) where pos.
// B: nullptr for the update's Σ_A, else the chain's Σ_B.
template <int NU, bool ROLL>
__device__ __forceinline__ double mwg_gsn_rw_lp(const MwgUpdate &u, const MixB *B, double c0, uint32_t n,
                                                double (&a)[NU], double (&b)[NU]) {
    constexpr int UJ = ROLL ? 1 : NU;
    const uint64_t pm = u.posmask;
    double x[NU], y[NU], r[NU];
    double lj = 0.0;
    bool first = true;
#pragma unroll UJ
    for (int i = 0; i < NU; ++i)
        if ((uint32_t)i < n && ((pm >> i) & 1ull)) {
            const double v = log_any(b[i]);
            lj = first ? v : lj + v;
            first = false;
        }
#pragma unroll UJ
    for (int i = 0; i < NU; ++i) {
        const bool pi = (uint32_t)i < n && ((pm >> i) & 1ull);
        x[i] = pi ? log_any(a[i]) : a[i];
        y[i] = pi ? log_any(b[i]) : b[i];
        r[i] = ((uint32_t)i < n) ? y[i] - x[i] : 0.0;
    }
    double lp = c0 - (B ? mwg_sqmahal_b<NU, ROLL>(*B, n, r) : mwg_sqmahal_u<NU, ROLL>(u, n, r)) / 2.0;
    if (pm) lp = lp + (-lj);
#pragma unroll UJ
    for (int i = 0; i < NU; ++i)
        if ((uint32_t)i < n && ((pm >> i) & 1ull)) {
            a[i] = exp_any(x[i]);
            b[i] = exp_any(y[i]);
        }
    return lp;
}

// The built-in target: loglikelihood(P°::GsnTargetLaw, obs) (gsn_target.jl:23-29),
// per observation or through the sufficient statistics.
struct GsnTarget {
    template <int D, int LLMODE, bool ROLL = false>
    __device__ __forceinline__ static double loglik(const MwgParams &a, const double (&mp)[D]) {
        constexpr int UJ = ROLL ? 1 : D;
        if constexpr (LLMODE == LL_PER_OBS) {
            double llp = 0.0;
            for (uint32_t k = 0; k < a.nobs; ++k) {
                double r[D];
#pragma unroll UJ
                for (int i = 0; i < D; ++i) r[i] = a.obs[(size_t)k * D + i] - mp[i];
                llp = llp + (a.t_c0 - mwg_sqmahal_t<D, ROLL>(a, r) / 2.0);
            }
            return llp;
        } else {
            double r[D];
#pragma unroll UJ
            for (int i = 0; i < D; ++i) r[i] = a.xbar[i] - mp[i];
            const double qv = mwg_sqmahal_t<D, ROLL>(a, r);
            return a.n_tc0 - (a.S_c + a.nobs_d * qv) * 0.5;
        }
    }
    // ∇_μ loglikelihood(P°, obs) = Σ_k Σ⁻¹(x_k − μ) = n·Σ⁻¹(x̄ − μ) (both likelihood
    // modes): y = L⁻¹(x̄ − μ) forward (as mwg_sqmahal_t), w = L⁻ᵀy backward
    // (w_i = (y_i − Σ_{j>i} L_ji w_j)/L_ii, j descending), g = n·w
    // (oracle orc_gsn_grad).  The hook MALA reads (compute_gradients_and_momenta!).
    template <int D, int LLMODE, bool ROLL = false>
    __device__ __forceinline__ static void grad(const MwgParams &a, const double (&mp)[D], double (&g)[D]) {
        constexpr int UJ = ROLL ? 1 : D;
        double y[D];
#pragma unroll UJ
        for (int i = 0; i < D; ++i) {
            double acc = a.xbar[i] - mp[i];
            if (!a.tdiag) {
#pragma unroll UJ
                for (int j = 0; j < i; ++j) acc = fma(-a.Lt[i * D + j], y[j], acc);
            }
            y[i] = acc * a.iLt[i];
        }
#pragma unroll UJ
        for (int ii = 0; ii < D; ++ii) {
            const int i = D - 1 - ii;
            double acc = y[i];
            if (!a.tdiag) {
#pragma unroll UJ
                for (int j = D - 1; j > i; --j) acc = fma(-a.Lt[j * D + i], g[j], acc);
            }
            g[i] = acc * a.iLt[i];
        }
#pragma unroll UJ
        for (int i = 0; i < D; ++i) g[i] = a.nobs_d * g[i];
    }
};

// ---- MALA (kind 4) on the general kernel -------------------------------------
// The reference stubs MALAUpdate (updates.jl:216-218) and gives a gradient-based
// update one hook, compute_gradients_and_momenta!, called on the current state
// in update_workspaces! (run.jl:110, __PREVIOUS) and on the proposal in
// compute_ll! (run.jl:259, __PROPOSAL).  The engine's definition over the
// update's n local coordinates (oracle orc_run_mwg kind 4):
//   g  = ∇ℓ(x)[coords], x = P°.θ with coords ← θ   (the vector whose ℓ the ratio
//        pairs with θ: the coordinates outside the update are P°'s)
//   θ° = m + ϵz, m = θ + h·g, h = ϵ²/2, z_j normal j of (chain, iter, update)
//   ltd_fwd = logpdf(MvNormal(m, ϵ²I), θ°), g° = ∇ℓ(P°.θ)[coords] after
//   set_proposal!, ltd_rev = logpdf(MvNormal(θ° + h·g°, ϵ²I), θ); both as the
//   update's diagonal Gaussian (L = ϵI: c0 − ‖(·)/ϵ‖²/2, the canonical sum).
// The prior enters the ratio as for any update; MALA has no proposal! redraw.
// eps0[0] = ϵ, eps0[1] = h (host-computed).
template <int NU, bool ROLL>
__device__ __forceinline__ void mwg_mala_forward(const MwgParams &a, const ZigTabs &zt, const MwgUpdate &u,
                                                 uint32_t n, uint32_t gid, uint32_t iter, uint32_t p,
                                                 const double (&tl)[NU], const double (&gl)[NU], double (&tp)[NU],
                                                 double &ltd_fwd, uint32_t &faults) {
    constexpr int UJ = ROLL ? 1 : NU;
    const double eps = u.eps0[0], h = u.eps0[1];
    double r[NU];
#pragma unroll UJ
    for (int j = 0; j < NU; ++j) {
        if ((uint32_t)j < n) {
            const double z = normal_draw(zt, a.key0, a.key1, gid, iter, p, (uint32_t)j, faults);
            const double m = tl[j] + h * gl[j];
            tp[j] = m + eps * z;
            r[j] = tp[j] - m;
        } else {
            tp[j] = 0.0;
            r[j] = 0.0;
        }
    }
    ltd_fwd = u.c0 - mwg_sqmahal_u<NU, ROLL>(u, n, r) / 2.0;
}
template <int NU, bool ROLL>
__device__ __forceinline__ double mwg_mala_reverse(const MwgUpdate &u, uint32_t n, const double (&tl)[NU],
                                                   const double (&tp)[NU], const double (&gp)[NU]) {
    constexpr int UJ = ROLL ? 1 : NU;
    const double h = u.eps0[1];
    double r[NU];
#pragma unroll UJ
    for (int j = 0; j < NU; ++j) r[j] = ((uint32_t)j < n) ? tl[j] - (tp[j] + h * gp[j]) : 0.0;
    return u.c0 - mwg_sqmahal_u<NU, ROLL>(u, n, r) / 2.0;
}
// gl[j] = g[coords[j]] for the update's local coordinates (selects over D)
template <int D, int NU, bool ROLL>
__device__ __forceinline__ void mwg_gather(const MwgUpdate &u, uint32_t n, const double (&g)[D], double (&gl)[NU]) {
    constexpr int UJ = ROLL ? 1 : NU;
#pragma unroll UJ
    for (int j = 0; j < NU; ++j) {
        double v = 0.0;
        if ((uint32_t)j < n) {
            const uint32_t cj = u.coords[j];
#pragma unroll
            for (int d = 0; d < D; ++d) v = (cj == (uint32_t)d) ? g[d] : v;
        }
        gl[j] = v;
    }
}

// ---- user updates (EMCMC_USER_UPDATE; emcmc_rtc.hip compiles the source) -----
// The draws a user proposal! makes come from the engine's counter-based stream,
// indexed, so the oracle (oracle/user_prelude.h) reproduces them: em_randn(j) is
// normal j of (chain, mcmciter, update) — the index space of the random walks'
// normals, blocks j/2 — and em_rand(j) the uniform [0, 1) from words (x, y) or
// (z, w) of block 2^31 + j/2, a range no other draw of the update uses.
struct UserRng {
    ZigTabs zt;
    uint32_t key0, key1, gid, iter, p;
    uint32_t faults;
};
__device__ __forceinline__ double user_randn(UserRng &r, uint32_t j) {
    return normal_draw(r.zt, r.key0, r.key1, r.gid, r.iter, r.p, j & 0x3FFFFFFFu, r.faults);
}
__device__ __forceinline__ double user_rand(const UserRng &r, uint32_t j) {
    const u32x4 w = draw(r.key0, r.key1, r.gid, r.iter, 0x80000000u | ((j & 0x3FFFFFFFu) >> 1), r.p, 0);
    return (j & 1u) ? u01_closed0(w.z, w.w) : u01_closed0(w.x, w.y);
}
// no user update in this kernel: the branch compiles away
struct NoUserUpdate {
    static constexpr bool kEnabled = false;
    static constexpr bool kMala = false;  // MALA updates (kind 4) compiled in
    __device__ __forceinline__ static void propose(UserRng &, const double *, double *, int, const double *) {}
    __device__ __forceinline__ static double ltd(const double *, const double *, int, const double *) { return 0.0; }
};
// MALA updates on the general kernel, no user update (compiled at run time)
struct MalaOnly : NoUserUpdate {
    static constexpr bool kMala = true;
};

// ---- one update step on the update's local coordinates (shared by both kernels)
// proposal! with resampling, log_transition_density both ways, and the two
// log-priors of the MH ratio.  tl: θ_local in (pos Gaussian: left as the
// reference's in-place round trips leave it); tp: θ° (proposal history, P°);
// ta: θ° as set_chain_param! copies it on accept.
template <int NU, bool ROLL = false, class UPD = NoUserUpdate, bool XT = false>
__device__ __forceinline__ void mwg_local_step(const MwgParams &a, const ZigTabs &zt, const MwgUpdate &u, uint32_t n,
                                               uint64_t chain, uint32_t gid, uint32_t iter, uint32_t p,
                                               double (&tl)[NU], double (&tp)[NU], double (&ta)[NU], double &ltd_fwd,
                                               double &ltd_rev, double &lpp, double &lpc, uint32_t &faults) {
    constexpr int UJ = ROLL ? 1 : NU;
    const uint64_t C = a.C;
    if constexpr (UPD::kEnabled) {
        if (u.kind == kKindUser) {  // wave-uniform: the update's kind
            // proposal!(updt, …) and log_transition_density(updt, θ, θ°) of the user's
            // update (updates.jl:42-93); the prior enters the ratio as for any update
            // (run.jl:374-385), proposal! has no redraw loop unless the user writes one
            UserRng rng{zt, a.key0, a.key1, gid, iter, p, 0u};
#pragma unroll UJ
            for (int j = 0; j < NU; ++j) tp[j] = 0.0;
            UPD::propose(rng, tl, tp, (int)n, u.L);
            faults |= rng.faults;
            ltd_fwd = UPD::ltd(tl, tp, (int)n, u.L);  // log_transition_density(__PREVIOUS): (θ, θ°)
            ltd_rev = UPD::ltd(tp, tl, (int)n, u.L);  // log_transition_density(__PROPOSAL): (θ°, θ)
#pragma unroll UJ
            for (int j = 0; j < NU; ++j) ta[j] = tp[j];
            lpp = 0.0;
            lpc = 0.0;
            if (u.prior != kPriorImproper) {
                lpp = mwg_log_prior<NU, ROLL>(u, n, tp);
                lpc = mwg_log_prior<NU, ROLL>(u, n, tl);
            }
            return;
        }
    }
    double t3[NU];  // θ as log_prior(::Previous) sees it (pos GaussianRandomWalk: after the round trips)
    // ---- proposal!: draw θ°; draw again while logpdf(prior, θ°) === −Inf
    // (updates.jl:191-196).  Resample r reads counter blocks (r << 16) | j/2.
    ltd_fwd = 0.0;
    ltd_rev = 0.0;
    double ev[NU];  // UniformRandomWalk ϵ of each local coordinate
    const uint64_t pm = u.posmask;  // positivity-restricted coordinates
    auto isp = [&](int i) { return ((pm >> i) & 1ull) != 0ull; };
    bool useB = false;  // GaussianRandomWalkMix: the last rand! picked gsn_B
    const MixB mb{a.mixpool + u.lb_off, a.mixpool + u.lbi_off, C, chain};
    for (uint32_t rs = 0;; ++rs) {
        if (u.kind == 1) {  // UniformRandomWalk: θ° = θ·1 + U, or θ·e^U where pos
#pragma unroll UJ
            for (int j = 0; j < NU; j += 2) {
                if ((uint32_t)j < n) {
                    const u32x4 r = draw(a.key0, a.key1, gid, iter, (rs << 16) | ((uint32_t)j >> 1), p, 0);
                    const double e0 = u.adapt ? a.eps[((uint64_t)p * kMwgMaxD + j) * C + chain] : u.eps0[j];
                    const double U0 = (-e0) + (e0 - (-e0)) * u01_closed0(r.x, r.y);
                    tp[j] = isp(j) ? tl[j] * exp_any(U0) + copysign(0.0, U0) : tl[j] * 1.0 + U0;
                    ev[j] = e0;
                    if (j + 1 < NU && (uint32_t)(j + 1) < n) {
                        const double e1 =
                            u.adapt ? a.eps[((uint64_t)p * kMwgMaxD + j + 1) * C + chain] : u.eps0[j + 1];
                        const double U1 = (-e1) + (e1 - (-e1)) * u01_closed0(r.z, r.w);
                        tp[j + 1] = isp(j + 1) ? tl[j + 1] * exp_any(U1) + copysign(0.0, U1) : tl[j + 1] * 1.0 + U1;
                        ev[j + 1] = e1;
                    }
                }
            }
        } else {  // GaussianRandomWalk over the update's coordinates; GaussianRandomWalkMix:
                  // pick_kernel at every rand! (B iff rand() ≤ λ, random_walk.jl:225-227),
                  // block 0xFFFFFFFE, attempt = the redraw
            if constexpr (XT) {
                if (u.kind == kKindMix) {
                    const u32x4 pr = draw(a.key0, a.key1, gid, iter, 0xFFFFFFFEu, p, rs);
                    useB = u01_closed0(pr.x, pr.y) <= u.lam;
                }
            }
            if (rs > 0 && pm != 0ull) {  // the previous rand! left θ ← exp(log θ) where pos
#pragma unroll UJ
                for (int i = 0; i < NU; ++i)
                    if ((uint32_t)i < n && isp(i)) tl[i] = exp_any(log_any(tl[i]));
            }
            double z[NU];
#pragma unroll UJ
            for (int j = 0; j < NU; ++j)
                z[j] = ((uint32_t)j < n) ? normal_draw(zt, a.key0, a.key1, gid, iter, p, (rs << 17) | (uint32_t)j,
                                                       faults)
                                         : 0.0;
#pragma unroll UJ
            for (int i = 0; i < NU; ++i) {
                if ((uint32_t)i < n) {
                    double lz;
                    if (XT && useB) {
                        lz = mb.L((uint32_t)i, 0) * z[0];
#pragma unroll UJ
                        for (int j = 1; j <= i; ++j) lz = fma(mb.L((uint32_t)i, (uint32_t)j), z[j], lz);
                    } else if (u.diag) {
                        lz = u.L[i * kMwgMaxD + i] * z[i];
                    } else {
                        lz = u.L[i * kMwgMaxD] * z[0];
#pragma unroll UJ
                        for (int j = 1; j <= i; ++j) lz = fma(u.L[i * kMwgMaxD + j], z[j], lz);
                    }
                    // remove_constraints!: θ_i ← log θ_i where pos (random_walk.jl:136, 145-147);
                    // reimpose_constraints!: θ°_i ← exp(θ°_i) (θ°₁)
                    const double v = (isp(i) ? log_any(tl[i]) : tl[i]) + lz;
                    tp[i] = isp(i) ? exp_any(v) : v;
                } else {
                    tp[i] = 0.0;
                }
            }
        }
        if (u.prior == kPriorImproper) break;
        if (!(mwg_log_prior<NU, ROLL>(u, n, tp) == -__builtin_inf())) break;
        if (rs >= (u.kind == 1 ? kMaxResample : kMaxResampleGsn)) {
            faults |= kFaultPriorResample;
            break;
        }
    }
      // θ as log_prior(::Previous) sees it (pos GaussianRandomWalk: after the round trips)
    if (u.kind == 1) {
        if (pm) {  // uniform branch: the mask is the update's
#pragma unroll UJ
            for (int j = 0; j < NU; ++j) {
                if ((uint32_t)j < n) {
                    const bool pj = isp(j);
                    const double c = pj ? -log_any(2.0 * ev[j]) : 0.0;
                    const double f = pj ? c - log_any(tp[j]) : 0.0;  // logpdf(rw, θ, θ°) term
                    const double g = pj ? c - log_any(tl[j]) : 0.0;  // logpdf(rw, θ°, θ) term
                    ltd_fwd = (j == 0) ? f : ltd_fwd + f;
                    ltd_rev = (j == 0) ? g : ltd_rev + g;
                }
            }
        }
    } else if (XT && u.kind == kKindMix) {
        // logpdf(rw::GaussianRandomWalkMix, a, b) = log((1−λ)·exp(logpdf(gsn_A, a, b)) +
        // λ·exp(logpdf(gsn_B, a, b))) (random_walk.jl:229-232), each component with its
        // round trips; ltd(__PROPOSAL) = logpdf(rw, θ°, θ) first (run.jl:271-277)
        const double c0B = a.mixpool[u.lbc_off + chain];
        double xa[NU], xb[NU];
#pragma unroll UJ
        for (int i = 0; i < NU; ++i) {
            xa[i] = tp[i];                                                        // θ°₁
            xb[i] = ((uint32_t)i < n && isp(i)) ? exp_any(log_any(tl[i])) : tl[i];  // θ₁
        }
#pragma unroll
        for (int dir = 0; dir < 2; ++dir) {
            const double lpA = mwg_gsn_rw_lp<NU, ROLL>(u, nullptr, u.c0, n, xa, xb);
            const double lpB = mwg_gsn_rw_lp<NU, ROLL>(u, &mb, c0B, n, xa, xb);
            const double t = log_any((1.0 - u.lam) * exp_any(lpA) + u.lam * exp_any(lpB));
            if (dir == 0) ltd_rev = t;
            else ltd_fwd = t;
#pragma unroll UJ
            for (int i = 0; i < NU; ++i) {  // the second call is logpdf(rw, θ, θ°)
                const double tmp = xa[i];
                xa[i] = xb[i];
                xb[i] = tmp;
            }
        }
        if (pm) {  // two swaps: xa is θ°₅ (set_chain_param!), xb θ₅ (log_prior(::Previous))
#pragma unroll UJ
            for (int i = 0; i < NU; ++i) {
                ta[i] = xa[i];
                t3[i] = xb[i];
            }
        }
    } else {
        double r[NU];
        if (pm == 0ull) {
#pragma unroll UJ
            for (int i = 0; i < NU; ++i) r[i] = tp[i] - tl[i];
            ltd_fwd = u.c0 - mwg_sqmahal_u<NU, ROLL>(u, n, r) / 2.0;
#pragma unroll UJ
            for (int i = 0; i < NU; ++i) r[i] = tl[i] - tp[i];
            ltd_rev = u.c0 - mwg_sqmahal_u<NU, ROLL>(u, n, r) / 2.0;
        } else {
            // The reference's in-place round trips, step by step (random_walk.jl:136-171):
            //   rand:   θ° ← exp(log θ + Lz), θ ← exp(log θ)               (θ°₁, θ₁)
            //   logpdf(θ°₁, θ₁): logJ = −Σ_pos log θ₁; MvNormal(log θ°₁) at log θ₁;
            //           then θ°₂ = exp(log θ°₁), θ₂ = exp(log θ₁)
            //   logpdf(θ₂, θ°₂): logJ = −Σ_pos log θ°₂; MvNormal(log θ₂) at log θ°₂;
            //           then θ°₃ = exp(log θ°₂) — the value an accept stores — and
            //           θ₃ = exp(log θ₂), the θ log_prior(::Previous) reads
            double t1[NU], a1[NU], b1[NU];
            double lj = 0.0;
            bool first = true;
#pragma unroll UJ
            for (int i = 0; i < NU; ++i) {
                if ((uint32_t)i < n) {
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
            ltd_rev = (u.c0 - mwg_sqmahal_u<NU, ROLL>(u, n, r) / 2.0) + (-lj);
            lj = 0.0;
            first = true;
#pragma unroll UJ
            for (int i = 0; i < NU; ++i) {
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
                    t3[i] = isp(i) ? exp_any(a2) : l2;                  // θ₃
                } else {
                    r[i] = 0.0;
                    t3[i] = 0.0;
                }
            }
            ltd_fwd = (u.c0 - mwg_sqmahal_u<NU, ROLL>(u, n, r) / 2.0) + (-lj);
        }
    }
    const bool rt = ((u.kind == 2 || (XT && u.kind == kKindMix)) && pm != 0ull);  // after the pos round trips
    if (!rt) {
#pragma unroll UJ
        for (int j = 0; j < NU; ++j) ta[j] = tp[j];
    }
    lpp = 0.0;
    lpc = 0.0;
    if (u.prior != kPriorImproper) {
        lpp = mwg_log_prior<NU, ROLL>(u, n, rt ? ta : tp);
        lpc = mwg_log_prior<NU, ROLL>(u, n, rt ? t3 : tl);
    }
}

// ---- accept bits, accept counts, rolling acceptance, AdaptationUnifRW of update p
__device__ __forceinline__ void mwg_register_step(const MwgParams &a, const MwgUpdate &u, uint32_t n, uint64_t chain,
                                                  uint32_t iter, uint32_t p, uint32_t s, uint32_t flags, uint64_t slot,
                                                  bool acc) {
    const uint64_t C = a.C;
    const uint64_t pc = (uint64_t)p * C + chain;
    {
        const uint64_t m = __ballot(acc);
        if ((threadIdx.x & 63) == 0) store_acc_bits<1>(a.hist_acc + slot * a.row_bytes, chain, m);
    }
    a.nacc[pc] += acc ? 1u : 0u;
    // update_stats!: rolling acceptance of update p (chain_statistics.jl:51-65)
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
    // update_adaptation!: AdaptationUnifRW on its own turn (run.jl:136-178, adaptation.jl:273-329)
    if (u.adapt == 1) {
        const uint32_t pr = a.aprop[pc] + 1, ac = a.aacc[pc] + (acc ? 1u : 0u);
        if (pr >= u.k) {  // proposed counts are equal across chains: uniform branch
            const double a_r = (double)ac / (double)pr;
            const bool up = a_r > u.target;
            for (uint32_t j = 0; j < n; ++j) {
                const double delta = u.ascale[j] / sqrt(fmax(1.0, (double)iter / (double)u.k - u.aoff[j]));
                double *ep = a.eps + ((uint64_t)p * kMwgMaxD + j) * C + chain;
                double e = *ep + (up ? delta : -delta);
                e = (e < u.amax[j]) ? e : u.amax[j];
                *ep = (e > u.amin[j]) ? e : u.amin[j];
            }
            a.aprop[pc] = 0;
            a.aacc[pc] = 0;
        } else {
            a.aprop[pc] = pr;
            a.aacc[pc] = ac;
        }
    }
}

// ---- GenericChainStats mean/cov and HaarioTypeAdaptation on the general kernel
// The rank-one recurrence (chain_statistics.jl:46-49, adaptation.jl:406-414) on
// n values, elementwise with each product rounded, over the packed lower
// triangle (the full matrix is symmetric bit for bit: each element's operands
// commute): old = (N−1)/N·cov + m m', m ← m·(N/(N+1)) + x/(N+1),
// new = old + (x x')/N, cov = new − (N+1)/N·(m m').  SoA [·][C].
template <int D, bool ROLL>
__device__ __forceinline__ void mwg_rank1(double *mean, double *cov, const double (&x)[D], uint32_t n, uint64_t C,
                                          uint64_t chain, uint64_t N) {
    constexpr int UJ = ROLL ? 1 : D;
    const double ka = (double)(N - 1) / (double)N, kb = (double)N / (double)(N + 1);
    const double kc = (double)(N + 1) / (double)N, Np1 = (double)(N + 1), Nd = (double)N;
    double mo[D], mn[D];
#pragma unroll UJ
    for (int i = 0; i < D; ++i) {
        if ((uint32_t)i < n) {
            mo[i] = mean[(uint64_t)i * C + chain];
            mn[i] = mo[i] * kb + x[i] / Np1;
            mean[(uint64_t)i * C + chain] = mn[i];
        }
    }
#pragma unroll UJ
    for (int i = 0; i < D; ++i) {
        if ((uint32_t)i < n) {
#pragma unroll UJ
            for (int j = 0; j <= i; ++j) {
                double &cv = cov[(uint64_t)tri_idx((uint32_t)i, (uint32_t)j) * C + chain];
                const double old = ka * cv + mo[i] * mo[j];
                const double nw = old + (x[i] * x[j]) / Nd;
                cv = nw - kc * (mn[i] * mn[j]);
            }
        }
    }
}

// readjust!(rw::GaussianRandomWalkMix, adpt, iter) (adaptation.jl:422-426): Σ_B =
// 2.38²/n·cov, its Cholesky factor in orc_cholesky's order into the scratch,
// then L_B, 1/L_B,ii and c0_B — or, if a pivot is not positive (the reference's
// PosDefException at the next MvNormal), fault bit 4 and the old factor kept.
__device__ __forceinline__ void mwg_readjust(const MwgParams &a, const MwgUpdate &v, uint64_t chain,
                                             uint32_t &faults) {
    const uint64_t C = a.C;
    const uint32_t n = v.nc;
    const double sB = (2.38 * 2.38) / (double)n;  // 2.38^2/length(rw)
    const double *cov = a.mixpool + v.hc_off;
    double *Ls = a.mixpool + v.lbs_off;
    auto S = [&](uint32_t i, uint32_t j) { return sB * cov[(uint64_t)tri_idx(i > j ? i : j, i > j ? j : i) * C + chain]; };
    auto LS = [&](uint32_t i, uint32_t j) -> double & { return Ls[(uint64_t)tri_idx(i, j) * C + chain]; };
    for (uint32_t col = 0; col < n; ++col) {
        double diag = S(col, col);
        for (uint32_t k = 0; k < col; ++k) {
            const double l = LS(col, k);
            diag = diag - l * l;
        }
        if (!(diag > 0.0)) {
            faults |= kFaultPosdefMwg;
            return;
        }
        const double ljj = sqrt(diag);
        LS(col, col) = ljj;
        for (uint32_t row = col + 1; row < n; ++row) {
            double t = S(col, row);
            for (uint32_t k = 0; k < col; ++k) t = t - LS(row, k) * LS(col, k);
            LS(row, col) = t / ljj;
        }
    }
    double *lb = a.mixpool + v.lb_off, *lbi = a.mixpool + v.lbi_off;
    double dd = 0.0;
    for (uint32_t i = 0; i < n; ++i) {
        for (uint32_t j = 0; j <= i; ++j) lb[(uint64_t)tri_idx(i, j) * C + chain] = LS(i, j);
        const double dg = LS(i, i);
        lbi[(uint64_t)i * C + chain] = 1.0 / dg;
        dd = dd + log_pos(dg);
    }
    a.mixpool[v.lbc_off + chain] = -((double)n * kLog2Pi + (dd + dd)) / 2.0;
}

// After step s of update p: update_stats!' mean/cov of the whole θ (when kept),
// then update_adaptation! of every HaarioTypeAdaptation — register! on every
// step (register_only_on_my_turn is false both ways), the global θ at the
// update's coordinates, log-transformed where pos and transformed back in place
// (remove/reimpose_constraints! on the view), and readjust! on its own turn
// when the host marks the step (flags bit 1: M reached k).  get(d) / set(d, v):
// the chain's global θ_d.
template <int D, bool ROLL, class GET, class SET>
__device__ __forceinline__ void mwg_post_step(const MwgParams &a, uint64_t chain, uint32_t p, uint32_t s,
                                              uint32_t flags, uint32_t &faults, GET get, SET set) {
    constexpr int UJ = ROLL ? 1 : D;
    const uint64_t N = a.N0 + s;
    if (a.chain_moments) {
        double x[D];
#pragma unroll UJ
        for (int d = 0; d < D; ++d) x[d] = get((uint32_t)d);
        mwg_rank1<D, ROLL>(a.smean, a.scov, x, (uint32_t)D, a.C, chain, N);
    }
    if (a.nhaario == 0) return;
    for (uint32_t q = 0; q < a.P; ++q) {
        const MwgUpdate &v = a.updates[q];
        if (!v.hk) continue;
        const uint32_t n = v.nc;
        const uint64_t pm = v.posmask;
        double x[D];
#pragma unroll UJ
        for (int j = 0; j < D; ++j) {
            x[j] = 0.0;
            if ((uint32_t)j < n) {
                const double t = get(v.coords[j]);
                x[j] = ((pm >> j) & 1ull) ? log_any(t) : t;
            }
        }
        mwg_rank1<D, ROLL>(a.mixpool + v.hm_off, a.mixpool + v.hc_off, x, n, a.C, chain, N);
        if (pm) {
#pragma unroll UJ
            for (int j = 0; j < D; ++j)
                if ((uint32_t)j < n && ((pm >> j) & 1ull)) set(v.coords[j], exp_any(x[j]));
        }
        if (q == p && (flags & 2u)) mwg_readjust(a, v, chain, faults);
    }
}

// One lane per chain; θ and P°.θ in registers, coordinates moved between global
// and update-local order by selects over the compile-time D (D ≤ 16).
// XT: GaussianRandomWalkMix updates, HaarioTypeAdaptation and GenericChainStats
// mean/cov compiled in (the ahead-of-time instantiations leave them out; the
// library compiles XT kernels at run time when a schedule needs them).
template <int D, bool FULL, int LLMODE, class TGT = GsnTarget, class UPD = NoUserUpdate, bool XT = false>
__global__ void __launch_bounds__(256) mwg_gsn_kernel(const MwgParams a) {
    static_assert(D <= 16, "register-state MWG kernel: D ≤ 16 (mwg_wide_kernel below for larger D)");
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
        // ---- update_workspaces!: θ_local ← θ[coords] (uniform coordinate indices)
        double tl[D], tp[D], ta[D];
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
        double ltd_fwd, ltd_rev, lpp, lpc;
        bool mala = false;
        if constexpr (UPD::kMala) mala = (u.kind == kKindMala);  // wave-uniform
        if constexpr (UPD::kMala) {
            if (mala) {  // compute_gradients_and_momenta!(__PREVIOUS) at P°.θ with coords ← θ
                double x[D], g[D], gl[D];
                if (mala_carry(a, n, (uint32_t)D) && s > 0) {  // ∇ℓ(θ) from the previous step
#pragma unroll
                    for (int d = 0; d < D; ++d) g[d] = a.gcache[state_pos(d, chain, C, D)];
                } else {
#pragma unroll
                    for (int d = 0; d < D; ++d) x[d] = mp[d];
#pragma unroll
                    for (int j = 0; j < D; ++j) {
                        if ((uint32_t)j < n) {
                            const uint32_t cj = u.coords[j];
#pragma unroll
                            for (int d = 0; d < D; ++d) x[d] = (cj == (uint32_t)d) ? tl[j] : x[d];
                        }
                    }
                    TGT::template grad<D, LLMODE>(a, x, g);
                    if (mala_carry(a, n, (uint32_t)D))
#pragma unroll
                        for (int d = 0; d < D; ++d) a.gcache[state_pos(d, chain, C, D)] = g[d];
                }
                mwg_gather<D, D, false>(u, n, g, gl);
                mwg_mala_forward<D, false>(a, zt, u, n, gid, iter, p, tl, gl, tp, ltd_fwd, faults);
#pragma unroll
                for (int j = 0; j < D; ++j) ta[j] = tp[j];
                ltd_rev = 0.0;
                lpp = 0.0;
                lpc = 0.0;
                if (u.prior != kPriorImproper) {
                    lpp = mwg_log_prior<D, false>(u, n, tp);
                    lpc = mwg_log_prior<D, false>(u, n, tl);
                }
            }
        }
        // XT kernels keep the update-local loops rolled: the mixture densities would
        // otherwise unroll four triangular solves per direction (minutes of hiprtc time)
        if (!mala)
            mwg_local_step<D, XT, UPD, XT>(a, zt, u, n, chain, gid, iter, p, tl, tp, ta, ltd_fwd, ltd_rev, lpp, lpc,
                                           faults);
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
        const double llp = TGT::template loglik<D, LLMODE>(a, mp);
        double gprop[UPD::kMala ? D : 1];  // ∇ℓ at the proposal: the next step's ∇ℓ(θ) if accepted
        if constexpr (UPD::kMala) {
            if (mala) {  // compute_gradients_and_momenta!(__PROPOSAL) at P°.θ
                double gp[D];
                TGT::template grad<D, LLMODE>(a, mp, gprop);
                mwg_gather<D, D, false>(u, n, gprop, gp);
                ltd_rev = mwg_mala_reverse<D, false>(u, n, tl, tp, gp);
            }
        }
        if (!(llp - llp == 0.0)) faults |= 1u;
        a.ll_prop[(uint64_t)p * C + chain] = llp;
        // ---- accept_reject! (run.jl:268-281)
        const double llr = ((((llp - ll) + ltd_rev) - ltd_fwd) + lpp) - lpc;
        const double E = exp_draw(zt, a.key0, a.key1, gid, iter, p, faults);
        const bool acc = E > -llr;
        if constexpr (FULL) {
#pragma unroll
            for (int d = 0; d < D; ++d)
                __builtin_nontemporal_store(prop[d], a.hist_prop + slot * D * C + state_pos(d, chain, C, D));
        }
        if (acc) {  // set_chain_param!: θ[coords] ← θ° (run.jl:312-318)
#pragma unroll
            for (int d = 0; d < D; ++d) th[d] = nst[d];
            ll = llp;
            if constexpr (UPD::kMala)
                if (mala && mala_carry(a, n, (uint32_t)D))
#pragma unroll
                    for (int d = 0; d < D; ++d) a.gcache[state_pos(d, chain, C, D)] = gprop[d];
        }
        if constexpr (FULL) {
#pragma unroll
            for (int d = 0; d < D; ++d)
                __builtin_nontemporal_store(th[d], a.hist_theta + slot * D * C + state_pos(d, chain, C, D));
            __builtin_nontemporal_store(ll, a.hist_ll + slot * C + chain);
        }
        mwg_register_step(a, u, n, chain, iter, p, s, flags, slot, acc);
        if (XT && (a.chain_moments | a.nhaario))
            mwg_post_step<D, true>(
                a, chain, p, s, flags, faults,
                [&](uint32_t c) {
                    double v = 0.0;
#pragma unroll
                    for (int d = 0; d < D; ++d) v = (c == (uint32_t)d) ? th[d] : v;
                    return v;
                },
                [&](uint32_t c, double v) {
#pragma unroll
                    for (int d = 0; d < D; ++d) th[d] = (c == (uint32_t)d) ? v : th[d];
                });
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

// One lane per chain for larger D: θ and P°.θ stay in HBM (SoA state_pos layout,
// L2/MALL-resident) and are read and written at the update's coordinates with
// wave-uniform indices, so no select network over D is needed; only the
// update's NU-sized local vectors and, for the likelihood, P°.θ live in
// registers.  The arithmetic is mwg_gsn_kernel's.
template <int D, int NU, bool FULL, int LLMODE, class TGT = GsnTarget, class UPD = NoUserUpdate, bool XT = false>
__global__ void __launch_bounds__(256) mwg_wide_kernel(const MwgParams a) {
    static_assert(NU <= D && D <= kMwgMaxD, "NU ≤ D ≤ 64");
    // loops over the update's NU coordinates and over the target's D stay rolled
    // only for the largest updates: unrolled, the local vectors live in registers
    constexpr bool RU = NU > 16 || XT;  // XT: rolled, as in mwg_gsn_kernel
    constexpr bool RT = NU > 16;
    const ZigTabs zt = stage_lds(nullptr, a.zig, nullptr, 0, nullptr, 0);
    const uint64_t chain = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (chain >= a.C) return;
    const uint64_t C = a.C;
    const uint32_t gid = a.chain0 + (uint32_t)chain;
    double ll = a.ll[chain];
    uint32_t faults = a.faults[chain];

    for (uint32_t s = 0; s < a.nsteps; ++s) {
        const uint32_t iter = a.steps[4 * s], pidx = a.steps[4 * s + 1], flags = a.steps[4 * s + 2];
        const uint32_t p = pidx - 1;
        const MwgUpdate &u = a.updates[p];
        const uint32_t n = u.nc;
        const uint64_t slot = (uint64_t)(iter - 1) * a.P + p;
        // ---- update_workspaces!: θ_local ← θ[coords]
        double tl[NU], tp[NU], ta[NU];
        for (int j = 0; j < NU; ++j) tl[j] = ((uint32_t)j < n) ? a.theta[state_pos(u.coords[j], chain, C, D)] : 0.0;
        double ltd_fwd, ltd_rev, lpp, lpc;
        bool mala = false;
        if constexpr (UPD::kMala) mala = (u.kind == kKindMala);  // wave-uniform
        if constexpr (UPD::kMala) {
            if (mala) {  // compute_gradients_and_momenta!(__PREVIOUS) at P°.θ with coords ← θ
                for (int j = 0; j < NU; ++j)
                    if ((uint32_t)j < n) a.mu_p[state_pos(u.coords[j], chain, C, D)] = tl[j];
                double x[D], g[D], gl[NU];
                if (mala_carry(a, n, (uint32_t)D) && s > 0) {  // ∇ℓ(θ) from the previous step
#pragma unroll
                    for (int d = 0; d < D; ++d) g[d] = a.gcache[state_pos(d, chain, C, D)];
                } else {
#pragma unroll
                    for (int d = 0; d < D; ++d) x[d] = a.mu_p[state_pos(d, chain, C, D)];
                    TGT::template grad<D, LLMODE, RT>(a, x, g);
                    if (mala_carry(a, n, (uint32_t)D))
#pragma unroll
                        for (int d = 0; d < D; ++d) a.gcache[state_pos(d, chain, C, D)] = g[d];
                }
                mwg_gather<D, NU, RU>(u, n, g, gl);
                mwg_mala_forward<NU, RU>(a, zt, u, n, gid, iter, p, tl, gl, tp, ltd_fwd, faults);
                for (int j = 0; j < NU; ++j) ta[j] = tp[j];
                ltd_rev = 0.0;
                lpp = 0.0;
                lpc = 0.0;
                if (u.prior != kPriorImproper) {
                    lpp = mwg_log_prior<NU, RU>(u, n, tp);
                    lpc = mwg_log_prior<NU, RU>(u, n, tl);
                }
            }
        }
        if (!mala)
            mwg_local_step<NU, RU, UPD, XT>(a, zt, u, n, chain, gid, iter, p, tl, tp, ta, ltd_fwd, ltd_rev, lpp, lpc,
                                            faults);
        // ---- set_proposal!: P°.θ[coords] ← θ°, then all of P°.θ for the likelihood
        for (int j = 0; j < NU; ++j)
            if ((uint32_t)j < n) a.mu_p[state_pos(u.coords[j], chain, C, D)] = tp[j];
        double mp[D];
#pragma unroll
        for (int d = 0; d < D; ++d) mp[d] = a.mu_p[state_pos(d, chain, C, D)];
        // ---- compute_ll!
        const double llp = TGT::template loglik<D, LLMODE, RT>(a, mp);
        double gprop[UPD::kMala ? D : 1];  // ∇ℓ at the proposal: the next step's ∇ℓ(θ) if accepted
        if constexpr (UPD::kMala) {
            if (mala) {  // compute_gradients_and_momenta!(__PROPOSAL) at P°.θ
                double gp[NU];
                TGT::template grad<D, LLMODE, RT>(a, mp, gprop);
                mwg_gather<D, NU, RU>(u, n, gprop, gp);
                ltd_rev = mwg_mala_reverse<NU, RU>(u, n, tl, tp, gp);
            }
        }
        if (!(llp - llp == 0.0)) faults |= 1u;
        a.ll_prop[(uint64_t)p * C + chain] = llp;
        // ---- accept_reject! (run.jl:268-281)
        const double llr = ((((llp - ll) + ltd_rev) - ltd_fwd) + lpp) - lpc;
        const double E = exp_draw(zt, a.key0, a.key1, gid, iter, p, faults);
        const bool acc = E > -llr;
        if constexpr (FULL) {  // proposal history: θ with coords ← θ° (run.jl:237-239)
            double *hp = a.hist_prop + slot * D * C;
#pragma unroll
            for (int d = 0; d < D; ++d) hp[state_pos(d, chain, C, D)] = a.theta[state_pos(d, chain, C, D)];
            for (int j = 0; j < NU; ++j)
                if ((uint32_t)j < n) hp[state_pos(u.coords[j], chain, C, D)] = tp[j];
        }
        if (acc) {  // set_chain_param!: θ[coords] ← θ° (run.jl:312-318)
            for (int j = 0; j < NU; ++j)
                if ((uint32_t)j < n) a.theta[state_pos(u.coords[j], chain, C, D)] = ta[j];
            ll = llp;
            if constexpr (UPD::kMala)
                if (mala && mala_carry(a, n, (uint32_t)D))
#pragma unroll
                    for (int d = 0; d < D; ++d) a.gcache[state_pos(d, chain, C, D)] = gprop[d];
        }
        if constexpr (FULL) {
            double *ht = a.hist_theta + slot * D * C;
#pragma unroll
            for (int d = 0; d < D; ++d)
                __builtin_nontemporal_store(a.theta[state_pos(d, chain, C, D)], ht + state_pos(d, chain, C, D));
            __builtin_nontemporal_store(ll, a.hist_ll + slot * C + chain);
        }
        mwg_register_step(a, u, n, chain, iter, p, s, flags, slot, acc);
        if (XT && (a.chain_moments | a.nhaario))
            mwg_post_step<D, true>(
                a, chain, p, s, flags, faults, [&](uint32_t c) { return a.theta[state_pos(c, chain, C, D)]; },
                [&](uint32_t c, double v) { a.theta[state_pos(c, chain, C, D)] = v; });
    }
    a.ll[chain] = ll;
    a.faults[chain] = faults;
    if (faults) *a.fault_flag = 1u;
}

}  // namespace emcmc
