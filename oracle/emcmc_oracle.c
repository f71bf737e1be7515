/*
 * emcmc_oracle.c — CPU oracle for the many-chain MH hot path.
 *
 * TEST INFRASTRUCTURE ONLY.  Only tests/, __graft_entry__.smoke() and the
 * cpu_baseline leg of bench.py may load liboracle.so.  The product
 * (extensiblemcmc.jl_amd/) never links or calls it.
 *
 * PARITY STATUS: the reference (Julia, /root/reference) cannot run in this
 * image (no julia; Distributions.jl unvendored and unpinned, Project.toml:9,
 * 14-15), and its own tests pin no number on the MH arithmetic (SURVEY §4,
 * §8c).  The MH arithmetic restated below is therefore "parity unpinned"
 * against the reference itself; it is pinned by (1) the Random123 Philox
 * known-answer vectors, (2) the reference's schedule and AdaptationUnifRW KATs
 * (test/runtests.jl:5-85, restated in the host layer and checked in tests/),
 * (3) an independent numpy restatement of the literal reference formulas
 * (oracle/literal.py: per-observation MvNormal logpdf via LAPACK Cholesky)
 * within fp64 tolerance, and (4) the analytic posterior N(x̄, Σ/n).
 *
 * What is restated (reference files under /root/reference/src):
 *   __run! loop, one update, P = 1 ............................ run.jl:64-83
 *   update_workspaces!: θ copy, ll carry (−Inf at step 1) ....... run.jl:101-112
 *   proposal!/rand!(GaussianRandomWalk): θ° = θ + L z ........... updates.jl:191-196,
 *                                                                 random_walk.jl:145-159
 *   set_proposal!: proposal history = θ with coords ← θ° ........ run.jl:221-240
 *   compute_ll!: ll° = Σ_k logpdf(MvNormal(θ°, Σ_t), x_k) ....... run.jl:251-260,
 *                                                                 gsn_target.jl:15-29
 *   accept_reject!: llr left-assoc, E ~ Exp(1), accept E > −llr . run.jl:268-281
 *   log_transition_density (both directions) ................... run.jl:344-367,
 *                                                                 random_walk.jl:161-171
 *   log_prior (ImproperPrior → 0.0) ............................ run.jl:374-385,
 *                                                                 priors.jl:18-19
 *   register_accept_reject_results!, set_chain_param! .......... run.jl:299-335
 *   update_stats! rolling acceptance (window W, N from 1) ....... chain_statistics.jl:41-65
 * MvNormal arithmetic (Distributions.jl, third-party, version unpinned by the
 * reference — Project.toml has no [compat] entry for it):
 *   logpdf = mvnormal_c0 − sqmahal/2, mvnormal_c0 = −(D·log2π + logdet Σ)/2,
 *   sqmahal = ‖L⁻¹(x − μ)‖², rand = μ + L z, L = cholesky(Symmetric(Σ)).L,
 *   logdet(::Cholesky) = dd + dd with dd = Σ log L_ii (LinearAlgebra).
 * Evaluation order of every sum is the engine's canonical order (DESIGN.md
 * §Numerics): blocked-8 pairwise for length-D sums, sequential over
 * observations.
 */
#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#include "oracle_math.h"

#define ORC_EXPORT __attribute__((visibility("default")))

static orc_zig_tables g_zig;
static int g_zig_ready = 0;
static const orc_zig_tables *zig(void) {
    if (!g_zig_ready) { /* first call happens outside any parallel region */
        orc_zig_build(&g_zig);
        g_zig_ready = 1;
    }
    return &g_zig;
}

/* ---- canonical helpers --------------------------------------------------- */

/* Cholesky of the upper-stored (column-major) symmetric Σ: row-major lower L.
 * Column-by-column, sums left to right, no fused multiply-add. */
ORC_EXPORT int orc_cholesky(const double *S, int D, double *L) {
    memset(L, 0, sizeof(double) * (size_t)D * D);
    for (int col = 0; col < D; ++col) {
        double diag = S[col + (size_t)col * D];
        for (int k = 0; k < col; ++k) {
            double l = L[(size_t)col * D + k];
            diag = diag - l * l;
        }
        if (!(diag > 0.0)) return -1; /* PosDefException in the reference */
        double ljj = sqrt(diag);
        L[(size_t)col * D + col] = ljj;
        for (int row = col + 1; row < D; ++row) {
            double t = S[col + (size_t)row * D];
            for (int k = 0; k < col; ++k) t = t - L[(size_t)row * D + k] * L[(size_t)col * D + k];
            L[(size_t)row * D + col] = t / ljj;
        }
    }
    return 0;
}

/* Length-D sum in the canonical order. */
ORC_EXPORT double orc_canon_sum(const double *v, int D) {
    int blk = (D % 8 == 0 && D >= 16) ? 8 : D;
    int nb = D / blk;
    double part[64];
    for (int b = 0; b < nb; ++b) {
        double s = v[b * blk];
        for (int i = 1; i < blk; ++i) s = s + v[b * blk + i];
        part[b] = s;
    }
    int n = nb;
    while (n > 1) {
        for (int i = 0; i < n / 2; ++i) part[i] = part[2 * i] + part[2 * i + 1];
        if (n & 1) part[n / 2] = part[n - 1];
        n = (n + 1) / 2;
    }
    return part[0];
}

/* Σ y_i² in the canonical order: same blocks and tree as orc_canon_sum, each
 * block accumulated as s = y0·y0, s = fma(y_i, y_i, s). */
ORC_EXPORT double orc_canon_sumsq(const double *y, int D) {
    int blk = (D % 8 == 0 && D >= 16) ? 8 : D;
    int nb = D / blk;
    double part[64];
    for (int b = 0; b < nb; ++b) {
        const double *yb = y + b * blk;
        double s = yb[0] * yb[0];
        for (int i = 1; i < blk; ++i) s = fma(yb[i], yb[i], s);
        part[b] = s;
    }
    int n = nb;
    while (n > 1) {
        for (int i = 0; i < n / 2; ++i) part[i] = part[2 * i] + part[2 * i + 1];
        if (n & 1) part[n / 2] = part[n - 1];
        n = (n + 1) / 2;
    }
    return part[0];
}

/* ‖L⁻¹ r‖² by forward substitution (PDMats sqmahal via chol.L \ r).  A unit
 * diagonal (Σ = I ⇒ L = I) makes y = r exactly, with or without the multiply. */
static double sqmahal(const double *L, const double *invdiag, const double *r, int D, int diag) {
    double y[64];
    for (int i = 0; i < D; ++i) {
        double acc = r[i];
        if (!diag)
            for (int j = 0; j < i; ++j) acc = fma(-L[(size_t)i * D + j], y[j], acc);
        y[i] = acc * invdiag[i];
    }
    return orc_canon_sumsq(y, D);
}

static double logdet_chol(const double *L, int D) {
    double dd = 0.0;
    for (int i = 0; i < D; ++i) dd = dd + orc_log(L[(size_t)i * D + i]);
    return dd + dd;
}

static double mvnormal_c0(int D, double logdet) { return -((double)D * ORC_LOG2PI + logdet) / 2.0; }

static int is_diag_upper(const double *S, int D) {
    for (int i = 0; i < D; ++i)
        for (int j = i + 1; j < D; ++j)
            if (S[i + (size_t)j * D] != 0.0) return 0;
    return 1;
}

/* ---- problem constants ----------------------------------------------------- */

typedef struct {
    int D, diag, ll_mode;
    /* faithful (ll_mode bit 9, CPU baseline only): every MvNormal construction
     * factorises its Σ again, as the reference does (random_walk.jl:147,167 for
     * rand and both logpdfs; gsn_target.jl:20 for set_parameters! of P° and of P),
     * and every logpdf recomputes its log-determinant.  Same bits as the
     * factor-once path (the same deterministic Cholesky of the same Σ). */
    int faithful;
    const double *rw_sigma, *t_sigma;
    uint64_t nobs;
    const double *obs;
    double Lrw[64 * 64], iLrw[64], Lt[64 * 64], iLt[64], xbar[64];
    double rw_c0, t_c0, S_c;
} orc_gsn;

/* constants: out[0]=rw_c0, out[1]=t_c0, out[2]=S_c, out[3..3+D)=x̄ */
static int gsn_prepare(orc_gsn *g, int D, const double *rw_sigma, const double *t_sigma, uint64_t nobs,
                       const double *obs, int ll_mode) {
    if (D < 1 || D > 64) return -2;
    g->D = D;
    g->nobs = nobs;
    g->obs = obs;
    g->ll_mode = ll_mode & 0xFF;
    g->faithful = (ll_mode & 0x200) != 0;
    g->rw_sigma = rw_sigma;
    g->t_sigma = t_sigma;
    if (orc_cholesky(rw_sigma, D, g->Lrw)) return -1;
    if (orc_cholesky(t_sigma, D, g->Lt)) return -1;
    /* ll_mode bit 8 forces the dense (general Cholesky) formulas even for a
     * diagonal Σ — used by tests to show both formulas give the same bits. */
    g->diag = !(ll_mode & 0x300) && is_diag_upper(rw_sigma, D) && is_diag_upper(t_sigma, D);
    for (int i = 0; i < D; ++i) {
        g->iLrw[i] = 1.0 / g->Lrw[(size_t)i * D + i];
        g->iLt[i] = 1.0 / g->Lt[(size_t)i * D + i];
    }
    g->rw_c0 = mvnormal_c0(D, logdet_chol(g->Lrw, D));
    g->t_c0 = mvnormal_c0(D, logdet_chol(g->Lt, D));
    for (int i = 0; i < D; ++i) {
        double s = 0.0;
        for (uint64_t k = 0; k < nobs; ++k) s = s + obs[k * D + i];
        g->xbar[i] = s / (double)nobs;
    }
    double Sc = 0.0;
    int dense_t = !is_diag_upper(t_sigma, D);
    for (uint64_t k = 0; k < nobs; ++k) {
        double r[64];
        for (int i = 0; i < D; ++i) r[i] = obs[k * D + i] - g->xbar[i];
        Sc = Sc + sqmahal(g->Lt, g->iLt, r, D, !dense_t);
    }
    g->S_c = Sc;
    return 0;
}

ORC_EXPORT int orc_gsn_constants(int D, const double *rw_sigma, const double *t_sigma, uint64_t nobs,
                                 const double *obs, double *out, double *Lrw_out, double *Lt_out) {
    orc_gsn *g = (orc_gsn *)malloc(sizeof(orc_gsn));
    int rc = gsn_prepare(g, D, rw_sigma, t_sigma, nobs, obs, 0);
    if (rc == 0) {
        out[0] = g->rw_c0;
        out[1] = g->t_c0;
        out[2] = g->S_c;
        for (int i = 0; i < D; ++i) out[3 + i] = g->xbar[i];
        if (Lrw_out) memcpy(Lrw_out, g->Lrw, sizeof(double) * (size_t)D * D);
        if (Lt_out) memcpy(Lt_out, g->Lt, sizeof(double) * (size_t)D * D);
    }
    free(g);
    return rc;
}

/* ---- one chain, `nsteps` steps of the single joint update ----------------- */

typedef struct {
    double *theta;  /* [D] in/out */
    double *ll;     /* in/out */
    double *ra;     /* in/out */
    uint64_t *ring; /* [2] in/out */
    uint32_t *nacc; /* in/out */
    uint32_t *faults;
} orc_chain;

/* A fresh MvNormal(·, Σ): Cholesky factor, 1/L_ii and c0 (PDMat construction +
 * mvnormal_c0's logdetcov at every logpdf call). */
typedef struct {
    double L[64 * 64], iL[64], c0;
} orc_mvn;
static void mvn_build(orc_mvn *m, const double *S, int D) {
    (void)orc_cholesky(S, D, m->L);
    for (int i = 0; i < D; ++i) m->iL[i] = 1.0 / m->L[(size_t)i * D + i];
    m->c0 = mvnormal_c0(D, logdet_chol(m->L, D));
}

/* The reference's per-step work without the factor-once shortcut (CPU baseline
 * "faithful" variant; iterations consecutive from iter0; dense formulas). */
static void run_chain_faithful(const orc_gsn *g, orc_chain st, uint32_t key0, uint32_t key1, uint32_t chain_id,
                               uint32_t iter0, uint32_t nsteps, uint64_t N0, uint32_t W, uint64_t C, uint64_t c,
                               double *hist_theta, double *hist_prop, double *hist_ll, uint8_t *hist_acc) {
    const int D = g->D;
    const orc_zig_tables *zt = zig();
    orc_mvn *m = (orc_mvn *)malloc(sizeof(orc_mvn));
    double th[64], thp[64], z[64], r[64];
    memcpy(th, st.theta, sizeof(double) * D);
    double ll = *st.ll, ra = *st.ra;
    uint64_t ring0 = st.ring[0], ring1 = st.ring[1];
    uint32_t nacc = *st.nacc, faults = *st.faults;
    volatile double sink = 0.0;
    for (uint32_t s = 0; s < nsteps; ++s) {
        const uint32_t iter = iter0 + s;
        mvn_build(m, g->rw_sigma, D); /* rand(MvNormal(θ, Σ)) */
        for (int j = 0; j < D; ++j) z[j] = orc_normal(zt, key0, key1, chain_id, iter, 0, (uint32_t)j, &faults);
        for (int i = 0; i < D; ++i) {
            double lz = m->L[(size_t)i * D] * z[0];
            for (int j = 1; j <= i; ++j) lz = fma(m->L[(size_t)i * D + j], z[j], lz);
            thp[i] = th[i] + lz;
        }
        mvn_build(m, g->t_sigma, D); /* set_parameters!(P°, …): MvNormal(μ, Symmetric(triu(Σ))) */
        double llp = 0.0;
        for (uint64_t k = 0; k < g->nobs; ++k) {
            for (int i = 0; i < D; ++i) r[i] = g->obs[k * D + i] - thp[i];
            const double c0 = mvnormal_c0(D, logdet_chol(m->L, D));
            llp = llp + (c0 - sqmahal(m->L, m->iL, r, D, 0) / 2.0);
        }
        if (!isfinite(llp)) faults |= 1u;
        mvn_build(m, g->rw_sigma, D); /* logpdf(MvNormal(θ°, Σ), θ) */
        for (int i = 0; i < D; ++i) r[i] = th[i] - thp[i];
        const double ltd_rev = m->c0 - sqmahal(m->L, m->iL, r, D, 0) / 2.0;
        mvn_build(m, g->rw_sigma, D); /* logpdf(MvNormal(θ, Σ), θ°) */
        for (int i = 0; i < D; ++i) r[i] = thp[i] - th[i];
        const double ltd_fwd = m->c0 - sqmahal(m->L, m->iL, r, D, 0) / 2.0;
        const double llr = ((((llp - ll) + ltd_rev) - ltd_fwd) + 0.0) - 0.0;
        const double E = orc_exponential(zt, key0, key1, chain_id, iter, 0, &faults);
        const int acc = E > -llr;
        if (hist_prop) memcpy(hist_prop + ((uint64_t)s * C + c) * D, thp, sizeof(double) * D);
        if (acc) {
            memcpy(th, thp, sizeof(double) * D);
            ll = llp;
            nacc += 1;
        }
        mvn_build(m, g->t_sigma, D); /* set_parameters!(::Previous): P rebuilt (dead work, kept) */
        sink = sink + m->L[(size_t)D * D - 1];
        if (hist_theta) memcpy(hist_theta + ((uint64_t)s * C + c) * D, th, sizeof(double) * D);
        if (hist_ll) hist_ll[(uint64_t)s * C + c] = ll;
        if (hist_acc) hist_acc[(uint64_t)s * C + c] = (uint8_t)acc;
        const uint64_t N = N0 + s;
        int outside = 0;
        if (iter > W) {
            uint32_t j = (iter - W) & 127u;
            outside = (int)((((j & 64u) ? ring1 : ring0) >> (j & 63u)) & 1u);
        }
        const uint64_t mn = N < (uint64_t)W ? N : (uint64_t)W;
        ra = (ra * (double)W + (double)(acc - outside)) / (double)mn;
        {
            uint32_t j = iter & 127u;
            uint64_t bit = 1ull << (j & 63u);
            if (j & 64u) ring1 = acc ? (ring1 | bit) : (ring1 & ~bit);
            else ring0 = acc ? (ring0 | bit) : (ring0 & ~bit);
        }
    }
    memcpy(st.theta, th, sizeof(double) * D);
    *st.ll = ll;
    *st.ra = ra;
    st.ring[0] = ring0;
    st.ring[1] = ring1;
    *st.nacc = nacc;
    *st.faults = faults;
    free(m);
}

static void run_chain(const orc_gsn *g, orc_chain st, uint32_t key0, uint32_t key1, uint32_t chain_id,
                      const uint32_t *iters, uint32_t iter0, uint32_t nsteps, uint64_t N0, uint32_t W,
                      uint64_t C, uint64_t c, double *hist_theta, double *hist_prop, double *hist_ll,
                      uint8_t *hist_acc) {
    const int D = g->D;
    const orc_zig_tables *zt = zig();
    double th[64], thp[64], z[64];
    memcpy(th, st.theta, sizeof(double) * D);
    double ll = *st.ll, ra = *st.ra;
    uint64_t ring0 = st.ring[0], ring1 = st.ring[1];
    uint32_t nacc = *st.nacc, faults = *st.faults;

    if (g->faithful) {
        run_chain_faithful(g, st, key0, key1, chain_id, iter0, nsteps, N0, W, C, c, hist_theta, hist_prop, hist_ll,
                           hist_acc);
        return;
    }
    for (uint32_t s = 0; s < nsteps; ++s) {
        const uint32_t iter = iters ? iters[s] : iter0 + s;
        /* proposal!  θ° = θ + L z  (random_walk.jl:147: rand(MvNormal(θ, Σ))) */
        for (int j = 0; j < D; ++j) z[j] = orc_normal(zt, key0, key1, chain_id, iter, 0, (uint32_t)j, &faults);
        for (int i = 0; i < D; ++i) {
            double lz;
            if (g->diag) {
                lz = g->Lrw[(size_t)i * D + i] * z[i];
            } else {
                lz = g->Lrw[(size_t)i * D] * z[0];
                for (int j = 1; j <= i; ++j) lz = fma(g->Lrw[(size_t)i * D + j], z[j], lz);
            }
            thp[i] = th[i] + lz;
        }
        /* log_transition_density(θ→θ°) and (θ°→θ): MvNormal logpdf of ±(θ°−θ);
         * the two sqmahal values are bitwise equal (random_walk.jl:161-171). */
        double r[64];
        for (int i = 0; i < D; ++i) r[i] = thp[i] - th[i];
        const double ltd_fwd = g->rw_c0 - sqmahal(g->Lrw, g->iLrw, r, D, g->diag) / 2.0;
        for (int i = 0; i < D; ++i) r[i] = th[i] - thp[i];
        const double ltd_rev = g->rw_c0 - sqmahal(g->Lrw, g->iLrw, r, D, g->diag) / 2.0;
        /* compute_ll!  (gsn_target.jl:23-29: ll = 0.0; for obs: ll += logpdf) */
        double llp;
        if (g->ll_mode == 0) {
            llp = 0.0;
            for (uint64_t k = 0; k < g->nobs; ++k) {
                for (int i = 0; i < D; ++i) r[i] = g->obs[k * D + i] - thp[i];
                llp = llp + (g->t_c0 - sqmahal(g->Lt, g->iLt, r, D, g->diag) / 2.0);
            }
        } else {
            for (int i = 0; i < D; ++i) r[i] = g->xbar[i] - thp[i];
            const double qv = sqmahal(g->Lt, g->iLt, r, D, g->diag);
            llp = (double)g->nobs * g->t_c0 - (g->S_c + (double)g->nobs * qv) * 0.5;
        }
        if (!isfinite(llp)) faults |= 1u;
        /* accept_reject!  (run.jl:271-278) — ImproperPrior: log_prior = 0.0 */
        const double lp_prop = 0.0, lp_prev = 0.0;
        const double llr = ((((llp - ll) + ltd_rev) - ltd_fwd) + lp_prop) - lp_prev;
        const double E = orc_exponential(zt, key0, key1, chain_id, iter, 0, &faults);
        const int acc = E > -llr;
        const uint64_t slot = (uint64_t)(s);
        if (hist_prop) memcpy(hist_prop + (slot * C + c) * D, thp, sizeof(double) * D);
        if (acc) {
            memcpy(th, thp, sizeof(double) * D);
            ll = llp;
            nacc += 1;
        }
        if (hist_theta) memcpy(hist_theta + (slot * C + c) * D, th, sizeof(double) * D);
        if (hist_ll) hist_ll[slot * C + c] = ll;
        if (hist_acc) hist_acc[slot * C + c] = (uint8_t)acc;
        /* update_stats! rolling acceptance (chain_statistics.jl:53-65) */
        const uint64_t N = N0 + s;
        int outside = 0;
        if (iter > W) {
            uint32_t j = (iter - W) & 127u;
            outside = (int)((((j & 64u) ? ring1 : ring0) >> (j & 63u)) & 1u);
        }
        const uint64_t mn = N < (uint64_t)W ? N : (uint64_t)W;
        /* rolling_ar[iter−1] of an iteration that did not run reads 0.0 */
        if (s > 0 && iter != (iters ? iters[s - 1] : iter0 + s - 1) + 1) ra = 0.0;
        ra = (ra * (double)W + (double)(acc - outside)) / (double)mn;
        {
            uint32_t j = iter & 127u;
            uint64_t bit = 1ull << (j & 63u);
            if (j & 64u) ring1 = acc ? (ring1 | bit) : (ring1 & ~bit);
            else ring0 = acc ? (ring0 | bit) : (ring0 & ~bit);
        }
    }
    memcpy(st.theta, th, sizeof(double) * D);
    *st.ll = ll;
    *st.ra = ra;
    st.ring[0] = ring0;
    st.ring[1] = ring1;
    *st.nacc = nacc;
    *st.faults = faults;
}

/*
 * Run `nsteps` iterations (P = 1) for chains [0, C) of a shard whose first
 * global chain id is chain0.  State arrays are in/out.  History outputs are
 * optional (NULL) and indexed by step s in [0, nsteps): hist_theta/hist_prop
 * [nsteps][C][D], hist_ll [nsteps][C], hist_acc [nsteps][C] (0/1 bytes).
 * Returns 0, or <0 on invalid input.
 */
ORC_EXPORT int orc_run_gsn(int D, uint64_t C, uint32_t chain0, uint64_t seed, const double *rw_sigma,
                           const double *t_sigma, uint64_t nobs, const double *obs, int ll_mode, uint32_t W,
                           const uint32_t *iters, uint32_t iter0, uint32_t nsteps, uint64_t N0, double *theta,
                           double *ll, double *ra, uint64_t *ring, uint32_t *nacc, uint32_t *faults,
                           double *hist_theta, double *hist_prop, double *hist_ll, uint8_t *hist_acc,
                           int nthreads) {
    orc_gsn *g = (orc_gsn *)malloc(sizeof(orc_gsn));
    if (!g) return -3;
    (void)zig();
    int rc = gsn_prepare(g, D, rw_sigma, t_sigma, nobs, obs, ll_mode);
    if (rc) {
        free(g);
        return rc;
    }
    const uint32_t k0 = (uint32_t)seed, k1 = (uint32_t)(seed >> 32);
#ifdef _OPENMP
#pragma omp parallel for schedule(static) num_threads(nthreads > 0 ? nthreads : 1)
#endif
    for (int64_t c = 0; c < (int64_t)C; ++c) {
        orc_chain st = {theta + (uint64_t)c * D, ll + c, ra + c, ring + 2 * (uint64_t)c, nacc + c, faults + c};
        run_chain(g, st, k0, k1, chain0 + (uint32_t)c, iters, iter0, nsteps, N0, W, C, (uint64_t)c, hist_theta,
                  hist_prop, hist_ll, hist_acc);
    }
    (void)nthreads;
    free(g);
    return 0;
}

/* ---- stream probes for tests ---------------------------------------------- */

ORC_EXPORT void orc_philox(const uint32_t ctr[4], const uint32_t key[2], uint32_t out[4]) {
    orc_u32x4 c = {{ctr[0], ctr[1], ctr[2], ctr[3]}};
    orc_u32x4 r = orc_philox4x32_10(c, key[0], key[1]);
    memcpy(out, r.v, sizeof r.v);
}

/* The D normals and the Exp(1) draw of (chain, iter, pidx0). */
ORC_EXPORT uint32_t orc_step_variates(uint64_t seed, uint32_t chain, uint32_t iter, uint32_t pidx0, int D, double *z,
                                      double *E) {
    const uint32_t k0 = (uint32_t)seed, k1 = (uint32_t)(seed >> 32);
    uint32_t faults = 0;
    for (int j = 0; j < D; ++j) z[j] = orc_normal(zig(), k0, k1, chain, iter, pidx0, (uint32_t)j, &faults);
    *E = orc_exponential(zig(), k0, k1, chain, iter, pidx0, &faults);
    return faults;
}

/* Bulk draws for distribution tests: n normals / exponentials from the stream. */
ORC_EXPORT void orc_normal_vec(uint64_t seed, uint32_t chain, uint32_t iter0, uint64_t n, double *out) {
    const uint32_t k0 = (uint32_t)seed, k1 = (uint32_t)(seed >> 32);
    uint32_t faults = 0;
    for (uint64_t i = 0; i < n; ++i)
        out[i] = orc_normal(zig(), k0, k1, chain, iter0 + (uint32_t)(i >> 6), 0, (uint32_t)(i & 63u), &faults);
}
ORC_EXPORT void orc_exp_vec(uint64_t seed, uint32_t chain, uint32_t iter0, uint64_t n, double *out) {
    const uint32_t k0 = (uint32_t)seed, k1 = (uint32_t)(seed >> 32);
    uint32_t faults = 0;
    for (uint64_t i = 0; i < n; ++i) out[i] = orc_exponential(zig(), k0, k1, chain + (uint32_t)i, iter0, 0, &faults);
}

ORC_EXPORT void orc_exp_nonpos_vec(const double *x, double *y, uint64_t n) {
    for (uint64_t i = 0; i < n; ++i) y[i] = orc_exp_nonpos(x[i]);
}

/* Ziggurat tables: an, fn (ORC_ZN_L + 2 each), ke, we, fe (256 each). */
ORC_EXPORT void orc_exp_le0_vec(const double *x, double *y, uint64_t n) {
    for (uint64_t i = 0; i < n; ++i) y[i] = orc_exp_le0(x[i]);
}
ORC_EXPORT void orc_log_1_2_vec(const double *x, double *y, uint64_t n) {
    for (uint64_t i = 0; i < n; ++i) y[i] = orc_log_1_2(x[i]);
}
ORC_EXPORT void orc_rcp_1_2_vec(const double *x, double *y, uint64_t n) {
    for (uint64_t i = 0; i < n; ++i) (void)orc_log_rcp_1_2(x[i], &y[i]);
}
ORC_EXPORT void orc_exp_any_vec(const double *x, double *y, uint64_t n) {
    for (uint64_t i = 0; i < n; ++i) y[i] = orc_exp_any(x[i]);
}

ORC_EXPORT void orc_log_any_vec(const double *x, double *y, uint64_t n) {
    for (uint64_t i = 0; i < n; ++i) y[i] = orc_log_any(x[i]);
}

ORC_EXPORT void orc_zig_tables_copy(double *an, double *fn, uint64_t *ke, double *we, double *fe) {
    const orc_zig_tables *t = zig();
    memcpy(an, t->an, sizeof t->an);
    memcpy(fn, t->fn, sizeof t->fn);
    memcpy(ke, t->ke, sizeof t->ke);
    memcpy(we, t->we, sizeof t->we);
    memcpy(fe, t->fe, sizeof t->fe);
}

ORC_EXPORT void orc_log_vec(const double *x, double *y, uint64_t n) {
    for (uint64_t i = 0; i < n; ++i) y[i] = orc_log(x[i]);
}


/* Checker for the device's rolling-acceptance quotient (emcmc_kernels.h
 * div_markstein): q = RN(x·y), y = RN(1/b), q' = RN(q + RN_exact(x − b·q)·y)
 * must equal the IEEE quotient x / b.  Returns the number of mismatches. */
ORC_EXPORT uint64_t orc_markstein_mismatches(double b, const double *x, uint64_t n) {
    const double y = 1.0 / b;
    uint64_t bad = 0;
    for (uint64_t i = 0; i < n; ++i) {
        const double q = x[i] * y;
        const double r = fma(-q, b, x[i]);
        const double q1 = fma(r, y, q);
        const double ref = x[i] / b;
        if (orc_d2u(q1) != orc_d2u(ref)) ++bad;
    }
    return bad;
}

/* ==========================================================================
 * General schedule path: P ≥ 1 RandomWalkUpdates over coordinate subsets
 * (Metropolis-within-Gibbs), UniformRandomWalk or GaussianRandomWalk,
 * NoAdaptation or AdaptationUnifRW, ImproperPrior, GsnTargetLaw target.
 *
 * Restated (reference files under /root/reference/src):
 *   schedule order, first step has no prev_ws ........... schedule.jl:56-89, run.jl:64-83
 *   update_workspaces!: θ_local ← θ[coords]; ll ← ll of the previous step's
 *     local workspace at its iteration (−Inf before the first step) .. run.jl:101-112
 *   UniformRandomWalk rand: U = a + (b − a)·u, a = −ϵ, b = ϵ (Distributions'
 *     Uniform), θ° = θ·(e^U·pos + 1·!pos) + U·!pos with Julia's Bool products
 *     (x·true = x, x·false = copysign(0, x)): pos = false ⇒ θ·1 + U,
 *     pos = true ⇒ θ·e^U + copysign(0, U) ............... random_walk.jl:63-73
 *   UniformRandomWalk logpdf(θ, θ°) = mapreduce(i → pos_i ? −log(2ϵ_i) −
 *     log θ°_i : 0.0, +, 1:n), a left fold ............... random_walk.jl:88-94
 *   GaussianRandomWalk over the update's coordinates ..... random_walk.jl:145-171
 *     with pos: on the log scale, with the in-place exp/log round trips of
 *     remove_/reimpose_constraints! in rand and both logpdf calls, and the
 *     log-Jacobian −sum(log θ[pos]) (see the code) ....... random_walk.jl:136-171
 *   set_parameters!(::Proposal): P°.θ[coords] ← θ°; P° persists across updates
 *     and starts as deepcopy(data.P) — the target's μ, not θinit
 *                                         updates.jl:198-205, workspaces.jl:225-233
 *   loglikelihood(ws, ::Proposal) = loglikelihood(P°, obs) ... workspaces.jl:236-238
 *   proposal history = θ with coords ← θ°; state history = θ after accept
 *                                                         run.jl:231-240, 312-320
 *   update_stats!: N counts every update step (from 1); ra_prev =
 *     rolling_ar[max(1, iter−1)][pidx], 0.0 when (iter−1, pidx) did not run
 *                                                         chain_statistics.jl:42-66
 *   AdaptationUnifRW on its own turn: accepted += a, proposed += 1; when
 *     proposed ≥ k: δ = scale/√max(1, iter/k − offset), a_r = accepted/proposed
 *     (counters reset), ϵ ← clamp(ϵ + (a_r > target ? δ : −δ), min, max)
 *                                              run.jl:136-178, adaptation.jl:273-329
 * Variates: uniform j of update p at iter from block (j/2, attempt 0) with
 * counter w = (p << 16): words (x,y) for even j, (z,w) for odd j, u ∈ [0,1)
 * from 53 bits; Gaussian normals as in the single-update path (index j local
 * to the update); the accept exponential as orc_exponential with pidx0 = p.
 * ========================================================================== */

#define ORC_MWG_MAXD 64
#define ORC_MAX_RESAMPLE 0xFFFEu     /* UniformRandomWalk: counter blocks (r << 16) | j/2 */
#define ORC_MAX_RESAMPLE_GSN 0x7FFEu /* GaussianRandomWalk: normal index (r << 17) | j < 2^32, never repeated */
#define ORC_FAULT_PRIOR_RESAMPLES 8u

/* priors.jl, restated: EMCMC_PRIOR_* kinds, EMCMC_DIST_* families */
enum { ORC_PRIOR_IMPROPER = 0, ORC_PRIOR_IMPROPER_POS = 1, ORC_PRIOR_PRODUCT = 2, ORC_PRIOR_STANDARD = 3 };
enum {
    ORC_DIST_NORMAL = 1, ORC_DIST_UNIFORM = 2, ORC_DIST_EXPONENTIAL = 3, ORC_DIST_GAMMA = 4, ORC_DIST_LOGNORMAL = 5,
    ORC_DIST_BETA = 6, ORC_DIST_INVERSE_GAMMA = 7, ORC_DIST_CAUCHY = 8, ORC_DIST_LAPLACE = 9, ORC_DIST_TDIST = 10,
    ORC_DIST_PRODUCT = 32, ORC_DIST_MVNORMAL = 33
};
#define ORC_LOGPI 1.1447298858494002 /* log π */

static double orc_log_real(double x) { return (x < 0.0) ? NAN : orc_log_any(x); }

/* logpdf of one univariate factor (Distributions.jl / StatsFuns forms; the
 * Distributions version is unpinned):
 *   Normal(μ, σ): normlogpdf(z) − log σ = −(z² + log2π)/2 − log σ, z = (x − μ)/σ
 *   Uniform(a, b): −log(b − a) on [a, b], else −Inf
 *   Exponential(θ): x < 0 ? −Inf : log λ − λx, λ = 1/θ
 *   Gamma(α, θ): x < 0 ? −Inf : −loggamma(α) − α log θ + (α − 1) log x − x/θ (left to right)
 *   LogNormal(μ, σ): x ≤ 0 ? −Inf : normlogpdf(μ, σ, log x) − log x
 *   Beta(α, β): x ∉ [0, 1] ? −Inf : xlogy(α − 1, x) + xlog1py(β − 1, −x) − logbeta(α, β)
 *   InverseGamma(α, θ): x ≤ 0 ? −Inf : α log θ − loggamma(α) − (α + 1) log x − θ/x
 *   Cauchy(μ, σ): −((log1psq(z) + log π) + log σ)  (Distributions.jl: −(log1psq(z) + logπ + log(σ))),
 *     log1psq(z) = |z| < 2^53 ? log1p(z²) : 2·log|z|  (StatsFuns / LogExpFunctions)
 *   Laplace(μ, θ): −(|x − μ|/θ + log(2θ))
 *   TDist(ν): loggamma((ν+1)/2) − loggamma(ν/2) − log(νπ)/2 − (ν+1)/2 · log1p(x²/ν)
 * (a, b) are the parameters as the device holds them (Exponential: b = 1/θ,
 * TDist: b = (ν+1)/2), c the constant the host computes once. */
static double orc_univariate_logpdf(uint32_t fam, double a, double b, double c, double x) {
    switch (fam) {
    case ORC_DIST_NORMAL: {
        const double z = (x - a) / b;
        return -(z * z + ORC_LOG2PI) / 2.0 - c;
    }
    case ORC_DIST_UNIFORM: return (x >= a && x <= b) ? c : -INFINITY;
    case ORC_DIST_EXPONENTIAL: return (x < 0.0) ? -INFINITY : c - b * x;
    case ORC_DIST_GAMMA: return (x < 0.0) ? -INFINITY : (c + (a - 1.0) * orc_log_real(x)) - x / b;
    case ORC_DIST_LOGNORMAL: {
        if (x != x) return x;
        if (x <= 0.0) return -INFINITY;
        const double lx = orc_log_any(x);
        const double z = (lx - a) / b;
        return (-(z * z + ORC_LOG2PI) / 2.0 - c) - lx;
    }
    case ORC_DIST_BETA: {
        if (x < 0.0 || x > 1.0) return -INFINITY;
        const double t1 = (a - 1.0 == 0.0) ? 0.0 : (a - 1.0) * orc_log_real(x); /* xlogy */
        const double t2 = (b - 1.0 == 0.0) ? 0.0 : (b - 1.0) * orc_log1p_any(-x); /* xlog1py */
        return (t1 + t2) - c;
    }
    case ORC_DIST_INVERSE_GAMMA:
        if (x != x) return x;
        if (x <= 0.0) return -INFINITY;
        return (c - (a + 1.0) * orc_log_any(x)) - b / x;
    case ORC_DIST_CAUCHY: {
        /* StatsFuns log1psq: log1p(z²) below maxintfloat = 2^53, else 2·log|z| (z² would
           lose z or overflow) */
        const double z = (x - a) / b, az = fabs(z);
        const double l = (az < 0x1p53) ? orc_log1p_any(az * az) : 2.0 * orc_log_any(az);
        return -((l + ORC_LOGPI) + c);
    }
    case ORC_DIST_LAPLACE: return -(fabs(x - a) / b + c);
    default: /* TDist */
        return c - b * orc_log1p_any((x * x) / a);
    }
}

/* (family, a, b) of a univariate factor → device parameters and constant
 * (engine host code); −1 on invalid parameters, −4 for a family with no plugin */
static int orc_prior_factor_consts(uint32_t fam, double a, double b, double *pa, double *pb, double *pc) {
    *pa = a, *pb = b;
    switch (fam) {
    case ORC_DIST_NORMAL:
    case ORC_DIST_LOGNORMAL:
        if (!(b > 0.0)) return -1;
        *pc = orc_log(b);
        return 0;
    case ORC_DIST_UNIFORM:
        if (!(a < b)) return -1;
        *pc = -orc_log(b - a);
        return 0;
    case ORC_DIST_EXPONENTIAL:
        if (!(a > 0.0)) return -1;
        *pb = 1.0 / a, *pc = orc_log(1.0 / a);
        return 0;
    case ORC_DIST_GAMMA:
        if (!(a > 0.0 && b > 0.0)) return -1;
        *pc = (-lgamma(a)) - a * orc_log(b);
        return 0;
    case ORC_DIST_BETA:
        if (!(a > 0.0 && b > 0.0)) return -1;
        *pc = (lgamma(a) + lgamma(b)) - lgamma(a + b);
        return 0;
    case ORC_DIST_INVERSE_GAMMA:
        if (!(a > 0.0 && b > 0.0)) return -1;
        *pc = a * orc_log(b) - lgamma(a);
        return 0;
    case ORC_DIST_CAUCHY:
        if (!(b > 0.0)) return -1;
        *pc = orc_log(b);
        return 0;
    case ORC_DIST_LAPLACE:
        if (!(b > 0.0)) return -1;
        *pc = orc_log(2.0 * b);
        return 0;
    case ORC_DIST_TDIST:
        if (!(a > 0.0)) return -1;
        *pb = (a + 1.0) / 2.0;
        *pc = (lgamma((a + 1.0) / 2.0) - lgamma(a / 2.0)) - orc_log(a * 3.141592653589793) / 2.0;
        return 0;
    }
    return -4;
}
typedef struct {
    uint32_t kind; /* 1 uniform, 2 gaussian */
    uint32_t nc;
    uint8_t pos[ORC_MWG_MAXD]; /* uniform: positivity flags */
    uint32_t coords[ORC_MWG_MAXD];
    double eps0[ORC_MWG_MAXD];
    double L[ORC_MWG_MAXD * ORC_MWG_MAXD], iL[ORC_MWG_MAXD], c0;
    int diag;
    uint32_t adapt, k;
    double target, scale[ORC_MWG_MAXD], amin[ORC_MWG_MAXD], amax[ORC_MWG_MAXD], offset[ORC_MWG_MAXD];
    /* prior: the factors with the local index each reads (priors.jl:64-79) */
    uint32_t prior, nfac;
    uint32_t ffam[ORC_MWG_MAXD], fcnt[ORC_MWG_MAXD], fstart[ORC_MWG_MAXD], fcomp[ORC_MWG_MAXD];
    double fa[ORC_MWG_MAXD], fb[ORC_MWG_MAXD], fc[ORC_MWG_MAXD];
    uint32_t cfam[ORC_MWG_MAXD]; /* Product components, in factor order */
    double ca[ORC_MWG_MAXD], cb[ORC_MWG_MAXD], cc[ORC_MWG_MAXD];
    double mmu[ORC_MWG_MAXD], mL[ORC_MWG_MAXD * ORC_MWG_MAXD], miL[ORC_MWG_MAXD]; /* MvNormal factors, by local index */
} orc_mwg_update;

/* logpdf(dist_f, θ[idx_f]) of factor f: a univariate at its one index; a
 * Product (Distributions' sum over its components, folded left); an MvNormal
 * c0 − ‖L⁻¹(θ − μ)‖²/2 (forward substitution, squares folded left). */
static double orc_factor_logpdf(const orc_mwg_update *u, uint32_t f, const double *x) {
    const uint32_t st = u->fstart[f], k = u->fcnt[f];
    if (u->ffam[f] == ORC_DIST_PRODUCT) {
        double s = 0.0;
        for (uint32_t i = 0; i < k; ++i) {
            const uint32_t q = u->fcomp[f] + i;
            const double v = orc_univariate_logpdf(u->cfam[q], u->ca[q], u->cb[q], u->cc[q], x[st + i]);
            s = (i == 0) ? v : s + v;
        }
        return s;
    }
    if (u->ffam[f] == ORC_DIST_MVNORMAL) {
        double y[ORC_MWG_MAXD], s = 0.0;
        for (uint32_t i = 0; i < k; ++i) {
            double acc = x[st + i] - u->mmu[st + i];
            for (uint32_t m = 0; m < i; ++m) acc = fma(-u->mL[(size_t)(st + i) * ORC_MWG_MAXD + st + m], y[m], acc);
            y[i] = acc * u->miL[st + i];
            s = (i == 0) ? y[i] * y[i] : fma(y[i], y[i], s);
        }
        return u->fc[f] - s / 2.0;
    }
    return orc_univariate_logpdf(u->ffam[f], u->fa[f], u->fb[f], u->fc[f], x[st]);
}

/* logpdf(prior, x) over the update's n local coordinates (priors.jl:18-88):
 * ImproperPosPrior −(x₁ + x₂ + …) of the logs; ProductPrior lp = 0.0;
 * lp += logpdf(dist, θ[idx]) per factor (priors.jl:82-88); StandardPrior
 * logpdf(dist, θ) (priors.jl:39). */
static double orc_mwg_log_prior(const orc_mwg_update *u, uint32_t n, const double *x) {
    if (u->prior == ORC_PRIOR_IMPROPER) return 0.0;
    if (u->prior == ORC_PRIOR_IMPROPER_POS) {
        double s = 0.0;
        for (uint32_t j = 0; j < n; ++j) {
            const double v = orc_log_real(x[j]);
            s = (j == 0) ? v : s + v;
        }
        return -s;
    }
    if (u->prior == ORC_PRIOR_STANDARD) return orc_factor_logpdf(u, 0, x);
    double lp = 0.0;
    for (uint32_t f = 0; f < u->nfac; ++f) lp += orc_factor_logpdf(u, f, x);
    return lp;
}

/* The prior of update u from the caller's tables: factor f = (ffam, fcnt, fa, fb);
 * Product components in cfam/ca/cb, consecutively in factor order; MvNormal
 * μ / Σ in mvmu / mvS placed at the factor's local index range (Σ column-major
 * in a 64 × 64 block).  The index each factor reads is the constructor's
 * (priors.jl:64-79): dims 1 → θ[1], dims k > 1 → θ[last:last+k−1], `last`
 * advancing by dims either way.  Returns 0, −2 (invalid) or −4 (a pairing the
 * reference raises a MethodError on: univariate over dims > 1, multivariate
 * over dims 1, a univariate StandardPrior). */
static int orc_build_prior(orc_mwg_update *u, uint32_t nfac, const uint32_t *ffam, const uint32_t *fcnt,
                           const double *fa, const double *fb, const uint32_t *cfam, const double *ca,
                           const double *cb, const double *mvmu, const double *mvS) {
    const uint32_t n = u->nc;
    if (nfac == 0 || nfac > ORC_MWG_MAXD) return -2;
    if (u->prior == ORC_PRIOR_STANDARD && nfac != 1) return -2;
    u->nfac = nfac;
    uint32_t last = 0, ncomp = 0;
    for (uint32_t f = 0; f < nfac; ++f) {
        const uint32_t fam = ffam[f], k = fcnt[f];
        const int multi = (fam == ORC_DIST_PRODUCT || fam == ORC_DIST_MVNORMAL);
        if (k == 0) return -2;
        if (u->prior == ORC_PRIOR_STANDARD) {
            if (!multi) return -4; /* logpdf(univariate, θ::Vector): no scalar in the reference */
            if (k != n) return -2;
        } else if (multi != (k > 1)) {
            return -4;
        }
        u->ffam[f] = fam;
        u->fcnt[f] = k;
        u->fstart[f] = (k == 1) ? 0u : last;
        last += k;
        if (last > n) return -2;
        if (fam == ORC_DIST_PRODUCT) {
            if (ncomp + k > ORC_MWG_MAXD) return -2;
            u->fcomp[f] = ncomp;
            for (uint32_t i = 0; i < k; ++i, ++ncomp) {
                u->cfam[ncomp] = cfam[ncomp];
                const int rc = orc_prior_factor_consts(cfam[ncomp], ca[ncomp], cb[ncomp], &u->ca[ncomp], &u->cb[ncomp],
                                                       &u->cc[ncomp]);
                if (rc) return rc == -4 ? -4 : -2;
            }
        } else if (fam == ORC_DIST_MVNORMAL) {
            const uint32_t st = u->fstart[f];
            double S[ORC_MWG_MAXD * ORC_MWG_MAXD], Lk[ORC_MWG_MAXD * ORC_MWG_MAXD];
            for (uint32_t j = 0; j < k; ++j)
                for (uint32_t i = 0; i < k; ++i) S[i + (size_t)j * k] = mvS[(st + i) + (size_t)(st + j) * ORC_MWG_MAXD];
            if (orc_cholesky(S, (int)k, Lk)) return -2;
            for (uint32_t i = 0; i < k; ++i) {
                u->mmu[st + i] = mvmu[st + i];
                u->miL[st + i] = 1.0 / Lk[(size_t)i * k + i];
                for (uint32_t m = 0; m <= i; ++m) u->mL[(size_t)(st + i) * ORC_MWG_MAXD + st + m] = Lk[(size_t)i * k + m];
            }
            u->fc[f] = mvnormal_c0((int)k, logdet_chol(Lk, (int)k));
        } else {
            const int rc = orc_prior_factor_consts(fam, fa[f], fb[f], &u->fa[f], &u->fb[f], &u->fc[f]);
            if (rc) return rc == -4 ? -4 : -2;
        }
    }
    return 0;
}

/* Test entry: logpdf(prior, x) for each of nx local vectors x (n entries each),
 * from the same factor tables as orc_run_mwg (one update).  Returns the
 * orc_build_prior status (0, −2 invalid, −4 a pairing the reference raises on). */
ORC_EXPORT int orc_eval_prior(uint32_t prior, uint32_t n, uint32_t nfac, const uint32_t *ffam, const uint32_t *fcnt,
                              const double *fa, const double *fb, const uint32_t *cfam, const double *ca,
                              const double *cb, const double *mvmu, const double *mvS, uint64_t nx, const double *x,
                              double *out) {
    if (n < 1 || n > ORC_MWG_MAXD) return -2;
    orc_mwg_update *u = (orc_mwg_update *)calloc(1, sizeof(orc_mwg_update));
    if (!u) return -3;
    u->nc = n;
    u->prior = prior;
    int rc = 0;
    if (prior == ORC_PRIOR_PRODUCT || prior == ORC_PRIOR_STANDARD)
        rc = orc_build_prior(u, nfac, ffam, fcnt, fa, fb, cfam, ca, cb, mvmu, mvS);
    if (rc == 0)
        for (uint64_t i = 0; i < nx; ++i) out[i] = orc_mwg_log_prior(u, n, x + i * n);
    free(u);
    return rc;
}

/* user target (EMCMC_TARGET_USER): loglikelihood(P°, obs) of a user function,
 * the same source the engine compiles for the device (tests/user_targets/) */
typedef double (*orc_user_loglik_fn)(const double *theta, int D, const double *obs, uint64_t nobs,
                                     const double *params);
/* user update (EMCMC_USER_UPDATE): proposal! and log_transition_density of the
 * same source the engine compiles (tests/user_updates/, oracle/user_prelude.h) */
typedef void (*orc_user_prop_fn)(const double *theta, double *theta_prop, int n, const double *params,
                                 emcmc_rng *rng);
typedef double (*orc_user_ltd_fn)(const double *x, const double *y, int n, const double *params);
/* a user law's gradient (EMCMC_USER_GRAD): ∇ loglikelihood(P°, obs) into grad[D] */
typedef void (*orc_user_grad_fn)(const double *theta, int D, const double *obs, uint64_t nobs, const double *params,
                                 double *grad);

#define ORC_FAULT_POSDEF 4u

static void mix_factor_consts(const double *L, int D, double *iL, double *c0) {
    for (int i = 0; i < D; ++i) iL[i] = 1.0 / L[(size_t)i * D + i];
    *c0 = mvnormal_c0(D, logdet_chol(L, D));
}

/* GaussianRandomWalkMix / HaarioTypeAdaptation / GenericChainStats mean-cov
 * state of the general schedule (kind 3 updates; chain moments for any P).
 * Per update p, per chain c: L_B (lower, row-major n_p × n_p) at
 * LB + off_sq[p] + c·n_p², the Haario mean at hmean + off_v[p] + c·n_p and cov
 * at hcov + off_sq[p] + c·n_p²; M_io[p] Haario's M (uniform over chains);
 * smean [C][D], scov [C][D][D] the chain's running mean/cov of θ. */
typedef struct orc_mwg_ext {
    const double *mix_lam;    /* [P] λ of each GaussianRandomWalkMix update */
    const uint32_t *haario_k; /* [P] adapt_every_k_steps, 0: no HaarioTypeAdaptation */
    uint32_t *M_io;           /* [P] */
    double *LB, *hmean, *hcov;
    const uint64_t *off_sq, *off_v;
    int chain_moments;
    int reserved;
    double *smean, *scov;
    orc_user_grad_fn user_grad; /* MALA (kind 4) with a user target: the law's EMCMC_USER_GRAD */
} orc_mwg_ext;

/* ∇_μ loglikelihood(GsnTargetLaw, obs) = Σ_k Σ⁻¹(x_k − μ) = n·Σ⁻¹(x̄ − μ), both
 * likelihood modes: y = L⁻¹(x̄ − μ) forward, w = L⁻ᵀy backward (w_i = (y_i −
 * Σ_{j>i} L_ji w_j)/L_ii, j descending), g = n·w — the device's GsnTarget::grad
 * (emcmc_mwg.h), the hook MALA reads (compute_gradients_and_momenta!). */
static void orc_gsn_grad(const orc_gsn *g, int D, int tdiag, const double *mp, double *out) {
    double y[64];
    for (int i = 0; i < D; ++i) {
        double acc = g->xbar[i] - mp[i];
        if (!tdiag)
            for (int j = 0; j < i; ++j) acc = fma(-g->Lt[(size_t)i * D + j], y[j], acc);
        y[i] = acc * g->iLt[i];
    }
    for (int i = D - 1; i >= 0; --i) {
        double acc = y[i];
        if (!tdiag)
            for (int j = D - 1; j > i; --j) acc = fma(-g->Lt[(size_t)j * D + i], out[j], acc);
        out[i] = acc * g->iLt[i];
    }
    for (int i = 0; i < D; ++i) out[i] = (double)g->nobs * out[i];
}

/* logpdf(rw::GaussianRandomWalk, a, b) (random_walk.jl:161-171) with its
 * in-place round trips: logJ = −sum(log b[pos]) (left fold; only where a
 * coordinate is restricted), logpdf(MvNormal(log a, Σ), log b) + logJ, then
 * a ← exp(log a), b ← exp(log b) at the restricted coordinates. */
static double orc_gsn_rw_lp(const double *L, const double *iL, double c0, int diag, const uint8_t *pos, uint32_t n,
                            int anypos, double *a, double *b) {
    double x[ORC_MWG_MAXD], y[ORC_MWG_MAXD], r[ORC_MWG_MAXD], lj = 0.0;
    int first = 1;
    for (uint32_t i = 0; i < n; ++i)
        if (pos[i]) {
            const double v = orc_log_any(b[i]);
            lj = first ? v : lj + v;
            first = 0;
        }
    for (uint32_t i = 0; i < n; ++i) {
        x[i] = pos[i] ? orc_log_any(a[i]) : a[i];
        y[i] = pos[i] ? orc_log_any(b[i]) : b[i];
        r[i] = y[i] - x[i];
    }
    double lp = c0 - sqmahal(L, iL, r, (int)n, diag) / 2.0;
    if (anypos) lp = lp + (-lj);
    for (uint32_t i = 0; i < n; ++i)
        if (pos[i]) {
            a[i] = orc_exp_any(x[i]);
            b[i] = orc_exp_any(y[i]);
        }
    return lp;
}

/* GenericChainStats / Haario register! recurrence on n values (chain_statistics.jl:46-49,
 * adaptation.jl:406-414): old = (N−1)/N·cov + m m', m ← m·(N/(N+1)) + θ/(N+1),
 * new = old + (θθ')/N, cov = new − (N+1)/N·(m m'), elementwise, products rounded */
static void orc_rank1_register(double *m, double *cv, const double *x, uint32_t n, uint64_t N) {
    const double a = (double)(N - 1) / (double)N;
    const double b = (double)N / (double)(N + 1);
    const double cN = (double)(N + 1) / (double)N;
    double mo[ORC_MWG_MAXD];
    memcpy(mo, m, sizeof(double) * n);
    for (uint32_t i = 0; i < n; ++i) m[i] = m[i] * b + x[i] / (double)(N + 1);
    for (uint32_t i = 0; i < n; ++i)
        for (uint32_t j = 0; j < n; ++j) {
            const double old_sq = a * cv[(size_t)i * n + j] + mo[i] * mo[j];
            const double new_sq = old_sq + (x[i] * x[j]) / (double)N;
            cv[(size_t)i * n + j] = new_sq - cN * (m[i] * m[j]);
        }
}

/* table layout from Python (ORC_MWG_MAXD = 64 slots per update):
 *   kind[P], nc[P], coords[P*64], eps[P*64], sigma[P*4096] (nc×nc column-major),
 *   pos[P*64] (uint8), adapt[P], k[P], aparams[P*257] = (target, scale[64], min[64], max[64], offset[64])
 *   (AdaptationUnifRW per coordinate; the scalar form repeats its values),
 *   prior[P], factor tables per update: nfac[P], ffam[P*64], fcnt[P*64], fa[P*64], fb[P*64];
 * ll_prop [P][C] out: sub_ws°.ll of each update's latest proposal (NULL: skip);
 * user_ll: NULL for GsnTargetLaw, else the user target (user_params its parameters). */
ORC_EXPORT int orc_run_mwg(int D, uint64_t C, uint32_t chain0, uint64_t seed, uint32_t P, const uint32_t *kind,
                           const uint32_t *nc, const uint32_t *coords, const double *eps, const double *sigma,
                           const uint8_t *pos, const uint32_t *adapt, const uint32_t *adapt_k, const double *aparams,
                           const double *t_sigma, uint64_t nobs, const double *obs, int ll_mode,
                           uint32_t W, uint32_t nsteps, const uint32_t *step_iter, const uint32_t *step_pidx,
                           uint64_t *N_io, uint32_t *last_iter_io, double *theta, double *mu_p, double *ll,
                           double *ra, uint64_t *ring, uint32_t *nacc, uint32_t *aprop, uint32_t *aacc,
                           double *eps_state, uint32_t *faults, double *hist_theta, double *hist_prop,
                           double *hist_ll, uint8_t *hist_acc, int nthreads, const uint32_t *prior_kind,
                           const uint32_t *nfac, const uint32_t *ffam, const uint32_t *fcnt, const double *fa,
                           const double *fb, double *ll_prop, orc_user_loglik_fn user_ll,
                           const double *user_params, const uint32_t *pcfam, const double *pca, const double *pcb,
                           const double *pmvmu, const double *pmvS, orc_user_prop_fn user_prop,
                           orc_user_ltd_fn user_ltd, const double *user_uparams, const orc_mwg_ext *ext) {
    if (D < 1 || D > ORC_MWG_MAXD || P < 1 || P > 64) return -2;
    (void)zig();
    orc_gsn *g = (orc_gsn *)malloc(sizeof(orc_gsn));
    orc_mwg_update *U = (orc_mwg_update *)calloc(P, sizeof(orc_mwg_update));
    if (!g || !U) return -3;
    /* target constants (the rw Σ argument is unused here: pass Σ_t twice) */
    /* a user target's observation rows have their own width: the Gaussian
     * constants are not used then, so they are built over no observations */
    int rc = gsn_prepare(g, D, t_sigma, t_sigma, user_ll ? 0 : nobs, obs, ll_mode | 0x100);
    if (rc) {
        free(g);
        free(U);
        return rc;
    }
    const int tdiag = is_diag_upper(t_sigma, D);
    for (uint32_t p = 0; p < P; ++p) {
        orc_mwg_update *u = &U[p];
        u->kind = kind[p];
        u->nc = nc[p];
        if (u->nc < 1 || u->nc > ORC_MWG_MAXD) {
            free(g);
            free(U);
            return -2;
        }
        for (uint32_t j = 0; j < u->nc; ++j) {
            u->coords[j] = coords[p * ORC_MWG_MAXD + j];
            u->eps0[j] = eps[p * ORC_MWG_MAXD + j];
            u->pos[j] = (pos && pos[p * ORC_MWG_MAXD + j]) ? 1 : 0;
            if (u->coords[j] >= (uint32_t)D) {
                free(g);
                free(U);
                return -2;
            }
        }
        if ((u->kind == 3 || (ext && ext->haario_k && ext->haario_k[p])) && !ext) {
            free(g);
            free(U);
            return -2;
        }
        if (u->kind == 4) { /* MALA: ϵ = eps[0]; its densities' MvNormal(·, ϵ²I) as the factor ϵI */
            const int n = (int)u->nc;
            const double e = u->eps0[0];
            if (!(e > 0.0) || (user_ll && !(ext && ext->user_grad))) {
                free(g);
                free(U);
                return -2;
            }
            memset(u->L, 0, sizeof(double) * (size_t)n * n);
            for (int i = 0; i < n; ++i) {
                u->L[(size_t)i * n + i] = e;
                u->iL[i] = 1.0 / e;
            }
            u->c0 = mvnormal_c0(n, logdet_chol(u->L, n));
            u->diag = 1;
        }
        if (u->kind == 2 || u->kind == 3) {
            const int n = (int)u->nc;
            if (orc_cholesky(sigma + (size_t)p * ORC_MWG_MAXD * ORC_MWG_MAXD, n, u->L)) {
                free(g);
                free(U);
                return -1;
            }
            for (int i = 0; i < n; ++i) u->iL[i] = 1.0 / u->L[(size_t)i * n + i];
            u->c0 = mvnormal_c0(n, logdet_chol(u->L, n));
            u->diag = is_diag_upper(sigma + (size_t)p * ORC_MWG_MAXD * ORC_MWG_MAXD, n);
        }
        u->adapt = adapt[p];
        u->k = adapt_k[p];
        {
            const double *ap = aparams + (size_t)p * (1 + 4 * ORC_MWG_MAXD);
            u->target = ap[0];
            for (int j = 0; j < ORC_MWG_MAXD; ++j) {
                u->scale[j] = ap[1 + j];
                u->amin[j] = ap[1 + ORC_MWG_MAXD + j];
                u->amax[j] = ap[1 + 2 * ORC_MWG_MAXD + j];
                u->offset[j] = ap[1 + 3 * ORC_MWG_MAXD + j];
            }
        }
        u->prior = prior_kind ? prior_kind[p] : ORC_PRIOR_IMPROPER;
        if (u->prior == ORC_PRIOR_PRODUCT || u->prior == ORC_PRIOR_STANDARD) {
            const size_t o = (size_t)p * ORC_MWG_MAXD;
            const int prc = orc_build_prior(u, nfac[p], ffam + o, fcnt + o, fa + o, fb + o, pcfam ? pcfam + o : NULL,
                                            pca ? pca + o : NULL, pcb ? pcb + o : NULL, pmvmu ? pmvmu + o : NULL,
                                            pmvS ? pmvS + o * ORC_MWG_MAXD : NULL);
            if (prc) {
                free(g);
                free(U);
                return prc;
            }
        }
    }
    const uint32_t k0 = (uint32_t)seed, k1 = (uint32_t)(seed >> 32);
    const orc_zig_tables *zt = zig();
    const uint64_t N_start = *N_io;
    uint32_t last0[64];
    for (uint32_t p = 0; p < P; ++p) last0[p] = last_iter_io[p];
#pragma omp parallel for num_threads(nthreads > 0 ? nthreads : 1) schedule(static)
    for (int64_t ci = 0; ci < (int64_t)C; ++ci) {
        const uint64_t c = (uint64_t)ci;
        const uint32_t chain_id = chain0 + (uint32_t)c;
        double th[ORC_MWG_MAXD], mp[ORC_MWG_MAXD];
        memcpy(th, theta + c * D, sizeof(double) * D);
        memcpy(mp, mu_p + c * D, sizeof(double) * D);
        double cll = ll[c];
        uint32_t f = faults[c];
        uint32_t last[64], Mloc[64];
        memcpy(last, last0, sizeof(uint32_t) * P);
        for (uint32_t q = 0; q < P; ++q) Mloc[q] = (ext && ext->M_io) ? ext->M_io[q] : 0u;
        for (uint32_t s = 0; s < nsteps; ++s) {
            const uint32_t iter = step_iter[s], p = step_pidx[s] - 1;
            const orc_mwg_update *u = &U[p];
            const uint32_t n = u->nc;
            double *ep = eps_state + ((size_t)p * C + c) * ORC_MWG_MAXD;
            double tl[ORC_MWG_MAXD], tp[ORC_MWG_MAXD], ta[ORC_MWG_MAXD];
            int accept_ta = 0; /* accepted values differ from the proposal (Gaussian with pos) */
            int useB = 0;      /* GaussianRandomWalkMix: the last rand! picked gsn_B */
            (void)useB;
            for (uint32_t j = 0; j < n; ++j) tl[j] = th[u->coords[j]];
            double ltd_fwd = 0.0, ltd_rev = 0.0;
            int anypos = 0;
            for (uint32_t j = 0; j < n; ++j) anypos |= u->pos[j];
            /* proposal! (updates.jl:191-196): rand!, again while logpdf(prior, θ°) === −Inf;
             * resample r reads counter blocks (r << 16) | j/2.  A user update
             * (kind 5): its own proposal! and log_transition_density
             * (updates.jl:42-93), compiled from the engine's source */
            if (u->kind == 5) {
                emcmc_rng rng = {zt, k0, k1, chain_id, iter, p, 0u};
                for (uint32_t j = 0; j < ORC_MWG_MAXD; ++j) tp[j] = 0.0;
                user_prop(tl, tp, (int)n, user_uparams + (size_t)p * ORC_MWG_MAXD * ORC_MWG_MAXD, &rng);
                f |= rng.faults;
                ltd_fwd = user_ltd(tl, tp, (int)n, user_uparams + (size_t)p * ORC_MWG_MAXD * ORC_MWG_MAXD);
                ltd_rev = user_ltd(tp, tl, (int)n, user_uparams + (size_t)p * ORC_MWG_MAXD * ORC_MWG_MAXD);
            }
            /* MALA (kind 4; the reference stubs MALAUpdate, updates.jl:216-218): g =
             * ∇ℓ(x)[coords] at x = P°.θ with coords ← θ (compute_gradients_and_momenta!
             * (__PREVIOUS), run.jl:110), m = θ + h·g, θ° = m + ϵz (normal j of (chain,
             * iter, update)), ltd_fwd = logpdf(MvNormal(m, ϵ²I), θ°); no redraw loop */
            const double mala_h = (u->eps0[0] * u->eps0[0]) / 2.0;
            if (u->kind == 4) {
                double x[ORC_MWG_MAXD], gg[ORC_MWG_MAXD], r[ORC_MWG_MAXD];
                memcpy(x, mp, sizeof(double) * D);
                for (uint32_t j = 0; j < n; ++j) x[u->coords[j]] = tl[j];
                if (user_ll) ext->user_grad(x, D, obs, nobs, user_params, gg);
                else orc_gsn_grad(g, D, tdiag, x, gg);
                for (uint32_t j = 0; j < n; ++j) {
                    const double z = orc_normal(zt, k0, k1, chain_id, iter, p, j, &f);
                    const double m = tl[j] + mala_h * gg[u->coords[j]];
                    tp[j] = m + u->eps0[0] * z;
                    r[j] = tp[j] - m;
                }
                ltd_fwd = u->c0 - sqmahal(u->L, u->iL, r, (int)n, 1) / 2.0;
            }
            for (uint32_t rs = 0; u->kind != 5 && u->kind != 4; ++rs) {
                if (u->kind == 1) { /* UniformRandomWalk */
                    for (uint32_t j = 0; j < n; ++j) {
                        const orc_u32x4 r = orc_draw(k0, k1, chain_id, iter, (rs << 16) | (j >> 1), p, 0);
                        const double uu = (j & 1u) ? orc_u01_closed0(r.v[2], r.v[3]) : orc_u01_closed0(r.v[0], r.v[1]);
                        const double e = ep[j];
                        const double a = -e, b = e;
                        const double Uv = a + (b - a) * uu;
                        tp[j] = u->pos[j] ? tl[j] * orc_exp_any(Uv) + copysign(0.0, Uv) : tl[j] * 1.0 + Uv;
                    }
                } else { /* GaussianRandomWalk over the update's coordinates; GaussianRandomWalkMix:
                          * pick_kernel (B iff rand() ≤ λ, random_walk.jl:225-227) at every rand!,
                          * from block 0xFFFFFFFE, attempt = the redraw */
                    const double *Lx = u->L;
                    int dg = u->diag;
                    if (u->kind == 3) {
                        const orc_u32x4 pr = orc_draw(k0, k1, chain_id, iter, 0xFFFFFFFEu, p, rs);
                        useB = orc_u01_closed0(pr.v[0], pr.v[1]) <= ext->mix_lam[p];
                        if (useB) Lx = ext->LB + ext->off_sq[p] + c * (uint64_t)n * n, dg = 0;
                    }
                    if (rs > 0) /* the previous rand! left θ ← exp(log θ) where pos */
                        for (uint32_t i = 0; i < n; ++i)
                            if (u->pos[i]) tl[i] = orc_exp_any(orc_log_any(tl[i]));
                    double z[ORC_MWG_MAXD];
                    for (uint32_t j = 0; j < n; ++j) z[j] = orc_normal(zt, k0, k1, chain_id, iter, p, (rs << 17) | j, &f);
                    for (uint32_t i = 0; i < n; ++i) {
                        double lz;
                        if (dg) {
                            lz = Lx[(size_t)i * n + i] * z[i];
                        } else {
                            lz = Lx[(size_t)i * n] * z[0];
                            for (uint32_t j = 1; j <= i; ++j) lz = fma(Lx[(size_t)i * n + j], z[j], lz);
                        }
                        /* remove_constraints!: θ_i ← log θ_i where pos (random_walk.jl:136);
                         * reimpose_constraints!: θ°_i ← exp θ°_i (θ°₁) */
                        const double v = (u->pos[i] ? orc_log_any(tl[i]) : tl[i]) + lz;
                        tp[i] = u->pos[i] ? orc_exp_any(v) : v;
                    }
                }
                if (u->prior == ORC_PRIOR_IMPROPER) break;
                if (!(orc_mwg_log_prior(u, n, tp) == -INFINITY)) break;
                if (rs >= (u->kind == 1 ? ORC_MAX_RESAMPLE : ORC_MAX_RESAMPLE_GSN)) {
                    f |= ORC_FAULT_PRIOR_RESAMPLES;
                    break;
                }
            }
            double t3[ORC_MWG_MAXD]; /* θ as log_prior(::Previous) reads it */
            if (u->kind == 5 || u->kind == 4) {
                /* transition densities done above (MALA's reverse one after compute_ll!) */
            } else if (u->kind == 3) {
                /* logpdf(rw::GaussianRandomWalkMix, a, b) = log((1−λ)·exp(logpdf(gsn_A, a, b)) +
                 * λ·exp(logpdf(gsn_B, a, b))) (random_walk.jl:229-232), each component's logpdf
                 * with its own round trips on a and b; ltd(__PROPOSAL) = logpdf(rw, θ°, θ) is
                 * evaluated first (run.jl:271-277) */
                const double lam = ext->mix_lam[p];
                const double *Lb = ext->LB + ext->off_sq[p] + c * (uint64_t)n * n;
                double iLb[ORC_MWG_MAXD], c0b;
                mix_factor_consts(Lb, (int)n, iLb, &c0b);
                double a[ORC_MWG_MAXD], b[ORC_MWG_MAXD];
                for (uint32_t i = 0; i < n; ++i) {
                    a[i] = tp[i];                                                 /* θ°₁ */
                    b[i] = u->pos[i] ? orc_exp_any(orc_log_any(tl[i])) : tl[i];  /* θ₁ */
                }
                for (int dir = 0; dir < 2; ++dir) {
                    const double lpA = orc_gsn_rw_lp(u->L, u->iL, u->c0, u->diag, u->pos, n, anypos, a, b);
                    const double lpB = orc_gsn_rw_lp(Lb, iLb, c0b, 0, u->pos, n, anypos, a, b);
                    const double t = orc_log_any((1.0 - lam) * orc_exp_any(lpA) + lam * orc_exp_any(lpB));
                    if (dir == 0) ltd_rev = t;
                    else ltd_fwd = t;
                    for (uint32_t i = 0; i < n; ++i) { /* the second call is logpdf(rw, θ, θ°) */
                        const double tmp = a[i];
                        a[i] = b[i];
                        b[i] = tmp;
                    }
                }
                if (anypos) { /* two swaps: a is θ° again, b is θ */
                    for (uint32_t i = 0; i < n; ++i) {
                        ta[i] = a[i]; /* θ°₅, what set_chain_param! copies */
                        t3[i] = b[i]; /* θ₅, what log_prior(::Previous) reads */
                    }
                    accept_ta = 1;
                }
            } else if (u->kind == 1) {
                /* logpdf(rw, θ, θ°) (subtracted) and logpdf(rw, θ°, θ) (added), left folds */
                for (uint32_t j = 0; j < n; ++j) {
                    const double c = u->pos[j] ? -orc_log_any(2.0 * ep[j]) : 0.0;
                    const double f1 = u->pos[j] ? c - orc_log_any(tp[j]) : 0.0;
                    const double g2 = u->pos[j] ? c - orc_log_any(tl[j]) : 0.0;
                    ltd_fwd = (j == 0) ? f1 : ltd_fwd + f1;
                    ltd_rev = (j == 0) ? g2 : ltd_rev + g2;
                }
            } else {
                double r[ORC_MWG_MAXD];
                if (!anypos) {
                    for (uint32_t i = 0; i < n; ++i) r[i] = tp[i] - tl[i];
                    ltd_fwd = u->c0 - sqmahal(u->L, u->iL, r, (int)n, u->diag) / 2.0;
                    for (uint32_t i = 0; i < n; ++i) r[i] = tl[i] - tp[i];
                    ltd_rev = u->c0 - sqmahal(u->L, u->iL, r, (int)n, u->diag) / 2.0;
                } else {
                    /* rand (random_walk.jl:145-151): θ°₁ = exp(log θ + Lz), θ₁ = exp(log θ)
                     * (reimpose_constraints! on both, in place);
                     * logpdf(rw, θ°₁, θ₁) (:166-171): logJ = −sum(log θ₁[pos]),
                     * logpdf(MvNormal(log θ°₁, Σ), log θ₁) + logJ, then θ°₂ = exp(log θ°₁),
                     * θ₂ = exp(log θ₁); logpdf(rw, θ₂, θ°₂) likewise, then
                     * θ°₃ = exp(log θ°₂), the value set_chain_param! copies on accept,
                     * and θ₃ = exp(log θ₂), the θ log_prior(::Previous) reads */
                    double t1[ORC_MWG_MAXD], a1[ORC_MWG_MAXD], b1[ORC_MWG_MAXD], lj = 0.0;
                    int first = 1;
                    for (uint32_t i = 0; i < n; ++i) {
                        t1[i] = u->pos[i] ? orc_exp_any(orc_log_any(tl[i])) : tl[i];
                        if (u->pos[i]) {
                            const double v = orc_log_any(t1[i]);
                            lj = first ? v : lj + v;
                            first = 0;
                        }
                        a1[i] = u->pos[i] ? orc_log_any(tp[i]) : tp[i];
                        b1[i] = u->pos[i] ? orc_log_any(t1[i]) : t1[i];
                        r[i] = b1[i] - a1[i];
                    }
                    ltd_rev = (u->c0 - sqmahal(u->L, u->iL, r, (int)n, u->diag) / 2.0) + (-lj);
                    lj = 0.0;
                    first = 1;
                    for (uint32_t i = 0; i < n; ++i) {
                        const double p2 = u->pos[i] ? orc_exp_any(a1[i]) : a1[i];
                        const double l2 = u->pos[i] ? orc_exp_any(b1[i]) : b1[i];
                        if (u->pos[i]) {
                            const double v = orc_log_any(p2);
                            lj = first ? v : lj + v;
                            first = 0;
                        }
                        const double a2 = u->pos[i] ? orc_log_any(l2) : l2;
                        const double b2 = u->pos[i] ? orc_log_any(p2) : p2;
                        r[i] = b2 - a2;
                        ta[i] = u->pos[i] ? orc_exp_any(b2) : p2;
                        t3[i] = u->pos[i] ? orc_exp_any(a2) : l2;
                    }
                    ltd_fwd = (u->c0 - sqmahal(u->L, u->iL, r, (int)n, u->diag) / 2.0) + (-lj);
                    accept_ta = 1;
                }
            }
            /* log_prior(::Proposal) − log_prior(::Previous) of the local states (run.jl:374-385) */
            double lpp = 0.0, lpc = 0.0;
            if (u->prior != ORC_PRIOR_IMPROPER) {
                lpp = orc_mwg_log_prior(u, n, accept_ta ? ta : tp);
                lpc = orc_mwg_log_prior(u, n, accept_ta ? t3 : tl);
            }
            /* set_proposal!: history θ with coords ← θ°; P°.θ[coords] ← θ° */
            double prop[ORC_MWG_MAXD];
            memcpy(prop, th, sizeof(double) * D);
            for (uint32_t j = 0; j < n; ++j) {
                prop[u->coords[j]] = tp[j];
                mp[u->coords[j]] = tp[j];
            }
            /* compute_ll!: loglikelihood(P°, obs) */
            double llp, r[ORC_MWG_MAXD];
            if (user_ll) {
                llp = user_ll(mp, D, obs, nobs, user_params);
            } else if (g->ll_mode == 0) {
                llp = 0.0;
                for (uint64_t kk = 0; kk < nobs; ++kk) {
                    for (int i = 0; i < D; ++i) r[i] = obs[kk * D + i] - mp[i];
                    llp = llp + (g->t_c0 - sqmahal(g->Lt, g->iLt, r, D, tdiag) / 2.0);
                }
            } else {
                for (int i = 0; i < D; ++i) r[i] = g->xbar[i] - mp[i];
                const double qv = sqmahal(g->Lt, g->iLt, r, D, tdiag);
                llp = (double)nobs * g->t_c0 - (g->S_c + (double)nobs * qv) * 0.5;
            }
            if (u->kind == 4) {
                /* compute_gradients_and_momenta!(__PROPOSAL) (run.jl:259) at P°.θ:
                 * ltd_rev = logpdf(MvNormal(θ° + h·g°, ϵ²I), θ) */
                double gg[ORC_MWG_MAXD], rr[ORC_MWG_MAXD];
                if (user_ll) ext->user_grad(mp, D, obs, nobs, user_params, gg);
                else orc_gsn_grad(g, D, tdiag, mp, gg);
                for (uint32_t j = 0; j < n; ++j) rr[j] = tl[j] - (tp[j] + mala_h * gg[u->coords[j]]);
                ltd_rev = u->c0 - sqmahal(u->L, u->iL, rr, (int)n, 1) / 2.0;
            }
            if (!isfinite(llp)) f |= 1u;
            if (ll_prop) ll_prop[(size_t)p * C + c] = llp;
            const double llr = ((((llp - cll) + ltd_rev) - ltd_fwd) + lpp) - lpc;
            const double E = orc_exponential(zt, k0, k1, chain_id, iter, p, &f);
            const int acc = E > -llr;
            if (hist_prop) memcpy(hist_prop + ((uint64_t)s * C + c) * D, prop, sizeof(double) * D);
            if (acc) { /* set_chain_param!: θ[coords] ← θ° of the local workspace (run.jl:312-318) */
                for (uint32_t j = 0; j < n; ++j) th[u->coords[j]] = accept_ta ? ta[j] : tp[j];
                cll = llp;
                nacc[(size_t)p * C + c] += 1;
            }
            if (hist_theta) memcpy(hist_theta + ((uint64_t)s * C + c) * D, th, sizeof(double) * D);
            if (hist_ll) hist_ll[(uint64_t)s * C + c] = cll;
            if (hist_acc) hist_acc[(uint64_t)s * C + c] = (uint8_t)acc;
            /* update_stats! rolling acceptance of update p */
            {
                const uint64_t N = N_start + s;
                uint64_t *rg = ring + ((size_t)p * C + c) * 2;
                int outside = 0;
                if (iter > W) {
                    uint32_t j = (iter - W) & 127u;
                    outside = (int)((((j & 64u) ? rg[1] : rg[0]) >> (j & 63u)) & 1u);
                }
                const double ra_prev = (iter > 1 && last[p] == iter - 1) ? ra[(size_t)p * C + c] : 0.0;
                const uint64_t mn = N < (uint64_t)W ? N : (uint64_t)W;
                ra[(size_t)p * C + c] = (ra_prev * (double)W + (double)(acc - outside)) / (double)mn;
                uint32_t j = iter & 127u;
                uint64_t bit = 1ull << (j & 63u);
                if (j & 64u) rg[1] = acc ? (rg[1] | bit) : (rg[1] & ~bit);
                else rg[0] = acc ? (rg[0] | bit) : (rg[0] & ~bit);
                last[p] = iter;
            }
            /* update_adaptation!: only the update whose turn it is registers */
            if (u->adapt == 1) {
                uint32_t *pr = aprop + (size_t)p * C + c, *ac = aacc + (size_t)p * C + c;
                *ac += (uint32_t)acc;
                *pr += 1;
                if (*pr >= u->k) {
                    /* δ = scale/√max(1, iter/k − offset) and the clamp, per coordinate
                     * (adaptation.jl:312-329; the scalar form repeats its values) */
                    const double a_r = (*pr == 0) ? 0.0 : (double)*ac / (double)*pr;
                    *pr = 0;
                    *ac = 0;
                    for (uint32_t j = 0; j < n; ++j) {
                        const double delta =
                            u->scale[j] / sqrt(fmax(1.0, (double)iter / (double)u->k - u->offset[j]));
                        const double step = (a_r > u->target) ? delta : -delta;
                        double e = ep[j] + step;
                        e = e < u->amax[j] ? e : u->amax[j];
                        ep[j] = e > u->amin[j] ? e : u->amin[j];
                    }
                }
            }
            if (ext) {
                const uint64_t N = N_start + s;
                /* update_stats!: GenericChainStats mean/cov of the whole θ after every
                 * update (chain_statistics.jl:46-49), before update_adaptation! */
                if (ext->chain_moments) orc_rank1_register(ext->smean + c * D, ext->scov + c * D * D, th, D, N);
                /* update_adaptation! (run.jl:136-178): every HaarioTypeAdaptation registers on
                 * every step — register_only_on_my_turn is false both ways (adaptation.jl:399-404)
                 * — the global θ at its coordinates, log-transformed where pos and transformed
                 * back in place (remove/reimpose_constraints! on the view, :407,412); M += 1
                 * and the readjust only on its own turn */
                for (uint32_t q = 0; q < P; ++q) {
                    const uint32_t hk = ext->haario_k ? ext->haario_k[q] : 0u;
                    if (!hk) continue;
                    const orc_mwg_update *v = &U[q];
                    const uint32_t nq = v->nc;
                    double x[ORC_MWG_MAXD];
                    for (uint32_t j = 0; j < nq; ++j) {
                        const double t = th[v->coords[j]];
                        x[j] = v->pos[j] ? orc_log_any(t) : t;
                    }
                    double *hm = ext->hmean + ext->off_v[q] + c * (uint64_t)nq;
                    double *hc = ext->hcov + ext->off_sq[q] + c * (uint64_t)nq * nq;
                    orc_rank1_register(hm, hc, x, nq, N);
                    for (uint32_t j = 0; j < nq; ++j)
                        if (v->pos[j]) th[v->coords[j]] = orc_exp_any(x[j]);
                    if (q == p && ++Mloc[q] >= hk) { /* time_to_update: readjust!(rw, adpt, iter) */
                        Mloc[q] = 0;
                        const double sB = (2.38 * 2.38) / (double)nq; /* 2.38^2/length(rw) */
                        double S[ORC_MWG_MAXD * ORC_MWG_MAXD], Ln[ORC_MWG_MAXD * ORC_MWG_MAXD];
                        for (uint32_t i = 0; i < nq; ++i)
                            for (uint32_t j = 0; j < nq; ++j) S[(size_t)j * nq + i] = sB * hc[(size_t)i * nq + j];
                        if (orc_cholesky(S, (int)nq, Ln))
                            f |= ORC_FAULT_POSDEF;
                        else
                            memcpy(ext->LB + ext->off_sq[q] + c * (uint64_t)nq * nq, Ln, sizeof(double) * nq * nq);
                    }
                }
            }
        }
        memcpy(theta + c * D, th, sizeof(double) * D);
        memcpy(mu_p + c * D, mp, sizeof(double) * D);
        ll[c] = cll;
        faults[c] = f;
    }
    *N_io = N_start + nsteps;
    for (uint32_t s = 0; s < nsteps; ++s) last_iter_io[step_pidx[s] - 1] = step_iter[s];
    if (ext && ext->M_io && ext->haario_k) /* M advances by the own-turn steps, uniform over chains */
        for (uint32_t s = 0; s < nsteps; ++s) {
            const uint32_t q = step_pidx[s] - 1;
            if (ext->haario_k[q] && ++ext->M_io[q] >= ext->haario_k[q]) ext->M_io[q] = 0;
        }
    free(g);
    free(U);
    return 0;
}

/* ---- GaussianRandomWalkMix + HaarioTypeAdaptation + GenericChainStats mean/cov
 *
 * One joint update (P = 1) on coords 1:D, BASELINE cfg 4.  Restated from
 * (src/ under /root/reference):
 *   pick_kernel: B iff rand() ≤ λ (Bernoulli(λ)) ........ random_walk.jl:225-227
 *   rand(gsn_X, θ): θ° = θ + L_X z ........................ random_walk.jl:145-151
 *   logpdf(mix) = log((1−λ)·exp(lp_A) + λ·exp(lp_B)),
 *   lp_X = logpdf(MvNormal(θ, Σ_X), θ°) + logJ (logJ = −0.0 without
 *   positivity constraints, so the addition is the identity) .. random_walk.jl:161-171,
 *                                                              229-232
 *   update_stats!: running mean/cov, phantom zero sample
 *   (N = 1, mean = 0, cov = 0 at construction) ............ chain_statistics.jl:23-49
 *   HaarioTypeAdaptation: M += 1 on its own turn, register! θ with the same
 *   rank-one recurrence (so for P = 1 its mean/cov equal the chain-stats
 *   mean/cov and are kept once), readjust at M ≥ k:
 *   Σ_B = 2.38²/D·cov, λ = fλ(λ, N, iter) (identity) ...... adaptation.jl:399-426
 * cholesky(Symmetric(Σ_B)) of the next MvNormal throws PosDefException in the
 * reference; here the chain's EMCMC fault bit 4 is set and L_B stays as it was.
 *
 * mix = 0: plain GaussianRandomWalk(Σ_A) with on-device chain moments (bitwise
 * the orc_run_gsn chain plus mean/cov).  haario requires mix.
 * State: mean [C][D], cov [C][D][D] (symmetric, row-major), LB [C][D][D]
 * (lower, row-major) in/out; *N_io = GenericChainStats.N (= Haario N),
 * *M_io = Haario M (uniform over chains).
 */

ORC_EXPORT int orc_run_mix(int D, uint64_t C, uint32_t chain0, uint64_t seed, const double *sigma_a, int mix,
                           double lam, int haario, uint32_t k, const double *t_sigma, uint64_t nobs,
                           const double *obs, int ll_mode, uint32_t W, uint32_t iter0, uint32_t nsteps,
                           uint64_t *N_io, uint32_t *M_io, double *theta, double *ll, double *ra, uint64_t *ring,
                           uint32_t *nacc, uint32_t *faults, double *mean, double *cov, double *LB,
                           double *hist_theta, double *hist_prop, double *hist_ll, uint8_t *hist_acc,
                           int nthreads) {
    if (D < 1 || D > 64 || (haario && (!mix || k < 1))) return -2;
    orc_gsn *g = (orc_gsn *)malloc(sizeof(orc_gsn));
    if (!g) return -3;
    (void)zig();
    int rc = gsn_prepare(g, D, sigma_a, t_sigma, nobs, obs, ll_mode);
    if (rc) {
        free(g);
        return rc;
    }
    const int adiag = is_diag_upper(sigma_a, D);
    const int tdiag = is_diag_upper(t_sigma, D);
    const uint32_t k0 = (uint32_t)seed, k1 = (uint32_t)(seed >> 32);
    const orc_zig_tables *zt = zig();
    const uint64_t N0 = *N_io;
    const uint32_t M0 = *M_io;
    const double sB = (2.38 * 2.38) / (double)D; /* 2.38^2/length(rw) */
#ifdef _OPENMP
#pragma omp parallel for schedule(static) num_threads(nthreads > 0 ? nthreads : 1)
#endif
    for (int64_t ci = 0; ci < (int64_t)C; ++ci) {
        const uint64_t c = (uint64_t)ci;
        const uint32_t gid = chain0 + (uint32_t)c;
        double th[64], thp[64], z[64], r[64], m[64], iLB[64], c0B = 0.0;
        double *cv = cov + c * D * D, *Lb = LB + c * D * D;
        memcpy(th, theta + c * D, sizeof(double) * D);
        memcpy(m, mean + c * D, sizeof(double) * D);
        double cll = ll[c], cra = ra[c];
        uint64_t ring0 = ring[2 * c], ring1 = ring[2 * c + 1];
        uint32_t na = nacc[c], f = faults[c], M = M0;
        if (mix) mix_factor_consts(Lb, D, iLB, &c0B);
        for (uint32_t s = 0; s < nsteps; ++s) {
            const uint32_t iter = iter0 + s;
            const uint64_t N = N0 + s;
            /* proposal!: pick, then θ° = θ + L z */
            int useB = 0;
            if (mix) {
                const orc_u32x4 pr = orc_draw(k0, k1, gid, iter, 0xFFFFFFFEu, 0, 0);
                useB = orc_u01_closed0(pr.v[0], pr.v[1]) <= lam;
            }
            for (int j = 0; j < D; ++j) z[j] = orc_normal(zt, k0, k1, gid, iter, 0, (uint32_t)j, &f);
            for (int i = 0; i < D; ++i) {
                double lz;
                if (useB) {
                    lz = Lb[(size_t)i * D] * z[0];
                    for (int j = 1; j <= i; ++j) lz = fma(Lb[(size_t)i * D + j], z[j], lz);
                } else if (adiag) {
                    lz = g->Lrw[(size_t)i * D + i] * z[i];
                } else {
                    lz = g->Lrw[(size_t)i * D] * z[0];
                    for (int j = 1; j <= i; ++j) lz = fma(g->Lrw[(size_t)i * D + j], z[j], lz);
                }
                thp[i] = th[i] + lz;
            }
            /* log_transition_density both ways */
            double t_fwd = 0.0, t_rev = 0.0;
            for (int dir = 0; dir < 2; ++dir) {
                for (int i = 0; i < D; ++i) r[i] = dir ? th[i] - thp[i] : thp[i] - th[i];
                const double lpA = g->rw_c0 - sqmahal(g->Lrw, g->iLrw, r, D, adiag) / 2.0;
                double t = lpA;
                if (mix) {
                    const double lpB = c0B - sqmahal(Lb, iLB, r, D, 0) / 2.0;
                    t = orc_log_any((1.0 - lam) * orc_exp_any(lpA) + lam * orc_exp_any(lpB));
                }
                if (dir) t_rev = t;
                else t_fwd = t;
            }
            /* compute_ll! */
            double llp;
            if (g->ll_mode == 0) {
                llp = 0.0;
                for (uint64_t kk = 0; kk < nobs; ++kk) {
                    for (int i = 0; i < D; ++i) r[i] = obs[kk * D + i] - thp[i];
                    llp = llp + (g->t_c0 - sqmahal(g->Lt, g->iLt, r, D, tdiag) / 2.0);
                }
            } else {
                for (int i = 0; i < D; ++i) r[i] = g->xbar[i] - thp[i];
                const double qv = sqmahal(g->Lt, g->iLt, r, D, tdiag);
                llp = (double)nobs * g->t_c0 - (g->S_c + (double)nobs * qv) * 0.5;
            }
            if (!isfinite(llp)) f |= 1u;
            const double llr = ((((llp - cll) + t_rev) - t_fwd) + 0.0) - 0.0;
            const double E = orc_exponential(zt, k0, k1, gid, iter, 0, &f);
            const int acc = E > -llr;
            if (hist_prop) memcpy(hist_prop + ((uint64_t)s * C + c) * D, thp, sizeof(double) * D);
            if (acc) {
                memcpy(th, thp, sizeof(double) * D);
                cll = llp;
                na += 1;
            }
            if (hist_theta) memcpy(hist_theta + ((uint64_t)s * C + c) * D, th, sizeof(double) * D);
            if (hist_ll) hist_ll[(uint64_t)s * C + c] = cll;
            if (hist_acc) hist_acc[(uint64_t)s * C + c] = (uint8_t)acc;
            /* update_stats!: running mean/cov of θ (chain_statistics.jl:46-49) */
            {
                const double a = (double)(N - 1) / (double)N;
                const double b = (double)N / (double)(N + 1);
                const double cN = (double)(N + 1) / (double)N;
                double mo[64];
                memcpy(mo, m, sizeof(double) * D);
                for (int i = 0; i < D; ++i) m[i] = m[i] * b + th[i] / (double)(N + 1);
                for (int i = 0; i < D; ++i)
                    for (int j = 0; j < D; ++j) {
                        const double old_sq = a * cv[(size_t)i * D + j] + mo[i] * mo[j];
                        const double new_sq = old_sq + (th[i] * th[j]) / (double)N;
                        cv[(size_t)i * D + j] = new_sq - cN * (m[i] * m[j]);
                    }
            }
            /* rolling acceptance (chain_statistics.jl:51-64) */
            {
                int outside = 0;
                if (iter > W) {
                    uint32_t j = (iter - W) & 127u;
                    outside = (int)((((j & 64u) ? ring1 : ring0) >> (j & 63u)) & 1u);
                }
                const uint64_t mn = N < (uint64_t)W ? N : (uint64_t)W;
                cra = (cra * (double)W + (double)(acc - outside)) / (double)mn;
                uint32_t j = iter & 127u;
                uint64_t bit = 1ull << (j & 63u);
                if (j & 64u) ring1 = acc ? (ring1 | bit) : (ring1 & ~bit);
                else ring0 = acc ? (ring0 | bit) : (ring0 & ~bit);
            }
            /* update_adaptation!: Haario M, readjust at M ≥ k */
            if (haario) {
                M += 1;
                if (M >= k) {
                    M = 0;
                    double S[64 * 64], Ln[64 * 64];
                    for (int i = 0; i < D; ++i)
                        for (int j = 0; j < D; ++j) S[(size_t)j * D + i] = sB * cv[(size_t)i * D + j];
                    if (orc_cholesky(S, D, Ln)) {
                        f |= ORC_FAULT_POSDEF;
                    } else {
                        memcpy(Lb, Ln, sizeof(double) * (size_t)D * D);
                        mix_factor_consts(Lb, D, iLB, &c0B);
                    }
                }
            }
        }
        memcpy(theta + c * D, th, sizeof(double) * D);
        memcpy(mean + c * D, m, sizeof(double) * D);
        ll[c] = cll;
        ra[c] = cra;
        ring[2 * c] = ring0;
        ring[2 * c + 1] = ring1;
        nacc[c] = na;
        faults[c] = f;
    }
    *N_io = N0 + nsteps;
    if (haario) *M_io = (uint32_t)((M0 + nsteps) % k);
    (void)nthreads;
    free(g);
    return 0;
}

/* ---- MALA on a logistic-regression target (row f2, BASELINE cfg 3) ----------
 *
 * The reference stubs MALAUpdate (updates.jl:216-218, "✗" at updates.jl:7) and
 * provides the hook a gradient-based update uses: compute_gradients_and_momenta!
 * on the current state (run.jl:110, __PREVIOUS) and on the proposal (run.jl:259,
 * __PROPOSAL).  No reference numbers exist ("parity unpinned" against the
 * reference): this is the engine's definition, checked against the literal numpy
 * restatement (oracle/literal.py run_mala_chain).
 *   target     ℓ(θ) = Σ_n [y_n η_n − log(1 + e^{η_n})], η = Xθ; ∇ℓ = Xᵀ(y − σ(η))
 *   proposal   m = θ + h∇ℓ(θ), θ° = m + ϵz, h = ϵ²/2, z ~ N(0, I)
 *   transition logpdf(MvNormal(m, ϵ²I), θ°) and back with m° = θ° + h∇ℓ(θ°)
 *   accept     the reference's left-associative llr, E ~ Exp(1) > −llr (run.jl:268-281)
 * ∇ℓ is carried with the state like ll (the __PREVIOUS hook's value is the
 * gradient of the current state); it is evaluated once at θinit.
 * Evaluation orders (the device's, see emcmc_mala.h):
 *   η_n   = fma chain over d = 0..D−1 from 0.0 (v_mfma_f64_16x16x4f64 is an fma
 *           chain over its k, scripts/ubench/mfma_f64_probe.hip)
 *   ∇ℓ_d  = fma chain over n = 0..N−1 from 0.0
 *   ℓ     = (S_0 + S_1) + (S_2 + S_3), S_g = Σ_{n ≡ g mod 4} ℓ_n in increasing n
 *   ‖v‖²  = (s_0 + s_1) + (s_2 + s_3), s_g = v_g² then fma over d ≡ g mod 4 ascending
 *   t = e^{−|η|} (orc_exp_le0), u = 1 + t, log(u) and v ≈ 1/u (≤ 2 ulp, no
 *   division) by orc_log_rcp_1_2,
 *   log1p(t) = t if u == 1 else log(u) − ((u − 1) − t)·v,
 *   softplus(η) = max(η, 0) + log1p(t), σ(η) = (η ≥ 0 ? 1 : t)·v.
 */
static inline void orc_logistic_terms(double eta, double y, double *ell, double *r) {
    const double t = orc_exp_le0(-fabs(eta));
    const double u = 1.0 + t;
    double v;
    const double lu = orc_log_rcp_1_2(u, &v);
    const double lp1 = (u == 1.0) ? t : lu - ((u - 1.0) - t) * v;
    const double sp = (eta > 0.0 ? eta : 0.0) + lp1;
    const double sig = (eta >= 0.0 ? 1.0 : t) * v;
    *ell = y * eta - sp;
    *r = y - sig;
}

static double orc_sq4(const double *v, int D) {
    double s[4] = {0.0, 0.0, 0.0, 0.0};
    for (int g = 0; g < 4 && g < D; ++g) {
        s[g] = v[g] * v[g];
        for (int d = g + 4; d < D; d += 4) s[g] = fma(v[d], v[d], s[g]);
    }
    return (s[0] + s[1]) + (s[2] + s[3]);
}

static void orc_logistic_eval(const double *X, const double *y, uint64_t N, int D, const double *th, double *ll,
                              double *G) {
    double S[4] = {0.0, 0.0, 0.0, 0.0};
    for (int d = 0; d < D; ++d) G[d] = 0.0;
    for (uint64_t n = 0; n < N; ++n) {
        const double *x = X + n * (uint64_t)D;
        double eta = 0.0;
        for (int d = 0; d < D; ++d) eta = fma(x[d], th[d], eta);
        double ell, r;
        orc_logistic_terms(eta, y[n], &ell, &r);
        S[n & 3] = S[n & 3] + ell;
        for (int d = 0; d < D; ++d) G[d] = fma(x[d], r, G[d]);
    }
    *ll = (S[0] + S[1]) + (S[2] + S[3]);
}

/* ℓ and ∇ℓ at theta [C][D] → ll [C] (may be NULL), grad [C][D]. */
ORC_EXPORT void orc_logistic_eval_batch(int D, uint64_t C, const double *X, const double *y, uint64_t N,
                                        const double *theta, double *ll, double *grad, int nthreads) {
#ifdef _OPENMP
#pragma omp parallel for schedule(static) num_threads(nthreads > 0 ? nthreads : 1)
#endif
    for (int64_t c = 0; c < (int64_t)C; ++c) {
        double l;
        orc_logistic_eval(X, y, N, D, theta + (uint64_t)c * D, &l, grad + (uint64_t)c * D);
        if (ll) ll[c] = l;
    }
    (void)nthreads;
}

ORC_EXPORT int orc_run_mala(int D, uint64_t C, uint32_t chain0, uint64_t seed, double eps, const double *X,
                            const double *y, uint64_t N, uint32_t W, uint32_t iter0, uint32_t nsteps, uint64_t N0,
                            double *theta, double *grad, double *ll, double *ra, uint64_t *ring, uint32_t *nacc,
                            uint32_t *faults, double *hist_theta, double *hist_prop, double *hist_ll,
                            uint8_t *hist_acc, int nthreads) {
    if (D < 1 || D > 64 || !(eps > 0.0)) return -2;
    (void)zig();
    const uint32_t k0 = (uint32_t)seed, k1 = (uint32_t)(seed >> 32);
    const orc_zig_tables *zt = zig();
    const double h = (eps * eps) / 2.0, ie = 1.0 / eps;
    double dd = 0.0;
    for (int d = 0; d < D; ++d) dd = dd + orc_log(eps);
    const double c0 = mvnormal_c0(D, dd + dd);
#ifdef _OPENMP
#pragma omp parallel for schedule(dynamic, 1) num_threads(nthreads > 0 ? nthreads : 1)
#endif
    for (int64_t ci = 0; ci < (int64_t)C; ++ci) {
        const uint64_t c = (uint64_t)ci;
        const uint32_t gid = chain0 + (uint32_t)c;
        double th[64], g[64], tp[64], gp[64], m[64], v[64];
        memcpy(th, theta + c * D, sizeof(double) * D);
        memcpy(g, grad + c * D, sizeof(double) * D);
        double cll = ll[c], cra = ra[c];
        uint64_t ring0 = ring[2 * c], ring1 = ring[2 * c + 1];
        uint32_t na = nacc[c], f = faults[c];
        for (uint32_t s = 0; s < nsteps; ++s) {
            const uint32_t iter = iter0 + s;
            for (int d = 0; d < D; ++d) {
                const double z = orc_normal(zt, k0, k1, gid, iter, 0, (uint32_t)d, &f);
                m[d] = th[d] + h * g[d];
                tp[d] = m[d] + eps * z;
                v[d] = (tp[d] - m[d]) * ie;
            }
            const double ltd_fwd = c0 - orc_sq4(v, D) / 2.0;
            double llp;
            orc_logistic_eval(X, y, N, D, tp, &llp, gp);
            for (int d = 0; d < D; ++d) v[d] = (th[d] - (tp[d] + h * gp[d])) * ie;
            const double ltd_rev = c0 - orc_sq4(v, D) / 2.0;
            if (!isfinite(llp)) f |= 1u;
            const double llr = ((((llp - cll) + ltd_rev) - ltd_fwd) + 0.0) - 0.0;
            const double E = orc_exponential(zt, k0, k1, gid, iter, 0, &f);
            const int acc = E > -llr;
            if (hist_prop) memcpy(hist_prop + ((uint64_t)s * C + c) * D, tp, sizeof(double) * D);
            if (acc) {
                memcpy(th, tp, sizeof(double) * D);
                memcpy(g, gp, sizeof(double) * D);
                cll = llp;
                na += 1;
            }
            if (hist_theta) memcpy(hist_theta + ((uint64_t)s * C + c) * D, th, sizeof(double) * D);
            if (hist_ll) hist_ll[(uint64_t)s * C + c] = cll;
            if (hist_acc) hist_acc[(uint64_t)s * C + c] = (uint8_t)acc;
            {
                const uint64_t Nn = N0 + s;
                int outside = 0;
                if (iter > W) {
                    uint32_t j = (iter - W) & 127u;
                    outside = (int)((((j & 64u) ? ring1 : ring0) >> (j & 63u)) & 1u);
                }
                const uint64_t mn = Nn < (uint64_t)W ? Nn : (uint64_t)W;
                cra = (cra * (double)W + (double)(acc - outside)) / (double)mn;
                uint32_t j = iter & 127u;
                uint64_t bit = 1ull << (j & 63u);
                if (j & 64u) ring1 = acc ? (ring1 | bit) : (ring1 & ~bit);
                else ring0 = acc ? (ring0 | bit) : (ring0 & ~bit);
            }
        }
        memcpy(theta + c * D, th, sizeof(double) * D);
        memcpy(grad + c * D, g, sizeof(double) * D);
        ll[c] = cll;
        ra[c] = cra;
        ring[2 * c] = ring0;
        ring[2 * c + 1] = ring1;
        nacc[c] = na;
        faults[c] = f;
    }
    (void)nthreads;
    return 0;
}
