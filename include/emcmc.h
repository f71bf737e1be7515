/*
 * emcmc.h — C ABI of the MI355X many-chain MCMC engine (libemcmc.so).
 *
 * This is the drop-in boundary for the hot path of ExtensibleMCMC.jl
 * (reference: JuliaDiffusionBayes/ExtensibleMCMC.jl, mounted read-only at
 * /root/reference).  The reference has no FFI of its own: its extension point
 * is the `MCMCBackend` dispatch (src/types.jl:110-117) together with the
 * workspace/update plugin surface (src/workspaces.jl:38,280; src/updates.jl:42-93).
 * A Julia `MI355XBackend <: MCMCBackend` (extensiblemcmc.jl_amd/julia/) binds
 * these entry points with `ccall`; Python binds them with `ctypes`
 * (extensiblemcmc.jl_amd/extensible_mcmc/_lib.py).  See INTEGRATION.md.
 *
 * Each entry point names the reference function(s) it replaces.
 *
 * Conventions
 *  - Plain C: POD structs, plain pointers + sizes, `emcmc_status` return codes.
 *    Nothing throws across the ABI.  `emcmc_last_error(h)` gives a message.
 *  - Indices crossing the ABI are 0-based (coords) except `mcmciter`/`pidx` in
 *    `emcmc_step`, which are 1-based exactly as `MCMCSchedule` yields them
 *    (src/schedule.jl:56-66).
 *  - Matrices Σ are column-major (Julia layout); only the upper triangle is
 *    read, like `Symmetric(Σ)` (uplo = :U) in src/transition_kernels/random_walk.jl:132
 *    and `Symmetric(triu(Σ))` in src/example/gsn_target.jl:19.
 *  - Chain state crossing the ABI is row-major [C][D] (chain-major).
 *  - Ownership: the library owns all device memory; the caller owns host
 *    buffers and keeps them alive for the duration of the call.
 *  - Threading: one handle = one host thread + one HIP stream on one device.
 *    Handles are independent; there is no global mutable state (the RNG is
 *    counter-based, keyed by (seed, global chain id)).
 *  - `emcmc_run` is asynchronous (enqueue only); every `emcmc_get_*` call and
 *    `emcmc_synchronize` wait for it.
 */
#ifndef EMCMC_H
#define EMCMC_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define EMCMC_ABI_VERSION 2u  /* 2: emcmc_prior_factor gained components / mu / sigma (round 3) */

typedef enum emcmc_status {
    EMCMC_OK = 0,
    EMCMC_INVALID_ARG = 1,        /* reference: @assert / error("…") in constructors */
    EMCMC_HIP_ERROR = 2,
    EMCMC_RCCL_ERROR = 3,         /* RCCL missing or a collective failed (emcmc_comm_*, emcmc_diagnostics) */
    EMCMC_UNSUPPORTED_PLUGIN = 4, /* update/target kind with no device plugin */
    EMCMC_CHAIN_FAULT = 5,        /* ≥1 chain raised a fault bit (see emcmc_get_faults) */
    EMCMC_OUT_OF_MEMORY = 6,
    EMCMC_NO_DEVICE = 7,
    EMCMC_STATE_ERROR = 8         /* call out of order (e.g. run before set_target) */
} emcmc_status;

/* Transition kernels — src/transition_kernels/random_walk.jl */
#define EMCMC_RW_UNIFORM 1u       /* UniformRandomWalk        random_walk.jl:45-94  */
#define EMCMC_RW_GAUSSIAN 2u      /* GaussianRandomWalk       random_walk.jl:123-171 */
#define EMCMC_RW_GAUSSIAN_MIX 3u  /* GaussianRandomWalkMix    random_walk.jl:193-232 */
#define EMCMC_MALA 4u             /* MALAUpdate: a stub in the reference (updates.jl:216-218); the engine's
                                     definition is in DESIGN.md §2.  epsilon[0] = step size ϵ.  ∇ℓ is the
                                     target's compute_gradients_and_momenta! (updates.jl:123-133): on the
                                     logistic-regression target the fused MFMA kernel (one joint update,
                                     ImproperPrior); on GsnTargetLaw (built-in ∇) or a user law whose source
                                     defines EMCMC_USER_GRAD, the general kernel (any coords and prior, any
                                     schedule); a user law without one: EMCMC_UNSUPPORTED_PLUGIN */
#define EMCMC_USER_UPDATE 5u      /* a user-defined MCMCParamUpdate: its proposal! and log_transition_density
                                     (updates.jl:42-93, the methods an update MUST implement) as device source
                                     compiled at run time; emcmc_update_desc.user_update */

/* Priors — src/priors.jl.  Evaluated on the update's local coordinates
 * (log_prior, updates.jl:104; run.jl:374-385); proposal! draws θ° again while
 * logpdf(prior, θ°) === −Inf (updates.jl:191-196).  Non-improper priors run on
 * the general schedule kernel (D ≤ 64). */
#define EMCMC_PRIOR_IMPROPER 0u     /* ImproperPrior     priors.jl:18-19: 0.0 */
#define EMCMC_PRIOR_IMPROPER_POS 1u /* ImproperPosPrior  priors.jl:25-26: −sum(log.(θ)) */
#define EMCMC_PRIOR_PRODUCT 2u      /* ProductPrior(dists, dims) priors.jl:60-88.  The factors are `dists` with
                                       count = dims[k]; the engine builds the index list as the constructor does
                                       (priors.jl:64-79): a factor with dims 1 reads local θ[1] (index 1, not
                                       the next coordinate), a factor with dims k > 1 reads θ[last:last+k−1],
                                       last advancing by dims either way; then lp = 0.0; lp += logpdf(dist, θ[idx])
                                       in factor order.  dims 1 needs a univariate family, dims > 1 a multivariate
                                       one (EMCMC_DIST_PRODUCT / EMCMC_DIST_MVNORMAL): the other pairings raise a
                                       MethodError in the reference and EMCMC_UNSUPPORTED_PLUGIN here */
#define EMCMC_PRIOR_STANDARD 3u     /* StandardPrior(dist) priors.jl:35-39: logpdf(dist, θ_local), one factor, dist
                                       multivariate with count = num_coords (a univariate dist on the local vector
                                       raises in the reference: EMCMC_UNSUPPORTED_PLUGIN) */
/* Families of a prior factor (Distributions.jl parameterisations, StatsFuns forms) */
#define EMCMC_DIST_NORMAL 1u        /* Normal(μ = a, σ = b) */
#define EMCMC_DIST_UNIFORM 2u       /* Uniform(a, b) */
#define EMCMC_DIST_EXPONENTIAL 3u   /* Exponential(θ = a), the scale */
#define EMCMC_DIST_GAMMA 4u         /* Gamma(α = a, θ = b), shape and scale */
#define EMCMC_DIST_LOGNORMAL 5u     /* LogNormal(μ = a, σ = b) */
#define EMCMC_DIST_BETA 6u          /* Beta(α = a, β = b) */
#define EMCMC_DIST_INVERSE_GAMMA 7u /* InverseGamma(α = a, θ = b), shape and scale */
#define EMCMC_DIST_CAUCHY 8u        /* Cauchy(μ = a, σ = b) */
#define EMCMC_DIST_LAPLACE 9u       /* Laplace(μ = a, θ = b) */
#define EMCMC_DIST_TDIST 10u        /* TDist(ν = a) */
#define EMCMC_DIST_PRODUCT 32u      /* Product([d_1, …, d_k]) of univariates: `components`, k = count */
#define EMCMC_DIST_MVNORMAL 33u     /* MvNormal(μ, Σ) over count coordinates: `mu`, `sigma` */

/* Adaptation — src/transition_kernels/adaptation.jl */
#define EMCMC_ADPT_NONE 0u      /* NoAdaptation          adaptation.jl:26 */
#define EMCMC_ADPT_UNIF_RW 1u   /* AdaptationUnifRW      adaptation.jl:51-329 */
#define EMCMC_ADPT_HAARIO 2u    /* HaarioTypeAdaptation  adaptation.jl:372-426 (GaussianRandomWalkMix only) */
#define EMCMC_ADPT_UNIF_RW_VEC 3u /* AdaptationUnifRW with per-coordinate scale/min/max/offset (its nonscalar
                                     form, adaptation.jl:155-188); see emcmc_unifrw_adaptation_vec */

/* Targets — src/example/gsn_target.jl */
#define EMCMC_TARGET_GSN 1u     /* GsnTargetLaw(μ, Σ) with coords ⊆ μ */
#define EMCMC_TARGET_LOGISTIC 2u /* logistic regression: obs = X (n×d), labels = y (n), ℓ = Σ y·η − log(1+e^η) */
#define EMCMC_TARGET_USER 3u     /* a user law compiled at run time (emcmc_set_user_target) */

/* How the Gaussian log-likelihood Σ_k logpdf(N(μ,Σ), x_k) is evaluated. */
#define EMCMC_LL_PER_OBS 0u   /* literal gsn_target.jl:23-29: one sqmahal per observation */
#define EMCMC_LL_SUFFSTAT 1u  /* same quantity via Σ_k‖L⁻¹(x_k−x̄)‖² + n‖L⁻¹(x̄−μ)‖² */

/* History retention — src/workspaces.jl:157-192, 413-476 */
#define EMCMC_HIST_FULL 0u         /* state, proposal, ll and accept histories */
#define EMCMC_HIST_ACCEPT_ONLY 1u  /* accept bits only (no per-step state streams) */

/* History selectors for emcmc_get_history / emcmc_history_device_ptr.
 * Host copies (emcmc_get_history*) use the layouts below.  In HBM the STATE and
 * PROPOSAL histories are tiled pair-interleaved SoA per slot, which is what
 * emcmc_history_device_ptr exposes: with T = 32 when C is a multiple of 32 (else
 * T = C, one tile), c0 = c − c mod T, element (d, c) of slot s is at
 *   s·D·C + c0·D + ((d/2)·T + (c − c0))·2 + d%2   (even D)
 *   s·D·C + c0·D + d·T + (c − c0)                 (odd D). */
#define EMCMC_H_STATE 0u     /* state_history[iter][pidx]          : double [M][P][C][D] */
#define EMCMC_H_PROPOSAL 1u  /* state_proposal_history[iter][pidx] : double [M][P][C][D] */
#define EMCMC_H_LL 2u        /* local_wss[pidx].sub_ws.ll_history  : double [M][P][C]    */
#define EMCMC_H_ACCEPT 3u    /* local_wss[pidx].acceptance_history : bits   [M][P][ceil(C/64)] u64 */

/* Per-chain fault bits (emcmc_get_faults) */
#define EMCMC_FAULT_NONFINITE_LL 1u  /* proposal log-likelihood NaN/±Inf */
#define EMCMC_FAULT_RNG_RETRIES 2u   /* a ziggurat draw exhausted its 65,535 attempt counters */
#define EMCMC_FAULT_POSDEF 4u        /* Haario readjust: 2.38²/D·cov not positive definite.  The reference
                                        throws PosDefException at the next MvNormal(θ, Σ_B)
                                        (random_walk.jl:147,167); the chain keeps its previous Σ_B factor */
#define EMCMC_FAULT_PRIOR_RESAMPLES 8u /* proposal! drew 65,535 proposals outside the prior's support
                                          (the reference loops forever, updates.jl:193-195); the last
                                          draw is kept and rejected (llr = NaN or −Inf) */

typedef struct emcmc_handle emcmc_handle;

/* Engine configuration.  Mirrors what `init!(mcmc, …)` (src/mcmc.jl:83-109)
 * and `init_global_workspace` (src/workspaces.jl:215-234) receive. */
typedef struct emcmc_config {
    uint32_t abi_version;      /* must be EMCMC_ABI_VERSION */
    uint32_t dim;              /* D = length(θinit) */
    uint64_t num_chains;       /* C: chains held by this handle (one shard); C·dim·8 bytes ≤ 4 GiB − 1
                                  (the state and one history slot are addressed with 32-bit offsets) */
    uint64_t first_chain_id;   /* global id of local chain 0 (sharding; RNG key) */
    uint64_t num_mcmc_steps;   /* M: history length, run.jl:34 `num_mcmc_steps` */
    uint64_t seed;             /* master seed of the counter-based stream */
    int32_t device;            /* HIP device ordinal */
    uint32_t history_mode;     /* EMCMC_HIST_* */
    uint32_t roll_window;      /* GenericChainStats roll_window (chain_statistics.jl:27); 0 → 100; ≤ 128 */
    uint32_t lanes_per_chain;  /* 0 = auto; else 1, 2 or 4 (must divide the work layout) */
    uint32_t steps_per_launch; /* 0 = auto (64) */
    uint32_t kernel_variant;   /* 0 = auto; EMCMC_VARIANT_* tuning flags (results are identical) */
    uint32_t chain_moments;    /* 1 = keep GenericChainStats mean/cov (chain_statistics.jl:46-49) on
                                  device, after every update step of any schedule (always on with a
                                  single joint GaussianRandomWalkMix); read with emcmc_get_chain_moments */
    uint32_t history_ring;     /* iterations of history kept on device as a ring (0 = all num_mcmc_steps);
                                  older iterations are streamed out with emcmc_stream_history */
    uint32_t reserved[4];
} emcmc_config;

/* kernel_variant flags: performance-only choices among kernels the library keeps for other
 * shapes, bit-identical results (A/B timing).  Bits 1 and 2 selected register-capped builds of
 * the diagonal kernel that lost their A/B; they are retired and ignored. */
#define EMCMC_VARIANT_SCALAR_OBS 4u      /* diagonal Σ: one lane per chain, observations as SGPR operands */
#define EMCMC_VARIANT_MIX_STREAM 8u      /* GaussianRandomWalkMix: stream L_B from HBM every step (mix_gsn_kernel)
                                            instead of keeping it in registers (mix_res_kernel) */
#define EMCMC_VARIANT_NO_XCD_ORDER 16u   /* blocks in blockIdx order instead of one contiguous chain range per XCD */
#define EMCMC_VARIANT_NO_RTC_CHOL 32u    /* a correlated Σ at a D without an ahead-of-time rwm_gsn_chol_kernel runs on
                                            the general kernel instead of the chol kernel compiled at run time */
#define EMCMC_VARIANT_NO_MIX_CHOL 64u    /* GaussianRandomWalkMix / chain moments with a dense Σ_A or Σ_t at D = 16 or
                                            32: the general kernel instead of mix_chol_kernel */
#define EMCMC_VARIANT_UNCAPPED 128u      /* diagonal fused kernel without the 2-waves-per-SIMD register cap
                                            (D = 16, 32, 64 build it at MINW = 2 by default) */
#define EMCMC_VARIANT_NO_BLOCK 256u      /* one MALA / user update over all 17 ≤ D ≤ 64 coordinates, or a schedule
                                            of random-walk updates at 17 ≤ D ≤ 64: the general wide kernel
                                            instead of mwg_block_kernel / mwg_rw_block_kernel */
#define EMCMC_VARIANT_NO_FUSED_PRIOR 512u /* one update over all coordinates whose terms separate (diagonal
                                            GaussianRandomWalk or UniformRandomWalk with a Product of
                                            univariates / ImproperPosPrior): the schedule kernels instead of
                                            rwm_gsn_diag_kernel with those terms compiled in */

/* `AdaptationUnifRW(θ; adapt_every_k_steps, target_accpt_rate, scale, min,
 * max, offset)` in its scalar form (transition_kernels/adaptation.jl:51-118,
 * defaults 100, 0.234, 1.0, 1e-12, 1e7, 1e2).  Passed as
 * emcmc_update_desc.adaptation_params when adaptation == EMCMC_ADPT_UNIF_RW. */
typedef struct emcmc_unifrw_adaptation {
    uint32_t adapt_every_k_steps;
    uint32_t reserved;
    double target_accpt_rate;
    double scale;
    double min;
    double max;
    double offset;
} emcmc_unifrw_adaptation;

/* `AdaptationUnifRW(θ; scale = [...], min = ..., ...)` in its per-coordinate
 * form (AdaptationUnifRW{Vector{Float64}} / {SVector{N,Float64}},
 * adaptation.jl:155-188; the reference's constructor test, test/runtests.jl:65-84).
 * Each array has num_coords entries.  Passed as adaptation_params when
 * adaptation == EMCMC_ADPT_UNIF_RW_VEC.  The reference's readjust! evaluates
 * `scale/sqrt(max(1.0, iter/k - offset))` and `max.(min.(ϵ, max), min)`; with a
 * vector offset `Float64 - Vector` has no method in Julia 1.x, so the reference
 * stops with a MethodError at the first readjust.  The engine applies the
 * formula coordinate by coordinate: δ_i = scale_i/√max(1, iter/k − offset_i),
 * ϵ_i ← clamp(ϵ_i ± δ_i, min_i, max_i) — the scalar form's bits when all
 * entries are equal. */
typedef struct emcmc_unifrw_adaptation_vec {
    uint32_t adapt_every_k_steps;
    uint32_t reserved;
    double target_accpt_rate;
    const double *scale;
    const double *min;
    const double *max;
    const double *offset;
} emcmc_unifrw_adaptation_vec;

/* `HaarioTypeAdaptation(θ; adapt_every_k_steps, scale, f)` (adaptation.jl:372-397,
 * defaults 100, 2.38², identity).  Passed as emcmc_update_desc.adaptation_params
 * when adaptation == EMCMC_ADPT_HAARIO.  `scale` is carried but, as in the
 * reference, readjust! uses the literal 2.38² (adaptation.jl:423); fλ is the
 * identity unless emcmc_set_mix_lambda_fn installs one. */
typedef struct emcmc_haario_adaptation {
    uint32_t adapt_every_k_steps;
    uint32_t reserved;
    double scale;
} emcmc_haario_adaptation;

/* One factor of a ProductPrior (one of its `dists`, with its `dims` entry as
 * count) or the `dist` of a StandardPrior (count = its length). */
typedef struct emcmc_prior_factor {
    uint32_t family;      /* EMCMC_DIST_* */
    uint32_t count;       /* dims[k] (ProductPrior) / length(dist) (StandardPrior); 1 for a univariate */
    double a, b;          /* univariate parameters (EMCMC_DIST_* above) */
    const struct emcmc_prior_factor *components; /* EMCMC_DIST_PRODUCT: count univariate factors, else NULL */
    const double *mu;     /* EMCMC_DIST_MVNORMAL: μ, count doubles, else NULL */
    const double *sigma;  /* EMCMC_DIST_MVNORMAL: Σ, count² column-major (upper triangle read), else NULL */
} emcmc_prior_factor;

/* emcmc_update_desc.prior_params for EMCMC_PRIOR_PRODUCT / EMCMC_PRIOR_STANDARD:
 * the factors in the order given to the reference constructor. */
typedef struct emcmc_prior_desc {
    uint32_t num_factors;
    uint32_t reserved;
    const emcmc_prior_factor *factors;
} emcmc_prior_desc;

/* A user-defined update (EMCMC_USER_UPDATE): the reference's update plugin
 * surface (updates.jl:42-93) — `proposal!(updt, gws, ws, step)` writing
 * state°(ws) from state(ws), and `log_transition_density(updt, θ, θ°)` — as
 *
 *     EMCMC_USER_PROPOSAL {   // in scope: const double *theta (state(ws), n entries),
 *         …                   //   double *theta_prop (state°(ws), out), int n,
 *     }                       //   const double *params (num_params); em_randn(j), em_rand(j)
 *     EMCMC_USER_LTD {        // in scope: const double *x, const double *y, int n, params:
 *         return …;           //   log_transition_density(updt, x, y)
 *     }
 *
 * in the C subset both hiprtc and a C compiler accept (emcmc_user_target_desc's
 * rules; em_randn(j) = normal j, em_rand(j) = uniform [0, 1) j of the engine's
 * stream for (chain, mcmciter, update), j < 2^30).  The MH ratio adds
 * ltd(θ°, θ) − ltd(θ, θ°) and the prior as run.jl:268-281 does; set_parameters!
 * is P°.θ[coords] ← θ° (updates.jl:198-205).  Every user update of a handle
 * shares one source (updates differ by coords, params and prior); it runs on
 * the general schedule kernel, beside the built-in updates, with any target. */
typedef struct emcmc_user_update_desc {
    const char *source;   /* EMCMC_USER_PROPOSAL { … } EMCMC_USER_LTD { … } */
    const char *options;  /* extra hiprtc options, or NULL */
    uint64_t num_params;  /* ≤ 4096 */
    const double *params;
} emcmc_user_update_desc;

/* One `RandomWalkUpdate(rw, coords; prior, adpt)` (src/updates.jl:163-183).
 * Any number of updates, each on any coordinate subset (Metropolis-within-Gibbs,
 * BASELINE cfg 1 and the reference's own test, test/runtests.jl:87-114).  A single
 * GaussianRandomWalk update on coords 1:D without adaptation runs on the fused
 * kernels; a single GaussianRandomWalkMix update on coords 1:D (optionally with
 * HaarioTypeAdaptation, BASELINE cfg 4) runs on the mix kernels, which also keep
 * the chain moments; every other schedule runs on the general schedule kernel
 * (D ≤ 64). */
typedef struct emcmc_update_desc {
    uint32_t kernel;          /* EMCMC_RW_UNIFORM, EMCMC_RW_GAUSSIAN or EMCMC_RW_GAUSSIAN_MIX */
    uint32_t prior;           /* EMCMC_PRIOR_* */
    uint32_t adaptation;      /* EMCMC_ADPT_NONE, EMCMC_ADPT_UNIF_RW / EMCMC_ADPT_UNIF_RW_VEC
                                 (UniformRandomWalk) or EMCMC_ADPT_HAARIO (GaussianRandomWalkMix) */
    uint32_t num_coords;      /* length(coords) */
    const uint32_t *coords;   /* 0-based indices into θ (reference coords are 1-based), any order */
    const double *sigma;      /* GaussianRandomWalk Σ, GaussianRandomWalkMix Σ_A: num_coords² column-major */
    const double *epsilon;    /* UniformRandomWalk ϵ: num_coords */
    const uint8_t *pos;       /* positivity flags or NULL (all false): UniformRandomWalk (θ° = θ·e^U,
                                 random_walk.jl:63-94), GaussianRandomWalk and GaussianRandomWalkMix (log
                                 scale with the in-place round trips, random_walk.jl:136-232; D ≤ 64) */
    const void *adaptation_params; /* const emcmc_unifrw_adaptation* (EMCMC_ADPT_UNIF_RW),
                                      const emcmc_unifrw_adaptation_vec* (EMCMC_ADPT_UNIF_RW_VEC) or
                                      const emcmc_haario_adaptation* (EMCMC_ADPT_HAARIO) */
    const double *sigma_b;    /* GaussianRandomWalkMix Σ_B: num_coords² column-major */
    const emcmc_prior_desc *prior_params; /* EMCMC_PRIOR_PRODUCT / EMCMC_PRIOR_STANDARD factors, else NULL */
    const struct emcmc_user_update_desc *user_update; /* EMCMC_USER_UPDATE: its source and parameters, else NULL */
    double mix_lambda;        /* GaussianRandomWalkMix λ ∈ [0, 1] (B is picked iff rand() ≤ λ) */
    double reserved_f64[3];
} emcmc_update_desc;

/* `data = (P = GsnTargetLaw(μ, Σ), obs = [x_1, …, x_n])` (src/example/gsn_target.jl:1-29,
 * docs/src/get_started/basic_use.md:112). */
typedef struct emcmc_target_desc {
    uint32_t kind;        /* EMCMC_TARGET_GSN or EMCMC_TARGET_LOGISTIC (the MALA update's target) */
    uint32_t dim;         /* d = length(μ) */
    const double *mu;     /* μ at construction: P.θ[1:d] */
    const double *sigma;  /* Σ: d×d column-major (upper triangle read) */
    uint64_t num_obs;     /* n */
    const double *obs;    /* n×d row-major: obs[k*d + i] = x_k[i] */
    uint32_t ll_mode;     /* EMCMC_LL_* (GSN) */
    uint32_t reserved;
    const double *labels; /* EMCMC_TARGET_LOGISTIC: y, n doubles (0/1 or any real) */
} emcmc_target_desc;

/* A user-defined target law: `data = (P = MyLaw(θ), obs = …)` with the law's
 * `set_parameters!(P, idx, θ)` + `loglikelihood(P, obs)` (the plugin surface of
 * src/example/gsn_target.jl:15-29 and docs/src/get_started/basic_use.md:84-112).
 * set_parameters! is the engine's P°.θ[coords] ← θ° (updates.jl:198-205, P°
 * starting at theta0 as deepcopy(data.P), workspaces.jl:225-233); loglikelihood
 * is `source`, compiled with hiprtc for gfx950 into the general schedule kernel:
 *
 *     EMCMC_USER_LOGLIK {   // in scope: const double *theta (P°.θ, D entries), int D,
 *         …                 //   const double *obs (num_obs × obs_dim), uint64_t nobs,
 *         return ll;        //   const double *params (num_params)
 *     }
 *
 * in the C subset both hiprtc and a C compiler accept: + − × ÷, fma, sqrt, fabs,
 * copysign, em_exp(x), em_log(x) (the engine's exp / log, NaN below 0;
 * oracle/user_prelude.h maps them to their CPU restatement).  Every update kind, prior and adaptation
 * of the general kernel runs with it; D ≤ 64.  A law may also define its gradient, the
 * compute_gradients_and_momenta! hook MALA reads (updates.jl:123-133, run.jl:110, 259):
 *
 *     EMCMC_USER_GRAD {     // in scope: theta, D, obs, nobs, params as above and
 *         …                 //   double *grad (out, D entries): ∇ loglikelihood(P°, obs)
 *     }
 */
typedef struct emcmc_user_target_desc {
    uint32_t dim;           /* length(P.θ) = D */
    uint32_t obs_dim;       /* doubles per observation row (the source's business) */
    const double *theta0;   /* P.θ at construction (NULL: zeros) */
    uint64_t num_obs;
    const double *obs;      /* num_obs × obs_dim, row-major */
    uint64_t num_params;
    const double *params;   /* constants of the law (NULL if none) */
    const char *source;     /* EMCMC_USER_LOGLIK { … } */
    const char *options;    /* extra hiprtc options (e.g. "-DN_FEATURES=4"), or NULL */
} emcmc_user_target_desc;

/* One element of the `MCMCSchedule` iteration (src/schedule.jl:56-66). */
typedef struct emcmc_step {
    uint32_t mcmciter;  /* 1-based */
    uint32_t pidx;      /* 1-based update index */
} emcmc_step;

/* Cross-chain moments of θ over an iteration window, for split-R̂
 * (new functionality; BASELINE cfg 5).  out3d = [m̄ | M2 | Σ var] over the
 * chains of this handle: not sums.  Shards combine by an all-gather of every
 * rank's 3·D + 3 doubles and chain count, merged in rank order with Chan's
 * pairwise update (extensible_mcmc/diagnostics.py). */
typedef struct emcmc_moments {
    uint64_t num_chains;   /* chains summed (×2 halves when split) */
    uint64_t num_draws;    /* draws per (half-)chain */
    uint64_t accepted;     /* accepted proposals in the window, all chains */
    uint64_t proposed;
} emcmc_moments;

/* ---- lifecycle --------------------------------------------------------- */

/* Number of HIP devices visible (0 with no GPU).  Never fails on a CPU host. */
emcmc_status emcmc_device_count(int *count);

/* Replaces init_global_workspace(::GenericMCMCBackend, …) (workspaces.jl:215-234)
 * and create_workspaces (workspaces.jl:362-371): allocates SoA device state and
 * history buffers for C chains. */
emcmc_status emcmc_create(emcmc_handle **h, const emcmc_config *cfg);

/* Appends one update (→ pidx = number of updates added so far).  Replaces the
 * per-update plugin methods proposal!/log_transition_density/log_prior/
 * set_parameters! (updates.jl:185-214, run.jl:344-385) with device code. */
emcmc_status emcmc_add_update(emcmc_handle *h, const emcmc_update_desc *u);

/* Replaces set_parameters!(P::GsnTargetLaw, …) + loglikelihood(P, obs)
 * (gsn_target.jl:15-29): uploads observations and the factorised Σ. */
emcmc_status emcmc_set_target(emcmc_handle *h, const emcmc_target_desc *t);

/* Replaces set_parameters!(P::MyLaw, …) + loglikelihood(P::MyLaw, obs) of a
 * user-defined law (gsn_target.jl:15-29 is the reference's example of the
 * interface): compiles `source` for gfx950 (hiprtc; cached per process) and
 * uploads obs / params.  A compile error returns EMCMC_INVALID_ARG with the
 * compiler log in emcmc_last_error. */
emcmc_status emcmc_set_user_target(emcmc_handle *h, const emcmc_user_target_desc *t);

/* Compile-only check of a user log-likelihood for dimension dim (no device
 * needed): EMCMC_OK, or EMCMC_INVALID_ARG with the compiler log in log_out
 * (truncated to log_len bytes, NUL-terminated; log_out may be NULL). */
emcmc_status emcmc_check_user_target(const char *source, uint32_t dim, const char *options, char *log_out,
                                     size_t log_len);
/* The same for a user update's source (emcmc_user_update_desc) at dimension dim. */
emcmc_status emcmc_check_user_update(const char *source, uint32_t dim, const char *options, char *log_out,
                                     size_t log_len);

/* Compile (no device needed) the run-time rwm_gsn_chol_kernel for a correlated Σ at a
 * dimension 2 ≤ dim ≤ 64 the library has no ahead-of-time instantiation of (it has 16, 24
 * and 32: those return EMCMC_OK without compiling) into the on-disk code-object cache
 * (emcmc_rtc_info), so the first handle of a deployment loads it instead of compiling it
 * (≈ 1 minute at dim ≥ 40). */
emcmc_status emcmc_prebuild_chol_kernel(uint32_t dim, uint32_t history_mode, uint32_t ll_mode, char *log_out,
                                        size_t log_len);
/* The same for mwg_block_kernel, the kernel a handle with ONE MALA update (update_source =
 * NULL) or ONE user update (its EMCMC_USER_PROPOSAL/EMCMC_USER_LTD source) over coordinates
 * 1:dim, ImproperPrior, selects at 17 ≤ dim ≤ 64: on the built-in GsnTargetLaw
 * (target_source = NULL; dense_target != 0 for a non-diagonal Σ) or on a user law
 * (target_source, its options).  MALA on GsnTargetLaw at dim = 32 is ahead of time (EMCMC_OK,
 * nothing compiled). */
emcmc_status emcmc_prebuild_block_kernel(uint32_t dim, uint32_t history_mode, uint32_t ll_mode, int dense_target,
                                         const char *target_source, const char *target_options,
                                         const char *update_source, const char *update_options, char *log_out,
                                         size_t log_len);

/* The same for mwg_rw_block_kernel, the kernel a handle whose schedule is 1 ≤ P ≤ 8
 * UniformRandomWalk / GaussianRandomWalk updates (any coordinate subsets, priors, positivity
 * flags, AdaptationUnifRW on a UniformRandomWalk) selects at 17 ≤ dim ≤ 64 — unless it is one
 * GaussianRandomWalk over 0..dim-1 with ImproperPrior and no flags on the built-in target, which
 * the fused kernels take.  The kernel is compiled for the schedule's structure (kinds, coordinates,
 * diagonal Σ, pos flags, adaptation, prior families), so `updates` are the num_updates
 * emcmc_update_desc the handle will be given, in order (their values may differ: they are read at
 * run time).  The built-in GsnTargetLaw (target_source = NULL; dense_target != 0 for a
 * non-diagonal Σ) or a user law (target_source, its options). */
emcmc_status emcmc_prebuild_rw_block_kernel(uint32_t dim, uint32_t history_mode, uint32_t ll_mode, int dense_target,
                                            const emcmc_update_desc *updates, uint32_t num_updates,
                                            const char *target_source, const char *target_options, char *log_out,
                                            size_t log_len);

/* The same for the fused diagonal step with the update's separable terms compiled in
 * (rwm_gsn_diag_kernel + FusedUpdate), the kernel a handle selects for ONE update over 0..dim-1
 * without adaptation — a GaussianRandomWalk with a diagonal Σ or a UniformRandomWalk, positivity
 * flags allowed on either — whose prior is ImproperPosPrior or one ProductPrior / StandardPrior
 * factor: a Product of dim univariates or an MvNormal over all dim coordinates (ImproperPrior too
 * with flags or a UniformRandomWalk), families and flags repeating across the chain's lanes,
 * dim / lanes = 8·2^k with more than one lane, on the built-in GsnTargetLaw with a diagonal Σ
 * (unit_target != 0: Σ = I).  lanes_per_chain as in emcmc_config (0 = automatic).  Compiles both
 * occupancies the handle may try (two waves per SIMD, then one). */
emcmc_status emcmc_prebuild_fused_prior_kernel(uint32_t dim, uint32_t lanes_per_chain, uint32_t history_mode,
                                               uint32_t ll_mode, int unit_target, const emcmc_update_desc *update,
                                               char *log_out, size_t log_len);

/* θinit for every chain (row-major [C][D]); ll = NULL means the reference's
 * initial ll = -Inf (workspaces.jl:425), i.e. the first step always accepts.
 * Also resets the rolling-acceptance statistics (chain_statistics.jl:23-36). */
emcmc_status emcmc_set_state(emcmc_handle *h, const double *theta, const double *ll);

/* Replaces the body of __run! (run.jl:64-83) for the given schedule steps:
 * update_workspaces! → update! (proposal!, set_proposal!, compute_ll!,
 * accept_reject!, update_stats!) → update_adaptation!, fused over all chains.
 * Asynchronous. */
emcmc_status emcmc_run(emcmc_handle *h, const emcmc_step *steps, uint64_t num_steps);

/* Wait for all queued work; returns EMCMC_CHAIN_FAULT if any chain faulted. */
emcmc_status emcmc_synchronize(emcmc_handle *h);

void emcmc_destroy(emcmc_handle *h);
const char *emcmc_last_error(const emcmc_handle *h);

/* ---- state and histories ------------------------------------------------ */

/* Current θ ([C][D]) and ll ([C]) — state(global_ws), ll(local_ws). Either may be NULL. */
emcmc_status emcmc_get_state(emcmc_handle *h, double *theta, double *ll);

/* Current rolling acceptance (chain_statistics.jl:61-64: the value of
 * rolling_ar[last iteration][pidx]) and accepted counts, per update and chain:
 * [P][C] each.  Either may be NULL. */
emcmc_status emcmc_get_chain_stats(emcmc_handle *h, double *rolling_ar, uint64_t *accepted);

/* Adaptation state of update `pidx` (1-based), per chain: the UniformRandomWalk
 * ϵ as adapted (updt.rw.ϵ; [C][num_coords]) and AdaptationUnifRW's `proposed` /
 * `accepted` counters ([C] each) (adaptation.jl:51-70).  Any pointer may be NULL. */
emcmc_status emcmc_get_update_state(emcmc_handle *h, uint32_t pidx, double *epsilon, uint32_t *proposed,
                                    uint32_t *accepted);

/* GenericChainStats running mean and covariance of θ (chain_statistics.jl:46-49,
 * phantom zero sample included), updated after every update step, per chain:
 * mean [C][D], cov [C][D][D] (symmetric).  Kept on device with
 * emcmc_config.chain_moments (any schedule) and with a single joint
 * GaussianRandomWalkMix update; EMCMC_STATE_ERROR otherwise.  Either may be NULL.
 * With HaarioTypeAdaptation and P = 1 these equal the adaptation's mean/cov
 * (same recurrence on the same θ, adaptation.jl:406-414). */
emcmc_status emcmc_get_chain_moments(emcmc_handle *h, double *mean, double *cov);

/* HaarioTypeAdaptation mean and cov of update `pidx` (adaptation.jl:372-414):
 * its own running moments of the update's coordinates (log scale where pos), per
 * chain: mean [C][n], cov [C][n][n].  They register after every update step of
 * the schedule (register_only_on_my_turn is false both ways); for a single joint
 * update they equal emcmc_get_chain_moments.  Either may be NULL. */
emcmc_status emcmc_get_adaptation_moments(emcmc_handle *h, uint32_t pidx, double *mean, double *cov);

/* GaussianRandomWalkMix state of update `pidx`: the lower Cholesky factor of
 * each chain's current Σ_B ([C][n][n], row-major, zeros above the diagonal),
 * and HaarioTypeAdaptation's M (own-turn steps since the last readjust).
 * Either may be NULL. */
emcmc_status emcmc_get_mix_state(emcmc_handle *h, uint32_t pidx, double *chol_sigma_b, uint32_t *steps_since_adapt);

/* HaarioTypeAdaptation's fλ (adaptation.jl:372-397, 425: `rw.λ = adpt.fλ(rw.λ,
 * adpt.N, mcmc_iter)` at every readjust!).  N and mcmc_iter are the same for
 * every chain (P = 1: N = 1 + the iterations registered), so λ stays one
 * number: the library calls f on the host, when emcmc_run enqueues the
 * readjust, and the launches that follow use the new λ.  f = NULL restores the
 * identity (the reference's default (x, y, z) -> x). */
typedef double (*emcmc_lambda_fn)(double lambda, int64_t N, int64_t mcmciter, void *ctx);
emcmc_status emcmc_set_mix_lambda_fn(emcmc_handle *h, uint32_t pidx, emcmc_lambda_fn f, void *ctx);
/* The current λ of GaussianRandomWalkMix update `pidx` (rw.λ). */
emcmc_status emcmc_get_mix_lambda(emcmc_handle *h, uint32_t pidx, double *lambda);

/* Per-chain fault bits (EMCMC_FAULT_*), [C] uint32. */
emcmc_status emcmc_get_faults(emcmc_handle *h, uint32_t *faults);

/* `ll°(local_ws)` = sub_ws°.ll of every update (workspaces.jl:316-337): the
 * log-likelihood of the update's most recent proposal, per chain: [P][C]
 * (NaN for an update that has not run since emcmc_set_state).  REPLCallback's
 * ll° and llr (callbacks.jl:305-307, workspaces.jl:378) read it. */
emcmc_status emcmc_get_proposal_ll(emcmc_handle *h, double *ll_prop);

/* Copies iterations [iter_first, iter_first+num_iters) (1-based) of one history
 * to host.  Layout per EMCMC_H_* above, restricted to the window. */
emcmc_status emcmc_get_history(emcmc_handle *h, uint32_t which, uint64_t iter_first,
                               uint64_t num_iters, void *host_out, size_t host_bytes);

/* Same, restricted to chains [chain_first, chain_first+num_chains) (STATE,
 * PROPOSAL, LL only): out is [num_iters][P][num_chains][D] / [..][num_chains]. */
emcmc_status emcmc_get_history_chains(emcmc_handle *h, uint32_t which, uint64_t iter_first,
                                      uint64_t num_iters, uint64_t chain_first, uint64_t num_chains,
                                      void *host_out, size_t host_bytes);

/* ---- history streaming (ring buffers on device) -------------------------
 * With emcmc_config.history_ring = R, iteration i of every history lives in
 * ring slot (i−1) mod R and is overwritten by iteration i + R.  The getters
 * above accept only resident iterations (the last R run); older ones return
 * EMCMC_STATE_ERROR.  Histories leave the device while later steps run: */

/* Enqueue an asynchronous copy of iterations iter_first, iter_first+thin, …
 * (num_iters of them) of history `which` into host_out, in the emcmc_get_history
 * layout of a num_iters window ([n][P][C][D], [n][P][C] or [n][P][⌈C/64⌉] u64).
 * The copy runs on the handle's copy stream: after every emcmc_run enqueued so
 * far, and before any later step that reuses those ring slots; later steps
 * overlap it otherwise.  host_out must stay valid until emcmc_stream_wait; use
 * pinned memory (emcmc_host_alloc) for the copy to be asynchronous. */
emcmc_status emcmc_stream_history(emcmc_handle *h, uint32_t which, uint64_t iter_first, uint64_t num_iters,
                                  uint64_t thin, void *host_out, size_t host_bytes);
/* Wait for every enqueued history copy. */
emcmc_status emcmc_stream_wait(emcmc_handle *h);
/* Page-locked host memory for streamed histories (hipHostMalloc / hipHostFree). */
emcmc_status emcmc_host_alloc(size_t bytes, void **ptr);
emcmc_status emcmc_host_free(void *ptr);

/* Device pointer + byte size of a whole history buffer (zero-copy interop;
 * history_ring iterations when a ring is configured). */
emcmc_status emcmc_history_device_ptr(emcmc_handle *h, uint32_t which, void **dptr,
                                      size_t *bytes);

/* ---- diagnostics (new; BASELINE cfg 5) --------------------------------- */

/* Per-dimension moments over the chains of this handle of the (split) chain
 * means and unbiased variances of θ over iterations [iter_first, iter_first+num_iters):
 * out3d = [m̄ = mean of the chain means | M2 = Σ_c (m_c − m̄)² | Σ_c var_c], 3·D doubles,
 * with info->num_chains (half-)chains.  M2 comes from a Welford/Chan reduction, so
 * shards merge without cancellation (Chan et al. 1979; extensible_mcmc/diagnostics.py).
 * split != 0 treats each chain as two halves (split-R̂). */
emcmc_status emcmc_moments_window(emcmc_handle *h, uint64_t iter_first, uint64_t num_iters,
                                  int split, double *out3d, emcmc_moments *info);

/* Cross-chain diagnostics over every rank (SURVEY.md §8(b) `emcmc_diagnostics`; new: the
 * reference's GenericChainStats, src/chain_statistics.jl:16-66, is single-chain).  Chains are
 * sharded one handle per GPU; a communicator joins the handles of one job:
 *   - RCCL (emcmc_comm_init): rank 0 draws an id with emcmc_comm_unique_id, the caller
 *     broadcasts its 128 bytes (MPI, torch.distributed, a file), every rank calls
 *     emcmc_comm_init on its own GPU; the all-gather runs over xGMI (ncclAllGather).
 *     librccl.so.1 is opened at the first call (the copy already loaded, e.g. by torch, or
 *     the system's); without it these calls return EMCMC_RCCL_ERROR.
 *   - host callback (emcmc_comm_init_host): the caller's own all-gather of doubles
 *     (MPI.Allgather!, gloo), for callers that already hold a process group.
 * The per-rank record is the 3·D + 3 doubles [num_chains | m̄ (D) | M2 (D) | Σvar (D) |
 * accepted | proposed] (emcmc_moments_window's moments); every rank merges the gathered
 * records in rank order with Chan's pairwise update and forms split-R̂ (BDA3 §11.4):
 *   B = n/(m−1)·M2, W = Σvar/m, var⁺ = (n−1)/n·W + B/n, R̂ = √(var⁺/W),
 * m (half-)chains of n draws: the arithmetic of extensible_mcmc/diagnostics.py, bit for bit. */
typedef struct emcmc_comm emcmc_comm;
#define EMCMC_COMM_ID_BYTES 128
/* all-gather of `count` doubles per rank: recv = nranks·count doubles in rank order; 0 = ok */
typedef int (*emcmc_allgather_fn)(const double *send, double *recv, uint64_t count, void *ctx);

emcmc_status emcmc_comm_unique_id(uint8_t id[EMCMC_COMM_ID_BYTES]);
emcmc_status emcmc_comm_init(emcmc_comm **comm, int nranks, int rank, int device,
                             const uint8_t id[EMCMC_COMM_ID_BYTES]);
emcmc_status emcmc_comm_init_host(emcmc_comm **comm, int nranks, int rank, emcmc_allgather_fn fn, void *ctx);
void emcmc_comm_destroy(emcmc_comm *comm);
const char *emcmc_comm_last_error(const emcmc_comm *comm);  /* comm = NULL: why this thread's last
                                                              emcmc_comm_init / _unique_id / comm-less
                                                              emcmc_diagnostics_merge failed */
/* HIP runtime images (libamdhip64.so*) mapped into this process; their paths, newline-separated,
 * in paths_out (truncated to len bytes, NUL-terminated; may be NULL).  More than one means a
 * second runtime was loaded beside the one libemcmc.so is bound to (e.g. torch's bundled copy
 * when libemcmc.so was loaded first): emcmc_comm_init / emcmc_comm_unique_id then refuse with
 * EMCMC_HIP_ERROR and say so in emcmc_comm_last_error(NULL), and the Python layer warns. */
int emcmc_hip_runtime_images(char *paths_out, size_t len);

typedef struct emcmc_diag {
    uint64_t num_chains;  /* (half-)chains merged over every rank */
    uint64_t num_draws;   /* draws per (half-)chain */
    uint64_t accepted;    /* accepted proposals in the window, every rank */
    uint64_t proposed;
    double accept_rate;   /* accepted / max(1, proposed) */
    double max_rhat;      /* max over the dimensions of R̂ (NaN if any is) */
    uint32_t dim;         /* out: D */
    uint32_t nranks;      /* out: records merged */
    double *mean;         /* caller-owned [D] arrays, each may be NULL: m̄ (the chain-mean mean) */
    double *m2;           /*   M2 = Σ_c (m_c − m̄)² */
    double *sum_var;      /*   Σ_c var_c */
    double *W;            /*   within-chain variance */
    double *B;            /*   between-chain variance */
    double *rhat;         /*   split-R̂ */
} emcmc_diag;

/* emcmc_moments_window of this handle's chains, all-gathered over `comm` (NULL: this
 * handle alone) and merged; every rank gets the same result.  Collective: every rank of
 * comm calls it with the same window.  An RCCL comm must be on the handle's device. */
emcmc_status emcmc_diagnostics(emcmc_handle *h, emcmc_comm *comm, uint64_t iter_first, uint64_t num_iters,
                               int split, emcmc_diag *out);
/* The same from a caller-made record (3·dim + 3 doubles as above) and draws per
 * (half-)chain; no handle, and no device with a host comm or comm = NULL.  Fewer than 2
 * (half-)chains over all ranks: EMCMC_INVALID_ARG (B = n·M2/(m − 1) is undefined). */
emcmc_status emcmc_diagnostics_merge(emcmc_comm *comm, const double *record, uint32_t dim, uint64_t num_draws,
                                     emcmc_diag *out);

/* ---- timing (bench / roofline) ----------------------------------------- */

/* Enable per-launch HIP-event timing on the handle's stream. */
emcmc_status emcmc_set_timing(emcmc_handle *h, int enable);
/* Sum of per-launch kernel durations (ms) and number of step-kernel launches
 * since the last reset; also returns algorithmic bytes moved by those launches. */
emcmc_status emcmc_get_timing(emcmc_handle *h, double *total_ms, uint64_t *launches,
                              double *algorithmic_bytes, int reset);

/* Human-readable name of the kernel variant `emcmc_run` dispatches to. */
emcmc_status emcmc_kernel_name(emcmc_handle *h, char *buf, size_t buflen);

/* How the handle's run-time compiled kernel (hiprtc: user laws and updates, the
 * general kernel at other D, the chol kernel at other D) was obtained: origin
 * 0 = this process's cache, 1 = the on-disk code-object cache (EMCMC_RTC_CACHE,
 * else rtc_cache/ beside libemcmc.so), 2 = compiled now, 3 = compiled now because the cache
 * directory exists but is not private to this user (owned by the effective uid, not group- or
 * world-writable; the library also says so once on stderr); seconds = the time it took.
 * EMCMC_STATE_ERROR when the selected kernel is compiled ahead of time. */
emcmc_status emcmc_rtc_info(emcmc_handle *h, uint32_t *origin, double *seconds);

/* ---- self-test probes (run the device's own math on given inputs) ------- */

/* For each of n (chain, iter) pairs: the dim normals and the Exp(1) accept draw
 * the step kernels use at (seed, chain, iter, pidx0).  z: [n][dim], E: [n]. */
emcmc_status emcmc_probe_variates(int device, uint64_t seed, uint32_t pidx0, uint32_t dim, uint64_t n,
                                  const uint32_t *chains, const uint32_t *iters, double *z, double *E);
/* y[i] = device log_pos(x[i]) (the hot path's log, x finite normal > 0). */
emcmc_status emcmc_probe_log(int device, const double *x, double *y, uint64_t n);

#ifdef __cplusplus
}
#endif

#endif /* EMCMC_H */
