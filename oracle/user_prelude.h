/*
 * user_prelude.h — TEST INFRASTRUCTURE ONLY.
 *
 * Host side of the user-target source protocol (include/emcmc.h
 * emcmc_user_target_desc): a C compiler sees the same EMCMC_USER_LOGLIK source
 * the engine compiles for the device with hiprtc, with em_exp / em_log bound to
 * the oracle's restatement of the engine's exp / log (oracle_math.h).  The
 * resulting function is what orc_run_mwg calls as `user_ll`
 * (oracle/emcmc_oracle.c, orc_user_loglik_fn), and a user update's
 * emcmc_user_proposal / emcmc_user_ltd what it calls as user_prop / user_ltd.
 * Build: oracle/Makefile (lib/user_<name>.so from tests/user_targets/<name>.c,
 * lib/userupd_<name>.so from tests/user_updates/<name>.c).
 */
#ifndef ORACLE_USER_PRELUDE_H
#define ORACLE_USER_PRELUDE_H

#include <math.h>
#include <stdint.h>

#include "oracle_math.h"

#define EMCMC_USER_LOGLIK                                                                              \
    double emcmc_user_loglik(const double *restrict theta, int D, const double *restrict obs, uint64_t nobs, \
                             const double *restrict params)
/* the law's gradient, ∇ loglikelihood(P°, obs) into grad[D] (optional; MALA reads it) */
#define EMCMC_USER_GRAD                                                                                \
    void emcmc_user_grad(const double *restrict theta, int D, const double *restrict obs, uint64_t nobs,   \
                         const double *restrict params, double *restrict grad)
/* a user update (include/emcmc.h emcmc_user_update_desc): proposal! and
 * log_transition_density, with the engine's draws by index (oracle_math.h) */
#define EMCMC_USER_PROPOSAL                                                                                  \
    void emcmc_user_proposal(const double *restrict theta, double *restrict theta_prop, int n,             \
                             const double *restrict params, emcmc_rng *restrict rng)
#define EMCMC_USER_LTD                                                                                       \
    double emcmc_user_ltd(const double *restrict x, const double *restrict y, int n, const double *restrict params)
#define em_randn(j) orc_user_randn(rng, (uint32_t)(j))
#define em_rand(j) orc_user_rand(rng, (uint32_t)(j))
#define em_exp(x) orc_exp_any(x)
/* log: NaN below 0 (Julia's log throws DomainError there), −Inf at 0 */
static inline double orc_user_log(double x) { return (x < 0.0) ? NAN : orc_log_any(x); }
#define em_log(x) orc_user_log(x)

#endif
