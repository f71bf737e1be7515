/* A multiplicative (log-normal) random walk on positive coordinates as a user
 * update: θ°_i = θ_i·exp(σ_i z_i), so
 *   log_transition_density(x, y) = Σ_i [logpdf(N(log x_i, σ_i), log y_i) − log y_i]
 * (the Jacobian term keeps the two directions from cancelling).  With
 * probability params[0] the step uses the scales params[1 + n + i] instead of
 * params[1 + i] (one em_rand draw per proposal): a two-scale mixture whose
 * density is the mixture of both.  params = [w, σ_1…σ_n, τ_1…τ_n]. */
EMCMC_USER_PROPOSAL {
    const int big = em_rand(0) < params[0];
    for (int i = 0; i < n; ++i) {
        const double sd = big ? params[1 + n + i] : params[1 + i];
        theta_prop[i] = theta[i] * em_exp(sd * em_randn(i));
    }
}

EMCMC_USER_LTD {
    const double w = params[0];
    double la = 0.0, lb = 0.0, lj = 0.0;
    for (int i = 0; i < n; ++i) {
        const double ly = em_log(y[i]);
        const double d = ly - em_log(x[i]);
        const double sa = params[1 + i], sb = params[1 + n + i];
        la = la + ((-0.91893853320467274178 - em_log(sa)) - 0.5 * ((d / sa) * (d / sa)));
        lb = lb + ((-0.91893853320467274178 - em_log(sb)) - 0.5 * ((d / sb) * (d / sb)));
        lj = lj + ly;
    }
    return em_log((1.0 - w) * em_exp(la) + w * em_exp(lb)) - lj;
}
