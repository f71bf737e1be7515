/* Robust linear regression with Student-t errors: y_k = x_kᵀβ + σ·ε_k, ε_k ~ t_ν.
 * θ = β (D coefficients); observation row k = (x_k[0], …, x_k[D−1], y_k);
 * params = (ν, σ, c) with c = lgamma((ν+1)/2) − lgamma(ν/2) − log(σ·√(νπ))
 * computed by the caller.  loglikelihood = Σ_k c − (ν+1)/2 · log(1 + z_k²/ν),
 * z_k = (y_k − x_kᵀβ)/σ (Distributions.jl's TDist logpdf of the scaled residual). */
EMCMC_USER_LOGLIK {
    const double nu = params[0], sigma = params[1], c = params[2];
    const double h = (nu + 1.0) / 2.0;
    double ll = 0.0;
    for (uint64_t k = 0; k < nobs; ++k) {
        const double *row = obs + k * (uint64_t)(D + 1);
        double eta = row[0] * theta[0];
        for (int i = 1; i < D; ++i) eta = fma(row[i], theta[i], eta);
        const double z = (row[D] - eta) / sigma;
        ll = ll + (c - h * em_log(1.0 + z * z / nu));
    }
    return ll;
}
