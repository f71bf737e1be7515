/* Poisson regression with the log link: y_k ~ Poisson(exp(x_kᵀβ)).
 * θ = β (D coefficients); observation row k = (x_k[0], …, x_k[D−1], y_k);
 * params[0] = Σ_k log(y_k!) computed by the caller.
 * loglikelihood = Σ_k (y_k·η_k − exp(η_k)) − Σ_k log(y_k!),  η_k = x_kᵀβ. */
EMCMC_USER_LOGLIK {
    double ll = 0.0;
    for (uint64_t k = 0; k < nobs; ++k) {
        const double *row = obs + k * (uint64_t)(D + 1);
        double eta = row[0] * theta[0];
        for (int i = 1; i < D; ++i) eta = fma(row[i], theta[i], eta);
        ll = ll + (row[D] * eta - em_exp(eta));
    }
    return ll - params[0];
}
