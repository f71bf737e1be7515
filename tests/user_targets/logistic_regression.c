/* Logistic regression with its gradient: y_k ~ Bernoulli(σ(x_kᵀβ)).
 * θ = β (D coefficients); observation row k = (x_k[0], …, x_k[D−1], y_k).
 * loglikelihood = Σ_k y_k·η_k − softplus(η_k),  η_k = x_kᵀβ,
 *   softplus(η) = max(η, 0) + log(1 + e^{−|η|});
 * gradient      = Σ_k x_k·(y_k − σ(η_k)),  σ(η) = (η ≥ 0 ? 1 : e^{−|η|}) / (1 + e^{−|η|}).
 * The gradient is the law's compute_gradients_and_momenta! hook (MALA). */
EMCMC_USER_LOGLIK {
    double ll = 0.0;
    for (uint64_t k = 0; k < nobs; ++k) {
        const double *row = obs + k * (uint64_t)(D + 1);
        double eta = row[0] * theta[0];
        for (int i = 1; i < D; ++i) eta = fma(row[i], theta[i], eta);
        const double t = em_exp(-fabs(eta));
        const double sp = (eta > 0.0 ? eta : 0.0) + em_log(1.0 + t);
        ll = ll + (row[D] * eta - sp);
    }
    return ll;
}
EMCMC_USER_GRAD {
    for (int i = 0; i < D; ++i) grad[i] = 0.0;
    for (uint64_t k = 0; k < nobs; ++k) {
        const double *row = obs + k * (uint64_t)(D + 1);
        double eta = row[0] * theta[0];
        for (int i = 1; i < D; ++i) eta = fma(row[i], theta[i], eta);
        const double t = em_exp(-fabs(eta));
        const double sig = (eta >= 0.0 ? 1.0 : t) / (1.0 + t);
        const double r = row[D] - sig;
        for (int i = 0; i < D; ++i) grad[i] = fma(row[i], r, grad[i]);
    }
}
