/* Haario, Saksman & Tamminen's (1999) "banana": a D-dimensional Gaussian
 * N(0, diag(100, 1, …, 1)) twisted by φ(θ)_2 = θ_2 + b·θ_1² − 100·b (params[0] = b).
 * No observations.  loglikelihood = −θ_1²/200 − φ_2²/2 − Σ_{i≥3} θ_i²/2. */
EMCMC_USER_LOGLIK {
    const double b = params[0];
    const double p2 = theta[1] + b * (theta[0] * theta[0]) - 100.0 * b;
    double s = -(theta[0] * theta[0]) / 200.0 - (p2 * p2) / 2.0;
    for (int i = 2; i < D; ++i) s = s - (theta[i] * theta[i]) / 2.0;
    return s;
}
