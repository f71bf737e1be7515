/* A preconditioned Crank–Nicolson (autoregressive) proposal as a user update —
 * a non-random-walk MCMCParamUpdate whose transition density does not cancel:
 *   θ°_i = m_i + ρ(θ_i − m_i) + s·z_i,  s = σ·√(1 − ρ²),  z ~ N(0, 1)
 *   log_transition_density(x, y) = Σ_i logpdf(N(m_i + ρ(x_i − m_i), s), y_i)
 * params = [ρ, σ, m_1, …, m_n].  Compiled by hiprtc for the device and by gcc
 * for the oracle (include/emcmc.h emcmc_user_update_desc). */
EMCMC_USER_PROPOSAL {
    const double rho = params[0];
    const double s = params[1] * sqrt(1.0 - rho * rho);
    for (int i = 0; i < n; ++i) {
        const double m = params[2 + i];
        theta_prop[i] = (m + rho * (theta[i] - m)) + s * em_randn(i);
    }
}

EMCMC_USER_LTD {
    const double rho = params[0];
    const double s = params[1] * sqrt(1.0 - rho * rho);
    const double c = -0.91893853320467274178 - em_log(s); /* −log(2π)/2 − log s */
    double lp = 0.0;
    for (int i = 0; i < n; ++i) {
        const double m = params[2 + i];
        const double z = (y[i] - (m + rho * (x[i] - m))) / s;
        lp = lp + (c - 0.5 * (z * z));
    }
    return lp;
}
