/* GsnTargetLaw(μ = θ, I) (src/example/gsn_target.jl:23-29) written as a user law,
 * in the engine's canonical summation order for D < 16 (one left-to-right fma
 * chain per observation): loglikelihood = Σ_k (c0 − ‖x_k − θ‖²/2), with
 * params[0] = c0 = −D·log(2π)/2.  Observation rows have D entries.  The device
 * run must match the built-in GsnTargetLaw kernel bit for bit. */
EMCMC_USER_LOGLIK {
    const double c0 = params[0];
    double ll = 0.0;
    for (uint64_t k = 0; k < nobs; ++k) {
        const double *x = obs + k * (uint64_t)D;
        const double r0 = x[0] - theta[0];
        double s = r0 * r0;
        for (int i = 1; i < D; ++i) {
            const double r = x[i] - theta[i];
            s = fma(r, r, s);
        }
        ll = ll + (c0 - s / 2.0);
    }
    return ll;
}
