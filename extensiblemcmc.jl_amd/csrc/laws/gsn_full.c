/* GsnTargetLaw with its whole parameter vector θ = [μ; vec Σ] (d + d² entries,
 * src/example/gsn_target.jl:1-29).  set_parameters! may write any entry; the law
 * then rebuilds MvNormal(μ, Symmetric(triu(Σ))) — a Cholesky factor of the
 * upper triangle — and loglikelihood sums logpdf over the observations
 * (gsn_target.jl:15-29).  Here the factor is rebuilt at every evaluation, in the
 * engine's canonical order (csrc/emcmc.hip cholesky_upper_colmajor, logdet_chol,
 * mvnormal_c0, the forward substitution and blocked sum of squares of
 * emcmc_mwg.h), so with Σ fixed the chain equals the built-in GsnTargetLaw's bit
 * for bit.  params[0] = d (≤ 8); observation rows have d entries.  A Σ that is
 * not positive definite — the reference's PosDefException — gives NaN: the
 * proposal is rejected and the chain's fault bit 1 is set. */
EMCMC_USER_LOGLIK {
    const int d = (int)params[0];
    const double *S = theta + d; /* column-major: Σ(i, j) = S[i + j·d] */
    double L[64], iL[8];
    for (int j = 0; j < d; ++j) {
        double s = S[j + j * d];
        for (int k = 0; k < j; ++k) s = s - L[j * 8 + k] * L[j * 8 + k];
        if (!(s > 0.0)) return __builtin_nan("");
        const double ljj = sqrt(s);
        L[j * 8 + j] = ljj;
        for (int i = j + 1; i < d; ++i) {
            double t = S[j + i * d]; /* Σ(j, i): the upper triangle */
            for (int k = 0; k < j; ++k) t = t - L[i * 8 + k] * L[j * 8 + k];
            L[i * 8 + j] = t / ljj;
        }
    }
    double dd = 0.0;
    for (int i = 0; i < d; ++i) {
        iL[i] = 1.0 / L[i * 8 + i];
        dd = dd + em_log(L[i * 8 + i]);
    }
    const double c0 = -((double)d * 1.8378770664093454835606594728112 + (dd + dd)) / 2.0;
    double ll = 0.0;
    for (uint64_t k = 0; k < nobs; ++k) {
        const double *x = obs + k * (uint64_t)d;
        double y[8], s = 0.0;
        for (int i = 0; i < d; ++i) {
            double acc = x[i] - theta[i];
            for (int j = 0; j < i; ++j) acc = fma(-L[i * 8 + j], y[j], acc);
            y[i] = acc * iL[i];
            s = (i == 0) ? y[0] * y[0] : fma(y[i], y[i], s);
        }
        ll = ll + (c0 - s / 2.0);
    }
    return ll;
}
