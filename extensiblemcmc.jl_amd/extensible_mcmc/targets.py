"""Target laws (reference src/example/gsn_target.jl).

``GsnTargetLaw(μ, Σ)`` keeps the reference's parameter vector θ = [μ; vec(Σ)]
(gsn_target.jl:1-13).  Device plugin: ``set_parameters!(P, coords, θ)`` +
``loglikelihood(P, obs)`` run inside the fused step kernel with coords ⊆ μ.
"""
from __future__ import annotations

import numpy as np


class GsnTargetLaw:
    def __init__(self, mu, Sigma=None):
        mu = np.atleast_1d(np.asarray(mu, dtype=float))
        d = mu.size
        S = np.eye(d) if Sigma is None else np.asarray(Sigma, dtype=float).reshape(d, d)
        self.d = d
        self.theta = np.zeros(d * (d + 1))
        self.theta[:d] = mu
        self.theta[d:] = S.ravel(order="F")  # vec(Σ), column-major

    @property
    def mu(self):
        return self.theta[: self.d]

    @property
    def Sigma(self):
        # set_parameters! rebuilds Symmetric(triu(Σ)) (gsn_target.jl:17-20): upper triangle wins
        S = self.theta[self.d :].reshape(self.d, self.d, order="F")
        U = np.triu(S)
        return U + np.triu(U, 1).T

    def set_parameters(self, loc2glob_idx, theta):
        """set_parameters!(P, idx, θ) (gsn_target.jl:15-21), 1-based indices."""
        idx = np.asarray(loc2glob_idx, dtype=int) - 1
        self.theta[idx] = theta

    def to_device(self, engine, ll_mode, obs):
        engine.set_gsn_target(self.mu, self.Sigma, obs, ll_mode=ll_mode)


class LogisticRegressionLaw:
    """Logistic regression ``ℓ(θ) = Σ_n y_n x_nᵀθ − log(1 + exp(x_nᵀθ))`` with
    ``obs = (X, y)``: the target of BASELINE cfg 3 (MALA, N = 1e5, D = 64).  It
    has no counterpart in the reference beyond its target-law interface
    (``set_parameters!`` + ``loglikelihood(P, obs)``, gsn_target.jl:15-29)."""

    def __init__(self, d):
        self.d = int(d)
        self.theta = np.zeros(self.d)

    def set_parameters(self, loc2glob_idx, theta):
        idx = np.asarray(loc2glob_idx, dtype=int) - 1
        self.theta[idx] = theta

    def to_device(self, engine, ll_mode, obs):
        X, y = obs
        engine.set_logistic_target(X, y)


class UserTargetLaw:
    """A user-defined target law (the reference's plugin surface for laws:
    ``set_parameters!(P, idx, θ)`` + ``loglikelihood(P, obs)``,
    gsn_target.jl:15-29, docs/src/get_started/basic_use.md:84-112).

    ``source`` is the law's log-likelihood as an ``EMCMC_USER_LOGLIK { … }``
    function body over ``theta`` (P.θ, length d), ``obs``/``nobs`` and
    ``params`` (include/emcmc.h emcmc_user_target_desc); the engine compiles it
    for the device with hiprtc.  ``set_parameters`` keeps the reference's
    meaning: P.θ[idx] ← θ (the device does the same on P° every update)."""

    def __init__(self, source: str, theta, params=None, options: str = ""):
        self.source = source
        self.theta = np.atleast_1d(np.asarray(theta, dtype=float)).copy()
        self.d = self.theta.size
        self.params = None if params is None else np.asarray(params, dtype=float)
        self.options = options

    def set_parameters(self, loc2glob_idx, theta):
        idx = np.asarray(loc2glob_idx, dtype=int) - 1
        self.theta[idx] = theta

    def to_device(self, engine, ll_mode, obs):
        engine.set_user_target(self.source, obs=obs, params=self.params, theta0=self.theta, options=self.options)


def make_data(P, obs):
    """The ``data = (P = …, obs = …)`` NamedTuple of the reference (basic_use.md:112)."""
    return {"P": P, "obs": np.asarray(obs, dtype=float)}
