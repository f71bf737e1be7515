"""User-defined target laws used by the tests (sources in tests/user_targets/).

Each case is the data of a ``run!`` with ``data = (P = MyLaw(θ), obs)`` where
MyLaw's ``loglikelihood(P, obs)`` is the EMCMC_USER_LOGLIK source: the engine
compiles it for the device with hiprtc, the oracle runs the gcc build of the
same text (oracle/Makefile, oracle/user_prelude.h).  Synthetic data from fixed
numpy seeds; the numpy restatements below pin the sources' formulas.
"""
import math
from dataclasses import dataclass, field

import numpy as np

LOG2PI = float("1.8378770664093454835606594728112")  # csrc/emcmc_math.h kLog2Pi


@dataclass
class UserCase:
    name: str           # tests/user_targets/<name>.c
    D: int
    obs: np.ndarray     # [nobs][obs_dim]
    params: np.ndarray
    theta0: np.ndarray  # P.θ at construction and the chains' θinit
    seed: int = 20261016
    extra: dict = field(default_factory=dict)


def student_t(D=4, n=50):
    rng = np.random.default_rng(1)
    X = np.column_stack([np.ones(n), rng.normal(size=(n, D - 1))])
    beta = np.array([1.0, -2.0, 0.5, 3.0, 0.25, -1.0, 0.75, 2.0][:D])
    nu, sigma = 4.0, 0.7
    y = X @ beta + sigma * rng.standard_t(nu, size=n)
    c = math.lgamma((nu + 1) / 2) - math.lgamma(nu / 2) - math.log(sigma * math.sqrt(nu * math.pi))
    return UserCase("student_t_regression", D, np.column_stack([X, y]), np.array([nu, sigma, c]),
                    np.zeros(D), extra={"beta": beta})


def poisson(D=3, n=40):
    rng = np.random.default_rng(2)
    X = np.column_stack([np.ones(n), rng.normal(scale=0.5, size=(n, D - 1))])
    beta = np.array([0.5, 1.0, -0.5, 0.3][:D])
    y = rng.poisson(np.exp(X @ beta)).astype(float)
    lfact = sum(math.lgamma(v + 1.0) for v in y)
    return UserCase("poisson_regression", D, np.column_stack([X, y]), np.array([lfact]), np.zeros(D),
                    extra={"beta": beta})


def banana(D=8, b=0.03):
    return UserCase("banana", D, np.zeros((0, 1)), np.array([b]), np.zeros(D))


def gsn_identity(D=3, n=10):
    rng = np.random.default_rng(3)
    mu = np.arange(1.0, D + 1.0)
    obs = mu + rng.normal(size=(n, D))
    c0 = -(D * LOG2PI + 0.0) / 2.0  # Distributions.mvnormal_c0 with logdet I = 0.0
    return UserCase("gsn_identity", D, obs, np.array([c0]), mu.copy())


def gsn_full(d=2, n=10):
    """GsnTargetLaw(μ, Σ) with θ = [μ; vec Σ] (gsn_target.jl:1-13): the reference
    test's target (test/runtests.jl:94-111) with its 10 observations drawn here."""
    rng = np.random.default_rng(4)
    mu = np.array([1.0, 2.0, -1.0, 0.5][:d])
    S = np.array([[1.0, 0.5, 0.0, 0.0], [0.5, 1.0, 0.2, 0.0], [0.0, 0.2, 1.5, 0.1], [0.0, 0.0, 0.1, 0.8]])[:d, :d]
    obs = rng.multivariate_normal(mu, S, size=n)
    theta0 = np.concatenate([np.zeros(d), np.eye(d).ravel(order="F")])
    return UserCase("gsn_full", d + d * d, obs, np.array([float(d)]), theta0, extra={"d": d, "mu": mu, "S": S})


def numpy_loglik(case: UserCase, theta):
    """The sources' formulas in numpy (libm exp/log: agree to ~1e-13 relative)."""
    th = np.asarray(theta, dtype=float)
    D = case.D
    if case.name in ("student_t_regression", "poisson_regression"):
        X, y = case.obs[:, :D], case.obs[:, D]
        eta = X @ th
        if case.name == "poisson_regression":
            return float(np.sum(y * eta - np.exp(eta)) - case.params[0])
        nu, sigma, c = case.params
        z = (y - eta) / sigma
        return float(np.sum(c - (nu + 1) / 2 * np.log1p(z * z / nu)))
    if case.name == "banana":
        b = case.params[0]
        p2 = th[1] + b * th[0] ** 2 - 100 * b
        return float(-th[0] ** 2 / 200 - p2 ** 2 / 2 - np.sum(th[2:] ** 2) / 2)
    if case.name == "gsn_full":
        d = case.extra["d"]
        mu, S = th[:d], th[d:].reshape(d, d, order="F")
        U = np.triu(S)
        S = U + np.triu(U, 1).T  # Symmetric(triu(Σ)) (gsn_target.jl:19)
        Li = np.linalg.inv(np.linalg.cholesky(S))
        r = (case.obs - mu) @ Li.T
        return float(np.sum(-(d * LOG2PI + np.linalg.slogdet(S)[1]) / 2 - np.sum(r * r, axis=1) / 2))
    if case.name == "gsn_identity":
        return float(np.sum(case.params[0] - np.sum((case.obs - th) ** 2, axis=1) / 2))
    raise KeyError(case.name)
