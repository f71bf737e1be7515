"""Synthetic workloads named in BASELINE.json / SURVEY.md §8(d).

cfg1  single-chain 2-D Gaussian (the reference's CPU-runnable case; isotropic
      target as BASELINE.json configs[0], plus the dense Σ = [1 .5; .5 1] of
      test/runtests.jl:88-111 as ``ref_test``)
cfg2  65,536 independent RWM chains, D = 32, GsnTargetLaw(μ*, I₃₂), n = 10,
      GaussianRandomWalk(σ²I₃₂), σ = 2.38/√(D·n), θinit = 0, seed 0xC0FFEE
cfg4  131,072 chains of cfg2's target with GaussianRandomWalkMix(σ²I, σ²I, λ=0.5)
      + HaarioTypeAdaptation(adapt_every_k_steps=200) and the GenericChainStats
      mean/cov on device (k = 200 rather than the constructor default 100: with
      fewer than ~D accepted moves per window the empirical covariance is
      rank-deficient and cholesky throws PosDefException in the reference)
cfg3  32,768 MALA chains on a logistic-regression target, N = 100,000 observations, D = 64
cfg5  cfg2 with 1,048,576 chains sharded over GPUs, overdispersed θinit
There is no network: observations are drawn from fixed numpy seeds.
"""
from __future__ import annotations

from dataclasses import dataclass

import numpy as np

SEED = 0xC0FFEE
OBS_SEED = 20261015


@dataclass
class GsnWorkload:
    name: str
    D: int
    num_chains: int
    mu_true: np.ndarray
    t_sigma: np.ndarray
    rw_sigma: np.ndarray
    obs: np.ndarray
    theta_init: np.ndarray  # [D] or [C][D]
    seed: int = SEED
    sigma_b: np.ndarray = None  # GaussianRandomWalkMix Σ_B (cfg 4)
    lam: float = None
    haario_k: int = None

    @property
    def nobs(self):
        return self.obs.shape[0]


def cfg2(num_chains: int = 65536, D: int = 32, nobs: int = 10) -> GsnWorkload:
    mu = (np.arange(D) - 15.5) / 8.0 if D == 32 else (np.arange(D) - (D - 1) / 2.0) / 8.0
    eps = np.random.default_rng(OBS_SEED).standard_normal((nobs, D))
    obs = mu[None, :] + eps
    sigma = 2.38 / np.sqrt(D * nobs)
    return GsnWorkload(
        name=f"rwm_gsn_d{D}_c{num_chains}", D=D, num_chains=num_chains, mu_true=mu, t_sigma=np.eye(D),
        rw_sigma=(sigma * sigma) * np.eye(D), obs=obs, theta_init=np.zeros(D),
    )


def cfg4(num_chains: int = 1 << 17, D: int = 32, nobs: int = 10, lam: float = 0.5, k: int = 200) -> GsnWorkload:
    w = cfg2(num_chains, D, nobs)
    w.name = f"haario_mix_gsn_d{D}_c{num_chains}"
    w.sigma_b = w.rw_sigma.copy()
    w.lam = lam
    w.haario_k = k
    return w


@dataclass
class LogisticWorkload:
    name: str
    D: int
    num_chains: int
    X: np.ndarray       # [N][D]
    y: np.ndarray       # [N] in {0, 1}
    theta_true: np.ndarray
    eps: float
    seed: int = SEED

    @property
    def nobs(self):
        return self.X.shape[0]

    @property
    def theta_init(self):  # θinit = 0 (BASELINE cfg 3)
        return np.zeros(self.D)


def cfg3(num_chains: int = 1 << 15, D: int = 64, nobs: int = 100_000, eps: float = None) -> LogisticWorkload:
    """BASELINE cfg 3: MALA on a logistic-regression log-likelihood, N = 1e5, D = 64.
    X ~ N(0, 1/D) entries, θ* ~ N(0, 1), y ~ Bernoulli(σ(Xθ*)).  ϵ defaults to
    0.045 at the cfg 3 shape (≈ 61 % acceptance, measured with the oracle; the
    MALA optimum is ≈ 57 %), scaled as ϵ ∝ √(D/N)·D^{-1/6} for other shapes."""
    rng = np.random.default_rng(OBS_SEED + 3)
    X = rng.standard_normal((nobs, D)) / np.sqrt(D)
    theta = rng.standard_normal(D)
    p = 1.0 / (1.0 + np.exp(-(X @ theta)))
    y = (rng.random(nobs) < p).astype(np.float64)
    if eps is None:
        eps = 0.045 * np.sqrt((D / 64.0) * (100_000.0 / nobs)) * (D / 64.0) ** (-1.0 / 6.0)
    return LogisticWorkload(name=f"mala_logistic_d{D}_n{nobs}_c{num_chains}", D=D, num_chains=num_chains, X=X, y=y,
                            theta_true=theta, eps=float(eps))


def cfg5(num_chains: int = 1 << 20, D: int = 32, nobs: int = 10) -> GsnWorkload:
    w = cfg2(num_chains, D, nobs)
    xbar = w.obs.mean(axis=0)
    z = np.random.default_rng(OBS_SEED + 1).standard_normal((num_chains, D))
    w.theta_init = xbar[None, :] + 3.0 * z / np.sqrt(nobs)
    w.name = f"rwm_gsn_d{D}_c{num_chains}_overdispersed"
    return w


def cfg1(isotropic: bool = True, num_chains: int = 1) -> GsnWorkload:
    mu = np.array([1.0, 2.0])
    S = np.eye(2) if isotropic else np.array([[1.0, 0.5], [0.5, 1.0]])
    rng = np.random.default_rng(10)
    obs = rng.multivariate_normal(mu, S, size=10)
    return GsnWorkload(
        name="gsn2d_iso" if isotropic else "gsn2d_ref_test", D=2, num_chains=num_chains, mu_true=mu, t_sigma=S,
        rw_sigma=0.5 * np.eye(2), obs=obs, theta_init=np.zeros(2),
    )


def ref_test(num_chains: int = 1) -> GsnWorkload:
    """test/runtests.jl:88-111 target with the tutorial's joint GaussianRandomWalk(0.5·I)."""
    return cfg1(isotropic=False, num_chains=num_chains)
