"""Transition kernels, priors, adaptation schemes and updates — the reference's
plugin surface (src/transition_kernels/*.jl, src/priors.jl, src/updates.jl),
as host-side descriptors.

These classes carry the constructor semantics of the reference (argument
defaults, assertions, scalar/vector promotion).  The per-step arithmetic
(``rand!``, ``logpdf``, ``log_prior``, ``register!``/``readjust!``) runs on the
device; ``to_device`` packs a descriptor for ``emcmc_add_update`` and raises
``UnsupportedPlugin`` for combinations without a device kernel yet.
"""
from __future__ import annotations

from dataclasses import dataclass, field
from typing import Callable, Optional, Sequence

import numpy as np
from math import lgamma  # noqa: E402

from . import _lib as L


UnsupportedPlugin = L.UnsupportedPlugin  # also raised, as UnsupportedPluginError, for EMCMC_UNSUPPORTED_PLUGIN


# ---------------------------------------------------------------------------
# abstract hierarchy (src/types.jl:8-125)
class MCMCUpdate:
    pass


class MCMCParamUpdate(MCMCUpdate):
    pass


class MCMCGradientBasedUpdate(MCMCParamUpdate):
    pass


class MCMCConjugateUpdate(MCMCUpdate):
    pass


class MCMCConjugateParamUpdate(MCMCParamUpdate):
    pass


class MCMCImputation(MCMCUpdate):
    pass


class MCMCUpdateDecorator:
    pass


def isdecorator(u) -> bool:
    """types.jl:65"""
    return isinstance(u, MCMCUpdateDecorator)


class TransitionKernel:
    pass


class RandomWalk(TransitionKernel):
    pass


class Adaptation:
    pass


class MCMCBackend:
    pass


class Prior:
    def logpdf(self, theta):
        raise NotImplementedError(f"logpdf not implemented for prior {type(self).__name__}.")


# flags (types.jl:122-125)
class Previous:
    pass


class Proposal:
    pass


class PreMCMCStep:
    pass


class PostMCMCStep:
    pass


# ---------------------------------------------------------------------------
# priors (src/priors.jl)
class ImproperPrior(Prior):
    """Flat prior, logpdf = 0.0 (priors.jl:18-19)."""

    def logpdf(self, theta):
        return 0.0


class ImproperPosPrior(Prior):
    """Flat prior on positive coordinates, logpdf = −Σ log θ (priors.jl:25-26)."""

    def logpdf(self, theta):
        theta = np.asarray(theta, dtype=float)
        if np.any(theta < 0):
            raise ValueError("DomainError: log of a negative number (priors.jl:26)")
        return -float(np.sum(np.log(theta)))


# prior distributions with a device plugin (Distributions.jl parameterisations);
# logpdf here is a host restatement in numpy (libm), the device and the oracle
# compute the StatsFuns forms of DESIGN.md §2 (within ~1e-15 of these)
class UnivariateDistribution:
    family = 0
    a = b = 0.0

    def to_factor(self):
        return (self.family, 1, self.a, self.b)


class Normal(UnivariateDistribution):
    family = L.DIST_NORMAL

    def __init__(self, mu=0.0, sigma=1.0):
        assert sigma > 0
        self.a, self.b = float(mu), float(sigma)

    def logpdf(self, x):
        z = (np.asarray(x, dtype=float) - self.a) / self.b
        return -(z * z + np.log(2 * np.pi)) / 2.0 - np.log(self.b)


class Uniform(UnivariateDistribution):
    family = L.DIST_UNIFORM

    def __init__(self, a=0.0, b=1.0):
        assert a < b
        self.a, self.b = float(a), float(b)

    def logpdf(self, x):
        x = np.asarray(x, dtype=float)
        return np.where((x >= self.a) & (x <= self.b), -np.log(self.b - self.a), -np.inf)


class Exponential(UnivariateDistribution):
    family = L.DIST_EXPONENTIAL

    def __init__(self, theta=1.0):
        assert theta > 0
        self.a, self.b = float(theta), 0.0

    def logpdf(self, x):
        x = np.asarray(x, dtype=float)
        lam = 1.0 / self.a
        return np.where(x < 0, -np.inf, np.log(lam) - lam * x)


class Gamma(UnivariateDistribution):
    family = L.DIST_GAMMA

    def __init__(self, alpha=1.0, theta=1.0):
        assert alpha > 0 and theta > 0
        self.a, self.b = float(alpha), float(theta)

    def logpdf(self, x):
        x = np.asarray(x, dtype=float)
        with np.errstate(divide="ignore", invalid="ignore"):
            v = -lgamma(self.a) - self.a * np.log(self.b) + (self.a - 1) * np.log(x) - x / self.b
        return np.where(x < 0, -np.inf, v)


class LogNormal(UnivariateDistribution):
    family = L.DIST_LOGNORMAL

    def __init__(self, mu=0.0, sigma=1.0):
        assert sigma > 0
        self.a, self.b = float(mu), float(sigma)

    def logpdf(self, x):
        x = np.asarray(x, dtype=float)
        with np.errstate(divide="ignore", invalid="ignore"):
            lx = np.log(x)
            z = (lx - self.a) / self.b
            v = -(z * z + np.log(2 * np.pi)) / 2.0 - np.log(self.b) - lx
        return np.where(x <= 0, -np.inf, v)


class Beta(UnivariateDistribution):
    family = L.DIST_BETA

    def __init__(self, alpha=1.0, beta=1.0):
        assert alpha > 0 and beta > 0
        self.a, self.b = float(alpha), float(beta)

    def logpdf(self, x):
        x = np.asarray(x, dtype=float)
        with np.errstate(divide="ignore", invalid="ignore"):
            t1 = 0.0 if self.a == 1 else (self.a - 1) * np.log(x)
            t2 = 0.0 if self.b == 1 else (self.b - 1) * np.log1p(-x)
            v = t1 + t2 - (lgamma(self.a) + lgamma(self.b) - lgamma(self.a + self.b))
        return np.where((x < 0) | (x > 1), -np.inf, v)


class InverseGamma(UnivariateDistribution):
    family = L.DIST_INVERSE_GAMMA

    def __init__(self, alpha=1.0, theta=1.0):
        assert alpha > 0 and theta > 0
        self.a, self.b = float(alpha), float(theta)

    def logpdf(self, x):
        x = np.asarray(x, dtype=float)
        with np.errstate(divide="ignore", invalid="ignore"):
            v = self.a * np.log(self.b) - lgamma(self.a) - (self.a + 1) * np.log(x) - self.b / x
        return np.where(x <= 0, -np.inf, v)


class Cauchy(UnivariateDistribution):
    family = L.DIST_CAUCHY

    def __init__(self, mu=0.0, sigma=1.0):
        assert sigma > 0
        self.a, self.b = float(mu), float(sigma)

    def logpdf(self, x):
        z = np.abs((np.asarray(x, dtype=float) - self.a) / self.b)
        with np.errstate(over="ignore"):  # log1psq: z² overflows long before log(1 + z²) does
            l = np.where(z < 2.0 ** 53, np.log1p(z * z), 2.0 * np.log(z))
        return -(np.log(np.pi) + np.log(self.b) + l)


class Laplace(UnivariateDistribution):
    family = L.DIST_LAPLACE

    def __init__(self, mu=0.0, theta=1.0):
        assert theta > 0
        self.a, self.b = float(mu), float(theta)

    def logpdf(self, x):
        return -(np.abs(np.asarray(x, dtype=float) - self.a) / self.b + np.log(2 * self.b))


class TDist(UnivariateDistribution):
    family = L.DIST_TDIST

    def __init__(self, nu=1.0):
        assert nu > 0
        self.a, self.b = float(nu), 0.0

    def logpdf(self, x):
        x = np.asarray(x, dtype=float)
        nu = self.a
        return (lgamma((nu + 1) / 2) - lgamma(nu / 2) - np.log(nu * np.pi) / 2
                - (nu + 1) / 2 * np.log1p(x * x / nu))


class MultivariateDistribution:
    pass


class Product(MultivariateDistribution):
    """Distributions.Product of univariates: logpdf = Σ_i logpdf(v_i, x_i), folded left."""

    def __init__(self, dists):
        self.v = list(dists)
        assert all(isinstance(d, UnivariateDistribution) for d in self.v)

    def __len__(self):
        return len(self.v)

    def logpdf(self, x):
        x = np.asarray(x, dtype=float)
        if x.ndim != 1 or x.size != len(self.v):
            raise ValueError("DimensionMismatch: length(d) != length(x)")
        return sum(float(d.logpdf(xi)) for d, xi in zip(self.v, x))

    def to_factor(self):
        return (L.DIST_PRODUCT, len(self.v), [(d.family, d.a, d.b) for d in self.v])


class MvNormal(MultivariateDistribution):
    """MvNormal(μ, Σ): logpdf = −(k·log2π + logdet Σ + (x − μ)ᵀΣ⁻¹(x − μ))/2."""

    def __init__(self, mu, Sigma):
        self.mu = np.asarray(mu, dtype=float).reshape(-1)
        self.Sigma = np.asarray(Sigma, dtype=float).reshape(self.mu.size, self.mu.size)
        self.chol = np.linalg.cholesky(np.triu(self.Sigma) + np.triu(self.Sigma, 1).T)

    def __len__(self):
        return self.mu.size

    def logpdf(self, x):
        x = np.asarray(x, dtype=float)
        if x.ndim != 1 or x.size != self.mu.size:
            raise ValueError("DimensionMismatch")
        y = np.linalg.solve(self.chol, x - self.mu)
        k = self.mu.size
        return -(k * np.log(2 * np.pi) + 2 * np.sum(np.log(np.diag(self.chol))) + float(y @ y)) / 2.0

    def to_factor(self):
        return (L.DIST_MVNORMAL, self.mu.size, self.mu, self.Sigma)


_UNIVARIATE = (UnivariateDistribution,)


def _logpdf(dist, x):
    """Distributions.logpdf(dist, x) with Julia's dispatch: a univariate needs a
    scalar, a multivariate a vector (anything else is a MethodError there)."""
    if isinstance(dist, UnivariateDistribution):
        if np.ndim(x) != 0:
            raise TypeError(f"MethodError: no method matching logpdf(::{type(dist).__name__}, ::Vector{{Float64}})")
        return float(dist.logpdf(float(x)))
    if np.ndim(x) == 0:
        raise TypeError(f"MethodError: no method matching logpdf(::{type(dist).__name__}, ::Float64)")
    return float(dist.logpdf(x))


class StandardPrior(Prior):
    """StandardPrior(dist) (priors.jl:35-39): logpdf(dist, θ).  On a coordinate
    vector only a multivariate dist has a scalar value."""

    def __init__(self, dist):
        self.dist = dist

    def logpdf(self, theta):
        return _logpdf(self.dist, np.asarray(theta, dtype=float))


class ProductPrior(Prior):
    """ProductPrior(dists, dims) (priors.jl:60-88).  The constructor's index
    list, restated (priors.jl:64-79): a factor with dims 1 gets the index 1 — it
    reads θ[1], not the next coordinate — and a factor with dims k > 1 the range
    last:last+k−1; `last` advances by dims either way.  ``idx`` holds 0-based
    ints / slices."""

    def __init__(self, dists, dims):
        idx, last = [], 0
        for d in dims:
            if d == 1:
                idx.append(0)
                last += 1
            else:
                idx.append(slice(last, last + d))
                last += d
        self.dists, self.dims, self.idx = tuple(dists), tuple(int(d) for d in dims), tuple(idx)

    def logpdf(self, theta):
        theta = np.asarray(theta, dtype=float)
        lp = 0.0
        for dist, ix in zip(self.dists, self.idx):
            if isinstance(ix, slice) and ix.stop > theta.size:
                raise IndexError("BoundsError")
            lp += _logpdf(dist, theta[ix])
        return lp


# ---------------------------------------------------------------------------
# random walkers (src/transition_kernels/random_walk.jl)
def _pos_default(n, pos):
    return np.zeros(n, dtype=bool) if pos is None else np.asarray(pos, dtype=bool).reshape(n)


class UniformRandomWalk(RandomWalk):
    """``UniformRandomWalk(ϵ, pos=false)`` (random_walk.jl:45-56)."""

    def __init__(self, eps, pos=None):
        eps_a = np.atleast_1d(np.asarray(eps, dtype=float))
        assert np.all(eps_a > 0.0), "@assert all(ϵ .> 0.0)"
        self.eps = eps_a
        self.pos = _pos_default(eps_a.size, pos)

    def __len__(self):
        return self.eps.size


class GaussianRandomWalk(RandomWalk):
    """``GaussianRandomWalk(Σ, pos=nothing)`` (random_walk.jl:123-136)."""

    def __init__(self, Sigma, pos=None):
        S = np.asarray(Sigma, dtype=float)
        if S.ndim == 0:
            S = S.reshape(1, 1)
        if S.ndim == 1:  # a length-1 vector, as in GaussianRandomWalk([1.0])
            S = np.diag(S) if S.size > 1 else S.reshape(1, 1)
        assert S.shape[0] == S.shape[1], "@assert size(Σ, 1) == size(Σ, 2)"
        self.Sigma = S
        self.pos = _pos_default(S.shape[0], pos)

    def __len__(self):
        return self.Sigma.shape[0]


class GaussianRandomWalkMix(RandomWalk):
    """``GaussianRandomWalkMix(Σ_A, Σ_B, λ=0.5, pos=nothing)`` (random_walk.jl:193-210)."""

    def __init__(self, Sigma_A, Sigma_B, lam=0.5, pos=None):
        assert 0.0 <= lam <= 1.0, "@assert 0.0 <= λ <= 1.0"
        A, B = np.asarray(Sigma_A, dtype=float), np.asarray(Sigma_B, dtype=float)
        assert A.shape == B.shape, "@assert size(Σ_A) == size(Σ_B)"
        self.gsn_A = GaussianRandomWalk(A, pos)
        self.gsn_B = GaussianRandomWalk(B, pos)
        self.lam = float(lam)

    def __len__(self):
        return len(self.gsn_A)


# ---------------------------------------------------------------------------
# adaptation (src/transition_kernels/adaptation.jl)
class NoAdaptation(Adaptation):
    """adaptation.jl:26"""

    def __eq__(self, o):
        return isinstance(o, NoAdaptation)


_UNIF_DEFAULTS = (("scale", 1.0), ("min", 1e-12), ("max", 1e7), ("offset", 1e2))


def _assure_scalar(v):
    """utility_functions.jl:16-21"""
    if np.isscalar(v):
        return v
    v = list(np.atleast_1d(v))
    assert len(v) == 1
    return v[0]


class AdaptationUnifRW(Adaptation):
    """``AdaptationUnifRW(θ; adapt_every_k_steps=100, target_accpt_rate=0.234,
    scale=1.0, min=1e-12, max=1e7, offset=1e2)`` (adaptation.jl:51-105).

    Field semantics match the reference: scalar fields when every vector-like
    kwarg has length 1 (``T = Float64``), per-coordinate vectors otherwise; ``N``
    = length(θ).  ``kind`` records the reference's element type T
    ("scalar" | "vector" | "svector") so that ``==`` follows adaptation.jl:206-213.
    """

    FIELDS = ("proposed", "accepted", "target_accpt_rate", "adapt_every_k_steps", "scale", "min", "max",
              "offset", "N")

    def __init__(self, theta=None, *, _raw=None, static=False, **kwargs):
        if _raw is not None:  # AdaptationUnifRW{T}(trgt, steps, scale, min, max, offset, N)
            (self.target_accpt_rate, self.adapt_every_k_steps, self.scale, self.min, self.max, self.offset,
             self.N, self.kind) = _raw
            self.proposed = 0
            self.accepted = 0
            return
        theta = np.atleast_1d(np.asarray(theta, dtype=float))
        n = theta.size
        trgt = float(_assure_scalar(kwargs.pop("target_accpt_rate", 0.234)))
        steps = int(_assure_scalar(kwargs.pop("adapt_every_k_steps", 100)))
        lengths = {np.atleast_1d(v).size for v in kwargs.values()}
        assert len(lengths) <= 2
        scalar = len(lengths) == 0 or max(lengths) == 1
        vals = []
        for name, default in _UNIF_DEFAULTS:
            v = kwargs.get(name, default)
            if scalar:
                vals.append(float(np.atleast_1d(v)[0]))
            else:
                a = np.atleast_1d(np.asarray(v, dtype=float))
                if a.size == 1:
                    a = np.repeat(a, n)
                assert a.size == n
                vals.append(a)
        kind = "scalar" if scalar else ("svector" if static else "vector")
        self.__init__(_raw=(trgt, steps, *vals, n, kind))

    @classmethod
    def raw(cls, target_accpt_rate, adapt_every_k_steps, scale, min, max, offset, N, kind="scalar"):
        return cls(_raw=(target_accpt_rate, adapt_every_k_steps, scale, min, max, offset, N, kind))

    def _fields_equal(self, o, skip=()):
        if not isinstance(o, AdaptationUnifRW) or self.kind != o.kind:
            return False
        for f in self.FIELDS:
            if f in skip:
                continue
            a, b = getattr(self, f), getattr(o, f)
            if not np.array_equal(np.atleast_1d(a), np.atleast_1d(b)) or np.shape(a) != np.shape(b):
                return False
        return True

    def __eq__(self, o):
        return self._fields_equal(o)

    def isequal_except(self, o, *args):
        """adaptation.jl:223-235"""
        return self._fields_equal(o, skip=args)

    # host restatement of the scalar recipes (used by tests and by the device
    # readjust kernel's parity checks)
    def acceptance_rate(self):
        return 0.0 if self.proposed == 0 else self.accepted / self.proposed

    def compute_delta(self, mcmc_iter):
        """compute_δ (adaptation.jl:312-319)"""
        return np.asarray(self.scale) / np.sqrt(np.maximum(1.0, mcmc_iter / self.adapt_every_k_steps
                                                          - np.asarray(self.offset)))


def isequal_except(a, b, *args):
    return a.isequal_except(b, *args)


class HaarioTypeAdaptation(Adaptation):
    """``HaarioTypeAdaptation(state; adapt_every_k_steps=100, scale=2.38^2, f=(x,y,z)->x)``
    (adaptation.jl:372-397)."""

    def __init__(self, state, adapt_every_k_steps=100, scale=2.38 ** 2, f: Optional[Callable] = None):
        s = np.atleast_1d(np.asarray(state, dtype=float))
        self.mean = np.zeros_like(s)
        self.cov = np.zeros((s.size, s.size))
        self.adapt_every_k_steps = int(adapt_every_k_steps)
        self.scale = float(scale)
        self.N = 1
        self.M = 0
        self.identity_f = f is None
        self.f = f if f is not None else (lambda x, y, z: x)


def prior_to_device(prior, n):
    """(EMCMC_PRIOR_*, factors) of a prior over an update's n coordinates (priors.jl).
    ProductPrior(dists, dims): one factor per dist with its dims entry as count
    (the engine rebuilds the constructor's index list); StandardPrior(dist): the
    one multivariate dist.  The pairings the reference cannot evaluate (a
    univariate over dims > 1 or on the whole vector, a multivariate over dims 1)
    raise UnsupportedPlugin, as the engine does."""
    if isinstance(prior, ImproperPrior):
        return L.PRIOR_IMPROPER, None
    if isinstance(prior, ImproperPosPrior):
        return L.PRIOR_IMPROPER_POS, None
    if isinstance(prior, ProductPrior):
        fs = []
        for dist, d in zip(prior.dists, prior.dims):
            if not isinstance(dist, (UnivariateDistribution, Product, MvNormal)):
                raise UnsupportedPlugin(f"ProductPrior factor {type(dist).__name__} has no device plugin")
            if isinstance(dist, UnivariateDistribution) != (d == 1):
                raise UnsupportedPlugin(f"ProductPrior factor {type(dist).__name__} over dims {d}: a MethodError "
                                        "in the reference (priors.jl:68-72, 85)")
            f = dist.to_factor()
            fs.append((f[0], d) + tuple(f[2:]))
        return L.PRIOR_PRODUCT, fs
    if isinstance(prior, StandardPrior):
        d = prior.dist
        if isinstance(d, (Product, MvNormal)) and len(d) == n:
            return L.PRIOR_STANDARD, [d.to_factor()]
        raise UnsupportedPlugin(f"StandardPrior({type(d).__name__}) on {n} coordinates has no scalar logpdf in the "
                                "reference (priors.jl:39) and no device plugin")
    raise UnsupportedPlugin(f"prior {type(prior).__name__} has no device plugin")


# ---------------------------------------------------------------------------
# updates (src/updates.jl)
@dataclass
class RandomWalkUpdate(MCMCParamUpdate):
    """``RandomWalkUpdate(rw, idx_of_global; prior=ImproperPrior(), adpt=NoAdaptation())``
    (updates.jl:163-183).  ``coords`` are 1-based global indices, as in the reference."""

    rw: RandomWalk
    coords: Sequence[int]
    prior: Prior = field(default_factory=ImproperPrior)
    adpt: Adaptation = field(default_factory=NoAdaptation)

    def __post_init__(self):
        self.coords = [int(c) for c in np.atleast_1d(self.coords)]
        self.invcoords = {c: i + 1 for i, c in enumerate(self.coords)}

    def to_device(self, engine):
        """Register this update with the engine (emcmc_add_update)."""
        coords0 = np.asarray(self.coords, dtype=np.int64) - 1
        prior, factors = prior_to_device(self.prior, len(self.coords))
        adapt = None
        if isinstance(self.adpt, NoAdaptation):
            pass
        elif isinstance(self.adpt, HaarioTypeAdaptation) and isinstance(self.rw, GaussianRandomWalkMix):
            adapt = {"k": self.adpt.adapt_every_k_steps, "scale": self.adpt.scale}
        elif isinstance(self.adpt, AdaptationUnifRW) and isinstance(self.rw, UniformRandomWalk):
            a = self.adpt
            adapt = {"k": a.adapt_every_k_steps, "target": a.target_accpt_rate, "scale": a.scale, "min": a.min,
                     "max": a.max, "offset": a.offset}
        else:
            raise UnsupportedPlugin(f"adaptation {type(self.adpt).__name__} has no device plugin for "
                                    f"{type(self.rw).__name__} yet")
        if isinstance(self.rw, GaussianRandomWalkMix):
            # the same pos for both components (random_walk.jl:198-205)
            pos = self.rw.gsn_A.pos
            engine.add_gaussian_rw_mix_update(coords0, self.rw.gsn_A.Sigma, self.rw.gsn_B.Sigma, lam=self.rw.lam,
                                              haario_k=None if adapt is None else adapt["k"],
                                              haario_scale=2.38 ** 2 if adapt is None else adapt["scale"],
                                              prior=prior, prior_factors=factors,
                                              pos=pos if np.any(pos) else None)
            if isinstance(self.adpt, HaarioTypeAdaptation) and not self.adpt.identity_f:
                # fλ(λ, N, mcmc_iter): one λ for all chains, called on the host at each readjust
                engine.set_mix_lambda_fn(engine.num_updates, self.adpt.f)
        elif isinstance(self.rw, GaussianRandomWalk):
            engine.add_gaussian_rw_update(coords0, self.rw.Sigma, prior=prior, prior_factors=factors,
                                          pos=self.rw.pos if np.any(self.rw.pos) else None)
        elif isinstance(self.rw, UniformRandomWalk):
            engine.add_uniform_rw_update(coords0, self.rw.eps, adapt=adapt, prior=prior, prior_factors=factors,
                                         pos=self.rw.pos if np.any(self.rw.pos) else None)
        else:
            raise UnsupportedPlugin(f"transition kernel {type(self.rw).__name__} has no device plugin yet")

    def pull_device_state(self, engine, pidx):
        """After a run: the reference mutates updt.rw.ϵ and updt.adpt in place
        (adaptation.jl:273-279); with many chains each chain has its own, so
        ``self.rw.eps_chains`` / ``self.adpt.proposed_chains`` etc. hold [C] arrays."""
        if isinstance(self.rw, GaussianRandomWalkMix):
            # per chain: the lower factor of gsn_B.Σ and, with Haario, its
            # mean/cov (= GenericChainStats mean/cov for a single update) and M
            Lb, M = engine.get_mix_state(pidx)
            self.rw.gsn_B.chol_chains = Lb
            if isinstance(self.adpt, HaarioTypeAdaptation):
                self.adpt.mean_chains, self.adpt.cov_chains = engine.get_adaptation_moments(pidx)
                self.adpt.M = M
            self.rw.lam = engine.get_mix_lambda(pidx)  # rw.λ after fλ (adaptation.jl:425)
        if isinstance(self.rw, UniformRandomWalk):
            eps, pr, ac = engine.get_update_state(pidx, len(self.rw.eps))
            self.rw.eps_chains = eps
            if isinstance(self.adpt, AdaptationUnifRW):
                self.adpt.proposed_chains, self.adpt.accepted_chains = pr, ac


@dataclass
class UserUpdate(MCMCParamUpdate):
    """A user-defined ``MCMCParamUpdate`` (the reference's update plugin surface,
    updates.jl:42-93: ``proposal!``, ``log_transition_density``; docs
    manual/updates_and_decorators.md:58-87).  Its two methods are written once as
    an ``EMCMC_USER_PROPOSAL { … } EMCMC_USER_LTD { … }`` source in the C subset the
    device compiler (hiprtc) and a C compiler both accept (include/emcmc.h
    emcmc_user_update_desc); ``params`` are its constants.  ``set_parameters!`` is
    the generic ``P°.θ[coords] ← θ°`` (updates.jl:198-205) and the prior enters the
    ratio like any update's (run.jl:374-385).  ``coords`` are 1-based."""

    source: str
    coords: Sequence[int]
    params: Sequence[float] = ()
    prior: Prior = field(default_factory=ImproperPrior)
    adpt: Adaptation = field(default_factory=NoAdaptation)
    options: str = ""

    def __post_init__(self):
        self.coords = [int(c) for c in np.atleast_1d(self.coords)]
        self.invcoords = {c: i + 1 for i, c in enumerate(self.coords)}

    def to_device(self, engine):
        if not isinstance(self.adpt, NoAdaptation):
            raise UnsupportedPlugin("adaptation of a user update has no device plugin")
        prior, factors = prior_to_device(self.prior, len(self.coords))
        engine.add_user_update(np.asarray(self.coords, dtype=np.int64) - 1, self.source, self.params,
                               options=self.options, prior=prior, prior_factors=factors)


@dataclass
class MALAUpdate(MCMCGradientBasedUpdate):
    """``MALAUpdate`` — a stub in the reference (updates.jl:216-218, "✗" at
    updates.jl:7) whose hook is ``compute_gradients_and_momenta!`` (run.jl:110,
    259).  The engine's definition: θ° = θ + (ϵ²/2)∇ℓ(θ) + ϵz with the MvNormal
    transition density both ways and the reference's accept_reject!
    (DESIGN.md §2).  Device plugins: the logistic-regression target (fused fp64
    MFMA kernel, one joint update), and GsnTargetLaw or any user law whose source
    defines ``EMCMC_USER_GRAD`` — the law's ``compute_gradients_and_momenta!`` —
    on the general kernel (any coordinates and prior, in any schedule)."""

    eps: float
    coords: Sequence[int]
    prior: Prior = field(default_factory=ImproperPrior)
    adpt: Adaptation = field(default_factory=NoAdaptation)

    def __post_init__(self):
        self.coords = [int(c) for c in np.atleast_1d(self.coords)]
        assert self.eps > 0.0

    def to_device(self, engine):
        if not isinstance(self.adpt, NoAdaptation):
            raise UnsupportedPlugin("MALA step-size adaptation has no device plugin yet")
        prior, factors = prior_to_device(self.prior, len(self.coords))
        engine.add_mala_update(np.asarray(self.coords, dtype=np.int64) - 1, self.eps, prior=prior,
                               prior_factors=factors)


class HamiltonianMCUpdate(MCMCGradientBasedUpdate):
    """Stub in the reference (updates.jl:220-222)."""
