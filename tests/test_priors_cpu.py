"""Priors (src/priors.jl) on the CPU: the oracle's restatement (orc_eval_prior)
and the Python mirror, pinned against values derived by hand from priors.jl and
against scipy.stats.

priors.jl:64-79 builds ProductPrior's index list with `push!(dims_reformatted,
dim)` for dims == 1, i.e. the *integer 1*: every univariate factor reads θ[1],
whatever its position, while a factor with dims k > 1 reads last:last+k-1 with
`last` advanced by every factor's dims.  These tests pin exactly that."""
import math

import numpy as np
import pytest
from scipy import stats

from extensible_mcmc import (Beta, Cauchy, Exponential, Gamma, InverseGamma, Laplace, LogNormal, MvNormal, Normal,
                             Product, ProductPrior, StandardPrior, TDist, Uniform)
from extensible_mcmc import _lib as L
from extensible_mcmc.kernels import UnsupportedPlugin, prior_to_device

LOG2PI = math.log(2 * math.pi)


def normal_lp(mu, s, x):  # Distributions.logpdf(Normal(μ, σ), x) = normlogpdf((x−μ)/σ) − log σ
    z = (x - mu) / s
    return -(z * z + LOG2PI) / 2 - math.log(s)


def gamma_lp(a, t, x):  # Distributions.logpdf(Gamma(α, θ), x)
    return -math.lgamma(a) - a * math.log(t) + (a - 1) * math.log(x) - x / t


def test_verdict_case_every_dims1_factor_reads_theta1(oracle):
    """ProductPrior([Normal(1, .5), Gamma(4, .5)], [1, 1]) on a 2-coordinate update:
    logpdf = 0.0 + logpdf(Normal(1,.5), θ[1]) + logpdf(Gamma(4,.5), θ[1]) — θ[2] is never read."""
    pr = ProductPrior([Normal(1.0, 0.5), Gamma(4.0, 0.5)], [1, 1])
    assert pr.idx == (0, 0)
    xs = np.array([[0.7, 3.0], [0.7, -5.0], [1.9, 0.25], [2.5, 1e6]])
    want = np.array([(0.0 + normal_lp(1.0, 0.5, x1)) + gamma_lp(4.0, 0.5, x1) for x1, _ in xs])
    # −1.894986931449199 at θ = (0.7, ·), by hand: −0.405791… + (−1.489196…)
    assert want[0] == pytest.approx(-1.894986931449199, abs=1e-14)
    assert want[0] == want[1]  # θ[2] does not enter
    for x, w in zip(xs, want):
        assert pr.logpdf(x) == pytest.approx(w, rel=1e-14)
    kind, fs = prior_to_device(pr, 2)
    assert kind == L.PRIOR_PRODUCT and [f[:2] for f in fs] == [(L.DIST_NORMAL, 1), (L.DIST_GAMMA, 1)]
    got = oracle.eval_prior(kind, 2, fs, xs)
    np.testing.assert_allclose(got, want, rtol=2e-15, atol=0)


def test_constructor_index_list_mixed_dims(oracle):
    """ProductPrior([Normal(), MvNormal(μ, Σ), Exponential(2)], [1, 3, 1]) on 5 coordinates:
    idx = (1, 2:4, 1) — last starts at 1, becomes 2 after the dims-1 factor, 5 after the MvNormal."""
    rng = np.random.default_rng(1)
    B = rng.standard_normal((3, 3))
    S = B @ B.T + np.eye(3)
    mu = np.array([0.5, -1.0, 2.0])
    pr = ProductPrior([Normal(0.0, 2.0), MvNormal(mu, S), Exponential(2.0)], [1, 3, 1])
    assert pr.idx == (0, slice(1, 4), 0)
    xs = np.abs(rng.standard_normal((6, 5))) + 0.1
    want = np.array([((0.0 + stats.norm(0, 2).logpdf(x[0])) + stats.multivariate_normal(mu, S).logpdf(x[1:4]))
                     + stats.expon(scale=2.0).logpdf(x[0]) for x in xs])
    np.testing.assert_allclose([pr.logpdf(x) for x in xs], want, rtol=1e-13)
    kind, fs = prior_to_device(pr, 5)
    np.testing.assert_allclose(oracle.eval_prior(kind, 5, fs, xs), want, rtol=1e-13)


FAMILIES = [
    (Normal(0.3, 1.7), stats.norm(0.3, 1.7), 0.9),
    (Uniform(-2.0, 3.0), stats.uniform(-2.0, 5.0), 0.4),
    (Exponential(2.5), stats.expon(scale=2.5), 1.3),
    (Gamma(3.0, 0.7), stats.gamma(3.0, scale=0.7), 2.2),
    (LogNormal(0.2, 0.6), stats.lognorm(0.6, scale=math.exp(0.2)), 1.4),
    (Beta(2.5, 4.0), stats.beta(2.5, 4.0), 0.3),
    (InverseGamma(3.0, 2.0), stats.invgamma(3.0, scale=2.0), 0.8),
    (Cauchy(-1.0, 0.5), stats.cauchy(-1.0, 0.5), 0.2),
    (Laplace(0.5, 1.5), stats.laplace(0.5, 1.5), -0.7),
    (TDist(4.5), stats.t(4.5), 1.1),
]


@pytest.mark.parametrize("dist,ref,x0", FAMILIES, ids=[type(f[0]).__name__ for f in FAMILIES])
def test_univariate_family_against_scipy(oracle, dist, ref, x0):
    """Each family's logpdf (the StatsFuns form of DESIGN.md §2, engine exp/log) against scipy."""
    xs = x0 + np.linspace(-0.25, 0.25, 11)
    if isinstance(dist, Beta):
        xs = np.clip(xs, 0.01, 0.99)
    if isinstance(dist, (Exponential, Gamma, LogNormal, InverseGamma)):
        xs = np.abs(xs) + 0.05
    pr = ProductPrior([dist], [1])
    kind, fs = prior_to_device(pr, 1)
    got = oracle.eval_prior(kind, 1, fs, xs.reshape(-1, 1))
    want = 0.0 + ref.logpdf(xs)
    np.testing.assert_allclose(got, want, rtol=1e-12, atol=1e-13)
    np.testing.assert_allclose([pr.logpdf([x]) for x in xs], want, rtol=1e-12, atol=1e-13)


def test_cauchy_far_tail_stays_finite(oracle):
    """Cauchy's log(1 + z²) as StatsFuns' log1psq: past |z| = 2^53 it is 2·log|z|, so a
    far-tail θ (z² overflows at |z| > 1.34e154) still has a finite log density."""
    a, b = -1.0, 0.5
    xs = np.array([1e20, -1e20, 3e100, 1e200, -1e300, 1e16, 2.0 ** 53 * 0.5 + a])
    pr = ProductPrior([Cauchy(a, b)], [1])
    kind, fs = prior_to_device(pr, 1)
    z = np.abs((xs - a) / b)
    want = np.array([-(math.log1p(v * v) if v < 2.0 ** 53 else 2.0 * math.log(v)) - math.log(math.pi) - math.log(b)
                     for v in z])
    got = oracle.eval_prior(kind, 1, fs, xs.reshape(-1, 1))
    assert np.all(np.isfinite(got))
    np.testing.assert_allclose(got, want, rtol=2e-15, atol=0)
    np.testing.assert_allclose([pr.logpdf([x]) for x in xs], want, rtol=2e-15, atol=0)


@pytest.mark.parametrize("dist,x", [(Uniform(0.0, 1.0), 1.5), (Exponential(1.0), -0.1), (Gamma(2.0, 1.0), -1.0),
                                    (LogNormal(0.0, 1.0), -0.5), (LogNormal(0.0, 1.0), 0.0), (Beta(2.0, 2.0), 1.2),
                                    (Beta(2.0, 2.0), -0.2), (InverseGamma(2.0, 1.0), 0.0)])
def test_outside_support_is_minus_inf(oracle, dist, x):
    kind, fs = prior_to_device(ProductPrior([dist], [1]), 1)
    assert oracle.eval_prior(kind, 1, fs, [[x]])[0] == -np.inf


def test_standard_prior_of_product_and_mvnormal(oracle):
    comps = [f[0] for f in FAMILIES]
    pr = StandardPrior(Product(comps))
    rng = np.random.default_rng(7)
    xs = np.array([f[2] for f in FAMILIES]) + 0.05 * rng.standard_normal((5, len(comps)))
    want = np.array([sum(f[1].logpdf(xi) for f, xi in zip(FAMILIES, x)) for x in xs])
    kind, fs = prior_to_device(pr, len(comps))
    assert kind == L.PRIOR_STANDARD and fs[0][0] == L.DIST_PRODUCT
    np.testing.assert_allclose(oracle.eval_prior(kind, len(comps), fs, xs), want, rtol=1e-12)
    B = rng.standard_normal((6, 6))
    S = B @ B.T / 6 + np.eye(6)
    mu = rng.standard_normal(6)
    pr = StandardPrior(MvNormal(mu, S))
    xs = rng.standard_normal((5, 6))
    kind, fs = prior_to_device(pr, 6)
    want = stats.multivariate_normal(mu, S).logpdf(xs)
    np.testing.assert_allclose(oracle.eval_prior(kind, 6, fs, xs), want, rtol=1e-13)
    np.testing.assert_allclose([pr.logpdf(x) for x in xs], want, rtol=1e-13)


def test_pairings_the_reference_cannot_evaluate_are_refused(oracle):
    """A univariate over dims > 1 reads θ[a:b] (logpdf(::Normal, ::Vector): MethodError),
    a multivariate over dims 1 reads the scalar θ[1], a univariate StandardPrior reads the
    whole vector: the mirror raises UnsupportedPlugin and the oracle returns −4 (the engine
    EMCMC_UNSUPPORTED_PLUGIN, tests/test_gpu_priors.py)."""
    bad = [(ProductPrior([Normal()], [3]), 3), (ProductPrior([Product([Normal()])], [1]), 1),
           (StandardPrior(Normal()), 1)]
    for pr, n in bad:
        with pytest.raises(UnsupportedPlugin):
            prior_to_device(pr, n)
        with pytest.raises((TypeError, ValueError)):
            pr.logpdf(np.zeros(n))
    tables = [(L.PRIOR_PRODUCT, 3, [(L.DIST_NORMAL, 3, 0.0, 1.0)]),
              (L.PRIOR_PRODUCT, 1, [(L.DIST_PRODUCT, 1, [(L.DIST_NORMAL, 0.0, 1.0)])]),
              (L.PRIOR_STANDARD, 1, [(L.DIST_NORMAL, 1, 0.0, 1.0)])]
    for kind, n, fs in tables:
        with pytest.raises(ValueError, match="-4"):
            oracle.eval_prior(kind, n, fs, np.zeros((1, n)))
    # a dims > 1 factor past the update's coordinates: BoundsError in the reference
    with pytest.raises(ValueError, match="-2"):
        oracle.eval_prior(L.PRIOR_PRODUCT, 2, [(L.DIST_NORMAL, 1, 0.0, 1.0),
                                               (L.DIST_PRODUCT, 2, [(L.DIST_NORMAL, 0.0, 1.0)] * 2)], np.zeros((1, 2)))
    with pytest.raises(IndexError):
        ProductPrior([Normal(), Product([Normal(), Normal()])], [1, 2]).logpdf(np.zeros(2))
