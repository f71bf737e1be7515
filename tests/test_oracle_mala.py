"""Oracle pins for row f2 (BASELINE cfg 3): MALA on a logistic-regression
target.  The reference stubs MALAUpdate (updates.jl:216-218), so the engine's
definition is pinned by the literal numpy restatement
(oracle/literal.py run_mala_chain: BLAS products, np.logaddexp softplus, MvNormal
logpdf), by a finite-difference gradient check and by the posterior mode."""
import numpy as np
import pytest

from extensible_mcmc import workloads as W
from oracle import literal as LT


def _problem(N, D, seed=3):
    rng = np.random.default_rng(seed)
    X = rng.standard_normal((N, D)) / np.sqrt(D)
    tt = rng.standard_normal(D)
    y = (rng.random(N) < 1 / (1 + np.exp(-X @ tt))).astype(float)
    return X, y, tt


def test_loglik_and_gradient(oracle):
    X, y, _ = _problem(777, 16)
    th = np.random.default_rng(0).standard_normal((3, 16)) * 0.3
    ll, g = oracle.logistic_eval(X, y, th)
    for c in range(3):
        eta = X @ th[c]
        ref = np.sum(y * eta - np.logaddexp(0.0, eta))
        assert ll[c] == pytest.approx(ref, rel=1e-13)
        np.testing.assert_allclose(g[c], X.T @ (y - 1 / (1 + np.exp(-eta))), rtol=1e-11, atol=1e-11)
        h = 1e-6
        for d in (0, 7, 15):
            e = np.zeros(16)
            e[d] = h
            fd = (oracle.logistic_eval(X, y, th[c] + e)[0][0] - oracle.logistic_eval(X, y, th[c] - e)[0][0]) / (2 * h)
            assert g[c, d] == pytest.approx(fd, rel=1e-6, abs=1e-6)


def test_extreme_linear_predictors(oracle):
    """softplus / σ stay finite and exact in the tails (|η| up to 800)."""
    X = np.array([[1.0], [1.0], [1.0], [1.0]])
    y = np.array([1.0, 0.0, 1.0, 0.0])
    for t in (-800.0, -40.0, 0.0, 40.0, 800.0):
        ll, g = oracle.logistic_eval(X, y, [[t]])
        assert np.isfinite(ll[0]) and np.isfinite(g[0, 0])
        assert ll[0] == pytest.approx(2 * (t - np.logaddexp(0, t)) - 2 * np.logaddexp(0, t), rel=1e-14)


@pytest.mark.parametrize("D,eps", [(16, 0.08), (64, 0.3)])
def test_mala_matches_literal(oracle, D, eps):
    X, y, _ = _problem(1500, D)
    C, S = 4, 150
    st = oracle.MALAState(np.zeros((C, D)), X, y)
    h = oracle.run_mala(st, seed=11, eps=eps, X=X, y=y, iter0=1, nsteps=S)
    for c in range(C):
        o = LT.run_mala_chain(11, c, np.zeros(D), eps, X, y, S)
        assert np.array_equal(o["acc"], h["acc"][:, c]), f"chain {c}: accept stream"
        np.testing.assert_allclose(o["theta"], h["theta"][:, c], rtol=1e-10, atol=1e-12)
        np.testing.assert_allclose(o["ll"][1:], h["ll"][1:, c], rtol=1e-12)
        np.testing.assert_allclose(o["ra"][-1], st.ra[c], rtol=1e-13)
    assert 0.3 < h["acc"].mean() < 1.0


def test_mala_centres_on_the_posterior_mode(oracle):
    """θ after burn-in scatters around the MAP (flat prior = MLE, found by Newton)."""
    X, y, _ = _problem(2000, 16)
    th = np.zeros(16)
    for _ in range(30):
        p = 1 / (1 + np.exp(-X @ th))
        H = (X * (p * (1 - p))[:, None]).T @ X
        th = th + np.linalg.solve(H, X.T @ (y - p))
    C = 64
    st = oracle.MALAState(np.zeros((C, 16)), X, y, nthreads=8)
    h = oracle.run_mala(st, seed=5, eps=0.1, X=X, y=y, iter0=1, nsteps=400, nthreads=8)
    draws = h["theta"][200:].reshape(-1, 16)
    sd = np.sqrt(np.diag(np.linalg.inv(H)))
    assert np.all(np.abs(draws.mean(axis=0) - th) < 0.25 * sd)
    np.testing.assert_allclose(draws.std(axis=0), sd, rtol=0.2)


def test_cfg3_workload_shape():
    w = W.cfg3(4, nobs=1000)
    assert w.X.shape == (1000, 64) and set(np.unique(w.y)) <= {0.0, 1.0}
