"""MALA on the general schedule path — the engine's definition of the reference's
stub MALAUpdate (updates.jl:216-218) through the hook a gradient-based update
has, compute_gradients_and_momenta! (updates.jl:123-133, called at run.jl:110 on
the current state and run.jl:259 on the proposal): oracle pins.

The C restatement (orc_run_mwg, kind 4) is checked against the literal numpy
restatement (oracle/literal.py run_mwg_chain: ∇ℓ by LAPACK solves, MvNormal
logpdfs as written) to fp64 tolerance, with the accept/reject stream equal; the
user law's gradient (tests/user_targets/logistic_regression.c, EMCMC_USER_GRAD)
against its numpy formula.  The reference has no MALA numbers, so these pins are
the engine's definition ("parity unpinned" against the reference by nature)."""
from types import SimpleNamespace

import numpy as np
import pytest

from extensible_mcmc import _lib as L
from extensible_mcmc import workloads as W
from extensible_mcmc.schedule import MCMCSchedule
from oracle import literal as LT
from test_oracle_mwg import full_steps


def compare(oracle, w, ups, steps, C, mu0, theta0):
    st = oracle.MWGState(np.tile(np.asarray(theta0, dtype=float), (C, 1)), mu0, ups)
    h = oracle.run_mwg(st, ups, seed=w.seed, t_sigma=w.t_sigma, obs=w.obs, steps=steps)
    for c in range(C):
        o = LT.run_mwg_chain(w.seed, c, list(theta0), mu0, ups, w.t_sigma, w.obs, steps)
        assert np.array_equal(np.array(o["acc"]), h["acc"][:, c]), f"chain {c}: accept stream"
        np.testing.assert_allclose(np.array(o["theta"]), h["theta"][:, c], rtol=1e-11, atol=1e-12)
        np.testing.assert_allclose(np.array(o["prop"]), h["prop"][:, c], rtol=1e-11, atol=1e-12)
        llo = np.array(o["ll"])
        fin = np.isfinite(llo)
        np.testing.assert_allclose(llo[fin], h["ll"][fin, c], rtol=1e-11, atol=1e-10)
    return st, h


def test_joint_mala_on_reference_gsn_target(oracle):
    """The reference test's GsnTargetLaw([1,2], [1 .5; .5 1]) with 10 observations
    (test/runtests.jl:87-114), one joint MALA update, ϵ = 0.35."""
    w = W.ref_test()
    ups = [oracle.mwg_update(oracle.KIND_MALA, [0, 1], eps=[0.35])]
    st, h = compare(oracle, w, ups, full_steps(300, 1), 6, [1.0, 2.0], (0.0, 0.0))
    assert 0.2 < h["acc"][1:].mean() < 0.99
    # the chains find the posterior mean (flat prior: x̄)
    assert np.allclose(h["theta"][100:].mean(axis=(0, 1)), np.asarray(w.obs).mean(0), atol=0.15)


def test_mala_inside_a_gibbs_schedule(oracle):
    """MALA on coordinate 2 beside a GaussianRandomWalk on coordinate 1, update 1
    excluded on iterations 10:30: ∇ℓ at P°.θ with the update's coordinate at θ."""
    w = W.ref_test()
    ups = [oracle.mwg_update(2, [0], sigma=[[0.3]]), oracle.mwg_update(oracle.KIND_MALA, [1], eps=[0.4])]
    steps = [(s.mcmciter, s.pidx) for s in MCMCSchedule(200, 2, [(1, range(10, 31))])]
    compare(oracle, w, ups, steps, 5, [1.0, 2.0], (0.5, -0.5))


def test_mala_block_on_a_dense_four_dimensional_target(oracle):
    rng = np.random.default_rng(7)
    D = 4
    A = rng.normal(size=(D, D))
    S = A @ A.T / D + np.eye(D)
    mu = rng.normal(size=D)
    obs = rng.multivariate_normal(mu, S, size=12)
    w = SimpleNamespace(seed=20261017, t_sigma=S, obs=obs)
    ups = [oracle.mwg_update(oracle.KIND_MALA, [3, 0, 2], eps=[0.25]), oracle.mwg_update(1, [1], eps=[0.6])]
    compare(oracle, w, ups, full_steps(150, 2), 4, mu, np.zeros(D))


def _logistic_case(D=3, n=60, seed=5):
    rng = np.random.default_rng(seed)
    X = np.column_stack([np.ones(n), rng.normal(size=(n, D - 1))])
    beta = np.array([0.3, -1.0, 0.8, 0.5][:D])
    y = (rng.uniform(size=n) < 1.0 / (1.0 + np.exp(-(X @ beta)))).astype(float)
    return X, y


def _np_ll_grad(X, y, th):
    eta = X @ th
    ll = float(np.sum(y * eta - np.logaddexp(0.0, eta)))
    return ll, X.T @ (y - 1.0 / (1.0 + np.exp(-eta)))


def test_user_law_gradient_matches_its_formula(oracle):
    X, y = _logistic_case()
    fn, _ = oracle.user_loglik("logistic_regression")
    gfn = oracle.user_grad("logistic_regression")
    obs = np.ascontiguousarray(np.column_stack([X, y]))
    rng = np.random.default_rng(1)
    import ctypes as C
    dp = C.POINTER(C.c_double)
    for _ in range(5):
        th = np.ascontiguousarray(rng.normal(size=3))
        g = np.zeros(3)
        gfn(th.ctypes.data_as(dp), 3, obs.ctypes.data_as(dp), len(y), None, g.ctypes.data_as(dp))
        ll = fn(th.ctypes.data_as(dp), 3, obs.ctypes.data_as(dp), len(y), None)
        want_ll, want_g = _np_ll_grad(X, y, th)
        assert ll == pytest.approx(want_ll, rel=1e-13)
        np.testing.assert_allclose(g, want_g, rtol=1e-12, atol=1e-12)


def test_mala_on_a_user_law_with_gradient(oracle):
    """Joint MALA on the user logistic-regression law: the oracle's chain against
    a numpy MALA loop with the same variates (flat prior; P°.θ = θ for a joint update)."""
    X, y = _logistic_case()
    D, C, M, eps, seed = 3, 4, 120, 0.3, 99
    fn, _ = oracle.user_loglik("logistic_regression")
    gfn = oracle.user_grad("logistic_regression")
    obs = np.column_stack([X, y])
    ups = [oracle.mwg_update(oracle.KIND_MALA, range(D), eps=[eps])]
    st = oracle.MWGState(np.zeros((C, D)), np.zeros(D), ups)
    h = oracle.run_mwg(st, ups, seed=seed, t_sigma=None, obs=obs, steps=full_steps(M, 1), user_ll=fn,
                       user_grad=gfn)
    hm, Le = eps * eps / 2.0, eps * np.eye(D)
    for c in range(C):
        th, ll = np.zeros(D), -np.inf
        for it in range(1, M + 1):
            _, g = _np_ll_grad(X, y, th)
            z, E, _ = oracle.step_variates(seed, c, it, D)
            m = th + hm * g
            tp = m + eps * z
            llp, gp = _np_ll_grad(X, y, tp)
            llr = llp - ll + LT.mvnormal_logpdf(th, tp + hm * gp, Le) - LT.mvnormal_logpdf(tp, m, Le)
            acc = E > -llr
            assert acc == h["acc"][it - 1, c], (c, it)
            if acc:
                th, ll = tp, llp
            np.testing.assert_allclose(h["theta"][it - 1, c], th, rtol=1e-11, atol=1e-12)
    assert 0.3 < h["acc"][1:].mean() < 0.99


def test_mala_on_a_user_law_without_gradient_is_refused(oracle):
    fn, _ = oracle.user_loglik("poisson_regression")
    ups = [oracle.mwg_update(oracle.KIND_MALA, [0, 1, 2], eps=[0.1])]
    st = oracle.MWGState(np.zeros((2, 3)), np.zeros(3), ups)
    with pytest.raises(ValueError):
        oracle.run_mwg(st, ups, seed=1, t_sigma=None, obs=np.zeros((4, 4)), steps=[(1, 1)], user_ll=fn)


def test_law_with_gradient_compiles_for_the_device_with_mala():
    """hiprtc (gfx950) accepts the EMCMC_USER_GRAD law with the MALA path compiled in."""
    from pathlib import Path

    src = (Path(__file__).resolve().parent / "user_targets" / "logistic_regression.c").read_text()
    L.check_user_target(src, 3)
