"""Oracle pins for the general schedule path (P ≥ 1 updates, Metropolis-within-
Gibbs): the C restatement orc_run_mwg against the literal numpy restatement
(oracle/literal.py run_mwg_chain) on the reference's own test workload
(test/runtests.jl:87-114), the tutorial's adaptive and Gaussian single-site
setups (docs/src/tutorials/mean_of_bivariate_gaussian.md), schedules with
exclusions, and the analytic posterior."""
import numpy as np
import pytest

from extensible_mcmc import workloads as W
from extensible_mcmc.schedule import MCMCSchedule
from oracle import literal as LT

ADAPT = {"k": 50, "target": 0.234, "scale": 0.1, "min": 1e-12, "max": 1e7, "offset": 1e2}


def ref_updates(oracle, kind="uniform", eps=1.0, adapt=None):
    if kind == "uniform":
        return [oracle.mwg_update(1, [0], eps=[eps], adapt=adapt), oracle.mwg_update(1, [1], eps=[eps], adapt=adapt)]
    return [oracle.mwg_update(2, [0], sigma=[[1.0]]), oracle.mwg_update(2, [1], sigma=[[1.0]])]


def full_steps(M, P):
    return [(i, p) for i in range(1, M + 1) for p in range(1, P + 1)]


def compare_with_literal(oracle, w, ups, steps, C, mu0, theta0=(0.0, 0.0)):
    st = oracle.MWGState(np.tile(theta0, (C, 1)), mu0, ups)
    h = oracle.run_mwg(st, ups, seed=w.seed, t_sigma=w.t_sigma, obs=w.obs, steps=steps)
    for c in range(C):
        o = LT.run_mwg_chain(w.seed, c, list(theta0), mu0, ups, w.t_sigma, w.obs, steps)
        assert np.array_equal(np.array(o["acc"]), h["acc"][:, c]), f"chain {c}: accept stream"
        np.testing.assert_array_equal(np.array(o["theta"]), h["theta"][:, c])
        np.testing.assert_array_equal(np.array(o["prop"]), h["prop"][:, c])
        llo = np.array(o["ll"])
        fin = np.isfinite(llo)
        np.testing.assert_allclose(llo[fin], h["ll"][fin, c], rtol=1e-13, atol=1e-12)
        for p in range(len(ups)):
            last = [r for (it, q), r in zip(steps, o["ra"]) if q == p + 1][-1]
            np.testing.assert_allclose(st.ra[p, c], last, rtol=1e-13)
            if ups[p]["adapt"] is not None:
                np.testing.assert_array_equal(st.eps[p, c, :len(ups[p]["coords"])], o["eps"][-1][p])
    return st, h


def test_reference_test_workload(oracle):
    """test/runtests.jl:87-114: two single-site UniformRandomWalk([1.0]) updates,
    GsnTargetLaw([1,2], [1 .5; .5 1]), 10 observations, θinit = [0,0]."""
    w = W.ref_test()
    compare_with_literal(oracle, w, ref_updates(oracle), full_steps(300, 2), 8, [1.0, 2.0])


def test_tutorial_adaptive_uniform(oracle):
    """mean_of_bivariate_gaussian.md: UniformRandomWalk([0.1]) + AdaptationUnifRW(k=50, scale=0.1)."""
    w = W.ref_test()
    st, _ = compare_with_literal(oracle, w, ref_updates(oracle, eps=0.1, adapt=ADAPT), full_steps(400, 2), 6,
                                 [1.0, 2.0])
    assert np.all(st.eps[:, :, 0] != 0.1)  # ϵ moved at every readjust
    assert np.all(st.aprop == 400 % 50)


def test_tutorial_gaussian_single_site(oracle):
    w = W.ref_test()
    compare_with_literal(oracle, w, ref_updates(oracle, kind="gaussian"), full_steps(300, 2), 6, [1.0, 2.0])


def test_exclusions_schedule(oracle):
    """exclude_updates (run.jl:43, schedule.jl): update 2 skipped on iterations 5:40."""
    w = W.ref_test()
    sch = MCMCSchedule(120, 2, [(2, range(5, 41))])
    steps = [(s.mcmciter, s.pidx) for s in sch]
    assert (10, 2) not in steps and (10, 1) in steps
    compare_with_literal(oracle, w, ref_updates(oracle, eps=0.5), steps, 5, [1.0, 2.0])


def test_single_joint_update_matches_fused_oracle(oracle):
    """P = 1 joint GaussianRandomWalk over 1:D: the general path and the fused
    single-update restatement give the same bits."""
    w = W.cfg2(32)
    D = 16
    rw = w.rw_sigma[:D, :D]
    ts = w.t_sigma[:D, :D]
    obs = np.asarray(w.obs)[:, :D]
    mu = np.asarray(w.mu_true)[:D]
    ups = [oracle.mwg_update(2, list(range(D)), sigma=rw)]
    st = oracle.MWGState(np.zeros((32, D)), mu, ups)
    h = oracle.run_mwg(st, ups, seed=w.seed, t_sigma=ts, obs=obs, steps=full_steps(150, 1))
    so = oracle.OracleState(np.zeros((32, D)))
    ho = oracle.run_gsn(so, seed=w.seed, rw_sigma=rw, t_sigma=ts, obs=obs, iter0=1, nsteps=150)
    assert np.array_equal(h["acc"], ho["acc"])
    assert np.array_equal(h["theta"], ho["theta"])
    assert np.array_equal(h["ll"], ho["ll"])
    assert np.array_equal(st.ra[0], so.ra)


def test_pmu_quirk_is_reproduced(oracle):
    """P° starts at the target's μ (workspaces.jl:231-232 deepcopy(data.P)) and
    keeps each update's last *proposal* (updates.jl:198-205): the first ll is
    evaluated with μ₂ = 2.0, not θinit₂ = 0."""
    w = W.ref_test()
    ups = ref_updates(oracle)
    st = oracle.MWGState(np.zeros((1, 2)), [1.0, 2.0], ups)
    h = oracle.run_mwg(st, ups, seed=w.seed, t_sigma=w.t_sigma, obs=w.obs, steps=[(1, 1)])
    th1 = h["prop"][0, 0, 0]
    want = sum(LT.mvnormal_logpdf(x, [th1, 2.0], np.linalg.cholesky(w.t_sigma)) for x in np.asarray(w.obs))
    assert h["acc"][0, 0]  # step 1 auto-accepts (ll = −Inf)
    assert h["ll"][0, 0] == pytest.approx(want, rel=1e-13)
    assert st.mu_p[0, 1] == 2.0


def test_posterior_mean_single_site(oracle):
    """With P's μ equal to θinit (no start-up offset), single-site Gaussian
    updates centre on x̄.  Only the mean is checked: because P° keeps the other
    coordinate's last *proposal* (accepted or not), the reference's
    Metropolis-within-Gibbs chain is not exactly N(x̄, Σ/n) — its correlation is
    damped and its variances inflated (≈0.02 vs 0.05, ≈0.11 vs 0.10 here), and
    the engine reproduces that, not the textbook posterior."""
    w = W.ref_test()
    xbar = np.asarray(w.obs).mean(axis=0)
    ups = ref_updates(oracle, kind="gaussian")
    C, M = 2048, 600
    st = oracle.MWGState(np.tile(xbar, (C, 1)), xbar, ups)
    h = oracle.run_mwg(st, ups, seed=w.seed, t_sigma=w.t_sigma, obs=w.obs, steps=full_steps(M, 2), nthreads=8)
    draws = h["theta"][M:].reshape(-1, 2)
    se = np.sqrt(np.diag(np.asarray(w.t_sigma)) / len(w.obs) / (C * 10))  # ≥ 10 draws/chain of information
    assert np.all(np.abs(draws.mean(axis=0) - xbar) < 6 * se)


def test_uniform_rw_positivity_restricted_against_literal(oracle):
    """UniformRandomWalk(ϵ, pos) (random_walk.jl:63-94): θ° = θ·e^U where pos
    (θ + U elsewhere) and logpdf(θ, θ°) = Σ_pos −log(2ϵ) − log θ°, which no longer
    cancels between the two directions.  The literal restatement uses numpy's
    exp/log, the oracle its own: θ within 1e-14 relative, the accept stream equal."""
    w = W.ref_test()
    ups = [oracle.mwg_update(1, [0], eps=[0.5], pos=[True]), oracle.mwg_update(1, [1], eps=[0.8], pos=[False])]
    C, theta0 = 6, [1.5, 0.5]
    steps = full_steps(300, 2)
    st = oracle.MWGState(np.tile(theta0, (C, 1)), [1.0, 2.0], ups)
    h = oracle.run_mwg(st, ups, seed=w.seed, t_sigma=w.t_sigma, obs=w.obs, steps=steps)
    for c in range(C):
        o = LT.run_mwg_chain(w.seed, c, list(theta0), [1.0, 2.0], ups, w.t_sigma, w.obs, steps)
        assert np.array_equal(np.array(o["acc"]), h["acc"][:, c]), f"chain {c}: accept stream"
        np.testing.assert_allclose(np.array(o["theta"]), h["theta"][:, c], rtol=1e-14)
        np.testing.assert_allclose(np.array(o["prop"]), h["prop"][:, c], rtol=1e-14)
    assert np.all(h["theta"][:, :, 0] > 0)  # the restricted coordinate stays positive
    # the restricted coordinate's moves are multiplicative: log θ° − log θ = U ∈ [−ϵ, ϵ]
    lr = np.log(h["prop"][1:, :, 0]) - np.log(h["theta"][:-1, :, 0])
    moved = np.array([p == 1 for _, p in steps])[1:]
    assert np.all(np.abs(lr[moved]) <= 0.5 + 1e-12)


def test_gaussian_rw_positivity_restricted_against_literal(oracle):
    """GaussianRandomWalk(Σ, pos) (random_walk.jl:136-171): the walk on log θ for the
    restricted coordinates, the log-Jacobian −Σ_pos log θ in each transition density,
    and the reference's in-place exp/log round trips (the literal restatement
    mutates its arrays exactly as rand/logpdf do).  numpy exp/log against the
    oracle's own: θ within 1e-13 relative, the accept stream equal."""
    w = W.ref_test()
    ups = [oracle.mwg_update(2, [0, 1], sigma=[[0.09, 0.02], [0.02, 0.04]], pos=[True, False])]
    C, theta0 = 6, [1.5, 0.5]
    steps = full_steps(300, 1)
    st = oracle.MWGState(np.tile(theta0, (C, 1)), [1.0, 2.0], ups)
    h = oracle.run_mwg(st, ups, seed=w.seed, t_sigma=w.t_sigma, obs=w.obs, steps=steps)
    for c in range(C):
        o = LT.run_mwg_chain(w.seed, c, list(theta0), [1.0, 2.0], ups, w.t_sigma, w.obs, steps)
        assert np.array_equal(np.array(o["acc"]), h["acc"][:, c]), f"chain {c}: accept stream"
        np.testing.assert_allclose(np.array(o["theta"]), h["theta"][:, c], rtol=1e-13)
        np.testing.assert_allclose(np.array(o["prop"]), h["prop"][:, c], rtol=1e-13)
    assert np.all(h["theta"][:, :, 0] > 0) and np.all(h["prop"][:, :, 0] > 0)
    assert 0.05 < h["acc"].mean() < 0.95


VEC_ADAPT = {"k": 40, "target": 0.234, "scale": [0.05, 0.2], "min": [1e-12, 0.02], "max": [1e7, 0.5],
             "offset": [1e2, 3.0]}


def test_per_coordinate_adaptation_against_literal(oracle):
    """AdaptationUnifRW in its per-coordinate form (adaptation.jl:155-188) on a
    block UniformRandomWalk over both coordinates: δ_i = scale_i/√max(1, iter/k −
    offset_i) and clamp(·, min_i, max_i) coordinate by coordinate (the reference's
    readjust! has no method for `Float64 - Vector`; include/emcmc.h documents the
    elementwise reading)."""
    w = W.ref_test()
    ups = [oracle.mwg_update(1, [0, 1], eps=[0.1, 0.3], adapt=VEC_ADAPT)]
    st, _ = compare_with_literal(oracle, w, ups, full_steps(600, 1), 6, [1.0, 2.0])
    e = st.eps[0, :, :2]
    assert np.all(e[:, 1] <= 0.5) and np.all(e[:, 1] >= 0.02)  # per-coordinate clamp active
    assert not np.allclose(e[:, 0], e[:, 1])


def test_scalar_adaptation_equals_repeated_vector(oracle):
    """The scalar form is the per-coordinate form with repeated entries, bit for bit."""
    w = W.ref_test()
    sc = dict(ADAPT)
    vec = {k: ([v, v] if k in ("scale", "min", "max", "offset") else v) for k, v in sc.items()}
    runs = []
    for a in (sc, vec):
        ups = [oracle.mwg_update(1, [0, 1], eps=[0.1, 0.2], adapt=a)]
        st = oracle.MWGState(np.zeros((64, 2)), [1.0, 2.0], ups)
        oracle.run_mwg(st, ups, seed=w.seed, t_sigma=w.t_sigma, obs=w.obs, steps=full_steps(300, 1), history=False)
        runs.append(st)
    assert np.array_equal(runs[0].eps, runs[1].eps) and np.array_equal(runs[0].theta, runs[1].theta)
