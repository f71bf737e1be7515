"""The reference-shaped API end to end on the GPU: MCMC(...) + run(...) with the
MI355X backend, mirroring the reference's "mcmc" testset and tutorial
(test/runtests.jl:87-114, docs/src/tutorials/mean_of_bivariate_gaussian.md)."""
import numpy as np
import pytest

from extensible_mcmc import (MCMC, AdaptationUnifRW, GaussianRandomWalk, GaussianRandomWalkMix, GsnTargetLaw,
                             HaarioTypeAdaptation, ImproperPrior, MI355XBackend, RandomWalkUpdate, REPLCallback, SavingCallback,
                             UniformRandomWalk, UnsupportedPlugin, run)
from extensible_mcmc import workloads as W

from helpers import run_oracle

pytestmark = pytest.mark.gpu


@pytest.fixture(autouse=True)
def _gpu(require_gpu):
    pass


def test_run_bivariate_joint_gaussian_rw(oracle, tmp_path):
    w = W.ref_test()
    mcmc = MCMC([RandomWalkUpdate(GaussianRandomWalk(0.5 * np.eye(2)), [1, 2], prior=ImproperPrior())],
                backend=MI355XBackend(num_chains=256, seed=w.seed))
    lines = []
    saver = SavingCallback(path=str(tmp_path), chains=(0, 5))
    ws, lwss = run(mcmc, 1000, dict(P=GsnTargetLaw([1.0, 2.0], [[1.0, 0.5], [0.5, 1.0]]), obs=w.obs),
                   [0.0, 0.0], [saver, REPLCallback(print_every_k_iter=250, printer=lines.append)])
    o = run_oracle(oracle, w, 256, 1000)
    assert np.array_equal(ws.state, o["state"].theta)
    assert np.array_equal(lwss[0].acceptance_history(1, 1000), o["acc"])
    assert np.array_equal(ws.state_history(1, 1000)[:, 0], o["theta"])
    # SavingCallback: rows for iterations 1..M-1 (callbacks.jl:223), reference row format
    rows = (tmp_path / "mcmc_results_chain0.csv").read_text().splitlines()
    assert len(rows) == 999
    assert rows[0].startswith("1, 1, !, ") and rows[0].count("!") == 5
    vals = rows[10].split(", ")
    assert float(vals[3]) == o["theta"][10, 0, 0]
    # the whole row as Julia's "$x, " interpolation writes it (callbacks.jl:249-253)
    from extensible_mcmc.callbacks import julia_float_string as J
    k = 10
    want = (f"{k + 1}, 1, !, " + "".join(f"{J(v)}, " for v in o["theta"][k, 0]) + "!, "
            + "".join(f"{J(v)}, " for v in o["prop"][k, 0]) + f"!, {J(o['ll'][k, 0])}, !, 0.0, !,"
            + ("true" if o["acc"][k, 0] else "false") + ", ")
    assert rows[k] == want
    assert any("1000.1" in l for l in lines) and any("successful" in l for l in lines)


def test_unsupported_plugins_raise_not_fallback():
    """A plugin without a device implementation raises UnsupportedPlugin — no CPU fallback."""
    from extensible_mcmc import MALAUpdate, Normal, ProductPrior, StandardPrior

    w = W.ref_test()
    # a univariate StandardPrior on a coordinate vector has no scalar logpdf in the reference
    mcmc = MCMC([RandomWalkUpdate(GaussianRandomWalk(np.eye(1)), [1], prior=StandardPrior(Normal())),
                 RandomWalkUpdate(GaussianRandomWalk(np.eye(1)), [2])], backend=MI355XBackend(num_chains=8))
    with pytest.raises(UnsupportedPlugin):
        run(mcmc, 10, dict(P=GsnTargetLaw([1.0, 2.0]), obs=w.obs), [0.0, 0.0])
    # MALA's fused logistic-regression kernel takes ImproperPrior only (the library's
    # EMCMC_UNSUPPORTED_PLUGIN surfaces as UnsupportedPlugin)
    from extensible_mcmc import LogisticRegressionLaw
    X = np.random.default_rng(0).normal(size=(64, 16))
    y = (X[:, 0] > 0).astype(float)
    mcmc = MCMC([MALAUpdate(0.1, list(range(1, 17)), prior=ProductPrior([Normal()], [1]))],
                backend=MI355XBackend(num_chains=64))
    with pytest.raises(UnsupportedPlugin):
        run(mcmc, 10, dict(P=LogisticRegressionLaw(16), obs=(X, y)), np.zeros(16))


def test_positive_mixture_walk_beside_a_gaussian_walk_through_the_api(oracle):
    """GaussianRandomWalkMix with positivity flags on coordinate 1 and a GaussianRandomWalk on
    coordinate 2 through MCMC / run (general kernel): the device run equals the oracle's."""
    w = W.ref_test()
    mcmc = MCMC([RandomWalkUpdate(GaussianRandomWalkMix(0.3 * np.eye(1), 0.9 * np.eye(1), 0.3, [True]), [1]),
                 RandomWalkUpdate(GaussianRandomWalk(0.5 * np.eye(1)), [2])],
                backend=MI355XBackend(num_chains=64, seed=w.seed))
    gws, _ = run(mcmc, 150, dict(P=GsnTargetLaw([1.0, 2.0], w.t_sigma), obs=w.obs), [1.0, 2.0])
    ups = [oracle.mwg_update(oracle.KIND_MIX, [0], sigma=[[0.3]], sigma_b=[[0.9]], lam=0.3, pos=[True]),
           oracle.mwg_update(2, [1], sigma=[[0.5]])]
    st = oracle.MWGState(np.tile([1.0, 2.0], (64, 1)), [1.0, 2.0], ups)
    oracle.run_mwg(st, ups, seed=w.seed, t_sigma=w.t_sigma, obs=w.obs,
                   steps=[(i, p) for i in range(1, 151) for p in (1, 2)], history=False)
    assert np.array_equal(gws.state, st.theta) and np.all(gws.state[:, 0] > 0)


def test_positive_uniform_walk_through_the_api(oracle):
    """UniformRandomWalk([0.5], [true]) on coordinate 1 through MCMC/run: the
    device run equals the oracle's, and the restricted coordinate stays positive."""
    w = W.ref_test()
    mcmc = MCMC([RandomWalkUpdate(UniformRandomWalk([0.5], [True]), [1]),
                 RandomWalkUpdate(UniformRandomWalk([1.0]), [2])], backend=MI355XBackend(num_chains=64, seed=w.seed))
    gws, _ = run(mcmc, 200, dict(P=GsnTargetLaw([1.0, 2.0], w.t_sigma), obs=w.obs), [1.0, 0.0])
    ups = [oracle.mwg_update(1, [0], eps=[0.5], pos=[True]), oracle.mwg_update(1, [1], eps=[1.0])]
    st = oracle.MWGState(np.tile([1.0, 0.0], (64, 1)), [1.0, 2.0], ups)
    oracle.run_mwg(st, ups, seed=w.seed, t_sigma=w.t_sigma, obs=w.obs,
                   steps=[(i, p) for i in range(1, 201) for p in (1, 2)], history=False)
    th = gws.state
    assert np.array_equal(th, st.theta) and np.all(th[:, 0] > 0)


def test_haario_mix_through_the_api(oracle):
    """GaussianRandomWalkMix + HaarioTypeAdaptation (BASELINE cfg 4 shape at D = 2)
    through MCMC/run: final state, accept history, per-chain Σ_B factor and the
    adaptation's mean/cov equal the oracle's."""
    w = W.ref_test()
    S = 0.5 * np.eye(2)
    upd = RandomWalkUpdate(GaussianRandomWalkMix(S, 0.25 * S, 0.4), [1, 2],
                           adpt=HaarioTypeAdaptation([0.0, 0.0], adapt_every_k_steps=50))
    mcmc = MCMC([upd], backend=MI355XBackend(num_chains=300, seed=w.seed))
    ws, lwss = run(mcmc, 400, dict(P=GsnTargetLaw([1.0, 2.0], [[1.0, 0.5], [0.5, 1.0]]), obs=w.obs), [0.0, 0.0])
    st = oracle.MixState(np.zeros((300, 2)), sigma_b=0.25 * S)
    h = oracle.run_mix(st, seed=w.seed, sigma_a=S, t_sigma=w.t_sigma, obs=w.obs, iter0=1, nsteps=400, lam=0.4,
                       haario_k=50, nthreads=8)
    assert "mix_gsn_kernel" in ws.engine.kernel_name()
    assert np.array_equal(ws.state, st.theta)
    assert np.array_equal(lwss[0].acceptance_history(1, 400), h["acc"])
    assert np.array_equal(upd.rw.gsn_B.chol_chains, st.LB)
    assert np.array_equal(upd.adpt.cov_chains, st.cov) and np.array_equal(upd.adpt.mean_chains, st.mean)
    assert upd.adpt.M == 0
    stats = ws.chain_stats()
    assert np.array_equal(stats["cov"], st.cov)


def test_reference_mcmc_testset_through_the_api(oracle):
    """test/runtests.jl:87-114 as written (two single-site UniformRandomWalk([1.0])
    updates), through MCMC/run with the MI355X backend, against the oracle."""
    w = W.ref_test()
    mcmc = MCMC([RandomWalkUpdate(UniformRandomWalk([1.0]), [1]), RandomWalkUpdate(UniformRandomWalk([1.0]), [2])],
                backend=MI355XBackend(num_chains=300, seed=w.seed))
    ws, lwss = run(mcmc, 1000, dict(P=GsnTargetLaw([1.0, 2.0], [[1.0, 0.5], [0.5, 1.0]]), obs=w.obs), [0.0, 0.0])
    ups = [oracle.mwg_update(1, [0], eps=[1.0]), oracle.mwg_update(1, [1], eps=[1.0])]
    st = oracle.MWGState(np.zeros((300, 2)), [1.0, 2.0], ups)
    h = oracle.run_mwg(st, ups, seed=w.seed, t_sigma=w.t_sigma, obs=w.obs,
                       steps=[(i, p) for i in range(1, 1001) for p in (1, 2)], nthreads=8)
    assert "mwg_gsn_kernel" in ws.engine.kernel_name()
    assert np.array_equal(ws.state, st.theta)
    assert np.array_equal(lwss[0].acceptance_history(1, 1000), h["acc"][0::2])
    assert np.array_equal(lwss[1].acceptance_history(1, 1000), h["acc"][1::2])
    assert np.array_equal(ws.state_history(1, 1000)[:, 1], h["theta"][1::2])


def test_tutorial_adaptation_through_the_api(oracle):
    """mean_of_bivariate_gaussian.md: UniformRandomWalk([0.1]) with
    AdaptationUnifRW([0.0]; adapt_every_k_steps=50, scale=0.1): the adapted ϵ of
    every chain equals the oracle's."""
    w = W.ref_test()
    ups_api = [RandomWalkUpdate(UniformRandomWalk([0.1]), [i], prior=ImproperPrior(),
                                adpt=AdaptationUnifRW([0.0], adapt_every_k_steps=50, scale=0.1)) for i in (1, 2)]
    mcmc = MCMC(ups_api, backend=MI355XBackend(num_chains=256, seed=w.seed))
    ws, lwss = run(mcmc, 1000, dict(P=GsnTargetLaw([0.3, 0.7], [[1.0, 0.5], [0.5, 1.0]]), obs=w.obs), [0.0, 0.0])
    adapt = {"k": 50, "target": 0.234, "scale": 0.1, "min": 1e-12, "max": 1e7, "offset": 1e2}
    ups = [oracle.mwg_update(1, [0], eps=[0.1], adapt=adapt), oracle.mwg_update(1, [1], eps=[0.1], adapt=adapt)]
    st = oracle.MWGState(np.zeros((256, 2)), [0.3, 0.7], ups)
    oracle.run_mwg(st, ups, seed=w.seed, t_sigma=w.t_sigma, obs=w.obs,
                   steps=[(i, p) for i in range(1, 1001) for p in (1, 2)], history=False, nthreads=8)
    assert np.array_equal(ws.state, st.theta)
    for p in (0, 1):
        assert np.array_equal(ups_api[p].rw.eps_chains[:, 0], st.eps[p, :, 0])
        assert np.array_equal(ups_api[p].adpt.proposed_chains, st.aprop[p])
        assert np.array_equal(ups_api[p].adpt.accepted_chains, st.aacc[p])
