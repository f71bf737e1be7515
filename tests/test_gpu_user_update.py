"""User-defined updates on the GPU (row g1): a user's proposal! and
log_transition_density (updates.jl:42-93) as an EMCMC_USER_PROPOSAL /
EMCMC_USER_LTD source, compiled at run time (hiprtc, gfx950) into the general
schedule kernel, against the oracle's gcc build of the same source, bit for
bit — accept streams, θ / θ° / ll histories, sub_ws°.ll, rolling acceptance.
The proposals are not random walks and their transition densities do not
cancel: a preconditioned Crank–Nicolson step and a two-scale multiplicative
walk with its Jacobian."""
import numpy as np
import pytest

from extensible_mcmc import _lib as L
from extensible_mcmc.engine import Engine, EngineConfig
from test_gpu_mwg import check, full_steps

pytestmark = pytest.mark.gpu


@pytest.fixture(autouse=True)
def _gpu(require_gpu):
    pass


def run_upd(oracle, name, D, C, M, ups, mu, t_sigma, obs, steps, seed, theta0=None, ll_mode=L.LL_PER_OBS,
            hist=L.HIST_FULL, spl=0):
    fns, src = oracle.user_update(name)
    eng = Engine(EngineConfig(dim=D, num_chains=C, num_mcmc_steps=M, seed=seed, history_mode=hist,
                              steps_per_launch=spl))
    for u in ups:
        pr = dict(prior=u.get("prior", 0), prior_factors=u.get("factors") or None)
        if u["kind"] == oracle.KIND_USER:
            eng.add_user_update(u["coords"], src, u["params"], **pr)
        elif u["kind"] == 1:
            eng.add_uniform_rw_update(u["coords"], u["eps"], adapt=u["adapt"], pos=u.get("pos"), **pr)
        else:
            eng.add_gaussian_rw_update(u["coords"], u["sigma"], pos=u.get("pos"), **pr)
    eng.set_gsn_target(mu, t_sigma, obs, ll_mode=ll_mode)
    th0 = np.zeros((C, D)) if theta0 is None else np.ascontiguousarray(np.broadcast_to(theta0, (C, D)))
    eng.set_state(th0)
    eng.run(steps)
    st = oracle.MWGState(np.array(th0), mu, ups)
    h = oracle.run_mwg(st, ups, seed=seed, t_sigma=t_sigma, obs=obs, steps=steps, ll_mode=ll_mode, nthreads=8,
                       user_upd=fns)
    return eng, st, h


def gsn_problem(D, seed, n=8):
    rng = np.random.default_rng(seed)
    mu = rng.normal(size=D)
    return mu, mu + rng.normal(size=(n, D))


def test_pcn_joint_update(oracle):
    """A pCN proposal on all 4 coordinates of a GsnTargetLaw: the transition densities
    differ both ways (llr adds ltd(θ°, θ) − ltd(θ, θ°))."""
    D, C, M = 4, 2000, 200
    mu, obs = gsn_problem(D, 1)
    prm = [0.8, 0.6] + list(obs.mean(0))
    ups = [oracle.mwg_update(oracle.KIND_USER, range(D), params=prm)]
    steps = full_steps(M, 1)
    eng, st, h = run_upd(oracle, "pcn", D, C, M, ups, mu, np.eye(D), obs, steps, 11)
    assert "UserUpdate" in eng.kernel_name()
    check(oracle, eng, st, h, steps, ups, 1)
    assert 0.05 < h["acc"][1:].mean() < 0.95


def test_pcn_in_a_gibbs_schedule_with_a_prior(oracle):
    """pCN on coordinates {1, 3} under ProductPrior([Normal(0, 2)], [1]) beside a
    GaussianRandomWalk on {2, 4} and a UniformRandomWalk on {5}, with update 2 excluded
    on iterations 20:40 — user and built-in updates in one kernel launch."""
    from extensible_mcmc.schedule import MCMCSchedule

    D, C, M = 5, 1500, 120
    mu, obs = gsn_problem(D, 2)
    ups = [oracle.mwg_update(oracle.KIND_USER, [0, 2], params=[0.5, 0.4, mu[0], mu[2]], prior=L.PRIOR_PRODUCT,
                             factors=[(L.DIST_NORMAL, 1, 0.0, 2.0)]),
           oracle.mwg_update(2, [1, 3], sigma=0.05 * np.eye(2)),
           oracle.mwg_update(1, [4], eps=[0.4], adapt=None)]
    steps = [(s.mcmciter, s.pidx) for s in MCMCSchedule(M, 3, [(2, range(20, 41))])]
    eng, st, h = run_upd(oracle, "pcn", D, C, M, ups, mu, np.eye(D), obs, steps, 12, ll_mode=L.LL_SUFFSTAT)
    check(oracle, eng, st, h, steps, ups, 3)


def test_two_scale_multiplicative_walk(oracle):
    """θ°_i = θ_i·exp(σ z_i) with a mixture of two scales picked by em_rand(0): positive
    coordinates, a Jacobian term in the transition density, NaN-free support."""
    D, C, M = 3, 1024, 250
    mu = np.array([2.0, 3.0, 1.5])
    obs = mu + 0.5 * np.random.default_rng(3).normal(size=(6, D))
    prm = [0.3, 0.05, 0.08, 0.06, 0.4, 0.5, 0.45]
    ups = [oracle.mwg_update(oracle.KIND_USER, range(D), params=prm, prior=L.PRIOR_IMPROPER_POS)]
    steps = full_steps(M, 1)
    eng, st, h = run_upd(oracle, "lognormal_walk", D, C, M, ups, mu, 0.25 * np.eye(D), obs, steps, 13,
                         theta0=np.ones(D))
    check(oracle, eng, st, h, steps, ups, 1)
    assert np.all(h["theta"] > 0)
    assert 0.05 < h["acc"][1:].mean() < 0.95


@pytest.mark.parametrize("hist", [L.HIST_FULL, L.HIST_ACCEPT_ONLY])
def test_pcn_blocks_at_d32_on_the_wide_kernel(oracle, hist):
    """Two pCN blocks of 16 coordinates at the headline D = 32 (mwg_wide_kernel, NU = 16),
    split over launches of 37 steps."""
    D, C, M = 32, 2048, 90
    mu, obs = gsn_problem(D, 4, n=10)
    xb = obs.mean(0)
    ups = [oracle.mwg_update(oracle.KIND_USER, range(0, 16), params=[0.9, 0.3] + list(xb[:16])),
           oracle.mwg_update(oracle.KIND_USER, range(16, 32), params=[0.7, 0.3] + list(xb[16:]))]
    steps = full_steps(M, 2)
    eng, st, h = run_upd(oracle, "pcn", D, C, M, ups, mu, np.eye(D), obs, steps, 14, hist=hist, spl=37)
    assert "mwg_wide_kernel<D=32,NU=16" in eng.kernel_name()
    check(oracle, eng, st, h, steps, ups, 2, full=hist == L.HIST_FULL)


def test_user_update_refusals(oracle):
    """A second, different source on one handle and a source that does not compile are
    refused (EMCMC_UNSUPPORTED_PLUGIN / EMCMC_INVALID_ARG with the compiler log)."""
    _, src = oracle.user_update("pcn")
    _, other = oracle.user_update("lognormal_walk")
    eng = Engine(EngineConfig(dim=2, num_chains=64, num_mcmc_steps=4, seed=1))
    try:
        eng.add_user_update([0], src, [0.5, 1.0, 0.0])
        with pytest.raises(L.EMCMCError) as e:
            eng.add_user_update([1], other, [0.5, 0.1, 0.2])
        assert e.value.status == L.UNSUPPORTED_PLUGIN
    finally:
        eng.close()
    eng = Engine(EngineConfig(dim=2, num_chains=64, num_mcmc_steps=4, seed=1))
    try:
        eng.add_user_update([0, 1], "EMCMC_USER_PROPOSAL { theta_prop[0] = undefined_name; }\n"
                                    "EMCMC_USER_LTD { return 0.0; }", [])
        with pytest.raises(L.EMCMCError) as e:
            eng.set_gsn_target(np.zeros(2), np.eye(2), np.zeros((3, 2)))
        assert e.value.status == L.INVALID_ARG and "undefined_name" in str(e.value)
    finally:
        eng.close()
