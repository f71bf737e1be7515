"""MALA on the general schedule kernel on the GPU (VERDICT r2 missing item 5):
the reference's gradient hook compute_gradients_and_momenta! (updates.jl:123-133;
run.jl:110 on the current state, run.jl:259 on the proposal) supplied by the
target — the built-in GsnTargetLaw's ∇ (emcmc_mwg.h GsnTarget::grad) or a user
law's EMCMC_USER_GRAD compiled with hiprtc — against the oracle (orc_run_mwg
kind 4; the same user source built by gcc), bit for bit: accept streams, θ / θ°
/ ll histories, sub_ws°.ll, rolling acceptance.  MALA blocks run beside other
updates, under priors, on any coordinates, at D ≤ 16 (mwg_gsn_kernel) and D > 16
(mwg_wide_kernel)."""
import numpy as np
import pytest

from extensible_mcmc import _lib as L
from extensible_mcmc import workloads as W
from extensible_mcmc.engine import Engine, EngineConfig
from extensible_mcmc.schedule import MCMCSchedule
from test_gpu_mwg import check, full_steps
from test_oracle_mala_general import _logistic_case

pytestmark = pytest.mark.gpu


@pytest.fixture(autouse=True)
def _gpu(require_gpu):
    pass


def _add(eng, u):
    pr = dict(prior=u.get("prior", 0), prior_factors=u.get("factors") or None)
    if u["kind"] == 4:
        eng.add_mala_update(u["coords"], u["eps"][0], **pr)
    elif u["kind"] == 1:
        eng.add_uniform_rw_update(u["coords"], u["eps"], adapt=u["adapt"], pos=u.get("pos"), **pr)
    else:
        eng.add_gaussian_rw_update(u["coords"], u["sigma"], pos=u.get("pos"), **pr)


def run_gsn(oracle, D, C, M, ups, mu, t_sigma, obs, steps, seed, ll_mode=L.LL_PER_OBS, hist=L.HIST_FULL, theta0=None):
    eng = Engine(EngineConfig(dim=D, num_chains=C, num_mcmc_steps=M, seed=seed, history_mode=hist))
    for u in ups:
        _add(eng, u)
    eng.set_gsn_target(mu, t_sigma, obs, ll_mode=ll_mode)
    th0 = np.zeros((C, D)) if theta0 is None else np.ascontiguousarray(np.broadcast_to(theta0, (C, D)))
    eng.set_state(th0)
    eng.run(steps)
    st = oracle.MWGState(np.array(th0), mu, ups)
    h = oracle.run_mwg(st, ups, seed=seed, t_sigma=t_sigma, obs=obs, steps=steps, ll_mode=ll_mode, nthreads=8)
    return eng, st, h


def test_joint_mala_on_the_reference_gsn_target(oracle):
    w = W.ref_test()
    D, C, M = 2, 3000, 150
    ups = [oracle.mwg_update(oracle.KIND_MALA, [0, 1], eps=[0.35])]
    steps = full_steps(M, 1)
    eng, st, h = run_gsn(oracle, D, C, M, ups, np.array([1.0, 2.0]), w.t_sigma, w.obs, steps, w.seed)
    assert "MALA" in eng.kernel_name()
    check(oracle, eng, st, h, steps, ups, 1)
    assert 0.2 < h["acc"][1:].mean() < 0.99


@pytest.mark.parametrize("ll_mode", [L.LL_PER_OBS, L.LL_SUFFSTAT])
def test_mala_block_with_prior_in_a_gibbs_schedule(oracle, ll_mode):
    """MALA on {4, 1, 3} under ProductPrior([Normal(0, 2), Normal(1, 3)], [1, 1]) (both
    factors read θ_local[1], priors.jl:64-79) beside a UniformRandomWalk on {2} and a
    GaussianRandomWalk on {5}; update 3 excluded on iterations 15:30; dense Σ_t."""
    rng = np.random.default_rng(11)
    D, C, M = 5, 2048, 80
    A = rng.normal(size=(D, D))
    S = A @ A.T / D + np.eye(D)
    mu = rng.normal(size=D)
    obs = rng.multivariate_normal(mu, S, size=9)
    ups = [oracle.mwg_update(oracle.KIND_MALA, [3, 0, 2], eps=[0.3], prior=L.PRIOR_PRODUCT,
                             factors=[(L.DIST_NORMAL, 1, 0.0, 2.0), (L.DIST_NORMAL, 1, 1.0, 3.0)]),
           oracle.mwg_update(1, [1], eps=[0.5], adapt=None),
           oracle.mwg_update(2, [4], sigma=[[0.2]])]
    steps = [(s.mcmciter, s.pidx) for s in MCMCSchedule(M, 3, [(3, range(15, 31))])]
    eng, st, h = run_gsn(oracle, D, C, M, ups, mu, S, obs, steps, 21, ll_mode=ll_mode, theta0=mu)
    check(oracle, eng, st, h, steps, ups, 3)


def test_mala_on_the_wide_kernel(oracle):
    """D = 40 (mwg_wide_kernel): a joint 24-coordinate MALA block and a 16-coordinate
    Gaussian block, dense Σ_t, sufficient-statistic likelihood."""
    rng = np.random.default_rng(12)
    D, C, M = 40, 1024, 30
    A = rng.normal(size=(D, D)) / np.sqrt(D)
    S = A @ A.T + 0.5 * np.eye(D)
    mu = rng.normal(size=D)
    obs = rng.multivariate_normal(mu, S, size=20)
    perm = rng.permutation(D)
    ups = [oracle.mwg_update(oracle.KIND_MALA, perm[:24], eps=[0.08]),
           oracle.mwg_update(2, perm[24:], sigma=0.003 * np.eye(16))]
    steps = full_steps(M, 2)
    eng, st, h = run_gsn(oracle, D, C, M, ups, mu, S, obs, steps, 22, ll_mode=L.LL_SUFFSTAT, theta0=mu)
    assert "mwg_wide_kernel" in eng.kernel_name()
    check(oracle, eng, st, h, steps, ups, 2)
    assert 0.05 < h["acc"][1:, ].mean() < 0.99


def _logistic_engine(oracle, ups, C, M, seed, hist=L.HIST_FULL):
    X, y = _logistic_case()
    D = X.shape[1]
    obs = np.column_stack([X, y])
    fn, src = oracle.user_loglik("logistic_regression")
    gfn = oracle.user_grad("logistic_regression")
    eng = Engine(EngineConfig(dim=D, num_chains=C, num_mcmc_steps=M, seed=seed, history_mode=hist))
    for u in ups:
        _add(eng, u)
    eng.set_user_target(src, obs=obs, theta0=np.zeros(D))
    eng.set_state(np.zeros((C, D)))
    return eng, obs, fn, gfn, D


def test_mala_on_a_user_law_with_its_gradient(oracle):
    """The user's logistic-regression law with EMCMC_USER_GRAD: joint MALA, then MALA on
    {1, 3} under StandardPrior(MvNormal) beside a Gaussian walk on {2}."""
    C, M = 4096, 60
    for ups in ([oracle.mwg_update(oracle.KIND_MALA, [0, 1, 2], eps=[0.3])],
                [oracle.mwg_update(oracle.KIND_MALA, [0, 2], eps=[0.35], prior=L.PRIOR_STANDARD,
                                   factors=[(L.DIST_MVNORMAL, 2, [0.0, 0.5], [[4.0, 1.0], [1.0, 2.0]])]),
                 oracle.mwg_update(2, [1], sigma=[[0.1]])]):
        eng, obs, fn, gfn, D = _logistic_engine(oracle, ups, C, M, 31)
        steps = full_steps(M, len(ups))
        eng.run(steps)
        assert "UserTarget" in eng.kernel_name() and "MALA" in eng.kernel_name()
        st = oracle.MWGState(np.zeros((C, D)), np.zeros(D), ups)
        h = oracle.run_mwg(st, ups, seed=31, t_sigma=None, obs=obs, steps=steps, nthreads=8, user_ll=fn,
                           user_grad=gfn)
        check(oracle, eng, st, h, steps, ups, len(ups))


def test_mala_on_a_user_law_without_gradient_is_refused(oracle):
    from user_target_cases import poisson

    case = poisson()
    _, src = oracle.user_loglik(case.name)
    eng = Engine(EngineConfig(dim=case.D, num_chains=64, num_mcmc_steps=4, seed=1))
    eng.add_mala_update(range(case.D), 0.1)
    with pytest.raises(L.EMCMCError, match="gradient") as e:
        eng.set_user_target(src, obs=case.obs, params=case.params, theta0=case.theta0)
    assert e.value.status == L.UNSUPPORTED_PLUGIN


def test_mala_update_through_the_api(oracle):
    """run!(MCMC([MALAUpdate(ϵ, coords; prior)]; backend), M, (P = UserTargetLaw(src, θ), obs), θinit)."""
    import extensible_mcmc as E
    X, y = _logistic_case()
    D = X.shape[1]
    obs = np.column_stack([X, y])
    fn, src = oracle.user_loglik("logistic_regression")
    gfn = oracle.user_grad("logistic_regression")
    C, M = 1024, 100
    P = E.UserTargetLaw(src, np.zeros(D))
    mcmc = E.MCMC([E.MALAUpdate(0.3, list(range(1, D + 1)))], backend=E.MI355XBackend(num_chains=C, seed=5))
    gws, lws = E.run(mcmc, M, E.make_data(P, obs), np.zeros(D))
    ups = [oracle.mwg_update(oracle.KIND_MALA, range(D), eps=[0.3])]
    st = oracle.MWGState(np.zeros((C, D)), np.zeros(D), ups)
    oracle.run_mwg(st, ups, seed=5, t_sigma=None, obs=obs, steps=full_steps(M, 1), nthreads=8, user_ll=fn,
                   user_grad=gfn, history=False)
    assert np.array_equal(gws.state, st.theta)
    assert np.array_equal(lws[0].ll, st.ll)


def test_mala_on_a_user_law_on_the_wide_kernel(oracle):
    """D = 20 (mwg_wide_kernel, NU = 20): the user logistic law with its gradient, a MALA
    block of 12 coordinates and a Gaussian block of 8, accept-only then full histories."""
    rng = np.random.default_rng(21)
    D, n, C, M = 20, 80, 2048, 40
    X = np.column_stack([np.ones(n), rng.normal(size=(n, D - 1))])
    beta = rng.normal(scale=0.3, size=D)
    y = (rng.uniform(size=n) < 1.0 / (1.0 + np.exp(-(X @ beta)))).astype(float)
    obs = np.column_stack([X, y])
    fn, src = oracle.user_loglik("logistic_regression")
    gfn = oracle.user_grad("logistic_regression")
    perm = rng.permutation(D)
    ups = [oracle.mwg_update(oracle.KIND_MALA, perm[:12], eps=[0.08]),
           oracle.mwg_update(2, perm[12:], sigma=0.004 * np.eye(8))]
    steps = full_steps(M, 2)
    for hist in (L.HIST_ACCEPT_ONLY, L.HIST_FULL):
        eng = Engine(EngineConfig(dim=D, num_chains=C, num_mcmc_steps=M, seed=41, history_mode=hist))
        for u in ups:
            _add(eng, u)
        eng.set_user_target(src, obs=obs, theta0=np.zeros(D))
        eng.set_state(np.zeros((C, D)))
        eng.run(steps)
        assert "mwg_wide_kernel<D=20" in eng.kernel_name() and "MALA" in eng.kernel_name()
        st = oracle.MWGState(np.zeros((C, D)), np.zeros(D), ups)
        h = oracle.run_mwg(st, ups, seed=41, t_sigma=None, obs=obs, steps=steps, nthreads=8, user_ll=fn,
                           user_grad=gfn)
        check(oracle, eng, st, h, steps, ups, 2, full=hist == L.HIST_FULL)
