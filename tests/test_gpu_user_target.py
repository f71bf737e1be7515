"""User-defined target laws (row g1) on the GPU: each EMCMC_USER_LOGLIK source is
compiled at run time (hiprtc, gfx950) into the general schedule kernel and run
against the oracle's gcc build of the same source, bit for bit — accept
streams, θ / θ° / ll histories, sub_ws°.ll, rolling acceptance, adapted ϵ —
with joint and Metropolis-within-Gibbs updates, priors, AdaptationUnifRW,
dense Σ, D up to 24 (the wide kernel), and through the MCMC API."""
import numpy as np
import pytest

import user_target_cases as U
from extensible_mcmc import _lib as L
from extensible_mcmc.engine import Engine, EngineConfig
from test_gpu_mwg import ADAPT, check, full_steps

pytestmark = pytest.mark.gpu


@pytest.fixture(autouse=True)
def _gpu(require_gpu):
    pass


def run_user(oracle, case, ups, steps, C, M, hist=L.HIST_FULL, spl=0):
    fn, src = oracle.user_loglik(case.name)
    eng = Engine(EngineConfig(dim=case.D, num_chains=C, num_mcmc_steps=M, seed=case.seed, history_mode=hist,
                              steps_per_launch=spl))
    for u in ups:
        pr = dict(prior=u.get("prior", 0), prior_factors=u.get("factors") or None)
        if u["kind"] == 1:
            eng.add_uniform_rw_update(u["coords"], u["eps"], adapt=u["adapt"], pos=u.get("pos"), **pr)
        else:
            eng.add_gaussian_rw_update(u["coords"], u["sigma"], pos=u.get("pos"), **pr)
    eng.set_user_target(src, obs=case.obs, params=case.params, theta0=case.theta0)
    th0 = np.ascontiguousarray(np.broadcast_to(case.theta0, (C, case.D)))
    eng.set_state(th0)
    eng.run(steps)
    st = oracle.MWGState(th0, case.theta0, ups)
    h = oracle.run_mwg(st, ups, seed=case.seed, t_sigma=None, obs=case.obs, steps=steps, nthreads=8,
                       user_ll=fn, user_params=case.params)
    return eng, st, h


def test_student_t_joint_gaussian_walk(oracle):
    case = U.student_t()
    ups = [oracle.mwg_update(2, range(case.D), sigma=0.01 * np.eye(case.D))]
    steps = full_steps(300, 1)
    eng, st, h = run_user(oracle, case, ups, steps, 2000, 300)
    assert "UserTarget[hiprtc]" in eng.kernel_name()
    check(oracle, eng, st, h, steps, ups, 1)
    acc = eng.get_history(L.H_ACCEPT, 2, 299)[:, 0]
    assert 0.1 < acc.mean() < 0.9


def test_poisson_dense_sigma_with_normal_prior(oracle):
    case = U.poisson()
    S = np.array([[0.010, 0.002, 0.0], [0.002, 0.008, -0.001], [0.0, -0.001, 0.012]])
    fac = [(L.DIST_PRODUCT, case.D, [(L.DIST_NORMAL, 0.0, 10.0)] * case.D)]
    ups = [oracle.mwg_update(2, range(case.D), sigma=S, prior=L.PRIOR_PRODUCT, factors=fac)]
    steps = full_steps(250, 1)
    eng, st, h = run_user(oracle, case, ups, steps, 1537, 250, spl=37)
    check(oracle, eng, st, h, steps, ups, 1)


def test_student_t_metropolis_within_gibbs_with_adaptation(oracle):
    """Blocks {1,2} (GaussianRandomWalk) then single sites 3 and 4 (UniformRandomWalk +
    AdaptationUnifRW), with update 2 excluded on iterations 10:30."""
    from extensible_mcmc.schedule import MCMCSchedule
    case = U.student_t()
    ups = [oracle.mwg_update(2, [0, 1], sigma=0.02 * np.eye(2)),
           oracle.mwg_update(1, [2], eps=[0.1], adapt=ADAPT),
           oracle.mwg_update(1, [3], eps=[0.1], adapt=ADAPT)]
    steps = [(s.mcmciter, s.pidx) for s in MCMCSchedule(200, 3, [(2, range(10, 31))])]
    eng, st, h = run_user(oracle, case, ups, steps, 999, 200)
    check(oracle, eng, st, h, steps, ups, 3)


@pytest.mark.parametrize("D", [2, 24])
@pytest.mark.parametrize("hist", [L.HIST_FULL, L.HIST_ACCEPT_ONLY])
def test_banana(oracle, D, hist):
    case = U.banana(D)
    sig = np.full(D, 1.0)
    sig[0] = 10.0
    ups = [oracle.mwg_update(2, range(D), sigma=np.diag((2.38 ** 2 / D) * sig ** 2))]
    steps = full_steps(400, 1)
    eng, st, h = run_user(oracle, case, ups, steps, 1024, 400, hist=hist)
    check(oracle, eng, st, h, steps, ups, 1, full=hist == L.HIST_FULL)


def test_gsn_as_user_law_matches_builtin_device_run(oracle):
    """GsnTargetLaw(θ, I) as a user law equals the built-in law on the same
    general kernel (two updates force it), bit for bit."""
    case = U.gsn_identity()
    D, C, M = case.D, 2048, 200
    fn, src = oracle.user_loglik(case.name)
    steps = full_steps(M, 2)
    outs = []
    for user in (False, True):
        eng = Engine(EngineConfig(dim=D, num_chains=C, num_mcmc_steps=M, seed=case.seed))
        eng.add_gaussian_rw_update([0, 1], 0.2 * np.eye(2))
        eng.add_uniform_rw_update([2], [0.4])
        if user:
            eng.set_user_target(src, obs=case.obs, params=case.params, theta0=case.theta0)
        else:
            eng.set_gsn_target(case.theta0, np.eye(D), case.obs)
        eng.set_state(np.zeros((C, D)))
        eng.run(steps)
        eng.synchronize(allow_faults=True)
        outs.append((eng.get_state(), eng.get_history(L.H_ACCEPT, 1, M), eng.get_history(L.H_STATE, 1, M)))
    (a, aa, ah), (b, ba, bh) = outs
    assert np.array_equal(a[0], b[0]) and np.array_equal(a[1], b[1])
    assert np.array_equal(aa, ba) and np.array_equal(ah, bh)


def test_user_law_through_the_api(oracle):
    """run!(MCMC(updates; backend), M, (P = UserTargetLaw(src, θ), obs), θinit)."""
    import extensible_mcmc as E
    case = U.poisson()
    fn, src = oracle.user_loglik(case.name)
    C, M = 512, 150
    P = E.UserTargetLaw(src, case.theta0, params=case.params)
    mcmc = E.MCMC([E.RandomWalkUpdate(E.GaussianRandomWalk(0.01 * np.eye(case.D)), list(range(1, case.D + 1)))],
                  backend=E.MI355XBackend(num_chains=C, seed=case.seed))
    gws, lws = E.run(mcmc, M, E.make_data(P, case.obs), case.theta0)
    ups = [oracle.mwg_update(2, range(case.D), sigma=0.01 * np.eye(case.D))]
    st = oracle.MWGState(np.zeros((C, case.D)), case.theta0, ups)
    oracle.run_mwg(st, ups, seed=case.seed, t_sigma=None, obs=case.obs, steps=full_steps(M, 1), nthreads=8,
                   user_ll=fn, user_params=case.params, history=False)
    assert np.array_equal(gws.state, st.theta)
    assert np.array_equal(lws[0].ll, st.ll)


def test_full_gsn_law_updates_sigma_entries(oracle):
    """GsnTargetLaw with θ = [μ; vec Σ] (gsn_target.jl:1-29) as a user law: a joint
    Gaussian walk on μ and UniformRandomWalks on Σ₁₁, Σ₁₂ (the upper entry, the
    one Symmetric(triu(Σ)) reads) and Σ₂₂, the variances positivity-restricted;
    the law refactorises Σ at every evaluation like set_parameters! does."""
    case = U.gsn_full()
    ups = [oracle.mwg_update(2, [0, 1], sigma=0.1 * np.eye(2)),
           oracle.mwg_update(1, [2], eps=[0.2], pos=[True]),
           oracle.mwg_update(1, [4], eps=[1.5]),  # wide: some proposals leave the PD cone
           oracle.mwg_update(1, [5], eps=[0.2], pos=[True])]
    steps = full_steps(300, 4)
    eng, st, h = run_user(oracle, case, ups, steps, 1200, 300)
    check(oracle, eng, st, h, steps, ups, 4)
    th = eng.get_state()[0]
    assert np.all(th[:, 2] > 0) and np.all(th[:, 5] > 0)
    assert np.any(eng.get_faults() & L.FAULT_NONFINITE_LL)  # some Σ proposals were not positive definite


def test_full_gsn_law_with_fixed_sigma_matches_builtin_device_run(oracle):
    """μ-only updates of the θ = [μ; vec Σ] user law give the built-in
    GsnTargetLaw(μ, Σ) chain on the device, bit for bit."""
    case = U.gsn_full()
    d, C, M = 2, 2048, 200
    fn, src = oracle.user_loglik(case.name)
    th0 = np.concatenate([np.zeros(d), case.extra["S"].ravel(order="F")])
    steps = full_steps(M, 2)
    outs = []
    for user in (False, True):
        D = d + d * d if user else d
        eng = Engine(EngineConfig(dim=D, num_chains=C, num_mcmc_steps=M, seed=case.seed))
        eng.add_gaussian_rw_update([0], [[0.4]])
        eng.add_uniform_rw_update([1], [0.6])
        if user:
            eng.set_user_target(src, obs=case.obs, params=case.params, theta0=th0)
            eng.set_state(np.tile(th0, (C, 1)))
        else:
            eng.set_gsn_target(th0[:d], case.extra["S"], case.obs)
            eng.set_state(np.zeros((C, d)))
        eng.run(steps)
        eng.synchronize(allow_faults=True)
        th, ll = eng.get_state()
        outs.append((th[:, :d], ll, eng.get_history(L.H_ACCEPT, 1, M), eng.get_history(L.H_LL, 1, M)))
    for a, b in zip(*outs):
        assert np.array_equal(a, b)


def test_gsn_target_law_over_mu_and_sigma_through_the_api(oracle):
    """The reference's own interface: GsnTargetLaw(μ, Σ) with θinit covering
    θ = [μ; vec Σ] and updates on Σ coordinates (coords 3:6, 1-based) — the engine
    runs the shipped law csrc/laws/gsn_full.c; the oracle runs its gcc build."""
    import extensible_mcmc as E
    case = U.gsn_full()
    fn, _ = oracle.user_loglik("gsn_full")
    d, C, M = 2, 700, 250
    th0 = np.concatenate([np.zeros(d), np.eye(d).ravel(order="F")])
    mcmc = E.MCMC([E.RandomWalkUpdate(E.GaussianRandomWalk(0.1 * np.eye(2)), [1, 2]),
                   E.RandomWalkUpdate(E.UniformRandomWalk([0.2], [True]), [3]),
                   E.RandomWalkUpdate(E.UniformRandomWalk([0.3]), [5]),
                   E.RandomWalkUpdate(E.UniformRandomWalk([0.2], [True]), [6])],
                  backend=E.MI355XBackend(num_chains=C, seed=case.seed))
    gws, lws = E.run(mcmc, M, E.make_data(E.GsnTargetLaw(np.zeros(d), np.eye(d)), case.obs), th0)
    assert "UserTarget" in gws.engine.kernel_name()
    ups = [oracle.mwg_update(2, [0, 1], sigma=0.1 * np.eye(2)), oracle.mwg_update(1, [2], eps=[0.2], pos=[True]),
           oracle.mwg_update(1, [4], eps=[0.3]), oracle.mwg_update(1, [5], eps=[0.2], pos=[True])]
    st = oracle.MWGState(np.tile(th0, (C, 1)), th0, ups)
    oracle.run_mwg(st, ups, seed=case.seed, t_sigma=None, obs=case.obs, steps=full_steps(M, 4), nthreads=8,
                   user_ll=fn, user_params=np.array([float(d)]), history=False)
    assert np.array_equal(gws.state, st.theta)
    S = gws.state[:, d:].reshape(C, d, d).mean(axis=0)
    assert 0.25 < S[0, 0] / np.cov(case.obs.T)[0, 0] < 4.0  # the Σ draws sit at the data's scale
