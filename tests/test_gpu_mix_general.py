"""GaussianRandomWalkMix + HaarioTypeAdaptation and GenericChainStats mean/cov on
the general schedule kernel (rows a8, a13, a14): every shape the fused cfg 4
kernels do not cover — a correlated target with a dense Σ_A at D = 32,
positivity-restricted coordinates (the in-place exp/log round trips of
random_walk.jl:136-232 and register!'s log scale, adaptation.jl:407,412), a mix
block inside a Metropolis-within-Gibbs schedule, priors, a user target, fλ —
bit for bit against the oracle (orc_run_mwg kind 3)."""
import numpy as np
import pytest

import user_target_cases as U
from extensible_mcmc import _lib as L
from extensible_mcmc.engine import Engine, EngineConfig
from test_gpu_mwg import check, full_steps

pytestmark = pytest.mark.gpu


@pytest.fixture(autouse=True)
def _gpu(require_gpu):
    pass


def build(oracle, D, C, M, ups, seed, hist=L.HIST_FULL, spl=0, chain_moments=False, ll_mode=L.LL_PER_OBS,
          variant=0):
    eng = Engine(EngineConfig(dim=D, num_chains=C, num_mcmc_steps=M, seed=seed, history_mode=hist,
                              steps_per_launch=spl, chain_moments=chain_moments, kernel_variant=variant))
    for u in ups:
        pr = dict(prior=u.get("prior", 0), prior_factors=u.get("factors") or None)
        if u["kind"] == oracle.KIND_MIX:
            eng.add_gaussian_rw_mix_update(u["coords"], u["sigma"], u["sigma_b"], lam=u["lam"],
                                           haario_k=u.get("haario_k"), pos=u.get("pos"), **pr)
        elif u["kind"] == 1:
            eng.add_uniform_rw_update(u["coords"], u["eps"], adapt=u["adapt"], pos=u.get("pos"), **pr)
        else:
            eng.add_gaussian_rw_update(u["coords"], u["sigma"], pos=u.get("pos"), **pr)
    return eng


def check_mix(oracle, eng, st, ups, chain_moments=False):
    for p, u in enumerate(ups):
        if u["kind"] != oracle.KIND_MIX:
            continue
        n = len(u["coords"])
        Lb, M = eng.get_mix_state(p + 1)
        assert np.array_equal(Lb, st.lb(p, n)), f"L_B of update {p + 1}"
        if u.get("haario_k"):
            assert M == st.M[p]
            hm, hc = eng.get_adaptation_moments(p + 1)
            om, oc = st.haario(p, n)
            assert np.array_equal(hm, om) and np.array_equal(hc, oc), f"Haario moments of update {p + 1}"
    if chain_moments:
        m, v = eng.get_chain_moments()
        assert np.array_equal(m, st.smean) and np.array_equal(v, st.scov)


def run_both(oracle, D, C, M, ups, mu, ts, obs, steps, seed, theta0=None, chain_moments=False, **kw):
    eng = build(oracle, D, C, M, ups, seed, chain_moments=chain_moments, **kw)
    eng.set_gsn_target(mu, ts, obs, ll_mode=kw.get("ll_mode", L.LL_PER_OBS))
    th0 = np.zeros((C, D)) if theta0 is None else np.ascontiguousarray(np.broadcast_to(theta0, (C, D)))
    eng.set_state(th0)
    eng.run(steps)
    st = oracle.MWGState(np.array(th0), mu, ups, chain_moments=chain_moments)
    h = oracle.run_mwg(st, ups, seed=seed, t_sigma=ts, obs=obs, steps=steps, nthreads=8,
                       ll_mode=kw.get("ll_mode", 0))
    return eng, st, h


def test_haario_on_a_correlated_d32_target_through_two_readjusts(oracle):
    """The round-2 verdict's case: HaarioTypeAdaptation on GsnTargetLaw(μ, BBᵀ/32 + I) at
    D = 32 with a dense Σ_A, k = 100, 230 steps (two readjusts): the general kernel
    (EMCMC_VARIANT_NO_MIX_CHOL; the default is the fused mix_chol_kernel,
    tests/test_gpu_mix_chol.py), bitwise."""
    rng = np.random.default_rng(32)
    D, C, M, k = 32, 1024, 230, 100
    B = rng.standard_normal((D, D))
    ts = B @ B.T / D + np.eye(D)
    mu = rng.standard_normal(D)
    obs = rng.multivariate_normal(mu, ts, size=10)
    sa = 0.2 * (2.38 ** 2 / (D * 10)) * ts  # ≈ 60 % acceptance: 100 registrations span the space
    ups = [oracle.mwg_update(oracle.KIND_MIX, range(D), sigma=sa, sigma_b=0.5 * sa, lam=0.3, haario_k=k)]
    steps = full_steps(M, 1)
    eng, st, h = run_both(oracle, D, C, M, ups, mu, ts, obs, steps, 321, theta0=obs.mean(0), ll_mode=L.LL_SUFFSTAT,
                          variant=L.VARIANT_NO_MIX_CHOL)
    assert "mwg_wide_kernel<D=32" in eng.kernel_name()
    check(oracle, eng, st, h, steps, ups, 1)
    check_mix(oracle, eng, st, ups)
    assert st.M[0] == M % k
    # the readjusts took on (almost) every chain: Σ_B is no longer the initial factor
    posdef = (st.faults & L.FAULT_POSDEF) != 0
    assert posdef.mean() < 0.05
    L0 = np.linalg.cholesky(0.5 * sa)
    assert np.all(np.abs(st.lb(0, D)[~posdef] - L0).max(axis=(1, 2)) > 0)
    assert 0.3 < h["acc"][1:].mean() < 0.9


def test_mix_with_positivity_flags_at_d2(oracle):
    """GaussianRandomWalkMix(Σ_A, Σ_B, 0.4, pos = [true, false]) + Haario(k = 25) at D = 2."""
    mu = np.array([2.0, 0.5])
    ts = np.array([[0.5, 0.1], [0.1, 0.4]])
    obs = mu + np.random.default_rng(1).multivariate_normal(np.zeros(2), ts, size=6)
    ups = [oracle.mwg_update(oracle.KIND_MIX, [0, 1], sigma=0.05 * np.eye(2), sigma_b=[[0.2, 0.05], [0.05, 0.1]],
                             lam=0.4, haario_k=25, pos=[True, False])]
    steps = full_steps(200, 1)
    eng, st, h = run_both(oracle, 2, 2000, 200, ups, mu, ts, obs, steps, 77, theta0=[1.0, 0.0])
    check(oracle, eng, st, h, steps, ups, 1)
    check_mix(oracle, eng, st, ups)
    assert np.all(h["theta"][..., 0] > 0)


@pytest.mark.parametrize("hist", [L.HIST_FULL, L.HIST_ACCEPT_ONLY])
def test_mix_block_in_a_gibbs_schedule_with_chain_moments(oracle, hist):
    """A mix + Haario block {1, 2} (registering after both updates' steps) beside a
    GaussianRandomWalk on {3, 4} and GenericChainStats mean/cov after every step
    (chain_statistics.jl:46-49), in launches of 29 steps."""
    rng = np.random.default_rng(2)
    mu = rng.normal(size=4)
    obs = mu + rng.normal(size=(8, 4))
    ups = [oracle.mwg_update(oracle.KIND_MIX, [0, 1], sigma=0.2 * np.eye(2), sigma_b=0.1 * np.eye(2), lam=0.5,
                             haario_k=40),
           oracle.mwg_update(2, [2, 3], sigma=0.05 * np.eye(2))]
    steps = full_steps(200, 2)
    eng, st, h = run_both(oracle, 4, 1500, 200, ups, mu, np.eye(4), obs, steps, 78, theta0=mu, chain_moments=True,
                          hist=hist, spl=29)
    check(oracle, eng, st, h, steps, ups, 2, full=hist == L.HIST_FULL)
    check_mix(oracle, eng, st, ups, chain_moments=True)


def test_mix_with_a_product_prior_and_redraws(oracle):
    """A mix update under ProductPrior([Product([Uniform(−1, 3), Uniform(−2, 2)])], [2]):
    proposal! redraws pick the kernel again at every rand! (attempt = the redraw)."""
    mu = np.array([1.0, 0.0])
    obs = mu + np.random.default_rng(5).normal(size=(5, 2))
    fac = [(L.DIST_PRODUCT, 2, [(L.DIST_UNIFORM, -1.0, 3.0), (L.DIST_UNIFORM, -2.0, 2.0)])]
    ups = [oracle.mwg_update(oracle.KIND_MIX, [0, 1], sigma=1.0 * np.eye(2), sigma_b=3.0 * np.eye(2), lam=0.5,
                             haario_k=30, prior=L.PRIOR_PRODUCT, factors=fac)]
    steps = full_steps(150, 1)
    eng, st, h = run_both(oracle, 2, 1024, 150, ups, mu, np.eye(2), obs, steps, 79, theta0=mu)
    check(oracle, eng, st, h, steps, ups, 1)
    check_mix(oracle, eng, st, ups)
    assert np.all(h["prop"][..., 0] >= -1.0) and np.all(h["prop"][..., 0] <= 3.0)


def test_mix_with_a_user_target(oracle):
    """GaussianRandomWalkMix + Haario on a user law (the student-t regression)."""
    case = U.student_t()
    D = case.D
    fn, src = oracle.user_loglik(case.name)
    ups = [oracle.mwg_update(oracle.KIND_MIX, range(D), sigma=0.01 * np.eye(D), sigma_b=0.02 * np.eye(D), lam=0.5,
                             haario_k=40)]
    C, M = 1024, 120
    eng = build(oracle, D, C, M, ups, case.seed)
    eng.set_user_target(src, obs=case.obs, params=case.params, theta0=case.theta0)
    th0 = np.ascontiguousarray(np.broadcast_to(case.theta0, (C, D)))
    eng.set_state(th0)
    steps = full_steps(M, 1)
    eng.run(steps)
    st = oracle.MWGState(th0.copy(), case.theta0, ups)
    h = oracle.run_mwg(st, ups, seed=case.seed, t_sigma=None, obs=case.obs, steps=steps, nthreads=8, user_ll=fn,
                       user_params=case.params)
    assert "UserTarget" in eng.kernel_name()
    check(oracle, eng, st, h, steps, ups, 1)
    check_mix(oracle, eng, st, ups)


def _flam(lam, N, it):
    return 0.5 + 0.4 * np.sin(it / 37.0) * (N % 5) / 4.0


def test_custom_flambda_on_the_general_kernel(oracle):
    """fλ at every readjust of a mix block in a two-update schedule: the launch ends
    after the readjust and the next one reads the new λ; the oracle runs in pieces."""
    rng = np.random.default_rng(6)
    mu = rng.normal(size=3)
    obs = mu + rng.normal(size=(6, 3))
    k, M = 20, 100
    ups = [oracle.mwg_update(oracle.KIND_MIX, [0, 1], sigma=0.1 * np.eye(2), sigma_b=0.3 * np.eye(2), lam=0.5,
                             haario_k=k),
           oracle.mwg_update(2, [2], sigma=[[0.1]])]
    C = 700
    eng = build(oracle, 3, C, M, ups, 80)
    eng.set_mix_lambda_fn(1, _flam)
    eng.set_gsn_target(mu, np.eye(3), obs)
    eng.set_state(np.tile(mu, (C, 1)))
    steps = full_steps(M, 2)
    eng.run(steps)
    st = oracle.MWGState(np.tile(mu, (C, 1)), mu, ups)
    hs = []
    for it0 in range(1, M + 1, k):
        piece = [(i, p) for i in range(it0, it0 + k) for p in (1, 2)]
        hs.append(oracle.run_mwg(st, ups, seed=80, t_sigma=np.eye(3), obs=obs, steps=piece, nthreads=8))
        # the readjust is at the k-th own turn (iteration it0 + k − 1, update 1); adpt.N after its register!
        st.lam[0] = _flam(st.lam[0], int(st.N[0]) - 1, it0 + k - 1)
    h = {key: np.concatenate([x[key] for x in hs]) for key in hs[0]}
    check(oracle, eng, st, h, steps, ups, 2)
    check_mix(oracle, eng, st, ups)
    assert eng.get_mix_lambda(1) == st.lam[0]
