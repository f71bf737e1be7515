"""General schedule kernel (mwg_gsn_kernel) on the GPU against the oracle
(orc_run_mwg), bit for bit: several updates per iteration over coordinate
subsets in any order, UniformRandomWalk and GaussianRandomWalk, AdaptationUnifRW,
exclusion schedules, split runs, both likelihood modes, both history modes."""
import numpy as np
import pytest

from extensible_mcmc import _lib as L
from extensible_mcmc import workloads as W
from extensible_mcmc.engine import Engine, EngineConfig
from extensible_mcmc.schedule import MCMCSchedule

pytestmark = pytest.mark.gpu

ADAPT = {"k": 50, "target": 0.234, "scale": 0.1, "min": 1e-12, "max": 1e7, "offset": 1e2}


@pytest.fixture(autouse=True)
def _gpu(require_gpu):
    pass


def full_steps(M, P, first=1):
    return [(i, p) for i in range(first, M + 1) for p in range(1, P + 1)]


def make_engine(D, C, M, ups, mu, t_sigma, obs, seed, ll_mode=L.LL_PER_OBS, hist=L.HIST_FULL, spl=0, theta0=None,
                variant=0):
    eng = Engine(EngineConfig(dim=D, num_chains=C, num_mcmc_steps=M, seed=seed, history_mode=hist,
                              steps_per_launch=spl, kernel_variant=variant))
    for u in ups:
        pr = dict(prior=u.get("prior", 0), prior_factors=u.get("factors") or None)
        if u["kind"] == 1:
            eng.add_uniform_rw_update(u["coords"], u["eps"], adapt=u["adapt"], pos=u.get("pos"), **pr)
        else:
            eng.add_gaussian_rw_update(u["coords"], u["sigma"], pos=u.get("pos"), **pr)
    eng.set_gsn_target(mu, t_sigma, obs, ll_mode=ll_mode)
    eng.set_state(np.zeros((C, D)) if theta0 is None else theta0)
    return eng


def check(oracle, eng, st, h, steps, ups, P, full=True):
    eng.synchronize(allow_faults=True)
    th, ll = eng.get_state()
    assert np.array_equal(th, st.theta)
    assert np.array_equal(ll, st.ll)
    ra, nacc = eng.get_chain_stats()
    assert np.array_equal(ra, st.ra)
    assert np.array_equal(nacc, st.nacc)
    assert np.array_equal(eng.get_faults(), st.faults)
    assert np.array_equal(eng.get_proposal_ll(), st.ll_prop, equal_nan=True)
    iters = sorted({i for i, _ in steps})
    i0, n = iters[0], iters[-1] - iters[0] + 1
    acc = eng.get_history(L.H_ACCEPT, i0, n)
    hs = eng.get_history(L.H_STATE, i0, n) if full else None
    hp = eng.get_history(L.H_PROPOSAL, i0, n) if full else None
    hl = eng.get_history(L.H_LL, i0, n) if full else None
    for s, (it, p) in enumerate(steps):
        assert np.array_equal(acc[it - i0, p - 1], h["acc"][s]), f"accepts at step {s} ({it}, {p})"
        if full:
            assert np.array_equal(hs[it - i0, p - 1], h["theta"][s])
            assert np.array_equal(hp[it - i0, p - 1], h["prop"][s])
            assert np.array_equal(hl[it - i0, p - 1], h["ll"][s])
    for p, u in enumerate(ups):
        if u["kind"] == 1:
            eps, pr, ac = eng.get_update_state(p + 1, len(u["coords"]))
            assert np.array_equal(eps, st.eps[p, :, :len(u["coords"])])
            assert np.array_equal(pr, st.aprop[p]) and np.array_equal(ac, st.aacc[p])


def run_both(oracle, D, C, M, ups, mu, t_sigma, obs, steps, seed, **kw):
    eng = make_engine(D, C, M, ups, mu, t_sigma, obs, seed, **kw)
    eng.run(steps)
    th0 = kw.get("theta0")
    st = oracle.MWGState(np.zeros((C, D)) if th0 is None else np.array(th0, dtype=np.float64), mu, ups)
    h = oracle.run_mwg(st, ups, seed=seed, t_sigma=t_sigma, obs=obs, steps=steps,
                       ll_mode=kw.get("ll_mode", 0), nthreads=8)
    return eng, st, h


@pytest.mark.parametrize("kind", ["uniform", "gaussian", "adaptive"])
def test_reference_single_site(oracle, kind):
    """test/runtests.jl:87-114 and the tutorial variants: D = 2, P = 2."""
    w = W.ref_test()
    if kind == "gaussian":
        ups = [oracle.mwg_update(2, [0], sigma=[[1.0]]), oracle.mwg_update(2, [1], sigma=[[1.0]])]
    else:
        eps, ad = (0.1, ADAPT) if kind == "adaptive" else (1.0, None)
        ups = [oracle.mwg_update(1, [0], eps=[eps], adapt=ad), oracle.mwg_update(1, [1], eps=[eps], adapt=ad)]
    steps = full_steps(400, 2)
    eng, st, h = run_both(oracle, 2, 1000, 400, ups, [1.0, 2.0], w.t_sigma, w.obs, steps, w.seed)
    assert "mwg_gsn_kernel<D=2,P=2" in eng.kernel_name()
    check(oracle, eng, st, h, steps, ups, 2)


def test_exclusions_and_split_runs(oracle):
    """exclude_updates: update 2 off on iterations 5:40; the schedule is run in
    three calls with 7-step launches."""
    w = W.ref_test()
    ups = [oracle.mwg_update(1, [0], eps=[0.5]), oracle.mwg_update(1, [1], eps=[0.5])]
    steps = [(s.mcmciter, s.pidx) for s in MCMCSchedule(150, 2, [(2, range(5, 41))])]
    eng = make_engine(2, 333, 150, ups, [1.0, 2.0], w.t_sigma, w.obs, w.seed, spl=7)
    for a, b in ((0, 50), (50, 51), (51, len(steps))):
        eng.run(steps[a:b])
    st = oracle.MWGState(np.zeros((333, 2)), [1.0, 2.0], ups)
    h = oracle.run_mwg(st, ups, seed=w.seed, t_sigma=w.t_sigma, obs=w.obs, steps=steps, nthreads=8)
    check(oracle, eng, st, h, steps, ups, 2)


@pytest.mark.parametrize("ll_mode", [L.LL_PER_OBS, L.LL_SUFFSTAT])
@pytest.mark.parametrize("hist", [L.HIST_FULL, L.HIST_ACCEPT_ONLY])
def test_block_updates_mixed_kernels(oracle, ll_mode, hist):
    """D = 4: a dense GaussianRandomWalk block on coords (3, 1) and an adaptive
    UniformRandomWalk block on coords (4, 2) (1-based, out of order)."""
    w = W.cfg2(64)
    D = 4
    rng = np.random.default_rng(5)
    A = rng.standard_normal((D, D))
    ts = A @ A.T / D + np.eye(D)
    obs = rng.standard_normal((12, D)) + 0.5
    mu = np.array([0.1, -0.2, 0.3, 0.0])
    ups = [oracle.mwg_update(2, [2, 0], sigma=[[0.09, 0.02], [0.02, 0.04]]),
           oracle.mwg_update(1, [3, 1], eps=[0.3, 0.2], adapt=dict(ADAPT, k=20))]
    steps = full_steps(300, 2)
    eng, st, h = run_both(oracle, D, 900, 300, ups, mu, ts, obs, steps, w.seed, ll_mode=ll_mode, hist=hist)
    check(oracle, eng, st, h, steps, ups, 2, full=(hist == L.HIST_FULL))


@pytest.mark.parametrize("D,split", [(8, (8,)), (16, (8, 8)), (16, (16,)), (3, (1, 2))])
def test_dimensions_and_canonical_blocks(oracle, D, split):
    """Updates of 1, 2, 8 and 16 coordinates (the 16-coordinate update sums in
    two canonical blocks); coords reversed so the general path is taken."""
    w = W.cfg2(256)
    obs = np.asarray(w.obs)[:, :D]
    ts = np.asarray(w.t_sigma)[:D, :D]
    mu = np.asarray(w.mu_true)[:D]
    ups, c0 = [], 0
    for n in split:
        coords = list(range(c0, c0 + n))[::-1]
        ups.append(oracle.mwg_update(2, coords, sigma=0.02 * np.eye(n)))
        c0 += n
    steps = full_steps(120, len(ups))
    eng, st, h = run_both(oracle, D, 256, 120, ups, mu, ts, obs, steps, w.seed)
    check(oracle, eng, st, h, steps, ups, len(ups))


@pytest.mark.parametrize("adapt", [False, True])
def test_uniform_rw_positivity_restricted(oracle, adapt):
    """UniformRandomWalk(ϵ, pos) (random_walk.jl:63-94): θ° = θ·e^U on the restricted
    coordinates, θ + U on the others, and the transition densities
    Σ_pos −log(2ϵ) − log θ no longer cancel in the MH ratio; with and without
    AdaptationUnifRW, a block mixing restricted and free coordinates."""
    w = W.ref_test()
    D, C, M = 3, 300, 120
    mu = np.array([1.0, 2.0, 0.5])
    t_sigma = np.array([[1.0, 0.3, 0.0], [0.3, 1.0, 0.0], [0.0, 0.0, 0.25]])
    obs = np.random.default_rng(5).multivariate_normal(mu, t_sigma, 10)
    ups = [oracle.mwg_update(1, [0, 2], eps=[0.4, 0.3], pos=[True, False], adapt=ADAPT if adapt else None),
           oracle.mwg_update(1, [1], eps=[0.6], pos=[True])]
    theta0 = np.tile([1.5, 0.7, 0.2], (C, 1))
    steps = full_steps(M, 2)
    eng, st, h = run_both(oracle, D, C, M, ups, mu, t_sigma, obs, steps, w.seed, theta0=theta0)
    check(oracle, eng, st, h, steps, ups, 2)
    th, _ = eng.get_state()
    assert np.all(th[:, :2] > 0) and 0.05 < h["acc"].mean() < 0.95


@pytest.mark.parametrize("joint", [False, True])
def test_gaussian_rw_positivity_restricted(oracle, joint):
    """GaussianRandomWalk(Σ, pos) (random_walk.jl:136-171) on device: the log-scale
    walk, the log-Jacobian terms and the reference's in-place exp/log round trips
    (accepted states are θ° after two more round trips), bit for bit.  joint: one
    update on all coordinates (not the fused kernel: positivity routes it here)."""
    w = W.ref_test()
    D, C, M = 3, 300, 120
    mu = np.array([1.0, 2.0, 0.5])
    t_sigma = np.array([[1.0, 0.3, 0.0], [0.3, 1.0, 0.0], [0.0, 0.0, 0.25]])
    obs = np.random.default_rng(6).multivariate_normal(mu, t_sigma, 10)
    if joint:
        ups = [oracle.mwg_update(2, [0, 1, 2], sigma=0.02 * np.eye(3) + 0.005, pos=[True, False, True])]
    else:
        ups = [oracle.mwg_update(2, [2, 0], sigma=[[0.05, 0.01], [0.01, 0.04]], pos=[True, False]),
               oracle.mwg_update(1, [1], eps=[0.6], pos=[True])]
    theta0 = np.tile([1.5, 0.7, 0.2], (C, 1))
    steps = full_steps(M, len(ups))
    eng, st, h = run_both(oracle, D, C, M, ups, mu, t_sigma, obs, steps, w.seed, theta0=theta0)
    assert "mwg" in eng.kernel_name()
    check(oracle, eng, st, h, steps, ups, len(ups))
    assert h["acc"][len(ups):].sum() > 10  # moves beyond the first step's auto-accepts


def test_reference_schedule_kat_on_device(oracle, golden_dir):
    """The reference's schedule KAT (test/runtests.jl:5-31) driven through the
    general kernel: 4 updates with exclusions [(1, 3:8), (2, 4:2:10)], and at
    (5, 3) reschedule!(schedule, 2, [4], [(5, 8:9)]) grows the schedule to 6
    updates.  The host walks the schedule exactly as __run! does (run.jl:64-83)
    and hands each (iter, pidx) to emcmc_run; the step list must be the KAT's and
    every written slot, the rolling acceptance across the skipped iterations
    and the final state must equal the oracle's run of that list."""
    import json
    from extensible_mcmc import JRange, reschedule
    k = json.loads((golden_dir / "schedule_kat.json").read_text())
    jr = lambda t: JRange(t[0], t[1], t[2])  # noqa: E731
    D, C, M = 6, 777, k["num_mcmc_iter"]
    rng = np.random.default_rng(11)
    obs = rng.normal(size=(8, D))
    mu = np.zeros(D)
    ups = [oracle.mwg_update(1 if p % 2 else 2, [p], eps=[0.7] if p % 2 else None,
                             sigma=None if p % 2 else [[0.5]]) for p in range(D)]
    eng = make_engine(D, C, M, ups, mu, np.eye(D), obs, 4242)
    sched = MCMCSchedule(M, k["num_params"], [(i, jr(r)) for i, r in k["exclude_params"]])
    ra = k["reschedule_args"]
    steps = []
    for s in sched:
        steps.append((s.mcmciter, s.pidx))
        eng.run([(s.mcmciter, s.pidx)])
        if [s.mcmciter, s.pidx] == k["reschedule_at"]:
            reschedule(sched, ra["num_new_updates"], ra["idxes_to_remove"],
                       [(i, jr(r)) for i, r in ra["idxes_to_add"]])
    assert [list(t) for t in steps] == k["expected"]
    st = oracle.MWGState(np.zeros((C, D)), mu, ups)
    h = oracle.run_mwg(st, ups, seed=4242, t_sigma=np.eye(D), obs=obs, steps=steps, nthreads=8)
    check(oracle, eng, st, h, steps, ups, D)


def test_per_coordinate_adaptation(oracle):
    """AdaptationUnifRW's per-coordinate form on a UniformRandomWalk block, with a
    Gaussian single-site update beside it (include/emcmc.h
    emcmc_unifrw_adaptation_vec): every chain's adapted ϵ bitwise."""
    w = W.ref_test()
    vec = {"k": 40, "target": 0.234, "scale": [0.05, 0.2], "min": [1e-12, 0.02], "max": [1e7, 0.5],
           "offset": [1e2, 3.0]}
    ups = [oracle.mwg_update(1, [0, 1], eps=[0.1, 0.3], adapt=vec)]
    steps = full_steps(600, 1)
    eng, st, h = run_both(oracle, 2, 1500, 600, ups, [1.0, 2.0], w.t_sigma, w.obs, steps, w.seed)
    check(oracle, eng, st, h, steps, ups, 1)


def test_d64_general_kernel_blocks_and_dense(oracle):
    """D = 64 on the general kernel (compiled at run time): a diagonal Gaussian
    block of 16, a correlated Gaussian block of 40 (five canonical 8-blocks: the
    run-time tree 5 → 3 → 2 → 1) and a UniformRandomWalk block of 8 with a
    ProductPrior([Product(fill(Normal, 8))], [8]), against a dense D = 64 target."""
    rng = np.random.default_rng(9)
    D, C, M = 64, 700, 120
    A = rng.standard_normal((D, D))
    ts = A @ A.T / D + np.eye(D)
    mu = rng.normal(size=D)
    obs = mu + rng.normal(size=(6, D))
    B = rng.standard_normal((40, 40))
    S40 = 0.002 * (B @ B.T / 40 + np.eye(40))
    ups = [oracle.mwg_update(2, range(0, 16), sigma=0.01 * np.eye(16)),
           oracle.mwg_update(2, range(16, 56), sigma=S40),
           oracle.mwg_update(1, range(56, 64), eps=[0.05] * 8, prior=L.PRIOR_PRODUCT,
                             factors=[(L.DIST_PRODUCT, 8, [(L.DIST_NORMAL, 0.0, 3.0)] * 8)])]
    steps = full_steps(M, 3)
    eng, st, h = run_both(oracle, D, C, M, ups, mu, ts, obs, steps, 31)
    assert "D=64" in eng.kernel_name()
    # as mwg_rw_block_kernel this schedule needs scratch (θ, P°.θ, a dense 40-block and the
    # dense target's sweeps exceed the register file), so the wide kernel runs it
    assert eng.kernel_name().startswith("mwg_wide_kernel"), eng.kernel_name()
    check(oracle, eng, st, h, steps, ups, 3)


def test_d48_block_of_48(oracle):
    """A joint GaussianRandomWalk block of all 48 coordinates (six 8-blocks, tree
    6 → 3 → 2 → 1) beside nothing else, on a diagonal target: general kernel
    NU = 48 compiled at run time."""
    rng = np.random.default_rng(10)
    D, C, M = 48, 512, 80
    mu = rng.normal(size=D)
    obs = mu + rng.normal(size=(5, D))
    ups = [oracle.mwg_update(2, range(D), sigma=0.004 * np.eye(D), pos=[False] * D, prior=L.PRIOR_PRODUCT,
                             factors=[(L.DIST_PRODUCT, D, [(L.DIST_NORMAL, 0.0, 10.0)] * D)])]
    steps = full_steps(M, 1)
    eng, st, h = run_both(oracle, D, C, M, ups, mu, np.eye(D), obs, steps, 32)
    check(oracle, eng, st, h, steps, ups, 1)
