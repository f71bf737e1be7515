"""mwg_rw_block_kernel on the GPU: one UniformRandomWalk or
GaussianRandomWalk update over all 17 ≤ D ≤ 64 coordinates with a prior
(priors.jl:11-88), positivity flags (random_walk.jl:45-94, 136-171), the proposal!
redraw loop (updates.jl:191-196) and AdaptationUnifRW (adaptation.jl:273-329), the
update's structure compiled in at run time, against the oracle (orc_run_mwg kinds 1
and 2 — the restatement the general kernels are checked against), bit for bit:
accept streams, θ / θ° / ll histories, sub_ws°.ll, rolling acceptance, fault bits,
the adaptive ϵ.  The same schedules on the wide general kernel
(EMCMC_VARIANT_NO_BLOCK) give the same bits."""
import numpy as np
import pytest

from extensible_mcmc import _lib as L
from extensible_mcmc import workloads as W
from extensible_mcmc.engine import Engine, EngineConfig
from extensible_mcmc.schedule import MCMCSchedule
from test_gpu_mwg import ADAPT, check, full_steps

pytestmark = pytest.mark.gpu

N_, U_, E_, G_, LN_ = L.DIST_NORMAL, L.DIST_UNIFORM, L.DIST_EXPONENTIAL, L.DIST_GAMMA, L.DIST_LOGNORMAL
IG_, C_, LA_, T_ = L.DIST_INVERSE_GAMMA, L.DIST_CAUCHY, L.DIST_LAPLACE, L.DIST_TDIST
P_, MV_ = L.DIST_PRODUCT, L.DIST_MVNORMAL


@pytest.fixture(autouse=True)
def _gpu(require_gpu):
    pass


def problem(D, shift=0.0, dense_t=False, seed=5):
    """cfg 2's Gaussian target at dimension D, μ* shifted (a positive target for pos flags)."""
    w = W.cfg2(8, D=D)
    mu = np.asarray(w.mu_true) + shift
    obs = np.asarray(w.obs) - np.asarray(w.mu_true) + mu
    ts = np.eye(D)
    if dense_t:
        B = np.random.default_rng(seed).standard_normal((D, D))
        ts = B @ B.T / D + np.eye(D)
    return w.seed, mu, ts, obs


def engine_for(D, C, M, ups, mu, ts, obs, seed, ll_mode=L.LL_PER_OBS, hist=L.HIST_FULL, spl=0, variant=0,
               theta0=None, user=None, lanes=0):
    eng = Engine(EngineConfig(dim=D, num_chains=C, num_mcmc_steps=M, seed=seed, history_mode=hist,
                              steps_per_launch=spl, kernel_variant=variant, lanes_per_chain=lanes))
    for u in ups:
        pr = dict(prior=u.get("prior", 0), prior_factors=u.get("factors") or None)
        if u["kind"] == 1:
            eng.add_uniform_rw_update(u["coords"], u["eps"], adapt=u["adapt"], pos=u.get("pos"), **pr)
        else:
            eng.add_gaussian_rw_update(u["coords"], u["sigma"], pos=u.get("pos"), **pr)
    if user is None:
        eng.set_gsn_target(mu, ts, obs, ll_mode=ll_mode)
    else:
        eng.set_user_target(user, obs=obs, theta0=np.zeros(D))
    eng.set_state(np.zeros((C, D)) if theta0 is None else theta0)
    return eng


def run_pair(oracle, D, C, M, ups, mu, ts, obs, seed, theta0, steps=None, ll_mode=L.LL_PER_OBS, hist=L.HIST_FULL,
             spl=0, user=None, calls=None, variant=0, lanes=0):
    steps = steps or full_steps(M, 1)
    eng = engine_for(D, C, M, ups, mu, ts, obs, seed, ll_mode, hist, spl, variant=variant, theta0=theta0,
                     user=None if user is None else user[1], lanes=lanes)
    for a, b in (calls or [(0, len(steps))]):
        eng.run(steps[a:b])
    st = oracle.MWGState(np.array(theta0, dtype=np.float64), mu if user is None else np.zeros(D), ups)
    kw = {} if user is None else {"user_ll": user[0]}
    h = oracle.run_mwg(st, ups, seed=seed, t_sigma=ts, obs=obs, steps=steps, ll_mode=ll_mode, nthreads=8, **kw)
    return eng, st, h, steps


def assert_block(eng, D):
    assert eng.kernel_name().startswith(f"mwg_rw_block_kernel<D={D}"), eng.kernel_name()


def s2(D, n=10, f=1.0):
    return f * (2.38 / np.sqrt(D * n)) ** 2


@pytest.mark.parametrize("ll_mode", [L.LL_PER_OBS, L.LL_SUFFSTAT])
@pytest.mark.parametrize("hist", [L.HIST_FULL, L.HIST_ACCEPT_ONLY])
def test_d32_gaussian_rw_product_prior_normal(oracle, ll_mode, hist):
    """VERDICT shape 1: D = 32 joint GaussianRandomWalk + ProductPrior of Normal factors
    (one Product of 32 Normals: the logpdf folded left over the components), on the schedule
    kernel (EMCMC_VARIANT_NO_FUSED_PRIOR: by default the fused kernel takes it,
    tests/test_gpu_fprior.py)."""
    D, C, M = 32, 2048, 160
    seed, mu, ts, obs = problem(D)
    ups = [oracle.mwg_update(2, range(D), sigma=s2(D) * np.eye(D), prior=L.PRIOR_PRODUCT,
                             factors=[(P_, D, [(N_, 0.1 * j, 1.0 + 0.05 * j) for j in range(D)])])]
    th0 = np.tile(mu, (C, 1))
    eng, st, h, steps = run_pair(oracle, D, C, M, ups, mu, ts, obs, seed, th0, ll_mode=ll_mode, hist=hist,
                                 variant=L.VARIANT_NO_FUSED_PRIOR)
    assert_block(eng, D)
    check(oracle, eng, st, h, steps, ups, 1, full=(hist == L.HIST_FULL))
    assert 0.1 < h["acc"].mean() < 0.6


@pytest.mark.parametrize("variant", [L.VARIANT_NO_FUSED_PRIOR, 0])
def test_d32_gaussian_rw_standard_prior_mvnormal(oracle, variant):
    """VERDICT shape 2: D = 32 joint GaussianRandomWalk + StandardPrior(MvNormal(μ0, Σ0)),
    Σ0 dense (the forward substitution over the prior's factor, squares folded left) — on the
    schedule kernel and (variant 0) on the fused kernel, lane 1's rows after lane 0's."""
    D, C, M = 32, 2048, 160
    seed, mu, ts, obs = problem(D)
    B = np.random.default_rng(9).standard_normal((D, D))
    S0 = B @ B.T / D + 0.5 * np.eye(D)
    ups = [oracle.mwg_update(2, range(D), sigma=s2(D) * np.eye(D), prior=L.PRIOR_STANDARD,
                             factors=[(MV_, D, 0.3 * np.ones(D), S0)])]
    th0 = np.tile(mu, (C, 1))
    eng, st, h, steps = run_pair(oracle, D, C, M, ups, mu, ts, obs, seed, th0, variant=variant)
    if variant:
        assert_block(eng, D)
    else:
        assert eng.kernel_name().startswith("rwm_gsn_diag_kernel<D=32,LPC=2,"), eng.kernel_name()
    check(oracle, eng, st, h, steps, ups, 1)


@pytest.mark.parametrize("variant", [L.VARIANT_NO_FUSED_PRIOR, 0])
@pytest.mark.parametrize("prior", [L.PRIOR_IMPROPER, L.PRIOR_IMPROPER_POS])
def test_d32_uniform_rw_with_pos_flags(oracle, prior, variant):
    """VERDICT shape 3: D = 32 joint UniformRandomWalk with positivity flags (θ° = θ·e^U on
    24 of 32 coordinates, the −log(2ϵ) − log θ° density terms folded left), ImproperPrior
    and ImproperPosPrior — on the schedule kernel and (variant 0: the flags repeat every 4
    coordinates) on the fused kernel, the density sums folded lane to lane."""
    D, C, M = 32, 2048, 200
    seed, mu, ts, obs = problem(D, shift=4.0)
    pos = [j % 4 != 3 for j in range(D)]
    eps = [0.05 + 0.002 * j for j in range(D)]
    ups = [oracle.mwg_update(1, range(D), eps=eps, pos=pos, prior=prior)]
    th0 = np.tile(mu, (C, 1))
    eng, st, h, steps = run_pair(oracle, D, C, M, ups, mu, ts, obs, seed, th0, variant=variant)
    if variant:
        assert_block(eng, D)
    else:
        assert eng.kernel_name().startswith("rwm_gsn_diag_kernel<D=32,LPC=2"), eng.kernel_name()
    check(oracle, eng, st, h, steps, ups, 1)
    assert 0.05 < h["acc"].mean() < 0.9


def test_d32_adaptive_uniform_rw_with_pos(oracle):
    """AdaptationUnifRW (per-chain ϵ, readjusted every k = 25 proposals) on a D = 32
    UniformRandomWalk with positivity flags, split into launches of 7 steps."""
    D, C, M = 32, 1024, 150
    seed, mu, ts, obs = problem(D, shift=4.0)
    pos = [j % 2 == 0 for j in range(D)]
    ups = [oracle.mwg_update(1, range(D), eps=[0.08] * D, pos=pos, adapt=dict(ADAPT, k=25, scale=0.02))]
    th0 = np.tile(mu, (C, 1))
    eng, st, h, steps = run_pair(oracle, D, C, M, ups, mu, ts, obs, seed, th0, spl=7,
                                 calls=[(0, 40), (40, 41), (41, 150)])
    assert_block(eng, D)
    check(oracle, eng, st, h, steps, ups, 1)


def test_d24_dense_sigma_all_families_and_redraws(oracle):
    """D = 24, a dense Σ (column sweep of L z, row substitutions of the densities), a
    ProductPrior over the univariate families (dims-1 factors reading θ[1]), a Product factor
    and an MvNormal factor, and Uniform(1.6, 3.4) factors the target pushes the chains
    against: the proposal! redraw loop runs (normal indices (r << 17) | j) and the carried
    log-prior follows each accept."""
    D, C, M = 24, 1536, 120
    seed, mu, ts, obs = problem(D, shift=2.5, dense_t=True)
    A = np.random.default_rng(3).standard_normal((D, D))
    sig = s2(D, f=0.6) * (A @ A.T / D + np.eye(D))
    fam1 = [(N_, 1, 2.0, 1.5), (LN_, 1, 0.5, 1.0), (G_, 1, 2.0, 1.5), (E_, 1, 2.0, 0.0)]  # dims-1: read θ[1]
    fam_prod = (P_, 6, [(IG_, 3.0, 2.0), (C_, 1.0, 2.0), (LA_, 2.0, 1.0),
                        (T_, 5.0, 0.0), (N_, 2.5, 3.0), (G_, 3.0, 1.0)])
    mvn = (MV_, 8, 2.5 * np.ones(8), np.eye(8) + 0.2 * np.ones((8, 8)))
    unif = (P_, 6, [(U_, 1.6, 3.4)] * 6)
    ups = [oracle.mwg_update(2, range(D), sigma=sig, prior=L.PRIOR_PRODUCT, factors=fam1 + [fam_prod, mvn, unif])]
    th0 = np.tile(np.where(np.arange(D) >= 18, 2.5, mu), (C, 1))
    eng, st, h, steps = run_pair(oracle, D, C, M, ups, mu, ts, obs, seed, th0)
    assert_block(eng, D)
    check(oracle, eng, st, h, steps, ups, 1)
    prop = h["prop"][..., 18:]
    assert np.all((prop >= 1.6) & (prop <= 3.4))  # every stored θ° inside the Uniform support


@pytest.mark.parametrize("D", [20, 25, 33])
def test_gaussian_rw_with_pos_round_trips(oracle, D):
    """GaussianRandomWalk with positivity flags on half the coordinates: the reference's
    in-place exp/log round trips (θ°₃, θ₃), ImproperPosPrior (no log-prior carry), odd and
    even D, on the schedule kernel (EMCMC_VARIANT_NO_FUSED_PRIOR; tests/test_gpu_fprior.py runs
    the fused one).  At D = 33 the round trips' vectors exceed the register file (the code
    object needs scratch), so the schedule runs on the wide kernel: the same bits either way."""
    C, M = 1024, 120
    seed, mu, ts, obs = problem(D, shift=3.0)
    pos = [j % 2 == 1 for j in range(D)]
    ups = [oracle.mwg_update(2, range(D), sigma=s2(D, f=0.05) * np.eye(D), pos=pos, prior=L.PRIOR_IMPROPER_POS)]
    th0 = np.tile(mu, (C, 1))
    eng, st, h, steps = run_pair(oracle, D, C, M, ups, mu, ts, obs, seed, th0, variant=L.VARIANT_NO_FUSED_PRIOR)
    if D == 33:
        assert eng.kernel_name().startswith("mwg_wide_kernel<D=33"), eng.kernel_name()
    else:
        assert_block(eng, D)
    check(oracle, eng, st, h, steps, ups, 1)


def test_gaussian_rw_with_64_pos_flags_runs_on_the_wide_kernel(oracle):
    """GaussianRandomWalk over all 64 coordinates with every one flagged, off the fused kernel
    (EMCMC_VARIANT_NO_FUSED_PRIOR): the schedule kernel is not compiled (more than 32 flagged
    coordinates always need scratch, and at 64 the gfx950 backend aborts the compiling process),
    the wide kernel runs it with the oracle's bits."""
    D, C, M = 64, 512, 24
    seed, mu, ts, obs = problem(D, shift=3.0)
    ups = [oracle.mwg_update(2, range(D), sigma=s2(D, f=0.05) * np.eye(D), pos=[True] * D)]
    eng, st, h, steps = run_pair(oracle, D, C, M, ups, mu, ts, obs, seed, np.tile(mu, (C, 1)),
                                 variant=L.VARIANT_NO_FUSED_PRIOR)
    assert eng.kernel_name().startswith("mwg_wide_kernel<D=64"), eng.kernel_name()
    check(oracle, eng, st, h, steps, ups, 1)


@pytest.mark.parametrize("variant", [L.VARIANT_NO_FUSED_PRIOR, 0])
def test_schedule_gap_and_launch_cuts(oracle, variant):
    """The update excluded on iterations 31:50 (rolling_ar restarts from 0.0) and launches
    of 9 steps across three run calls: the log-prior is re-evaluated at each launch's
    first step and carried inside it — on the schedule kernel and on the fused kernel with the
    prior compiled in (variant 0: a Product of Cauchy factors is its shape)."""
    D, C, M = 32, 1024, 110
    seed, mu, ts, obs = problem(D)
    ups = [oracle.mwg_update(2, range(D), sigma=s2(D) * np.eye(D), prior=L.PRIOR_PRODUCT,
                             factors=[(P_, D, [(C_, 0.0, 3.0)] * D)])]
    steps = [(s.mcmciter, s.pidx) for s in MCMCSchedule(M, 1, [(1, range(31, 51))])]
    th0 = np.tile(mu, (C, 1))
    eng, st, h, steps = run_pair(oracle, D, C, M, ups, mu, ts, obs, seed, th0, steps=steps, spl=9,
                                 calls=[(0, 25), (25, 26), (26, len(steps))], variant=variant)
    if variant:
        assert_block(eng, D)
    else:
        assert eng.kernel_name().startswith("rwm_gsn_diag_kernel<D=32,LPC=2"), eng.kernel_name()
    check(oracle, eng, st, h, steps, ups, 1)


def test_user_law_with_prior(oracle):
    """A user law (logistic regression, EMCMC_USER_LOGLIK) under a D = 20 UniformRandomWalk
    with a ProductPrior of Normals: the block kernel with TGT = the user's law."""
    D, C, M, n = 20, 512, 80, 60
    rng = np.random.default_rng(12)
    X = rng.standard_normal((n, D)) / np.sqrt(D)
    beta = rng.normal(scale=0.3, size=D)
    y = (rng.uniform(size=n) < 1.0 / (1.0 + np.exp(-(X @ beta)))).astype(float)
    obs = np.column_stack([X, y])
    fn, src = oracle.user_loglik("logistic_regression")
    ups = [oracle.mwg_update(1, range(D), eps=[0.2] * D, prior=L.PRIOR_PRODUCT, factors=[(P_, D, [(N_, 0.0, 1.0)] * D)])]
    eng, st, h, steps = run_pair(oracle, D, C, M, ups, None, None, obs, 41, np.zeros((C, D)), user=(fn, src))
    assert_block(eng, D)
    assert "UserTarget" in eng.kernel_name()
    check(oracle, eng, st, h, steps, ups, 1)


def test_wide_kernel_gives_the_same_bits():
    """EMCMC_VARIANT_NO_BLOCK runs the same update on mwg_wide_kernel<D=32,NU=32>: every
    history and the final state equal the block kernel's."""
    D, C, M = 32, 1024, 60
    seed, mu, ts, obs = problem(D, shift=4.0)
    pos = [j % 3 == 0 for j in range(D)]
    fac = [(P_, D, [(G_, 4.0, 1.0)] * D)]
    out = []
    for variant in (0, L.VARIANT_NO_BLOCK):
        eng = Engine(EngineConfig(dim=D, num_chains=C, num_mcmc_steps=M, seed=seed, kernel_variant=variant))
        eng.add_uniform_rw_update(range(D), [0.07] * D, pos=pos, prior=L.PRIOR_PRODUCT, prior_factors=fac)
        eng.set_gsn_target(mu, ts, obs)
        eng.set_state(np.tile(mu, (C, 1)))
        eng.run_iters(1, M)
        eng.synchronize(allow_faults=True)
        out.append((eng.kernel_name(), eng.get_state(), eng.get_history(L.H_ACCEPT, 1, M),
                    eng.get_history(L.H_PROPOSAL, 1, M), eng.get_faults()))
        eng.close()
    assert out[0][0].startswith("mwg_rw_block_kernel") and out[1][0].startswith("mwg_wide_kernel<D=32")
    for a, b in zip(out[0][1:], out[1][1:]):
        if isinstance(a, tuple):
            for x, y in zip(a, b):
                assert np.array_equal(x, y)
        else:
            assert np.array_equal(a, b)


# ---- compiled schedules of several updates (Metropolis-within-Gibbs, round 6) ----------------
def sched_problem(D, shift=0.0):
    seed, mu, ts, obs = problem(D, shift=shift)
    return seed, mu, ts, obs, np.tile(mu, (1, 1))


@pytest.mark.parametrize("ll_mode", [L.LL_PER_OBS, L.LL_SUFFSTAT])
@pytest.mark.parametrize("hist", [L.HIST_FULL, L.HIST_ACCEPT_ONLY])
def test_d32_two_blocks_of_16(oracle, ll_mode, hist):
    """Two GaussianRandomWalk blocks of 16 coordinates (run.jl:64-83 over P = 2): the compiled
    schedule keeps θ, P°.θ and both blocks' vectors in registers; slots (iter−1)·2 + p."""
    D, C, M = 32, 2048, 100
    seed, mu, ts, obs, _ = sched_problem(D)
    ups = [oracle.mwg_update(2, range(0, 16), sigma=s2(16) * np.eye(16)),
           oracle.mwg_update(2, range(16, 32), sigma=s2(16) * np.eye(16))]
    th0 = np.tile(mu, (C, 1))
    eng, st, h, steps = run_pair(oracle, D, C, M, ups, mu, ts, obs, seed, th0, steps=full_steps(M, 2),
                                 ll_mode=ll_mode, hist=hist)
    assert_block(eng, D)
    assert "P=2" in eng.kernel_name()
    check(oracle, eng, st, h, steps, ups, 2, full=(hist == L.HIST_FULL))


def test_three_interleaved_updates_of_every_kind(oracle):
    """D = 33: a UniformRandomWalk with pos flags and AdaptationUnifRW on coords 0, 3, 6, …, a
    dense GaussianRandomWalk on 1, 4, 7, … (reversed) and a GaussianRandomWalk with a ProductPrior
    on 2, 5, 8, …; disjoint blocks, so every prior is carried."""
    D, C, M = 33, 1024, 90
    seed, mu, ts, obs, _ = sched_problem(D, shift=3.0)
    A = np.random.default_rng(4).standard_normal((11, 11))
    ups = [oracle.mwg_update(1, range(0, D, 3), eps=[0.1] * 11, pos=[True] * 11, adapt=dict(ADAPT, k=20)),
           oracle.mwg_update(2, list(range(1, D, 3))[::-1], sigma=s2(11, f=0.5) * (A @ A.T / 11 + np.eye(11))),
           oracle.mwg_update(2, range(2, D, 3), sigma=s2(11) * np.eye(11), prior=L.PRIOR_PRODUCT,
                             factors=[(P_, 11, [(G_, 6.0, 0.5)] * 11)])]
    th0 = np.tile(mu, (C, 1))
    eng, st, h, steps = run_pair(oracle, D, C, M, ups, mu, ts, obs, seed, th0, steps=full_steps(M, 3), spl=11)
    assert_block(eng, D)
    check(oracle, eng, st, h, steps, ups, 3)


def test_overlapping_updates_evaluate_both_priors(oracle):
    """Updates sharing coordinates 10..19 (no log-prior carry: the other update moves θ_local),
    an exclusion schedule (update 2 off on iterations 20:35) and three run calls."""
    D, C, M = 30, 1024, 80
    seed, mu, ts, obs, _ = sched_problem(D, shift=2.0)
    ups = [oracle.mwg_update(2, range(0, 20), sigma=s2(20) * np.eye(20), prior=L.PRIOR_PRODUCT,
                             factors=[(P_, 20, [(N_, 2.0, 2.0)] * 20)]),
           oracle.mwg_update(1, range(10, 30), eps=[0.15] * 20, prior=L.PRIOR_STANDARD,
                             factors=[(MV_, 20, 2.0 * np.ones(20), np.eye(20) + 0.1 * np.ones((20, 20)))])]
    steps = [(s.mcmciter, s.pidx) for s in MCMCSchedule(M, 2, [(2, range(20, 36))])]
    th0 = np.tile(mu, (C, 1))
    eng, st, h, steps = run_pair(oracle, D, C, M, ups, mu, ts, obs, seed, th0, steps=steps, spl=13,
                                 calls=[(0, 50), (50, 51), (51, len(steps))])
    assert_block(eng, D)
    check(oracle, eng, st, h, steps, ups, 2)


def test_d64_two_blocks_of_32_with_a_prior(oracle):
    """D = 64 as two GaussianRandomWalk blocks of 32 (the wide kernel's NU = 32 case), one with a
    ProductPrior of Normals."""
    D, C, M = 64, 1024, 60
    seed, mu, ts, obs, _ = sched_problem(D)
    ups = [oracle.mwg_update(2, range(0, 32), sigma=s2(32) * np.eye(32), prior=L.PRIOR_PRODUCT,
                             factors=[(P_, 32, [(N_, 0.0, 4.0)] * 32)]),
           oracle.mwg_update(2, range(32, 64), sigma=s2(32) * np.eye(32))]
    th0 = np.tile(mu, (C, 1))
    eng, st, h, steps = run_pair(oracle, D, C, M, ups, mu, ts, obs, seed, th0, steps=full_steps(M, 2))
    assert_block(eng, D)
    check(oracle, eng, st, h, steps, ups, 2)


def test_dense_target_three_blocks_d40(oracle):
    """D = 40 on a dense Σ_t (the GsnSweep<true> sweeps): a diagonal Gaussian block of 16, a
    correlated Gaussian block of 16 and a UniformRandomWalk block of 8 with a ProductPrior —
    test_gpu_mwg's D = 64 schedule at a size whose compiled kernel needs no scratch."""
    D, C, M = 40, 1024, 80
    seed, mu, ts, obs = problem(D, dense_t=True)
    B = np.random.default_rng(3).standard_normal((16, 16))
    ups = [oracle.mwg_update(2, range(0, 16), sigma=0.01 * np.eye(16)),
           oracle.mwg_update(2, range(16, 32), sigma=0.002 * (B @ B.T / 16 + np.eye(16))),
           oracle.mwg_update(1, range(32, 40), eps=[0.05] * 8, prior=L.PRIOR_PRODUCT,
                             factors=[(P_, 8, [(N_, 0.0, 3.0)] * 8)])]
    eng, st, h, steps = run_pair(oracle, D, C, M, ups, mu, ts, obs, seed, np.zeros((C, D)),
                                 steps=full_steps(M, 3))
    assert_block(eng, D)
    assert "DENSE_T" in eng.kernel_name()
    check(oracle, eng, st, h, steps, ups, 3)


def test_one_update_over_a_subset(oracle):
    """P = 1 over coordinates 5..24 of D = 30: P°.θ keeps the target's μ outside them
    (set_parameters! writes the update's coordinates only)."""
    D, C, M = 30, 1024, 80
    seed, mu, ts, obs, _ = sched_problem(D)
    ups = [oracle.mwg_update(1, range(5, 25), eps=[0.08] * 20, prior=L.PRIOR_PRODUCT,
                             factors=[(P_, 20, [(LA_, 0.0, 2.0)] * 20)])]
    th0 = np.tile(mu, (C, 1))
    eng, st, h, steps = run_pair(oracle, D, C, M, ups, mu, ts, obs, seed, th0)
    assert_block(eng, D)
    check(oracle, eng, st, h, steps, ups, 1)


def test_two_blocks_on_a_user_law(oracle):
    """Two UniformRandomWalk blocks on the user logistic law (D = 20, P = 2)."""
    D, C, M, n = 20, 512, 60, 60
    rng = np.random.default_rng(13)
    X = rng.standard_normal((n, D)) / np.sqrt(D)
    beta = rng.normal(scale=0.3, size=D)
    y = (rng.uniform(size=n) < 1.0 / (1.0 + np.exp(-(X @ beta)))).astype(float)
    obs = np.column_stack([X, y])
    fn, src = oracle.user_loglik("logistic_regression")
    ups = [oracle.mwg_update(1, range(0, 10), eps=[0.3] * 10),
           oracle.mwg_update(1, range(10, 20), eps=[0.3] * 10, prior=L.PRIOR_PRODUCT,
                             factors=[(P_, 10, [(N_, 0.0, 1.0)] * 10)])]
    eng, st, h, steps = run_pair(oracle, D, C, M, ups, None, None, obs, 43, np.zeros((C, D)), user=(fn, src),
                                 steps=full_steps(M, 2))
    assert_block(eng, D)
    check(oracle, eng, st, h, steps, ups, 2)


# ---- engine lifetime: run-time modules shared per process, handles created after others -------
def two_block_engine(C, M, variant=0, seed=None):
    w = W.cfg2(8)
    eng = Engine(EngineConfig(dim=32, num_chains=C, num_mcmc_steps=M, seed=w.seed if seed is None else seed,
                              kernel_variant=variant))
    for blk in (range(0, 16), range(16, 32)):
        eng.add_gaussian_rw_update(np.array(blk), np.asarray(w.rw_sigma)[:16, :16] * 2.0)
    eng.set_gsn_target(w.mu_true, w.t_sigma, w.obs)
    eng.set_state(np.zeros((C, 32)))
    return eng


def test_schedule_kernel_then_wide_kernel_at_full_size():
    """bench_general's in-process sequence at its size (65,536 chains, P = 2): the schedule
    kernel's handle destroyed, then a handle on the wide kernel — which once hung in its first
    launch (module and code-object lifetime).  The two kernels' bits agree over
    every chain: accept streams, θ and ll."""
    C, M = 65536, 60
    steps = full_steps(M, 2)
    out = []
    for variant in (0, L.VARIANT_NO_BLOCK):
        eng = two_block_engine(C, M, variant)
        eng.run(steps)
        eng.synchronize(allow_faults=True)
        out.append((eng.kernel_name(), eng.get_state(), eng.get_history(L.H_ACCEPT, 1, M)))
        eng.close()
    assert out[0][0].startswith("mwg_rw_block_kernel<D=32") and out[1][0].startswith("mwg_wide_kernel<D=32")
    for x, y in zip(out[0][1], out[1][1]):
        assert np.array_equal(x, y)
    assert np.array_equal(out[0][2], out[1][2])


def test_handles_share_a_module_and_outlive_each_other():
    """Two handles select the same compiled schedule (one module, loaded once per process); the
    first is destroyed between the second's launches, and the second's chains still equal a
    third handle's that ran alone afterwards."""
    C, M = 4096, 40
    steps = full_steps(M, 2)
    a, b = two_block_engine(C, M), two_block_engine(C, M)
    assert a.kernel_name() == b.kernel_name() and a.kernel_name().startswith("mwg_rw_block_kernel")
    a.run(steps[:40])
    b.run(steps[:40])
    a.synchronize(allow_faults=True)
    a.close()
    b.run(steps[40:])
    b.synchronize(allow_faults=True)
    got = (b.get_state(), b.get_history(L.H_ACCEPT, 1, M))
    b.close()
    c = two_block_engine(C, M)
    c.run(steps)
    c.synchronize(allow_faults=True)
    want = (c.get_state(), c.get_history(L.H_ACCEPT, 1, M))
    c.close()
    for x, y in zip(got[0], want[0]):
        assert np.array_equal(x, y)
    assert np.array_equal(got[1], want[1])
