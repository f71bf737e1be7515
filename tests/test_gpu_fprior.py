"""The fused diagonal step with the update's separable terms compiled in (rwm_gsn_diag_kernel +
FusedUpdate, emcmc_fused.h / emcmc_fprior.h): the joint GaussianRandomWalk with a diagonal Σ or
UniformRandomWalk (positivity flags) over coords 1:D on a diagonal GsnTargetLaw, with
ProductPrior([Product(u_1 … u_D)]), StandardPrior(Product(…)), one MvNormal(μ, Σ) over all D
or ImproperPosPrior
(priors.jl:18-88), the proposal! redraw loop (updates.jl:191-196) and the log-prior carry, every
left fold continued lane to lane across the chain's LPC lanes — against the oracle
(orc_run_mwg kind 2, the restatement the schedule kernels are checked against), bit for bit:
accept streams, θ / θ° / ll histories, rolling acceptance, fault bits.  EMCMC_VARIANT_NO_FUSED_PRIOR
runs the same update on the schedule kernel with the same bits."""
import numpy as np
import pytest

from extensible_mcmc import _lib as L
from extensible_mcmc.engine import Engine, EngineConfig
from test_gpu_mwg import check, full_steps
from test_gpu_rwblock import problem, run_pair

pytestmark = pytest.mark.gpu

N_, U_, E_, G_, LN_ = L.DIST_NORMAL, L.DIST_UNIFORM, L.DIST_EXPONENTIAL, L.DIST_GAMMA, L.DIST_LOGNORMAL
B_, IG_, C_, LA_, T_ = L.DIST_BETA, L.DIST_INVERSE_GAMMA, L.DIST_CAUCHY, L.DIST_LAPLACE, L.DIST_TDIST
P_, MV_ = L.DIST_PRODUCT, L.DIST_MVNORMAL


@pytest.fixture(autouse=True)
def _gpu(require_gpu):
    pass


def s2(D, n=10, f=1.0):
    return f * (2.38 / np.sqrt(D * n)) ** 2


def assert_fused(eng, D, lpc):
    name = eng.kernel_name()
    assert name.startswith(f"rwm_gsn_diag_kernel<D={D},LPC={lpc},") and "Prior" in name, name


def normals(D, sd=3.0):
    return [(P_, D, [(N_, 0.0, sd)] * D)]


@pytest.mark.parametrize("ll_mode", [L.LL_PER_OBS, L.LL_SUFFSTAT])
@pytest.mark.parametrize("hist", [L.HIST_FULL, L.HIST_ACCEPT_ONLY])
def test_d32_product_of_normals(oracle, ll_mode, hist):
    """The VERDICT r5 shape (GaussianRandomWalk(σ²I) + ProductPrior of 32 Normals) at two lanes per
    chain: each lane's 16 logpdfs, the fold continued from lane 0 to lane 1."""
    D, C, M = 32, 2048, 120
    seed, mu, ts, obs = problem(D)
    ups = [oracle.mwg_update(2, range(D), sigma=s2(D) * np.eye(D), prior=L.PRIOR_PRODUCT, factors=normals(D))]
    eng, st, h, steps = run_pair(oracle, D, C, M, ups, mu, ts, obs, seed, np.tile(mu, (C, 1)), ll_mode=ll_mode,
                                 hist=hist)
    assert_fused(eng, D, 2)
    check(oracle, eng, st, h, steps, ups, 1, full=(hist == L.HIST_FULL))


FAMILIES = [(N_, 2.0, 1.0), (G_, 4.0, 0.5), (LN_, 0.6, 0.4), (U_, 1.75, 2.4), (E_, 0.5, 0.0), (B_, 3.0, 2.0),
            (IG_, 3.0, 4.0), (C_, 2.0, 0.7), (LA_, 2.0, 0.5), (T_, 5.0, 0.0), (N_, 1.0, 0.2), (U_, 1.9, 2.2),
            (G_, 2.0, 1.5), (LN_, 0.7, 0.1), (B_, 5.0, 1.5), (LA_, 1.8, 1.0)]


def mixed_families(n, period=16):
    """The first `period` of 16 families / parameters, repeated (the families must repeat across
    the chain's lanes): supports that make proposal! redraw (Uniform, Beta, Gamma, LogNormal,
    Exponential, InverseGamma near their edges) beside unbounded ones."""
    return [FAMILIES[i % period] for i in range(n)]


def mixed_start(n, period=16):
    """θ inside every support: 2.0, the Beta coordinates at 0.5 / 0.8."""
    th = np.full(n, 2.0)
    for i in range(n):
        if FAMILIES[i % period][0] == B_:
            th[i] = 0.5 if (i % period) == 5 else 0.8
    return th


def test_d32_mixed_families_with_redraws(oracle):
    """Ten families across the two lanes, several with bounded support around the chains: the
    redraw loop runs (a chain whose θ° leaves a Uniform / Beta support draws again, r > 0
    normals), the carry holds across launches of 13 steps."""
    D, C, M = 32, 2048, 90
    seed, mu, ts, obs = problem(D)
    mu = mixed_start(D)
    obs = mu + np.random.default_rng(3).normal(scale=0.3, size=(10, D))
    ups = [oracle.mwg_update(2, range(D), sigma=s2(D, f=4.0) * np.eye(D), prior=L.PRIOR_PRODUCT,
                             factors=[(P_, D, mixed_families(D))])]
    eng, st, h, steps = run_pair(oracle, D, C, M, ups, mu, ts, obs, seed, np.tile(mu, (C, 1)), spl=13)
    assert_fused(eng, D, 2)
    check(oracle, eng, st, h, steps, ups, 1)


@pytest.mark.parametrize("D,lpc", [(16, 2), (64, 4), (24, 1)])
def test_lanes_per_chain(oracle, D, lpc):
    """The fold over 1, 2 and 4 lanes (auto_lpc: D = 24 → 1, 16 → 2, 64 → 4), StandardPrior(Product)
    at D = 64 (no 0.0 + in front of the fold), a non-unit diagonal Σ_t at D = 24."""
    C, M = 1024, 60
    seed, mu, ts, obs = problem(D)
    prior = L.PRIOR_STANDARD if D == 64 else L.PRIOR_PRODUCT
    if D == 24:
        ts = np.diag(np.linspace(0.5, 2.0, D))
    period = D // lpc if lpc > 1 else 16
    ups = [oracle.mwg_update(2, range(D), sigma=s2(D) * np.eye(D), prior=prior,
                             factors=[(P_, D, mixed_families(D, period) if D != 64 else [(N_, 0.0, 2.0)] * D)])]
    if D != 64:
        mu = mixed_start(D, period)
        obs = mu + np.random.default_rng(4).normal(scale=0.3, size=(10, D))
    th0 = np.tile(mu, (C, 1))
    eng, st, h, steps = run_pair(oracle, D, C, M, ups, mu, ts, obs, seed, th0)
    assert_fused(eng, D, lpc)
    check(oracle, eng, st, h, steps, ups, 1)


def test_forced_one_lane_per_chain_and_the_schedule_kernel_agree():
    """lanes_per_chain = 1 at D = 32 (the whole fold on one lane) and EMCMC_VARIANT_NO_FUSED_PRIOR
    (mwg_rw_block_kernel) give the default kernel's bits over every chain."""
    D, C, M = 32, 4096, 50
    seed, mu, ts, obs = problem(D)
    out = []
    for lanes, variant in ((0, 0), (1, 0), (0, L.VARIANT_NO_FUSED_PRIOR)):
        eng = Engine(EngineConfig(dim=D, num_chains=C, num_mcmc_steps=M, seed=seed, lanes_per_chain=lanes,
                                  kernel_variant=variant))
        eng.add_gaussian_rw_update(np.arange(D), s2(D) * np.eye(D), prior=L.PRIOR_PRODUCT,
                                   prior_factors=normals(D, 1.5))
        eng.set_gsn_target(mu, ts, obs)
        eng.set_state(np.tile(mu, (C, 1)))
        eng.run(full_steps(M, 1))
        eng.synchronize(allow_faults=True)
        out.append((eng.kernel_name(), eng.get_state(), eng.get_history(L.H_ACCEPT, 1, M),
                    eng.get_history(L.H_PROPOSAL, 1, M)))
        eng.close()
    assert out[0][0].startswith("rwm_gsn_diag_kernel<D=32,LPC=2")
    assert out[1][0].startswith("rwm_gsn_diag_kernel<D=32,LPC=1")
    assert out[2][0].startswith("mwg_rw_block_kernel<D=32")
    for o in out[1:]:
        for x, y in zip(out[0][1], o[1]):
            assert np.array_equal(x, y)
        assert np.array_equal(out[0][2], o[2]) and np.array_equal(out[0][3], o[3])


@pytest.mark.parametrize("D,lpc,prior", [(32, 2, L.PRIOR_PRODUCT), (64, 4, L.PRIOR_IMPROPER_POS),
                                         (24, 1, L.PRIOR_IMPROPER)])
def test_uniform_random_walk_with_pos_flags(oracle, D, lpc, prior):
    """UniformRandomWalk(ϵ_j) with positivity flags repeating across the lanes: θ·e^U, the two
    transition-density sums (−log 2ϵ_j − log θ°_j, 0.0 off the flags) folded lane to lane, with a
    Product of Gammas (redraws where a flag-less coordinate's θ° < 0), ImproperPosPrior or none."""
    C, M = 2048, 80
    seed, mu, ts, obs = problem(D, shift=3.0)
    dpl = D // lpc
    pos = [(j % dpl) % 3 != 1 for j in range(D)]
    eps = [0.04 + 0.003 * (j % dpl) for j in range(D)]
    fac = [(P_, D, [(G_, 6.0, 0.5)] * D)] if prior == L.PRIOR_PRODUCT else None
    ups = [oracle.mwg_update(1, range(D), eps=eps, pos=pos, prior=prior, factors=fac)]
    eng, st, h, steps = run_pair(oracle, D, C, M, ups, mu, ts, obs, seed, np.tile(mu, (C, 1)), spl=11)
    name = eng.kernel_name()
    assert name.startswith(f"rwm_gsn_diag_kernel<D={D},LPC={lpc},") and "UniformRandomWalk" in name, name
    check(oracle, eng, st, h, steps, ups, 1)


def test_gaussian_random_walk_with_improper_pos_prior(oracle):
    """GaussianRandomWalk (no flags) with ImproperPosPrior: −Σ log θ_j folded lane to lane; θ° ≤ 0
    makes the prior NaN / +Inf (log_real), which the ratio carries as the oracle does."""
    D, C, M = 32, 2048, 80
    seed, mu, ts, obs = problem(D, shift=2.0)
    ups = [oracle.mwg_update(2, range(D), sigma=s2(D) * np.eye(D), prior=L.PRIOR_IMPROPER_POS)]
    eng, st, h, steps = run_pair(oracle, D, C, M, ups, mu, ts, obs, seed, np.tile(mu, (C, 1)))
    assert_fused(eng, D, 2)
    check(oracle, eng, st, h, steps, ups, 1)


def dense_cov(D, seed=9):
    B = np.random.default_rng(seed).standard_normal((D, D))
    return B @ B.T / D + 0.5 * np.eye(D)


@pytest.mark.parametrize("D,lanes,prior,ll_mode", [(32, 0, L.PRIOR_STANDARD, L.LL_SUFFSTAT),
                                                   (32, 1, L.PRIOR_PRODUCT, L.LL_PER_OBS),
                                                   (16, 0, L.PRIOR_PRODUCT, L.LL_PER_OBS),
                                                   (32, 4, L.PRIOR_PRODUCT, L.LL_PER_OBS),
                                                   (64, 0, L.PRIOR_STANDARD, L.LL_PER_OBS)])
def test_mvnormal_prior(oracle, D, lanes, prior, ll_mode):
    """StandardPrior(MvNormal(μ0, Σ0)) / ProductPrior([MvNormal]) with Σ0 dense: y = L⁻¹(θ − μ0) row
    by row from the scalar-loaded factor, lane 1's rows continuing from lane 0's y's and sum of
    squares (two lanes per chain, auto at D = 16 and 32), one lane forced at D = 32; four lanes
    (forced at D = 32, auto at D = 64): lane k's rows take the earlier lanes' y's as quad
    broadcasts, one column at a time."""
    C, M = 2048, 100
    seed, mu, ts, obs = problem(D)
    ups = [oracle.mwg_update(2, range(D), sigma=s2(D) * np.eye(D), prior=prior,
                             factors=[(MV_, D, 0.3 * np.ones(D), dense_cov(D))])]
    eng, st, h, steps = run_pair(oracle, D, C, M, ups, mu, ts, obs, seed, np.tile(mu, (C, 1)), ll_mode=ll_mode,
                                 lanes=lanes)
    assert_fused(eng, D, lanes or (4 if D == 64 else 2))
    assert "MvNormal" in eng.kernel_name()
    check(oracle, eng, st, h, steps, ups, 1)


@pytest.mark.parametrize("D,lanes,factors", [(48, 0, "mvn"), (48, 2, "normals")])
def test_shapes_the_fused_kernel_declines(oracle, D, lanes, factors):
    """Shapes that run elsewhere with the oracle's bits: D = 48 on three lanes (auto) or two lanes
    of 24 (forced) — the likelihood's canonical sum (blocks of 8 under a pairwise tree) does not
    split into one subtree per lane."""
    C, M = 1024, 40
    seed, mu, ts, obs = problem(D)
    fac = [(MV_, D, 0.3 * np.ones(D), dense_cov(D))] if factors == "mvn" else normals(D)
    ups = [oracle.mwg_update(2, range(D), sigma=s2(D) * np.eye(D), prior=L.PRIOR_STANDARD, factors=fac)]
    eng, st, h, steps = run_pair(oracle, D, C, M, ups, mu, ts, obs, seed, np.tile(mu, (C, 1)), lanes=lanes)
    assert not eng.kernel_name().startswith("rwm_gsn_diag_kernel"), eng.kernel_name()
    check(oracle, eng, st, h, steps, ups, 1)


@pytest.mark.parametrize("D,lanes,pos,prior", [(32, 0, "all", L.PRIOR_IMPROPER), (32, 0, "odd", L.PRIOR_IMPROPER_POS),
                                               (64, 0, "all", L.PRIOR_IMPROPER), (24, 0, "all", L.PRIOR_IMPROPER),
                                               (16, 0, "all", L.PRIOR_PRODUCT), (32, 2, "odd", L.PRIOR_PRODUCT)])
def test_gaussian_random_walk_with_pos_round_trips(oracle, D, lanes, pos, prior):
    """GaussianRandomWalk with positivity flags on the fused kernel: θ° = exp(log θ + L z) where
    flagged, both densities through the reference's exp/log round trips (θ°₃ stored on accept,
    the prior at θ°₃ and θ₃, no carry), −Σ log θ₁ folded over the flagged coordinates lane to lane;
    with a Product of Gammas the flag-less coordinates leave the support and redraw, and each
    redraw round-trips the step's local θ first (cumulative over redraws)."""
    C, M = 2048, 60
    seed, mu, ts, obs = problem(D, shift=3.0)
    lpc = lanes or {16: 2, 24: 1, 32: 2, 64: 4}[D]
    dpl = D // lpc
    flags = [True] * D if pos == "all" else [(j % dpl) % 2 == 1 for j in range(D)]
    th0 = np.tile(mu, (C, 1))
    fac = None
    if prior == L.PRIOR_PRODUCT:  # Gammas where flagged, Uniform(2, 4) elsewhere: those redraw
        fac = [(P_, D, [(G_, 6.0, 0.5) if flags[j] else (U_, 2.0, 4.0) for j in range(D)])]
        th0 = np.full((C, D), 3.0)
    f = 2.0 if prior == L.PRIOR_PRODUCT else 0.05
    ups = [oracle.mwg_update(2, range(D), sigma=s2(D, f=f) * np.eye(D), pos=flags, prior=prior, factors=fac)]
    eng, st, h, steps = run_pair(oracle, D, C, M, ups, mu, ts, obs, seed, th0, lanes=lanes, spl=13)
    assert_fused(eng, D, lpc)
    check(oracle, eng, st, h, steps, ups, 1)


@pytest.mark.parametrize("shape", ["gauss_pos", "mvnormal"])
def test_accept_only_suffstat_launch_cuts_non_unit_target(oracle, shape):
    """The new shapes under the other modes: accept-only histories, the sufficient-statistic
    likelihood, a non-unit diagonal Σ_t, launches of 7 steps across three run calls (the round
    trips carry nothing; the MvNormal prior's carry is re-evaluated at each launch's start)."""
    D, C, M = 32, 2048, 70
    seed, mu, ts, obs = problem(D, shift=3.0)
    ts = np.diag(np.linspace(0.5, 2.0, D))
    if shape == "gauss_pos":
        ups = [oracle.mwg_update(2, range(D), sigma=s2(D, f=0.05) * np.eye(D), pos=[j % 4 != 0 for j in range(D)],
                                 prior=L.PRIOR_IMPROPER_POS)]
    else:
        ups = [oracle.mwg_update(2, range(D), sigma=s2(D) * np.eye(D), prior=L.PRIOR_STANDARD,
                                 factors=[(MV_, D, 3.0 * np.ones(D), dense_cov(D, seed=4))])]
    eng, st, h, steps = run_pair(oracle, D, C, M, ups, mu, ts, obs, seed, np.tile(mu, (C, 1)), ll_mode=L.LL_SUFFSTAT,
                                 hist=L.HIST_ACCEPT_ONLY, spl=7, calls=[(0, 17), (17, 40), (40, M)])
    assert_fused(eng, D, 2)
    assert "UNIT_T" not in eng.kernel_name()
    check(oracle, eng, st, h, steps, ups, 1, full=False)


def test_gaussian_round_trips_fused_and_schedule_kernel_agree_at_scale():
    """GaussianRandomWalk with every other coordinate flagged at D = 32 over 16,384 chains: the
    fused kernel (two lanes per chain) and the schedule path (EMCMC_VARIANT_NO_FUSED_PRIOR; with
    ImproperPosPrior the schedule kernel needs scratch, so the wide kernel runs it) give the same
    θ, ll and θ° / accept histories on every chain."""
    D, C, M = 32, 16384, 40
    seed, mu, ts, obs = problem(D, shift=3.0)
    out = []
    for variant in (0, L.VARIANT_NO_FUSED_PRIOR):
        eng = Engine(EngineConfig(dim=D, num_chains=C, num_mcmc_steps=M, seed=seed, kernel_variant=variant))
        eng.add_gaussian_rw_update(np.arange(D), s2(D, f=0.05) * np.eye(D), pos=[j % 2 for j in range(D)],
                                   prior=L.PRIOR_IMPROPER_POS)
        eng.set_gsn_target(mu, ts, obs)
        eng.set_state(np.tile(mu, (C, 1)))
        eng.run(full_steps(M, 1))
        eng.synchronize(allow_faults=True)
        out.append((eng.kernel_name(), eng.get_state(), eng.get_history(L.H_ACCEPT, 1, M),
                    eng.get_history(L.H_PROPOSAL, 1, M), eng.get_history(L.H_STATE, 1, M)))
        eng.close()
    assert out[0][0].startswith("rwm_gsn_diag_kernel<D=32,LPC=2"), out[0][0]
    assert out[1][0].startswith(("mwg_rw_block_kernel<D=32", "mwg_wide_kernel<D=32")), out[1][0]
    for x, y in zip(out[0][1], out[1][1]):
        assert np.array_equal(x, y)
    for k in (2, 3, 4):
        assert np.array_equal(out[0][k], out[1][k])


@pytest.mark.parametrize("kind", ["gaussian", "uniform"])
def test_mvnormal_prior_with_pos_flags(oracle, kind):
    """An MvNormal prior beside positivity flags: with GaussianRandomWalk's round trips it is
    evaluated at θ°₃ and θ₃ (no carry); with UniformRandomWalk it is carried and its −Inf-free
    values drive no redraws (an MvNormal has full support)."""
    D, C, M = 32, 2048, 60
    seed, mu, ts, obs = problem(D, shift=3.0)
    flags = [(j % 16) % 3 != 2 for j in range(D)]
    fac = [(MV_, D, 3.0 * np.ones(D), dense_cov(D, seed=7))]
    if kind == "gaussian":
        ups = [oracle.mwg_update(2, range(D), sigma=s2(D, f=0.05) * np.eye(D), pos=flags, prior=L.PRIOR_STANDARD,
                                 factors=fac)]
    else:
        ups = [oracle.mwg_update(1, range(D), eps=[0.03 + 0.002 * (j % 16) for j in range(D)], pos=flags,
                                 prior=L.PRIOR_PRODUCT, factors=fac)]
    eng, st, h, steps = run_pair(oracle, D, C, M, ups, mu, ts, obs, seed, np.tile(mu, (C, 1)), spl=9)
    name = eng.kernel_name()
    assert name.startswith("rwm_gsn_diag_kernel<D=32,LPC=2,") and "MvNormal" in name, name
    check(oracle, eng, st, h, steps, ups, 1)
