"""Row f1 on the GPU (BASELINE cfg 4): mix_gsn_kernel / mix_res_kernel + mix_readjust_kernel
against the oracle (orc_run_mix), bit for bit — accept stream, state, ll,
rolling acceptance, GenericChainStats mean/cov, each chain's Σ_B factor after
Haario readjusts, fault bits — through the C ABI."""
import numpy as np
import pytest

from extensible_mcmc import _lib as L
from extensible_mcmc import workloads as W
from extensible_mcmc.engine import Engine, EngineConfig

pytestmark = pytest.mark.gpu


@pytest.fixture(autouse=True)
def _gpu(require_gpu):
    pass


def _problem(D, dense=False):
    w = W.cfg2(8, D=D)
    obs = np.asarray(w.obs)[:, :D]
    ts = np.asarray(w.t_sigma)[:D, :D]
    mu = np.asarray(w.mu_true)[:D]
    sa = np.asarray(w.rw_sigma)[:D, :D]
    if dense:
        rng = np.random.default_rng(7)
        A = rng.standard_normal((D, D))
        ts = A @ A.T / D + np.eye(D)
        sa = 0.02 * (np.eye(D) + 0.3 * np.ones((D, D)))
    return w.seed, mu, ts, obs, sa


def _engine(D, C, M, seed, mu, ts, obs, sa, sb, lam, k, ll_mode, hist, spl=0, moments_only=False, variant=0):
    eng = Engine(EngineConfig(dim=D, num_chains=C, num_mcmc_steps=M, seed=seed, history_mode=hist,
                              steps_per_launch=spl, chain_moments=moments_only, kernel_variant=variant))
    if moments_only:
        eng.add_gaussian_rw_update(range(D), sa)
    else:
        eng.add_gaussian_rw_mix_update(range(D), sa, sb, lam=lam, haario_k=k or None)
    eng.set_gsn_target(mu, ts, obs, ll_mode=ll_mode)
    eng.set_state(np.zeros((C, D)))
    return eng


def _check(eng, st, hists, iters, full, mix=True):
    eng.synchronize(allow_faults=True)
    th, ll = eng.get_state()
    assert np.array_equal(th, st.theta)
    assert np.array_equal(ll, st.ll)
    ra, nacc = eng.get_chain_stats()
    assert np.array_equal(ra[0], st.ra)
    assert np.array_equal(nacc[0], st.nacc)
    assert np.array_equal(eng.get_faults(), st.faults)
    mean, cov = eng.get_chain_moments()
    assert np.array_equal(mean, st.mean)
    assert np.array_equal(cov, st.cov)
    if mix:
        Lb, M = eng.get_mix_state(1)
        assert np.array_equal(Lb, st.LB)
        assert M == st.M
    acc = np.concatenate([h["acc"] for h in hists])
    i0, n = iters[0], iters[-1] - iters[0] + 1
    rows = np.asarray(iters) - i0
    assert np.array_equal(eng.get_history(L.H_ACCEPT, i0, n)[rows, 0], acc)
    if full:
        for which, key in ((L.H_STATE, "theta"), (L.H_PROPOSAL, "prop"), (L.H_LL, "ll")):
            got = eng.get_history(which, i0, n)[rows, 0]
            assert np.array_equal(got, np.concatenate([h[key] for h in hists])), key


CASES = [  # D, lam, k, ll_mode, hist, dense
    (2, 0.5, 0, L.LL_PER_OBS, L.HIST_FULL, False),
    (4, 0.3, 25, L.LL_SUFFSTAT, L.HIST_FULL, True),
    (8, 0.5, 50, L.LL_PER_OBS, L.HIST_ACCEPT_ONLY, False),
    (8, 1.0, 40, L.LL_SUFFSTAT, L.HIST_FULL, True),
    (16, 0.5, 40, L.LL_SUFFSTAT, L.HIST_FULL, False),
    (32, 0.5, 100, L.LL_PER_OBS, L.HIST_FULL, False),
    (32, 0.25, 60, L.LL_SUFFSTAT, L.HIST_ACCEPT_ONLY, False),
]


@pytest.mark.parametrize("D,lam,k,ll_mode,hist,dense", CASES)
def test_mix_haario_matches_oracle(oracle, D, lam, k, ll_mode, hist, dense):
    """random_walk.jl:193-232, adaptation.jl:372-426, chain_statistics.jl:41-66."""
    seed, mu, ts, obs, sa = _problem(D, dense)
    sb = 0.5 * sa
    C, M = (1024 if D >= 16 else 777), 300
    eng = _engine(D, C, M, seed, mu, ts, obs, sa, sb, lam, k, ll_mode, hist, variant=L.VARIANT_MIX_STREAM)
    eng.run_iters(1, M)
    assert "mix_gsn_kernel<D=%d" % D in eng.kernel_name()
    st = oracle.MixState(np.zeros((C, D)), sigma_b=sb)
    h = oracle.run_mix(st, seed=seed, sigma_a=sa, t_sigma=ts, obs=obs, iter0=1, nsteps=M, lam=lam, haario_k=k,
                       ll_mode=ll_mode, nthreads=8)
    _check(eng, st, [h], list(range(1, M + 1)), hist == L.HIST_FULL)


RES_CASES = [  # lam, k, ll_mode, hist, unit Σ_t, nobs, C
    (0.5, 100, L.LL_PER_OBS, L.HIST_FULL, True, 10, 1024),
    (0.25, 60, L.LL_SUFFSTAT, L.HIST_ACCEPT_ONLY, True, 10, 1024),
    (0.5, 50, L.LL_PER_OBS, L.HIST_ACCEPT_ONLY, False, 37, 528),
    (0.7, 70, L.LL_SUFFSTAT, L.HIST_FULL, False, 10, 1040),
    (1.0, 40, L.LL_PER_OBS, L.HIST_FULL, False, 16, 1024),
]


@pytest.mark.parametrize("lam,k,ll_mode,hist,unit,nobs,C", RES_CASES)
def test_mix_res_kernel_matches_oracle(oracle, lam, k, ll_mode, hist, unit, nobs, C):
    """mix_res_kernel (L_B resident in registers, 16 lanes per chain), the default
    for D = 32 with diagonal Σ_A / Σ_t: the same bits as the oracle and as
    mix_gsn_kernel — identity or general diagonal Σ_t, 10 / 16 / 37 observations
    (one or three rounds of 16 observation lanes), FULL and ACCEPT_ONLY, Haario
    readjusts in the run (random_walk.jl:193-232, adaptation.jl:399-426)."""
    D, M = 32, 240
    w = W.cfg2(8, D=D, nobs=nobs)
    mu, obs, sa = np.asarray(w.mu_true), np.asarray(w.obs), np.asarray(w.rw_sigma)
    ts = np.eye(D) if unit else np.diag(0.5 + np.random.default_rng(3).random(D))
    sb = 0.5 * sa
    eng = _engine(D, C, M, w.seed, mu, ts, obs, sa, sb, lam, k, ll_mode, hist)
    eng.run_iters(1, M)
    assert "mix_res_kernel<D=32" in eng.kernel_name() and ("UNIT_T" in eng.kernel_name()) == unit
    st = oracle.MixState(np.zeros((C, D)), sigma_b=sb)
    h = oracle.run_mix(st, seed=w.seed, sigma_a=sa, t_sigma=ts, obs=obs, iter0=1, nsteps=M, lam=lam, haario_k=k,
                       ll_mode=ll_mode, nthreads=8)
    _check(eng, st, [h], list(range(1, M + 1)), hist == L.HIST_FULL)


def test_mix_res_kernel_falls_back_when_chains_do_not_fill_blocks(oracle):
    """C % 16 != 0: the mixture runs on mix_gsn_kernel (one lane per chain), same bits."""
    D, C, M = 32, 1000, 60
    seed, mu, ts, obs, sa = _problem(D)
    eng = _engine(D, C, M, seed, mu, ts, obs, sa, 0.5 * sa, 0.5, 30, L.LL_PER_OBS, L.HIST_FULL)
    eng.run_iters(1, M)
    assert "mix_gsn_kernel<D=32" in eng.kernel_name()
    st = oracle.MixState(np.zeros((C, D)), sigma_b=0.5 * sa)
    h = oracle.run_mix(st, seed=seed, sigma_a=sa, t_sigma=ts, obs=obs, iter0=1, nsteps=M, lam=0.5, haario_k=30,
                       nthreads=8)
    _check(eng, st, [h], list(range(1, M + 1)), True)


def test_split_calls_launch_cuts_and_gap(oracle):
    """Three emcmc_run calls, 7-step launches cut again at every readjust (k = 30),
    and a schedule gap (update excluded on iterations 51:60): rolling_ar restarts
    from 0.0 after the gap, N and M count steps that ran."""
    D, C, M, k = 8, 500, 130, 30
    seed, mu, ts, obs, sa = _problem(D)
    sb = sa.copy()
    eng = _engine(D, C, M, seed, mu, ts, obs, sa, sb, 0.5, k, L.LL_PER_OBS, L.HIST_FULL, spl=7)
    iters = list(range(1, 51)) + list(range(61, 131))
    for a, b in ((0, 33), (33, 80), (80, len(iters))):
        eng.run([(i, 1) for i in iters[a:b]])
    st = oracle.MixState(np.zeros((C, D)), sigma_b=sb)
    kw = dict(seed=seed, sigma_a=sa, t_sigma=ts, obs=obs, lam=0.5, haario_k=k, nthreads=8)
    hs = [oracle.run_mix(st, iter0=1, nsteps=50, **kw), oracle.run_mix(st, iter0=61, nsteps=70, **kw)]
    _check(eng, st, hs, iters, True)


def test_posdef_failure_sets_fault_and_keeps_factor(oracle):
    """Readjust after 3 steps at D = 8: 2.38²/D·cov has rank ≤ 4; the chains whose
    Cholesky fails raise EMCMC_FAULT_POSDEF (the reference: PosDefException) and
    keep their Σ_B factor; emcmc_synchronize reports EMCMC_CHAIN_FAULT."""
    D, C = 8, 256
    seed, mu, ts, obs, sa = _problem(D)
    eng = _engine(D, C, 20, seed, mu, ts, obs, sa, sa, 0.5, 3, L.LL_PER_OBS, L.HIST_FULL)
    eng.run_iters(1, 3)
    with pytest.raises(L.EMCMCError) as e:
        eng.synchronize()
    assert e.value.status == L.CHAIN_FAULT
    st = oracle.MixState(np.zeros((C, D)), sigma_b=sa)
    h = oracle.run_mix(st, seed=seed, sigma_a=sa, t_sigma=ts, obs=obs, iter0=1, nsteps=3, haario_k=3)
    assert ((st.faults & L.FAULT_POSDEF) != 0).sum() >= C // 2
    _check(eng, st, [h], [1, 2, 3], True)


@pytest.mark.parametrize("D", [8, 32])
def test_chain_moments_flag_on_plain_gaussian_rw(oracle, D):
    """emcmc_config.chain_moments with GaussianRandomWalk: the fused path's bits
    (orc_run_gsn) plus GenericChainStats mean/cov (orc_run_mix, mix off)."""
    seed, mu, ts, obs, sa = _problem(D)
    C, M = 1024, 200
    eng = _engine(D, C, M, seed, mu, ts, obs, sa, None, 0.0, 0, L.LL_SUFFSTAT, L.HIST_FULL, moments_only=True)
    eng.run_iters(1, M)
    assert "GSN_MOMENTS" in eng.kernel_name()
    st = oracle.MixState(np.zeros((C, D)))
    h = oracle.run_mix(st, seed=seed, sigma_a=sa, t_sigma=ts, obs=obs, iter0=1, nsteps=M, mix=False, ll_mode=1,
                       nthreads=8)
    so = oracle.OracleState(np.zeros((C, D)))
    ho = oracle.run_gsn(so, seed=seed, rw_sigma=sa, t_sigma=ts, obs=obs, iter0=1, nsteps=M, ll_mode=1, nthreads=8)
    assert np.array_equal(h["acc"], ho["acc"])
    _check(eng, st, [h], list(range(1, M + 1)), True, mix=False)


def test_shapes_outside_the_fused_kernels_run_on_the_general_kernel():
    """GaussianRandomWalkMix beside another update, and a dense Σ at D = 32, leave the
    fused cfg 4 kernels for the general schedule kernel (tests/test_gpu_mix_general.py
    checks their results); the fused kernels keep the shapes they instantiate."""
    seed, mu, ts, obs, sa = _problem(4)
    eng = Engine(EngineConfig(dim=4, num_chains=64, num_mcmc_steps=10, seed=seed))
    eng.add_gaussian_rw_mix_update([0, 1], sa[:2, :2], sa[:2, :2])
    eng.add_gaussian_rw_update([2, 3], sa[:2, :2])
    eng.set_gsn_target(mu, ts, obs)
    assert eng.kernel_name().startswith("mwg_gsn_kernel<D=4")
    eng.close()
    seed, mu, ts, obs, sa = _problem(32, dense=True)
    eng = Engine(EngineConfig(dim=32, num_chains=64, num_mcmc_steps=10, seed=seed))
    eng.add_gaussian_rw_mix_update(range(32), sa, sa)
    eng.set_gsn_target(mu, ts, obs)
    assert eng.kernel_name().startswith("mix_chol_kernel<D=32")  # round 4: dense Σ at D = 16 / 32 fused
    eng.close()
    eng = Engine(EngineConfig(dim=32, num_chains=64, num_mcmc_steps=10, seed=seed,
                              kernel_variant=L.VARIANT_NO_MIX_CHOL))
    eng.add_gaussian_rw_mix_update(range(32), sa, sa)
    eng.set_gsn_target(mu, ts, obs)
    assert eng.kernel_name().startswith("mwg_wide_kernel<D=32")
    eng.close()


@pytest.mark.parametrize("hist", [L.HIST_FULL, L.HIST_ACCEPT_ONLY])
def test_cfg4_shape_moments_match_oracle_on_sampled_chains(oracle, hist):
    """The cfg 4 shape (131,072 chains, D = 32): the moments kernel's grid is
    far larger than the chip, so tiles of one chain run at different times —
    every tile must see the launch's input means (regression: off-diagonal
    tiles read means already advanced by the diagonal tiles of the same chain).
    Sampled chains are replayed on the oracle through two readjusts."""
    D, C, M, k = 32, 131072, 60, 20
    w = W.cfg4(C, k=k)
    eng = _engine(D, C, M, w.seed, w.mu_true, w.t_sigma, w.obs, w.rw_sigma, w.sigma_b, w.lam, k, L.LL_PER_OBS, hist,
                  spl=20)
    eng.run_iters(1, 10)
    eng.run_iters(11, M - 10)
    eng.synchronize(allow_faults=True)
    th, ll = eng.get_state()
    mean, cov = eng.get_chain_moments()
    Lb, _ = eng.get_mix_state(1)
    acc = eng.get_history(L.H_ACCEPT, 1, M)[:, 0]
    faults = eng.get_faults()
    picks = [0, 1, 4095, 70001, C - 1]
    for c in picks:
        st = oracle.MixState(np.zeros((1, D)), sigma_b=w.sigma_b)
        h = oracle.run_mix(st, seed=w.seed, sigma_a=w.rw_sigma, t_sigma=w.t_sigma, obs=w.obs, iter0=1, nsteps=M,
                           lam=w.lam, haario_k=k, chain0=c)
        assert np.array_equal(acc[:, c], h["acc"][:, 0]), c
        assert np.array_equal(th[c], st.theta[0]) and ll[c] == st.ll[0], c
        assert np.array_equal(mean[c], st.mean[0]), c
        assert np.array_equal(cov[c], st.cov[0]), c
        assert np.array_equal(Lb[c], st.LB[0]), c
        assert faults[c] == st.faults[0], c


def test_cfg4_every_chain_through_two_readjusts(oracle):
    """The BASELINE cfg 4 shape as bench.py runs it (131,072 chains, D = 32, k = 200,
    one launch group per readjust period, full histories) over 400 iterations — two
    Haario readjusts — with EVERY chain compared bit for bit against orc_run_mix in its
    accept-only mode: the accept stream (run.jl:268-281), θ, ll, rolling acceptance,
    accept count, GenericChainStats mean/cov (chain_statistics.jl:41-66), each chain's
    Σ_B factor L_B after the readjusts (adaptation.jl:406-426) and the PosDef fault bits."""
    import os

    D, C, M, k = 32, 131072, 400, 200
    w = W.cfg4(C, k=k)
    eng = _engine(D, C, M, w.seed, w.mu_true, w.t_sigma, w.obs, w.rw_sigma, w.sigma_b, w.lam, k, L.LL_PER_OBS,
                  L.HIST_FULL, spl=k)
    eng.run_iters(1, M)
    eng.synchronize(allow_faults=True)
    kname = eng.kernel_name()
    st = oracle.MixState(np.zeros((C, D)), sigma_b=w.sigma_b)
    threads = max(1, min(16, int(os.environ.get("OMP_NUM_THREADS", "0") or 0) or (os.cpu_count() or 1)))
    h = oracle.run_mix(st, seed=w.seed, sigma_a=w.rw_sigma, t_sigma=w.t_sigma, obs=w.obs, iter0=1, nsteps=M,
                       lam=w.lam, haario_k=k, accept_only=True, nthreads=threads)
    bad = oracle.accept_mismatch_chains(eng.get_history_bits(1, M)[:, 0], oracle.pack_accept(h["acc"]), C)
    assert bad.size == 0, f"{kname}: {bad.size} of {C} accept streams differ (first: {bad[:8]})"
    th, ll = eng.get_state()
    assert np.array_equal(th, st.theta) and np.array_equal(ll, st.ll)
    ra, nacc = eng.get_chain_stats()
    assert np.array_equal(ra[0], st.ra) and np.array_equal(nacc[0], st.nacc)
    assert np.array_equal(eng.get_faults(), st.faults)
    mean, cov = eng.get_chain_moments()
    assert np.array_equal(mean, st.mean)
    assert np.array_equal(cov, st.cov)
    Lb, Mr = eng.get_mix_state(1)
    assert Mr == st.M == M % k  # Haario M counts steps since the last readjust
    assert np.array_equal(Lb, st.LB)
    eng.close()


def _flam(lam, N, it):
    """A custom HaarioTypeAdaptation fλ(λ, N, mcmc_iter) (adaptation.jl:425)."""
    return 0.5 + 0.4 * np.sin(it / 37.0) * (N % 5) / 4.0


def test_custom_flambda_matches_oracle(oracle):
    """fλ called on the host at every readjust (emcmc_set_mix_lambda_fn): λ changes
    every k = 40 steps; the oracle is run in readjust-sized pieces with the same
    fλ applied to (λ, N, iter) between them."""
    D, C, M, k = 8, 640, 240, 40
    seed, mu, ts, obs, sa = _problem(D)
    sb = 0.5 * sa
    eng = _engine(D, C, M, seed, mu, ts, obs, sa, sb, 0.5, k, L.LL_PER_OBS, L.HIST_FULL)
    eng.set_mix_lambda_fn(1, _flam)
    eng.run_iters(1, M)
    st = oracle.MixState(np.zeros((C, D)), sigma_b=sb)
    lam, hs = 0.5, []
    for it0 in range(1, M + 1, k):
        hs.append(oracle.run_mix(st, seed=seed, sigma_a=sa, t_sigma=ts, obs=obs, iter0=it0, nsteps=k, lam=lam,
                                 haario_k=k, nthreads=8))
        lam = _flam(lam, st.N, it0 + k - 1)  # rw.λ = fλ(rw.λ, adpt.N, mcmc_iter)
    _check(eng, st, hs, list(range(1, M + 1)), True)
    assert eng.get_mix_lambda(1) == lam


def test_custom_flambda_through_the_api(oracle):
    """HaarioTypeAdaptation(state; f = fλ) through MCMC / run: rw.λ is the adapted λ."""
    from extensible_mcmc import (MCMC, GaussianRandomWalkMix, GsnTargetLaw, HaarioTypeAdaptation, MI355XBackend,
                                 RandomWalkUpdate, run)
    D, C, M, k = 4, 256, 160, 40
    seed, mu, ts, obs, sa = _problem(D)
    sb = 0.5 * sa
    rw = GaussianRandomWalkMix(sa, sb, 0.5)
    mcmc = MCMC([RandomWalkUpdate(rw, list(range(1, D + 1)),
                                  adpt=HaarioTypeAdaptation(np.zeros(D), adapt_every_k_steps=k, f=_flam))],
                backend=MI355XBackend(num_chains=C, seed=seed))
    ws, _ = run(mcmc, M, dict(P=GsnTargetLaw(mu, ts), obs=obs), np.zeros(D))
    st = oracle.MixState(np.zeros((C, D)), sigma_b=sb)
    lam = 0.5
    for it0 in range(1, M + 1, k):
        oracle.run_mix(st, seed=seed, sigma_a=sa, t_sigma=ts, obs=obs, iter0=it0, nsteps=k, lam=lam, haario_k=k,
                       nthreads=8, history=False)
        lam = _flam(lam, st.N, it0 + k - 1)
    assert np.array_equal(ws.state, st.theta)
    assert rw.lam == lam
