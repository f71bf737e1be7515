"""Headline workload at full size (BASELINE cfg 2: 65,536 chains × 1,000
iterations, D = 32, full histories in HBM).  Every chain's accept stream and
final state are replayed on the oracle in its accept-only mode (6.6e7
chain-steps, a few seconds on the box's 16 cores); a random sample of chains is
also compared on the full θ / ll histories; size-independent properties
(first-step auto-accept, acceptance band, analytic posterior) on top."""
import os

import numpy as np
import pytest

from extensible_mcmc import _lib as L
from extensible_mcmc import rhat_from_moments
from extensible_mcmc import workloads as W

from helpers import run_engine

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def full_run(require_gpu):
    w = W.cfg2(65536)
    e = run_engine(w, 65536, 1000, fetch=False)
    return w, e


def test_sampled_chains_bitwise(oracle, full_run):
    w, e = full_run
    eng = e["engine"]
    rng = np.random.default_rng(11)
    picks = np.sort(rng.choice(65536, 24, replace=False))
    acc_all = eng.get_history(L.H_ACCEPT, 1, 1000)[:, 0]
    for c in picks:
        st = oracle.OracleState(np.zeros((1, 32)))
        h = oracle.run_gsn(st, seed=w.seed, rw_sigma=w.rw_sigma, t_sigma=w.t_sigma, obs=w.obs, iter0=1,
                           nsteps=1000, chain0=int(c))
        assert np.array_equal(acc_all[:, c], h["acc"][:, 0])
        th = eng.get_history_chains(L.H_STATE, 1, 1000, int(c), 1)[:, 0, 0]
        assert np.array_equal(th, h["theta"][:, 0])
        ll = eng.get_history_chains(L.H_LL, 1, 1000, int(c), 1)[:, 0, 0]
        assert np.array_equal(ll, h["ll"][:, 0])
        assert np.array_equal(e["theta"][c], st.theta[0])


def _threads():
    return max(1, min(16, int(os.environ.get("OMP_NUM_THREADS", "0") or 0) or (os.cpu_count() or 1)))


def test_every_chain_accept_stream_and_state_bitwise(oracle, full_run):
    """north_star's claim at the BASELINE cfg 2 shape: all 65,536 accept/reject streams
    over 1,000 iterations (run.jl:268-281) plus each chain's final θ, ll, rolling
    acceptance and accept count, bit for bit."""
    w, e = full_run
    eng = e["engine"]
    st = oracle.OracleState(np.zeros((65536, 32)))
    h = oracle.run_gsn(st, seed=w.seed, rw_sigma=w.rw_sigma, t_sigma=w.t_sigma, obs=w.obs, iter0=1, nsteps=1000,
                       accept_only=True, nthreads=_threads())
    got = eng.get_history_bits(1, 1000)[:, 0]
    bad = oracle.accept_mismatch_chains(got, oracle.pack_accept(h["acc"]), 65536)
    assert bad.size == 0, f"{bad.size} of 65536 chains' accept streams differ (first: {bad[:8]})"
    bad_th = np.flatnonzero((e["theta"] != st.theta).any(axis=1) | (e["ll"] != st.ll))
    assert bad_th.size == 0, f"{bad_th.size} chains' final θ/ll differ (first: {bad_th[:8]})"
    assert np.array_equal(e["ra"], st.ra)
    assert np.array_equal(e["nacc"], st.nacc.astype(e["nacc"].dtype))
    assert np.array_equal(e["faults"], st.faults)


def test_acceptance_and_first_step(full_run):
    w, e = full_run
    acc = e["engine"].get_history(L.H_ACCEPT, 1, 1000)[:, 0]
    assert acc[0].all()  # ll = −Inf before step 1 ⇒ always accept (workspaces.jl:425, run.jl:109)
    rate = acc[200:].mean()
    assert 0.20 < rate < 0.30, rate  # σ = 2.38/√(D·n): optimal-scaling acceptance ≈ 0.23–0.26
    assert e["nacc"].sum() == acc.sum()
    assert (e["faults"] == 0).all()


def test_posterior_matches_analytic(require_gpu):
    """ImproperPrior on μ of GsnTargetLaw(μ, I): posterior N(x̄, I/n) exactly.
    From θinit = 0 the chains need ~1,000 iterations of burn-in at D = 32
    (autocorrelation time of optimally scaled RWM ≈ 3·D), so this uses 8,192
    chains × 4,000 iterations and the second half for the moments."""
    w = W.cfg2(8192)
    e = run_engine(w, 8192, 4000, fetch=False)
    eng = e["engine"]
    m = eng.moments_window(2001, 2000, split=True)
    r = rhat_from_moments(m)
    xbar = w.obs.mean(axis=0)
    assert np.abs(r["mean"] - xbar).max() < 0.01
    post_var = r["W"] + r["B"] / m["num_draws"]
    assert np.abs(post_var / (1.0 / w.nobs) - 1.0).max() < 0.05
    # converged chains still give R̂ ≈ sqrt(1 + (τ−1)/n) with τ the integrated
    # autocorrelation time (≈ 100 here) and n = 1,000 draws per half-chain
    assert r["rhat"].max() < 1.1
    assert 0.20 < r["accept_rate"] < 0.30


def test_timing_reports_launches(full_run):
    w, _ = full_run
    e = run_engine(w, 65536, 128, fetch=False, hist=L.HIST_FULL, spl=64)
    eng = e["engine"]
    eng.set_timing(True)
    eng.run_iters(1, 128)
    eng.synchronize()
    ms, n, b = eng.get_timing()
    assert n == 2 and ms > 0
    # per launch: θ, ll, ra, ring, nacc, faults read and written, except θ's write-back: the
    # fused kernel leaves θ in its last history slot in FULL mode (emcmc.hip theta_live)
    assert b == pytest.approx(65536 * (128 * (16 * 32 + 8.125) + 2 * (8 * 32 + 80)))
