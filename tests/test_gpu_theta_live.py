"""θ left in the last history slot (emcmc.hip theta_live): the fused diagonal
kernel in FULL history mode does not write the state buffer back, the next launch reads θ
from the slot.  With EMCMC_THETA_LIVE=1 (default) and =0 (always write the state buffer) the
same runs give the same bits, in the cases where the slot's lifetime meets the ring and
stream machinery: a history ring streamed to the host across epoch wraps, a P = 2 schedule
(general kernel: theta_live inactive, checked for no interference), and a re-run of
iterations that overwrites the live slot itself."""
import os

import numpy as np
import pytest

from extensible_mcmc import _lib as L
from extensible_mcmc import workloads as W
from extensible_mcmc.engine import Engine, EngineConfig, PinnedArray

pytestmark = pytest.mark.gpu


@pytest.fixture(autouse=True)
def _gpu(require_gpu):
    pass


def engine(live, **kw):
    old = os.environ.get("EMCMC_THETA_LIVE")
    os.environ["EMCMC_THETA_LIVE"] = "1" if live else "0"  # read at emcmc_create
    try:
        return Engine(EngineConfig(**kw))
    finally:
        if old is None:
            del os.environ["EMCMC_THETA_LIVE"]
        else:
            os.environ["EMCMC_THETA_LIVE"] = old


def ring_streamed(live):
    """R = 40 ring, 16-step launches, 20-iteration chunks each streamed (θ, every 2nd
    iteration; ll; accept words) while the next chunk runs: epochs wrap at 40, 80."""
    w = W.cfg2(2048)
    eng = engine(live, dim=w.D, num_chains=2048, num_mcmc_steps=120, seed=w.seed, steps_per_launch=16,
                 history_ring=40)
    eng.add_gaussian_rw_update(np.arange(w.D), w.rw_sigma)
    eng.set_gsn_target(w.mu_true, w.t_sigma, w.obs)
    eng.set_state(np.zeros((2048, w.D)))
    name = eng.kernel_name()
    outs = []
    for c0 in range(1, 121, 20):
        eng.run_iters(c0, 20)
        outs.append(eng.stream_history(L.H_STATE, c0 + 1, 10, thin=2))
        outs.append(eng.stream_history(L.H_LL, c0, 20))
        outs.append(eng.stream_history(L.H_ACCEPT, c0, 20))
    eng.stream_wait()
    eng.synchronize()
    th, ll = eng.get_state()
    res = [np.array(o) for o in outs] + [th, ll, eng.get_history(L.H_STATE, 81, 40)]
    eng.close()
    return name, res


def two_updates(live):
    w = W.cfg2(1024)
    eng = engine(live, dim=w.D, num_chains=1024, num_mcmc_steps=60, seed=w.seed, steps_per_launch=9)
    for blk in (np.arange(0, 16), np.arange(16, 32)):
        eng.add_gaussian_rw_update(blk, 2.0 * np.asarray(w.rw_sigma)[:16, :16])
    eng.set_gsn_target(w.mu_true, w.t_sigma, w.obs)
    eng.set_state(np.zeros((1024, w.D)))
    eng.run([(i, p) for i in range(1, 61) for p in (1, 2)])
    eng.synchronize()
    th, ll = eng.get_state()
    res = [th, ll, eng.get_history(L.H_STATE, 1, 60), eng.get_history(L.H_ACCEPT, 1, 60)]
    name = eng.kernel_name()
    eng.close()
    return name, res


def rerun_over_live_slot(live):
    """Iterations 1..30 (θ lives in slot 30), then 25..40 again: the first launch of the
    re-run reads θ from slot 30 and overwrites it at its sixth step."""
    w = W.cfg2(2048)
    eng = engine(live, dim=w.D, num_chains=2048, num_mcmc_steps=40, seed=w.seed, steps_per_launch=8)
    eng.add_gaussian_rw_update(np.arange(w.D), w.rw_sigma)
    eng.set_gsn_target(w.mu_true, w.t_sigma, w.obs)
    eng.set_state(np.zeros((2048, w.D)))
    eng.run_iters(1, 30)
    eng.run_iters(25, 16)
    eng.synchronize()
    th, ll = eng.get_state()
    res = [th, ll, eng.get_history(L.H_STATE, 1, 40), eng.get_history(L.H_LL, 1, 40),
           eng.get_history(L.H_ACCEPT, 1, 40)]
    name = eng.kernel_name()
    eng.close()
    return name, res


@pytest.mark.parametrize("case", [ring_streamed, two_updates, rerun_over_live_slot])
def test_theta_live_on_and_off_give_the_same_bits(case):
    (n1, a), (n0, b) = case(True), case(False)
    assert n1 == n0
    if case is not two_updates:
        assert n1.startswith("rwm_gsn_diag_kernel")  # the kernel that leaves θ in its slot
    assert len(a) == len(b)
    for k, (x, y) in enumerate(zip(a, b)):
        assert np.array_equal(x, y), (case.__name__, k)


def test_rerun_matches_a_fresh_engine_from_the_same_state(oracle):
    """The re-run over the live slot is the reference's semantics: iterations 25..40 from
    the θ / ll after iteration 30, on a fresh handle with the same rolling statistics, give
    the same chains (the oracle replays the same schedule)."""
    w = W.cfg2(512)
    _, res = rerun_over_live_slot(True)
    st = oracle.OracleState(np.zeros((512, w.D)))
    oracle.run_gsn(st, seed=w.seed, rw_sigma=w.rw_sigma, t_sigma=w.t_sigma, obs=w.obs, iter0=1, nsteps=30)
    oracle.run_gsn(st, seed=w.seed, rw_sigma=w.rw_sigma, t_sigma=w.t_sigma, obs=w.obs, iter0=25, nsteps=16)
    assert np.array_equal(res[0][:512], st.theta) and np.array_equal(res[1][:512], st.ll)
