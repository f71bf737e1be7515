"""BASELINE cfg 5 on one MI355X: the 1,048,576-chain job as 8 shard handles of
131,072 chains (first_chain_id = r·131072, what rank r of the 8-GPU run owns)
against one 1M-chain handle, with history rings (the full 1M × 1000-step
history would need 550 GB).  Chains are keyed by global id, so
the shards must reproduce the unsharded job bit for bit; their Chan-merged
split-chain moments must equal the 1M handle's reduction; and sampled chains of
every one of the 1,048,576 chains must replay bitwise on the oracle in its
accept-only mode — the accept stream over the ring window and the final θ / ll
(run.jl:64-83 per chain)."""
import os

import numpy as np
import pytest

from extensible_mcmc import _lib as L
from extensible_mcmc import diagnostics as DG
from extensible_mcmc import workloads as W
from extensible_mcmc.engine import Engine, EngineConfig

pytestmark = pytest.mark.gpu

TOTAL, SHARDS, S, RING = 1 << 20, 8, 200, 100


@pytest.fixture(autouse=True)
def _gpu(require_gpu):
    pass


def _run(w, theta0, C, chain0):
    eng = Engine(EngineConfig(dim=w.D, num_chains=C, num_mcmc_steps=S, seed=w.seed, first_chain_id=chain0,
                              history_mode=L.HIST_FULL, history_ring=RING))
    eng.add_gaussian_rw_update(np.arange(w.D), w.rw_sigma)
    eng.set_gsn_target(w.mu_true, w.t_sigma, w.obs)
    eng.set_state(np.ascontiguousarray(theta0))
    eng.run_iters(1, S)
    eng.synchronize()
    out = {"kernel": eng.kernel_name(), "faults": int(np.count_nonzero(eng.get_faults()))}
    out["theta"], out["ll"] = eng.get_state()
    out["acc"] = eng.get_history(L.H_ACCEPT, S - RING + 1, RING)[:, 0]
    out["mom"] = eng.moments_window(S - RING + 1, RING, split=True)
    eng.close()
    return out


def test_cfg5_eight_shards_equal_the_1m_chain_job(oracle):
    w = W.cfg5(TOTAL)
    per = TOTAL // SHARDS
    shards = [_run(w, w.theta_init[r * per:(r + 1) * per], per, r * per) for r in range(SHARDS)]
    full = _run(w, w.theta_init, TOTAL, 0)
    assert full["faults"] == 0 and all(s["faults"] == 0 for s in shards)
    # per-chain results do not depend on the sharding (RNG keyed by global chain id)
    assert np.array_equal(np.concatenate([s["theta"] for s in shards]), full["theta"])
    assert np.array_equal(np.concatenate([s["ll"] for s in shards]), full["ll"])
    assert np.array_equal(np.concatenate([s["acc"] for s in shards], axis=1), full["acc"])
    # the diagnostics the 8 ranks all-gather, merged in rank order, equal the 1M handle's
    merged = DG.merge([s["mom"] for s in shards])
    ref = full["mom"]
    assert merged["num_chains"] == ref["num_chains"] == 2 * TOTAL
    assert merged["accepted"] == ref["accepted"] and merged["proposed"] == ref["proposed"]
    np.testing.assert_allclose(merged["mean"], ref["mean"], rtol=1e-12, atol=1e-13)
    np.testing.assert_allclose(merged["m2"], ref["m2"], rtol=1e-10)
    np.testing.assert_allclose(merged["sum_var"], ref["sum_var"], rtol=1e-12)
    r = DG.rhat_from_moments(merged)
    assert 0.15 < r["accept_rate"] < 0.4
    assert np.all(np.isfinite(r["rhat"]))
    # every chain of the 1M-chain job replays bitwise on the oracle (accept-only mode:
    # 2.1e8 chain-steps on the box's 16 cores, no θ history formed)
    threads = max(1, min(16, int(os.environ.get("OMP_NUM_THREADS", "0") or 0) or (os.cpu_count() or 1)))
    st = oracle.OracleState(np.ascontiguousarray(w.theta_init, dtype=np.float64))
    h = oracle.run_gsn(st, seed=w.seed, rw_sigma=w.rw_sigma, t_sigma=w.t_sigma, obs=w.obs, iter0=1, nsteps=S,
                       accept_only=True, nthreads=threads)
    want = h["acc"][S - RING:]
    bad = np.flatnonzero((full["acc"] != want).any(axis=0))
    assert bad.size == 0, f"{bad.size} of {TOTAL} accept streams differ in the ring window (first: {bad[:8]})"
    bad = np.flatnonzero((full["theta"] != st.theta).any(axis=1) | (full["ll"] != st.ll))
    assert bad.size == 0, f"{bad.size} of {TOTAL} chains' final θ/ll differ (first: {bad[:8]})"
