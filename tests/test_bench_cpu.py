"""bench.py's host side on CPU: every workload carries what the line needs (θinit
broadcast to the chain count, the metric's config), and the CPU-baseline leg
runs on each (tiny samples; the oracle is the baseline there, never the product)."""
import sys
from pathlib import Path

import numpy as np
import pytest

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))
import bench  # noqa: E402
from extensible_mcmc import workloads as W  # noqa: E402


@pytest.mark.parametrize("make", [lambda: W.cfg2(256), lambda: W.cfg3(2, nobs=500), lambda: W.cfg4(256),
                                  lambda: W.cfg5(512)])
def test_workload_theta_init_broadcasts(make):
    w = make()
    C = 8
    th = np.broadcast_to(np.asarray(w.theta_init, dtype=np.float64)[-C:] if np.ndim(w.theta_init) == 2
                         else np.asarray(w.theta_init, dtype=np.float64), (C, w.D))
    assert th.shape == (C, w.D) and np.all(np.isfinite(th))


@pytest.mark.parametrize("name", ["cfg2", "cfg3", "cfg4"])
def test_cpu_baseline_leg_runs(name, monkeypatch):
    monkeypatch.setenv("OMP_NUM_THREADS", "2")
    w = {"cfg2": lambda: W.cfg2(256), "cfg3": lambda: W.cfg3(2, nobs=500), "cfg4": lambda: W.cfg4(256)}[name]()
    out = bench.cpu_baseline(w, 0.3, 0)
    assert out["value"] > 0 and out["cores"] == 2 and out["kind"] == "port"
    assert out["single_core"]["value"] > 0


def _bench_line(args, env_extra, drop_world=True):
    import json
    import os
    import subprocess

    env = dict(os.environ, EMCMC_BENCH_STUB_ENGINE="1", **env_extra)
    if drop_world:
        for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK"):
            env.pop(k, None)
    r = subprocess.run([sys.executable, str(ROOT / "bench.py"), *args], cwd=ROOT, env=env, capture_output=True,
                       text=True, timeout=240)
    lines = [x for x in r.stdout.splitlines() if x.startswith("{")]
    return r, (json.loads(lines[-1]) if lines else None)


STUB_ARGS = ["--steps", "20", "--warmup", "5", "--no-cpu", "--no-parity", "--settle-ms", "0", "--reps", "1"]


def test_gpus_n_launches_n_ranks():
    """`python bench.py --gpus 2` with no launcher runs 2 ranks (a torch.distributed.run
    child, gloo under the stub engine) and rank 0's line reports them: the per-GPU shape
    stays cfg 2's, the total doubles, and the diagnostics are merged over both shards."""
    r, line = _bench_line(["--gpus", "2", *STUB_ARGS], {})
    assert r.returncode == 0, r.stderr[-3000:]
    assert line["stub_engine"] is True and line["n_gpus"] == 2
    assert line["config"]["chains_per_gpu"] == 65536 and line["config"]["total_chains"] == 131072
    assert line["config"]["process_group"] == "gloo"
    assert line["config"]["first_chain_id"] == 0
    one = _bench_line(["--gpus", "1", *STUB_ARGS], {})[1]
    assert one["n_gpus"] == 1 and one["config"]["total_chains"] == 65536
    key = "plumbing_check_split_rhat_max"  # a 6–25 window from θinit = 0 is burn-in: labelled, not convergence
    assert "plumbing check, burn-in window" in line["diagnostics"]["purpose"]
    assert line["diagnostics"]["window_iterations"] == [6, 25]
    assert line["diagnostics"][key] != one["diagnostics"][key]  # rank 1's shard merged
    assert line["diagnostics"]["chains_merged"] == 2 * 131072  # split halves of both shards
    assert "host all-gather (gloo), 2 ranks" in line["diagnostics"]["via"]


def test_gpus_must_match_the_launchers_world_size():
    r, line = _bench_line(["--gpus", "4", *STUB_ARGS], {"WORLD_SIZE": "2", "RANK": "0", "LOCAL_RANK": "0"},
                          drop_world=False)
    assert r.returncode != 0 and line is None
    assert "--gpus 4 but WORLD_SIZE=2" in r.stderr


def test_diagnostics_watchdog():
    """The diagnostics collective after the timed region runs under a watchdog: a result, an
    exception (then bench.py retries through torch's all-gather) or a timeout (then the line
    is printed without diagnostics and the rank exits without waiting on the collective)."""
    import time

    assert bench.watchdog(lambda: 3, 5.0) == (3, None)
    v, err = bench.watchdog(lambda: 1 / 0, 5.0)
    assert v is None and err.startswith("ZeroDivisionError")
    assert bench.watchdog(lambda: time.sleep(3.0), 0.2) == (None, "timeout")


class _ReplayEngine:
    """The engine surface parity_replay reads, backed by an oracle run (CPU): a
    'GPU' whose results are the oracle's, optionally with one chain's stream flipped."""

    def __init__(self, O, w, S, flip=None):
        self.st = O.OracleState(np.zeros((w.num_chains, w.D)))
        h = O.run_gsn(self.st, seed=w.seed, rw_sigma=w.rw_sigma, t_sigma=w.t_sigma, obs=w.obs, iter0=1, nsteps=S,
                      accept_only=True, nthreads=2)
        self.bits = O.pack_accept(h["acc"])[:, None, :]
        if flip is not None:
            it, c = flip
            self.bits[it, 0, c // 64] ^= np.uint64(1 << (c % 64))

    def get_history_bits(self, i0, n):
        return self.bits[i0 - 1:i0 - 1 + n]

    def get_state(self):
        return self.st.theta, self.st.ll


@pytest.mark.parametrize("flip", [None, (7, 130)])
def test_parity_replay_counts_mismatched_chains(oracle, flip):
    """bench.py's replay: every chain within the budget, mismatches counted."""
    import types

    w = W.cfg2(256)
    a = types.SimpleNamespace(warmup=5, steps=10)
    eng = _ReplayEngine(oracle, w, 5 + 10 * 2, flip)
    par = bench.parity_replay(eng, w, a, 0, first=0, reps=2)
    assert par["chains_replayed"] == 256 and par["iterations"] == 25
    assert par["mismatched_chains"] == (0 if flip is None else 1)
    assert par["accept_stream_bitwise"] == (flip is None)
    assert par["final_theta_ll_bitwise"]
