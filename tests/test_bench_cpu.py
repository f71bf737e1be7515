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
