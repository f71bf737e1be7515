#!/usr/bin/env python3
"""Where the wall of bench.py's short window goes (cfg 2, 65,536 chains, D = 32, full
histories): the Python wall of eng.run + eng.synchronize against the library's own host
time in emcmc_run and emcmc_synchronize (EMCMC_HOST_TIMING=1, printed at handle close)
and the kernel time from HIP events.  EMCMC_SYNC selects how emcmc_synchronize waits.

  EMCMC_HOST_TIMING=1 EMCMC_SYNC=0 python3 scripts/host_gap.py [--steps 20] [--reps 200]
"""
import argparse
import json
import os
import sys
import time
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parents[1]
sys.path[:0] = [str(ROOT), str(ROOT / "extensiblemcmc.jl_amd")]
from extensible_mcmc import workloads as W  # noqa: E402
from extensible_mcmc.engine import Engine, EngineConfig  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--reps", type=int, default=200)
    a = ap.parse_args()
    C = 65536
    w = W.cfg2(C)
    spl = 100
    # a ring of one launch's iterations: the windows run forever without filling HBM
    eng = Engine(EngineConfig(dim=w.D, num_chains=C, num_mcmc_steps=1 << 20, seed=w.seed, steps_per_launch=spl,
                              history_ring=spl))
    eng.add_gaussian_rw_update(np.arange(w.D), w.rw_sigma)
    eng.set_gsn_target(w.mu_true, w.t_sigma, w.obs)
    eng.set_state(np.zeros((C, w.D)))
    it = 1
    t0 = time.perf_counter()
    while time.perf_counter() - t0 < 0.3:  # settle the clock
        eng.run_iters(it, spl)
        eng.synchronize()
        it += spl
    it = ((it + spl - 1) // spl) * spl + 1  # windows inside one ring epoch
    walls, runs, syncs = [], [], []
    for r in range(a.reps):
        if (it - 1) % spl + a.steps > spl:
            it = ((it + spl - 1) // spl) * spl + 1
        steps = np.stack([np.arange(it, it + a.steps, dtype=np.uint32), np.ones(a.steps, dtype=np.uint32)], axis=1)
        eng.synchronize()
        t0 = time.perf_counter()
        eng.run(steps)
        t1 = time.perf_counter()
        eng.synchronize()
        t2 = time.perf_counter()
        walls.append(t2 - t0)
        runs.append(t1 - t0)
        syncs.append(t2 - t1)
        it += a.steps
    eng.set_timing(True)
    kern = []
    for r in range(20):
        if (it - 1) % spl + a.steps > spl:
            it = ((it + spl - 1) // spl) * spl + 1
        eng.run_iters(it, a.steps)
        eng.synchronize()
        ms, n, _ = eng.get_timing(reset=True)
        kern.append(ms / n * 1e3)
        it += a.steps
    med = lambda x: float(np.median(x)) * 1e6  # noqa: E731
    print(json.dumps({"steps": a.steps, "sync_mode": os.environ.get("EMCMC_SYNC", "0"),
                      "wall_us": med(walls), "py_run_us": med(runs), "py_sync_us": med(syncs),
                      "kernel_us": float(np.median(kern)), "wall_p10_us": float(np.percentile(walls, 10)) * 1e6}),
          flush=True)
    eng.close()


if __name__ == "__main__":
    main()
