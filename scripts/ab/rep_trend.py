#!/usr/bin/env python3
"""Why the first 20-step windows of a bench run are slower than the later ones: the kernel
time (dispatch events) of consecutive 20-step launches of the cfg 2 step kernel on one
handle, (a) back to back, (b) with an idle gap before each launch, (c) after 100 ms of
launches on the SAME handle, (d) after 100 ms on ANOTHER handle (what bench.py's settle does).

  python3 scripts/ab/rep_trend.py [--launches 15] [--gap-ms 5]
"""
import argparse
import json
import sys
import time
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parents[2]
sys.path[:0] = [str(ROOT), str(ROOT / "extensiblemcmc.jl_amd")]
from extensible_mcmc import workloads as W  # noqa: E402
from extensible_mcmc.engine import Engine, EngineConfig  # noqa: E402


RING = 100  # a history ring of one 100-step launch: the windows run as long as needed without filling HBM


def aligned(it, steps):
    """the first iteration ≥ it from which `steps` iterations stay inside one ring epoch"""
    return it if (it - 1) % RING + steps <= RING else ((it - 1) // RING + 1) * RING + 1


def make(w, C):
    eng = Engine(EngineConfig(dim=w.D, num_chains=C, num_mcmc_steps=1 << 20, seed=w.seed, steps_per_launch=100,
                              history_ring=RING))
    eng.add_gaussian_rw_update(np.arange(w.D), w.rw_sigma)
    eng.set_gsn_target(w.mu_true, w.t_sigma, w.obs)
    eng.set_state(np.zeros((C, w.D)))
    return eng


def trend(eng, it, n, steps, gap_s):
    out = []
    for _ in range(n):
        if gap_s:
            time.sleep(gap_s)
        it = aligned(it, steps)
        eng.set_timing(True)
        eng.run_iters(it, steps)
        eng.synchronize()
        ms, k, _ = eng.get_timing(reset=True)
        out.append(round(ms / k * 1e3, 1))
        it += steps
    return out, it


def burn(eng, it, ms, steps=100):
    t0 = time.perf_counter()
    while time.perf_counter() - t0 < ms / 1e3:
        it = aligned(it, steps)
        eng.run_iters(it, steps)
        eng.synchronize()
        it += steps
    return it


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--launches", type=int, default=15)
    ap.add_argument("--gap-ms", type=float, default=5.0)
    a = ap.parse_args()
    C, S = 65536, 20
    w = W.cfg2(C)
    eng = make(w, C)
    it = 1
    eng.run_iters(it, 5)
    eng.synchronize()
    it += 5
    res = {}
    res["back_to_back"], it = trend(eng, it, a.launches, S, 0.0)
    res["gap_%gms" % a.gap_ms], it = trend(eng, it, a.launches, S, a.gap_ms / 1e3)
    it = burn(eng, it, 100.0)
    res["after_100ms_same_handle"], it = trend(eng, it, a.launches, S, 0.0)
    other = make(w, C)
    burn(other, 1, 100.0)
    res["after_100ms_other_handle"], it = trend(eng, it, a.launches, S, 0.0)
    other.close()
    eng.close()
    for k, v in res.items():
        print(json.dumps({"case": k, "kernel_us": v}), flush=True)


if __name__ == "__main__":
    main()
