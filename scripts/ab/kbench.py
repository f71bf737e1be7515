#!/usr/bin/env python3
"""Kernel-variant sweep on the headline workload (one process, interleaved
rounds, median of rounds; §5.4 rule 24).  Prints one JSON line per variant."""
import argparse
import json
import sys
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT))
sys.path.insert(0, str(ROOT / "extensiblemcmc.jl_amd"))

from extensible_mcmc import _lib as L  # noqa: E402
from extensible_mcmc import workloads as W  # noqa: E402
from extensible_mcmc.engine import Engine, EngineConfig  # noqa: E402


def make(w, C, S, lpc, variant, ll_mode, hist, spl):
    eng = Engine(EngineConfig(dim=w.D, num_chains=C, num_mcmc_steps=S, seed=w.seed, history_mode=hist,
                              lanes_per_chain=lpc, steps_per_launch=spl, kernel_variant=variant))
    eng.add_gaussian_rw_update(np.arange(w.D), w.rw_sigma)
    eng.set_gsn_target(w.mu_true, w.t_sigma, w.obs, ll_mode=ll_mode)
    eng.set_state(np.zeros((C, w.D)))
    return eng


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--chains", type=int, default=65536)
    ap.add_argument("--steps", type=int, default=400)
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--variants", default="all")
    ap.add_argument("--grid", default="", help="lpc:variant,... (overrides --variants)")
    ap.add_argument("--hist", default="full,accept_only")
    ap.add_argument("--ll", default="per_obs,suffstat")
    a = ap.parse_args()
    w = W.cfg2(a.chains)
    grid = []
    hists = [{"full": L.HIST_FULL, "accept_only": L.HIST_ACCEPT_ONLY}[h] for h in a.hist.split(",")]
    lls = [{"per_obs": L.LL_PER_OBS, "suffstat": L.LL_SUFFSTAT}[x] for x in a.ll.split(",")]
    if a.grid:
        lv = tuple(tuple(int(v) for v in g.split(":")) for g in a.grid.split(","))
    else:
        lv = {"all": ((1, 0), (2, 0), (4, 0), (4, 1)), "lpc14": ((1, 0), (4, 0)),
              "lpc4": ((4, 0), (4, 1))}[a.variants]
    for hist in hists:
        for ll in lls:
            for lpc, var in lv:
                grid.append((lpc, var, ll, hist, 100))
    S = 100 + a.steps * a.rounds
    res = {g: [] for g in grid}
    for r in range(a.rounds):
        for g in grid:
            lpc, var, ll, hist, spl = g
            eng = make(w, a.chains, 100 + a.steps, lpc, var, ll, hist, spl)
            eng.run_iters(1, 100)
            eng.synchronize()
            eng.set_timing(True)
            eng.run_iters(101, a.steps)
            eng.synchronize()
            ms, n, b = eng.get_timing(reset=True)
            res[g].append((ms, n, b, eng.kernel_name()))
            eng.close()
            print(f"round {r} {g} {ms:.2f} ms", file=sys.stderr, flush=True)
    for g, v in res.items():
        ms = float(np.median([x[0] for x in v]))
        n, b, name = v[0][1], v[0][2], v[0][3]
        cs = a.chains * a.steps / (ms / 1e3)
        print(json.dumps({"kernel": name, "lpc": g[0], "variant": g[1], "ll_mode": g[2], "hist": g[3],
                          "chain_steps_per_s": cs, "ms": ms, "launches": n,
                          "GBps": b / (ms / 1e3) / 1e9, "frac_8TBs": b / (ms / 1e3) / 8e12}))


if __name__ == "__main__":
    main()
