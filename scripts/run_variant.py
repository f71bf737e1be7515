#!/usr/bin/env python3
"""Run one kernel variant on the headline workload (for rocprofv3 passes)."""
import argparse
import sys
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT))
sys.path.insert(0, str(ROOT / "extensiblemcmc.jl_amd"))
from extensible_mcmc import _lib as L  # noqa: E402
from extensible_mcmc import workloads as W  # noqa: E402
from extensible_mcmc.engine import Engine, EngineConfig  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--chains", type=int, default=65536)
ap.add_argument("--steps", type=int, default=200)
ap.add_argument("--spl", type=int, default=100)
ap.add_argument("--lpc", type=int, default=1)
ap.add_argument("--hist", choices=["full", "accept_only"], default="accept_only")
ap.add_argument("--ll", choices=["per_obs", "suffstat"], default="suffstat")
ap.add_argument("--variant", type=int, default=0)
a = ap.parse_args()
w = W.cfg2(a.chains)
eng = Engine(EngineConfig(dim=w.D, num_chains=a.chains, num_mcmc_steps=a.steps, seed=w.seed,
                          history_mode=L.HIST_FULL if a.hist == "full" else L.HIST_ACCEPT_ONLY,
                          lanes_per_chain=a.lpc, steps_per_launch=a.spl, kernel_variant=a.variant))
eng.add_gaussian_rw_update(np.arange(w.D), w.rw_sigma)
eng.set_gsn_target(w.mu_true, w.t_sigma, w.obs, ll_mode=L.LL_PER_OBS if a.ll == "per_obs" else L.LL_SUFFSTAT)
eng.set_state(np.zeros((a.chains, w.D)))
eng.set_timing(True)
eng.run_iters(1, a.steps)
eng.synchronize()
ms, n, b = eng.get_timing()
print(f"{eng.kernel_name()} {a.chains * a.steps / (ms / 1e3) / 1e9:.3f} Gchain-steps/s ({ms:.2f} ms, {n} launches)")
