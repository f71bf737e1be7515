#!/usr/bin/env python3
"""Dense (correlated) Σ_rw / Σ_t, one joint GaussianRandomWalk on coords 1:D, at D
without an ahead-of-time rwm_gsn_chol_kernel: the chol kernel compiled at run time
against the general kernel (EMCMC_VARIANT_NO_RTC_CHOL, the round-2 route), one JSON
line each.  Kernel time from the engine's HIP events; 65,536 chains, FULL history,
per-observation likelihood over 10 observations."""
import argparse
import json
import sys
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parent.parent
for p in (ROOT, ROOT / "extensiblemcmc.jl_amd", ROOT / "tests"):
    sys.path.insert(0, str(p))
from extensible_mcmc import _lib as L  # noqa: E402
from extensible_mcmc.engine import Engine, EngineConfig  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--chains", type=int, default=65536)
    ap.add_argument("--iters", type=int, default=100)
    ap.add_argument("--dims", default="12,20,40,48,64")
    ap.add_argument("--ll", choices=["per_obs", "suffstat"], default="per_obs")
    ap.add_argument("--general", type=int, default=1, help="also time the general-kernel route")
    a = ap.parse_args()
    llm = L.LL_PER_OBS if a.ll == "per_obs" else L.LL_SUFFSTAT
    C, M = a.chains, a.iters
    for D in [int(x) for x in a.dims.split(",")]:
        rng = np.random.default_rng(D)
        A = rng.standard_normal((D, D))
        S = A @ A.T / D + np.eye(D)
        mu = rng.standard_normal(D)
        obs = rng.multivariate_normal(mu, S, size=10)
        B = rng.standard_normal((D, D))
        R = (2.38 ** 2 / (D * 10)) * (B @ B.T / D + np.eye(D))
        for variant in (0, L.VARIANT_NO_RTC_CHOL) if a.general else (0,):
            eng = Engine(EngineConfig(dim=D, num_chains=C, num_mcmc_steps=3 * M, seed=D, kernel_variant=variant,
                                      steps_per_launch=M))
            eng.add_gaussian_rw_update(np.arange(D), R)
            eng.set_gsn_target(mu, S, obs, ll_mode=llm)
            eng.set_state(np.tile(mu, (C, 1)))
            eng.run_iters(1, M)  # warm-up (and the run-time compile)
            eng.synchronize(allow_faults=True)
            eng.set_timing(True)
            eng.get_timing(reset=True)
            best = None
            for r in range(2):
                eng.run_iters(M + 1 + r * M // 2, M // 2)
                eng.synchronize(allow_faults=True)
                ms, n, b = eng.get_timing(reset=True)
                best = ms / (M // 2) if best is None else min(best, ms / (M // 2))
            print(json.dumps({"D": D, "ll": a.ll, "kernel": eng.kernel_name(), "chains": C, "ms_per_step": best,
                              "chain_steps_per_s": C / (best / 1e3)}), flush=True)
            eng.close()


if __name__ == "__main__":
    main()
