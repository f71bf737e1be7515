#!/usr/bin/env python3
"""Throughput of the general schedule kernel (mwg_gsn_kernel / mwg_wide_kernel,
including the run-time-compiled user-law variants) on a few workloads; one JSON
line each.  Kernel time from the engine's HIP events (emcmc_get_timing);
"update_steps_per_s" counts (chain, update) steps, i.e. a P-update iteration
counts P.  Run under rocprofv3 --kernel-trace --stats for the per-kernel view."""
import argparse
import json
import sys
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parent.parent
for p in (ROOT, ROOT / "extensiblemcmc.jl_amd", ROOT / "tests"):
    sys.path.insert(0, str(p))
from extensible_mcmc import _lib as L  # noqa: E402
from extensible_mcmc import workloads as W  # noqa: E402
from extensible_mcmc.engine import Engine, EngineConfig  # noqa: E402


def timed(eng, steps, reps=3):
    eng.run(steps[: len(steps) // 10])  # warm-up (first launch also compiles any run-time kernel)
    eng.synchronize(allow_faults=True)
    eng.set_timing(True)
    eng.get_timing(reset=True)
    best = None
    for _ in range(reps):
        eng.run(steps)
        eng.synchronize(allow_faults=True)
        ms, n, b = eng.get_timing(reset=True)
        best = ms if best is None else min(best, ms)
    return best, b


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--chains", type=int, default=65536)
    ap.add_argument("--iters", type=int, default=200)
    a = ap.parse_args()
    C, M = a.chains, a.iters
    w = W.cfg2(8)
    out = []

    def report(name, eng, P, ms, nbytes):
        n = C * M * P
        out.append({"workload": name, "kernel": eng.kernel_name(), "chains": C, "iters": M, "updates": P,
                    "ms": ms, "update_steps_per_s": n / (ms / 1e3), "GBps_algorithmic": nbytes / (ms / 1e3) / 1e9})
        print(json.dumps(out[-1]), flush=True)

    # (1) D = 32, two GaussianRandomWalk blocks of 16 coordinates (Metropolis-within-Gibbs)
    eng = Engine(EngineConfig(dim=32, num_chains=C, num_mcmc_steps=2 * M, seed=w.seed))
    for blk in (range(0, 16), range(16, 32)):
        eng.add_gaussian_rw_update(np.array(blk), np.asarray(w.rw_sigma)[:16, :16] * 2.0)
    eng.set_gsn_target(w.mu_true, w.t_sigma, w.obs)
    eng.set_state(np.zeros((C, 32)))
    steps = [(i, p) for i in range(1, 2 * M + 1) for p in (1, 2)]
    ms, b = timed(eng, steps[: 2 * M], reps=3)
    report("mwg_d32_two_blocks", eng, 2, ms, b)
    eng.close()

    # (2) D = 32, one joint update with correlated proposal and target Σ
    rng = np.random.default_rng(5)
    A = rng.standard_normal((32, 32))
    St = A @ A.T / 32 + np.eye(32)
    Sr = 0.01 * (np.eye(32) + 0.2 * np.ones((32, 32)))
    eng = Engine(EngineConfig(dim=32, num_chains=C, num_mcmc_steps=2 * M, seed=w.seed))
    eng.add_gaussian_rw_update(np.arange(32), Sr)
    eng.set_gsn_target(w.mu_true, St, w.obs)
    eng.set_state(np.zeros((C, 32)))
    ms, b = timed(eng, [(i, 1) for i in range(1, M + 1)], reps=3)
    report("dense_d32_joint", eng, 1, ms, b)
    eng.close()
    # (2b) the same with the sufficient-statistic likelihood (one solve per step)
    eng = Engine(EngineConfig(dim=32, num_chains=C, num_mcmc_steps=2 * M, seed=w.seed))
    eng.add_gaussian_rw_update(np.arange(32), Sr)
    eng.set_gsn_target(w.mu_true, St, w.obs, ll_mode=L.LL_SUFFSTAT)
    eng.set_state(np.zeros((C, 32)))
    ms, b = timed(eng, [(i, 1) for i in range(1, M + 1)], reps=3)
    report("dense_d32_joint_suffstat", eng, 1, ms, b)
    eng.close()

    # (3) user law: student-t regression, D = 4, 50 observations (run-time compiled)
    import user_target_cases as U
    case = U.student_t()
    src = (ROOT / "tests" / "user_targets" / f"{case.name}.c").read_text()
    eng = Engine(EngineConfig(dim=case.D, num_chains=2 * C, num_mcmc_steps=2 * M, seed=case.seed))
    eng.add_gaussian_rw_update(np.arange(case.D), 0.01 * np.eye(case.D))
    eng.set_user_target(src, obs=case.obs, params=case.params, theta0=case.theta0)
    eng.set_state(np.zeros((2 * C, case.D)))
    C0 = C
    C = 2 * C0
    ms, b = timed(eng, [(i, 1) for i in range(1, M + 1)], reps=3)
    report("user_student_t_d4", eng, 1, ms, b)
    C = C0
    eng.close()


if __name__ == "__main__":
    main()
