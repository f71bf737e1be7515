#!/usr/bin/env python3
"""Fill the on-disk code-object cache (extensiblemcmc.jl_amd/lib/rtc_cache, or
EMCMC_RTC_CACHE) with the run-time chol kernels the GPU tests and benches use, on
the CPU (hiprtc needs no device).  The cache travels with the tree to the GPU box,
where a handle then loads instead of compiling (run-time compilation).

  python scripts/prebuild_rtc.py [D ...]      (default: the D the GPU tests use)
"""
import sys
import time
from concurrent.futures import ThreadPoolExecutor
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path[:0] = [str(ROOT), str(ROOT / "extensiblemcmc.jl_amd")]
from extensible_mcmc import _lib as L  # noqa: E402

# (D, history mode, ll mode) of tests/test_gpu_chol.py, tests/test_gpu_api.py and scripts/bench_dense.py
DEFAULT = [(9, 0, 0), (12, 0, 1), (20, 0, 0), (20, 1, 0), (27, 0, 0), (33, 0, 0), (40, 0, 1), (48, 0, 0),
           (49, 0, 0), (64, 0, 0)]


def one(job):
    D, hist, ll = job
    t = time.time()
    L.prebuild_chol_kernel(D, hist, ll)
    return f"D={D} hist={hist} ll={ll}: {time.time() - t:.1f} s"


if __name__ == "__main__":
    jobs = [(int(d), 0, 0) for d in sys.argv[1:]] or DEFAULT
    with ThreadPoolExecutor(4) as ex:
        for line in ex.map(one, jobs):
            print(line, flush=True)
