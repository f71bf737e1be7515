#!/usr/bin/env python3
"""Fill the on-disk code-object cache (extensiblemcmc.jl_amd/lib/rtc_cache, or
EMCMC_RTC_CACHE) with the run-time chol kernels the GPU tests and benches use, on
the CPU (hiprtc needs no device).  The cache travels with the tree to the GPU box,
where a handle then loads instead of compiling (run-time compilation).

  python scripts/prebuild_rtc.py [D ...]      (default: the D the GPU tests use)
"""
import sys
import time
from concurrent.futures import ProcessPoolExecutor
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path[:0] = [str(ROOT), str(ROOT / "extensiblemcmc.jl_amd")]
from extensible_mcmc import _lib as L  # noqa: E402

# (D, history mode, ll mode) of tests/test_gpu_chol.py, tests/test_gpu_api.py and scripts/bench_dense.py
DEFAULT = [(9, 0, 0), (12, 0, 1), (20, 0, 0), (20, 1, 0), (27, 0, 0), (33, 0, 0), (40, 0, 1), (48, 0, 0),
           (49, 0, 0), (53, 0, 0), (56, 0, 1), (64, 0, 0)]


# mwg_block_kernel (one MALA / user update over all coordinates) of tests/test_gpu_block.py and
# scripts/bench_general.py: (D, history mode, ll mode, dense target, user law, user update)
BLOCK = [(20, 0, 0, True, None, None), (40, 0, 0, True, None, None), (32, 0, 0, True, None, "pcn"),
         (20, 0, 0, True, "logistic_regression", None)]


# mwg_rw_block_kernel shapes of scripts/bench_general.py rw_prior (D = 32, FULL, per observation,
# diagonal target): (name, update-desc factory)
def rw_shapes():
    import numpy as np
    from extensible_mcmc.engine import Engine

    D = 32
    s2 = (2.38 / np.sqrt(D * 10)) ** 2
    B = np.random.default_rng(9).standard_normal((D, D))
    return [
        ("rw_product_normal_d32", lambda: Engine.gaussian_rw_desc(
            np.arange(D), s2 * np.eye(D), prior=L.PRIOR_PRODUCT,
            prior_factors=[(L.DIST_PRODUCT, D, [(L.DIST_NORMAL, 0.0, 3.0)] * D)])),
        ("rw_standard_mvnormal_d32", lambda: Engine.gaussian_rw_desc(
            np.arange(D), s2 * np.eye(D), prior=L.PRIOR_STANDARD,
            prior_factors=[(L.DIST_MVNORMAL, D, np.zeros(D), B @ B.T / D + np.eye(D))])),
        ("unif_pos_d32", lambda: Engine.uniform_rw_desc(np.arange(D), 0.06, pos=np.ones(D))),
    ]


def one_rw(i):
    name, make = rw_shapes()[i]
    t = time.time()
    u, keep = make()
    L.prebuild_rw_block_kernel(32, [u], 0, 0, False)
    return f"rw block {name}: {time.time() - t:.1f} s"


def one(job):
    D, hist, ll = job
    t = time.time()
    L.prebuild_chol_kernel(D, hist, ll)
    return f"D={D} hist={hist} ll={ll}: {time.time() - t:.1f} s"


def one_block(job):
    D, hist, ll, dense, law, upd = job
    t = time.time()
    tsrc = (ROOT / "tests" / "user_targets" / f"{law}.c").read_text() if law else ""
    usrc = (ROOT / "tests" / "user_updates" / f"{upd}.c").read_text() if upd else ""
    L.prebuild_block_kernel(D, hist, ll, dense, target_source=tsrc, update_source=usrc)
    return f"block D={D} hist={hist} ll={ll} law={law} update={upd or 'MALA'}: {time.time() - t:.1f} s"


if __name__ == "__main__":
    jobs = [(int(d), 0, 0) for d in sys.argv[1:]] or DEFAULT
    # processes, not threads: hiprtc compiles one program at a time per process
    with ProcessPoolExecutor(8) as ex:
        futs = [ex.submit(one, j) for j in jobs]
        if not sys.argv[1:]:
            futs += [ex.submit(one_block, j) for j in BLOCK]
            futs += [ex.submit(one_rw, i) for i in range(3)]
        for f in futs:
            print(f.result(), flush=True)
