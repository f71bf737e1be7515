#!/usr/bin/env python3
"""Compile the bench schedules of mwg_rw_block_kernel (scripts/bench_general.py) on the CPU with
hiprtc into a private temporary cache and print each code object's register / spill / scratch
metadata: the A/B check of a build option before it goes to the GPU.
  EMCMC_RTC_EXTRA="-DEMCMC_RW_WAVES_PER_EU=2" python3 scripts/rw_block_resources.py [names]"""
import os
import re
import subprocess
import sys
import tempfile
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
for p in (ROOT / "extensiblemcmc.jl_amd", ROOT / "tests", ROOT):
    sys.path.insert(0, str(p))
import numpy as np  # noqa: E402

READELF = "/opt/rocm/lib/llvm/bin/llvm-readelf"
KEYS = ["vgpr_count", "agpr_count", "vgpr_spill_count", "sgpr_spill_count", "private_segment_fixed_size"]


def shapes():
    from extensible_mcmc import _lib as L
    from extensible_mcmc import workloads as W
    from extensible_mcmc.engine import Engine
    w = W.cfg2(8)
    D = 32
    s2 = (2.38 / np.sqrt(D * 10)) ** 2
    B = np.random.default_rng(9).standard_normal((D, D))
    s64 = (2.38 / np.sqrt(32 * 10)) ** 2
    return {
        "mwg_d32_two_blocks": (32, lambda: [Engine.gaussian_rw_desc(np.arange(a, a + 16),
                                                                    np.asarray(w.rw_sigma)[:16, :16] * 2.0)
                                            for a in (0, 16)]),
        "rw_product_normal_d32": (32, lambda: [Engine.gaussian_rw_desc(
            np.arange(D), s2 * np.eye(D), prior=L.PRIOR_PRODUCT,
            prior_factors=[(L.DIST_PRODUCT, D, [(L.DIST_NORMAL, 0.0, 3.0)] * D)])]),
        "rw_standard_mvnormal_d32": (32, lambda: [Engine.gaussian_rw_desc(
            np.arange(D), s2 * np.eye(D), prior=L.PRIOR_STANDARD,
            prior_factors=[(L.DIST_MVNORMAL, D, np.zeros(D), B @ B.T / D + np.eye(D))])]),
        "unif_pos_d32": (32, lambda: [Engine.uniform_rw_desc(np.arange(D), 0.06, pos=np.ones(D))]),
        "mwg_d64_two_blocks": (64, lambda: [
            Engine.gaussian_rw_desc(np.arange(32), s64 * np.eye(32), prior=L.PRIOR_PRODUCT,
                                    prior_factors=[(L.DIST_PRODUCT, 32, [(L.DIST_NORMAL, 0.0, 4.0)] * 32)]),
            Engine.gaussian_rw_desc(np.arange(32, 64), s64 * np.eye(32))]),
    }


def main():
    want = sys.argv[1:]
    with tempfile.TemporaryDirectory() as tmp:
        os.chmod(tmp, 0o700)
        os.environ["EMCMC_RTC_CACHE"] = tmp
        from extensible_mcmc import _lib as L
        for name, (dim, make) in shapes().items():
            if want and name not in want:
                continue
            descs = make()
            before = set(os.listdir(tmp))
            L.prebuild_rw_block_kernel(dim, [d for d, _ in descs], 0, 0, False)
            new = sorted(set(os.listdir(tmp)) - before)
            for f in new:
                data = Path(tmp, f).read_bytes()
                elf = Path(tmp, f + ".elf")
                elf.write_bytes(data[data.find(b"\x7fELF"):])
                notes = subprocess.run([READELF, "--notes", str(elf)], capture_output=True, text=True).stdout
                vals = {k: re.search(r"\." + k + r":\s+(\d+)", notes).group(1) for k in KEYS}
                print(name, " ".join(f"{k}={v}" for k, v in vals.items()), flush=True)


if __name__ == "__main__":
    main()
