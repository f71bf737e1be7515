#!/usr/bin/env python3
"""Per-wave timeline of the cfg 2 step kernel (timing-only trace build).

EMCMC_LIB=extensiblemcmc.jl_amd/lib/libemcmc_trace.so python3 scripts/trace_diag.py --steps 20

Runs the headline workload (65,536 chains, D = 32, full histories), settles the
clock, then launches `--steps` steps as one launch with dispatch events, fetches
the per-wave s_memrealtime stamps (100 MHz) the trace build records (start,
tables staged, state arrived, end of each step, stores issued, stores drained)
and prints one JSON line: dispatch skew, staging and state-load time, per-step
time, the tail (last wave's drain to the event's end) — where the launch's
fixed cost goes.
"""
import argparse
import ctypes as C
import json
import sys
import time
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT))
sys.path.insert(0, str(ROOT / "extensiblemcmc.jl_amd"))
from extensible_mcmc import _lib as L  # noqa: E402
from extensible_mcmc import workloads as W  # noqa: E402
from extensible_mcmc.engine import Engine, EngineConfig  # noqa: E402

SLOTS, WAVES = 128, 16384
TICK_US = 0.01  # 100 MHz


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--chains", type=int, default=65536)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--settle-ms", type=float, default=150.0)
    ap.add_argument("--variant", type=int, default=0, help="kernel_variant (128: uncapped registers)")
    ap.add_argument("--dump", default="", help="save the raw per-wave stamps to <dump>_rep<k>.npz")
    a = ap.parse_args()
    assert a.steps + 5 <= SLOTS
    lib = L.lib()
    fetchers = [lib.emcmc_trace_fetch, lib.emcmc_trace_fetch2]  # MINW = 1 and MINW = 2 units
    for f in fetchers:
        f.restype = C.c_int
        f.argtypes = [C.c_void_p, C.c_size_t, C.c_int]
    buf = np.zeros((WAVES, SLOTS), dtype=np.uint64)
    tmp = np.zeros_like(buf)

    def fetch(_ptr, _n, clear):
        buf[:] = 0
        for f in fetchers:
            if f(tmp.ctypes.data, tmp.nbytes, clear) != 0:
                return -1
            buf[:] |= tmp  # one unit's buffer holds the launch, the other stays zero
        return 0

    w = W.cfg2(a.chains)
    # full histories into a ring of one launch (the clock-settling launches run for ~150 ms)
    eng = Engine(EngineConfig(dim=w.D, num_chains=a.chains, num_mcmc_steps=1 << 22, seed=w.seed, lanes_per_chain=2,
                              steps_per_launch=a.steps, history_ring=a.steps,
                              kernel_variant=a.variant))
    eng.add_gaussian_rw_update(np.arange(w.D), w.rw_sigma)
    eng.set_gsn_target(w.mu_true, w.t_sigma, w.obs)
    eng.set_state(np.zeros((a.chains, w.D)))
    eng.run_iters(1, a.steps)
    eng.synchronize()
    it = 1 + a.steps
    out = []
    for rep in range(a.reps):
        t0 = time.perf_counter()
        while time.perf_counter() - t0 < a.settle_ms / 1e3:  # settle on the same handle
            eng.run_iters(it, a.steps)
            eng.synchronize()
            it += a.steps
        assert fetch(buf.ctypes.data, buf.nbytes, 1) == 0  # clear
        eng.set_timing(True)
        eng.run_iters(it, a.steps)
        eng.synchronize()
        it += a.steps
        ms, n, _ = eng.get_timing(reset=True)
        eng.set_timing(False)
        assert fetch(buf.ctypes.data, buf.nbytes, 0) == 0
        nw = a.chains * 2 // 64
        t = buf[:nw].astype(np.int64)
        assert (t[:, 0] > 0).all() and (t[:, SLOTS - 1] > 0).all(), "trace incomplete"
        base = t[:, 0].min()
        rel = (t - base) * TICK_US
        start, staged, state = rel[:, 0], rel[:, 1], rel[:, 2]
        steps = rel[:, 3:3 + a.steps]
        issued, drained = rel[:, SLOTS - 2], rel[:, SLOTS - 1]
        per_step = np.diff(np.concatenate([state[:, None], steps], axis=1), axis=1)
        r = {
            "kernel": eng.kernel_name(), "rep": rep, "event_us": ms * 1e3, "waves": int(nw),
            "start_skew_us": float(start.max()), "start_p50_us": float(np.median(start)),
            "staging_us_p50": float(np.median(staged - start)), "staging_us_max": float((staged - start).max()),
            "state_us_p50": float(np.median(state - staged)), "state_us_max": float((state - staged).max()),
            "step_us_p50": float(np.median(per_step)), "step_us_mean": float(per_step.mean()),
            "first_step_us_p50": float(np.median(per_step[:, 0])), "last_step_us_p50": float(np.median(per_step[:, -1])),
            "step_p50_by_step": [round(float(x), 2) for x in np.median(per_step, axis=0)],
            "last_issue_us": float(issued.max()), "last_drain_us": float(drained.max()),
            "drain_us_p50": float(np.median(drained - issued)),
            "wave_span_us_p50": float(np.median(drained - start)), "wave_span_us_max": float((drained - start).max()),
            "end_p10_p50_p90_us": [float(np.percentile(drained, q)) for q in (10, 50, 90)],
            "event_minus_trace_us": ms * 1e3 - float(drained.max()),
        }
        # where the spread of end times comes from: per XCD (XCC_ID) and per SIMD slot
        hw = buf[:nw, 124].astype(np.int64)
        xcc = buf[:nw, 125].astype(np.int64) & 0xF
        cu = (hw >> 8) & 0xF
        se = (hw >> 13) & 0x7
        simd = (hw >> 4) & 0x3
        r["end_p50_by_xcc_us"] = [round(float(np.median(drained[xcc == x])), 1) for x in range(8)]
        r["end_max_by_xcc_us"] = [round(float(drained[xcc == x].max()), 1) if (xcc == x).any() else None
                                  for x in range(8)]
        slot = (xcc * 8 + se) * 16 * 4 + cu * 4 + simd  # one id per SIMD
        u, cnt = np.unique(slot, return_counts=True)
        r["waves_per_simd_hist"] = {int(k): int(v) for k, v in zip(*np.unique(cnt, return_counts=True))}
        r["cus_used"] = int(len(np.unique((xcc * 8 + se) * 16 + cu)))
        # end-time spread within one SIMD's waves vs across SIMDs
        per = {}
        for sid, d in zip(slot, drained):
            per.setdefault(int(sid), []).append(float(d))
        simd_end = np.array([max(v) for v in per.values()])
        r["simd_end_p10_p50_p90_max_us"] = [round(float(np.percentile(simd_end, q)), 1) for q in (10, 50, 90, 100)]
        if a.dump:
            np.savez_compressed(f"{a.dump}_rep{rep}.npz", t=buf[:nw, :3 + a.steps], end=buf[:nw, SLOTS - 2:],
                                hw=hw, xcc=xcc)
        out.append(r)
        print(json.dumps(r), flush=True)
    eng.close()


if __name__ == "__main__":
    main()
