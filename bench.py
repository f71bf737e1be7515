#!/usr/bin/env python3
"""bench.py — MCMC steps×chains/sec on the D=32 Gaussian target (BASELINE cfg 2).

--workload cfg4 measures BASELINE cfg 4 instead: GaussianRandomWalkMix +
HaarioTypeAdaptation with the per-chain running mean/cov kept on device
(131,072 chains by default); same metric and JSON contract.
--workload cfg3 measures BASELINE cfg 3: MALA on a logistic-regression
log-likelihood (N = 100,000, D = 64, 32,768 chains), fp64 MFMA-bound.

One "step" = one MCMC iteration of every chain on every GPU: proposal,
log-prior, log-likelihood, MH accept/reject, rolling acceptance and the full
per-step histories (θ, θ°, ll, accept bit) written to HBM — the reference's
run! outputs (src/run.jl:237-239, 319, 333-334).  Chains are sharded
embarrassingly: rank r owns global chain ids [r·C, (r+1)·C) (weak scaling,
no data-path collective).  Diagnostics (split-R̂, acceptance) are combined once
after the timed region: an all-gather of every rank's moments, Chan-merged.

  python bench.py [--gpus N] [--steps K] [--warmup W]
  torchrun --nproc-per-node N bench.py --gpus N ...

`python bench.py --gpus N` with N > 1 and no WORLD_SIZE in the environment starts
`torch.distributed.run --nproc-per-node N` on this same command line as a child
process (before anything here imports torch or touches a GPU) and exits with its
return code; rank 0 of the child prints the line.  Under a launcher, WORLD_SIZE
must equal --gpus (when given): a mismatch exits non-zero instead of measuring a
different N than the one asked for.

Prints ONE JSON line on rank 0.
"""
import argparse
import json
import os
import sys
import time
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parent
sys.path.insert(0, str(ROOT))
sys.path.insert(0, str(ROOT / "extensiblemcmc.jl_amd"))

HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec (MI355X_MICROARCH.md, chip-level parameters)
HBM_ACHIEVABLE_GBS = 6290.0  # measured achievable, float4 copy (MI355X_MICROARCH.md:36)
FP64_MFMA_PEAK_TFS = 78.6  # MI355X FP64 matrix peak (AMD spec; equal to the FP64 vector peak)
FP64_MFMA_MEASURED_TFS = 47.8  # v_mfma_f64_16x16x4f64 issue ceiling measured on MI355X (profiles/r3_mfma_f64_ubench.txt)
FP64_VALU_MEASURED_TFS = 50.5  # v_fma_f64, 8 independent chains, 2 waves/SIMD (profiles/r3_valu_f64_ubench.txt)
FP64_VALU_PEAK_TFS = 78.6  # MI355X FP64 vector peak: 1,024 SIMDs x 16 fma lanes x 2 flop x 2.4 GHz


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=None,
                    help="GPUs = ranks (default: WORLD_SIZE under a launcher, else 1); N > 1 without a launcher "
                         "runs N ranks through a torch.distributed.run child")
    ap.add_argument("--steps", type=int, default=1000)
    ap.add_argument("--warmup", type=int, default=100)
    ap.add_argument("--workload", choices=["cfg2", "cfg3", "cfg4", "cfg5"], default="cfg2",
                    help="cfg2: 65,536 chains per GPU at every N (the scaling line: the per-GPU shape does "
                         "not change with N); cfg5: 131,072 chains per GPU, overdispersed θinit (1,048,576 "
                         "chains at 8 GPUs), its own line")
    ap.add_argument("--shard", type=int, default=-1,
                    help="single-process run of shard r: global chains [r·C, (r+1)·C) (default: this rank's)")
    ap.add_argument("--chains-per-gpu", type=int, default=0,
                    help="0: 65,536 (cfg2) / 32,768 (cfg3) / 131,072 (cfg4)")
    ap.add_argument("--haario-k", type=int, default=200)
    ap.add_argument("--history-ring", type=int, default=0,
                    help="keep this many iterations of history on device (0 = all)")
    ap.add_argument("--stream-thin", type=int, default=0,
                    help="stream every k-th iteration's θ history to pinned host memory inside the timed "
                         "region (needs --history-ring; reports the PCIe-inclusive rate)")
    ap.add_argument("--history", choices=["full", "accept_only"], default="full")
    ap.add_argument("--ll-mode", choices=["per_obs", "suffstat"], default="per_obs")
    ap.add_argument("--lpc", type=int, default=0)
    ap.add_argument("--steps-per-launch", type=int, default=None,
                    help="steps per kernel launch (default 100; cfg 4: its readjust period k = 200, so every "
                         "launch group runs up to a readjust — +2.5%% against 100, profiles/r3_cfg4_k)")
    ap.add_argument("--variant", type=int, default=0,
                    help="emcmc_config.kernel_variant (EMCMC_VARIANT_* flags; same results, for A/B timing)")
    ap.add_argument("--reps", type=int, default=0,
                    help="repeat the timed region, report the median (0: 5 when the histories fit in 96 GB, else 1)")
    ap.add_argument("--cpu-seconds", type=float, default=10.0)
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--no-parity", action="store_true",
                    help="skip the oracle replay of each rank's first 4,096 chains (all, within the replay budget)")
    ap.add_argument("--no-kernel-timing", action="store_true",
                    help="A/B only: no dispatch events in the timed region (the line then has no kernel roofline)")
    ap.add_argument("--settle-ms", type=float, default=150.0,
                    help="run the same step kernel on a throwaway handle for this long before the warm-up steps, "
                         "so the timed steps see the steady-state clock (DESIGN.md §6: the clock bursts, dips, "
                         "then settles over ~40 ms of load); 0 disables")
    return ap.parse_args()


def host_info():
    """Host CPU facts for the baseline line: model, nproc, the cores this process may run on."""
    model = None
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                model = line.split(":", 1)[1].strip()
                break
    except OSError:
        pass
    try:
        affinity = len(os.sched_getaffinity(0))
    except AttributeError:
        affinity = os.cpu_count()
    quota = None  # the cgroup CPU quota in cores (cgroup v2 cpu.max "quota period"), if any
    try:
        q, per = open("/sys/fs/cgroup/cpu.max").read().split()[:2]
        if q != "max":
            quota = int(q) / int(per)
    except (OSError, ValueError):
        pass
    return {"cpu_model": model, "nproc": os.cpu_count(), "affinity_cores": affinity,
            "omp_num_threads_env": os.environ.get("OMP_NUM_THREADS"), "cgroup_cpu_quota_cores": quota}


def _time_oracle(step, chunk, seconds):
    step(1)  # warm (page faults, caches)
    it, steps = 1 + chunk, 0
    t0 = time.perf_counter()
    while time.perf_counter() - t0 < seconds:
        step(it)
        it += chunk
        steps += chunk
    return steps, time.perf_counter() - t0


def cpu_baseline(w, seconds, ll_mode):
    """The oracle (C restatement, OpenMP over chains) on a bounded sample of the
    same workload, histories included.  Threads = this GPU's CPU share: the
    OMP_NUM_THREADS the box sets (16 per GPU), else the cores in this process's
    affinity mask.  Also timed on 1 core, and (cfg 2) in the "faithful" variant
    that re-factorises Σ at every MvNormal construction like the reference
    (random_walk.jl:147,167; gsn_target.jl:20)."""
    from oracle import oracle as O

    hi = host_info()
    threads = int(os.environ.get("OMP_NUM_THREADS", "0") or 0) or hi["affinity_cores"] or 1
    mix = getattr(w, "haario_k", None) is not None
    mala = hasattr(w, "X")

    def make(T, faithful=False):
        if mala:  # cfg 3: MALA on the logistic target
            C, chunk = T, 2
            st = O.MALAState(np.zeros((C, w.D)), w.X, w.y, nthreads=T)

            def step(it):
                O.run_mala(st, seed=w.seed, eps=w.eps, X=w.X, y=w.y, iter0=it, nsteps=chunk, nthreads=T)
        elif mix:
            C, chunk = 256 * T, 50
            st = O.MixState(np.zeros((C, w.D)), sigma_b=w.sigma_b)

            def step(it):
                O.run_mix(st, seed=w.seed, sigma_a=w.rw_sigma, t_sigma=w.t_sigma, obs=w.obs, iter0=it, nsteps=chunk,
                          lam=w.lam, haario_k=w.haario_k, ll_mode=ll_mode, nthreads=T)
        else:
            C, chunk = 256 * T, (10 if faithful else 50)
            st = O.OracleState(np.zeros((C, w.D)))
            hist = O.alloc_history(C, w.D, chunk)
            mode = ll_mode | (0x200 if faithful else 0)

            def step(it):
                O.run_gsn(st, seed=w.seed, rw_sigma=w.rw_sigma, t_sigma=w.t_sigma, obs=w.obs, iter0=it, nsteps=chunk,
                          ll_mode=mode, nthreads=T, hist=hist)
        return C, chunk, step

    def rate(T, secs, faithful=False):
        C, chunk, step = make(T, faithful)
        steps, dt = _time_oracle(step, chunk, secs)
        return C * steps / dt, C, steps, dt

    v, C, steps, dt = rate(threads, 0.5 * seconds)
    v1, C1, steps1, dt1 = rate(1, 0.2 * seconds)
    out = {"value": v, "unit": "chain-steps/s", "cores": threads, "kind": "port", **hi,
           "single_core": {"value": v1, "sample": f"{C1} chains x {steps1} iterations, {dt1:.1f} s"},
           # the GPU box grants one GPU's process a CPU share (OMP_NUM_THREADS, 16) and asks that
           # pools stay within it; nproc / the affinity mask show the whole machine.  The whole
           # host's rate is therefore not measured: this is the single-core rate times the
           # affinity mask's cores (chains are independent; an upper bound, no memory contention)
           "all_host_cores_extrapolated": {"value": v1 * (hi["affinity_cores"] or 1),
                                           "cores": hi["affinity_cores"],
                                           "note": "single_core.value x affinity_cores, not measured: the box's "
                                                   "CPU share for one GPU is OMP_NUM_THREADS"}}
    if mala:
        out["sample"] = (f"{C} chains x {steps} iterations of the same MALA logistic workload (N={w.nobs}, D={w.D}), "
                         f"oracle/liboracle.so, {threads} threads, {dt:.1f} s")
        return out
    if not mix:
        vf, Cf, stepsf, dtf = rate(threads, 0.3 * seconds, faithful=True)
        out["faithful"] = {"value": vf, "cores": threads,
                           "sample": f"{Cf} chains x {stepsf} iterations, {dtf:.1f} s: a Cholesky of Σ at every "
                                     "MvNormal construction (rand, both logpdfs, P° and P set_parameters!) and a "
                                     "logdet per logpdf, as the reference; same bits as the factor-once oracle"}
    ac = hi["affinity_cores"] or 1
    if ac > threads:  # every core of the affinity mask, measured (the cgroup quota still caps their CPU time)
        va, Ca, stepsa, dta = rate(ac, 0.2 * seconds)
        out["all_affinity_cores_measured"] = {
            "value": va, "cores": ac, "sample": f"{Ca} chains x {stepsa} iterations, {dta:.1f} s",
            "note": "one OpenMP thread per core of the affinity mask; the box's cgroup CPU quota "
                    "(cgroup_cpu_quota_cores) caps the CPU time they get, so this is not the whole host's rate"}
        if not mix:
            vfa, Cfa, stepsfa, dtfa = rate(ac, 0.2 * seconds, faithful=True)
            out["all_affinity_cores_measured"]["faithful"] = {
                "value": vfa, "sample": f"{Cfa} chains x {stepsfa} iterations, {dtfa:.1f} s"}
    what = ("GaussianRandomWalkMix + HaarioTypeAdaptation(k=%d) + chain mean/cov" % w.haario_k) if mix else "RWM"
    out["sample"] = (f"{C} chains x {steps} iterations of the same D=32 {what} workload ({w.nobs} obs, "
                     f"{'per-observation' if ll_mode == 0 else 'sufficient-statistic'} log-likelihood, "
                     f"full histories), oracle/liboracle.so factor-once, {threads} threads, {dt:.1f} s")
    return out


def chains_per_gpu(workload, override=0):
    """Chains per GPU of a workload: the same for every world size, so a 1→8 GPU
    run is weak scaling of one per-GPU shape (cfg 5's 131,072 only when asked for)."""
    if override:
        return override
    return {"cfg2": 65536, "cfg3": 32768, "cfg4": 131072, "cfg5": 131072}[workload]


def timed_rep(eng, steps, barrier, run=None):
    """One timed repetition: barrier and synchronize on both sides, the clock
    between the two synchronizes only, so neither barrier's latency is inside the
    window (in a 0.18 ms window it would be a visible share).  Returns (this rank's
    seconds, the closing barrier's seconds); the caller takes the max over ranks."""
    barrier()
    eng.synchronize()
    t0 = time.perf_counter()
    (run or eng.run)(steps)
    eng.synchronize()
    dt = time.perf_counter() - t0
    tb = time.perf_counter()
    barrier()
    return dt, time.perf_counter() - tb


def reduce_over_ranks(x, dist, dev=None, op="max"):
    """max (times) or min (AND of 0/1 flags) of a float over every rank."""
    if dist is None:
        return x
    import torch

    t = torch.tensor([float(x)], dtype=torch.float64, device=dev)
    dist.all_reduce(t, op=dist.ReduceOp.MAX if op == "max" else dist.ReduceOp.MIN)
    return float(t.item())


STUB_ENV = "EMCMC_BENCH_STUB_ENGINE"


def engine_classes():
    """(Engine, EngineConfig) of the measured path: extensible_mcmc.engine over libemcmc.so.
    EMCMC_BENCH_STUB_ENGINE=1 swaps in tests/bench_stub.py, a do-nothing engine with the
    same methods, so CPU tests can drive the launcher and the rank plumbing of this file
    with gloo; such a line says "stub_engine": true and measures nothing."""
    if os.environ.get(STUB_ENV) == "1":
        import importlib.util

        spec = importlib.util.spec_from_file_location("bench_stub", ROOT / "tests" / "bench_stub.py")
        mod = importlib.util.module_from_spec(spec)
        spec.loader.exec_module(mod)
        return mod.Engine, mod.EngineConfig
    from extensible_mcmc.engine import Engine, EngineConfig

    return Engine, EngineConfig


def settle_clock(w, Cg, device, a, first, cfg3, cfg4, ll_mode):
    """Bring the GPU to its steady-state clock right before the timed steps: the same step
    kernel (same workload shape, full histories into a ring of one launch) on a throwaway
    handle for a.settle_ms of wall time.  Under this load the clock bursts for ~1 ms, dips
    for ~10 ms, then settles; the measured handle's chains are untouched.
    Returns (handle, info); the caller closes the handle after the timed region."""
    from extensible_mcmc import _lib as L

    Engine, EngineConfig = engine_classes()
    spl = 1 if cfg3 else a.steps_per_launch
    eng = Engine(EngineConfig(dim=w.D, num_chains=Cg, num_mcmc_steps=1 << 20,
                              seed=w.seed ^ 0x5E77, first_chain_id=first, device=device,
                              history_mode=L.HIST_FULL, lanes_per_chain=a.lpc, steps_per_launch=spl,
                              history_ring=spl, kernel_variant=a.variant))
    if cfg3:
        eng.add_mala_update(np.arange(w.D), w.eps)
        eng.set_logistic_target(w.X, w.y)
    elif cfg4:
        eng.add_gaussian_rw_mix_update(np.arange(w.D), w.rw_sigma, w.sigma_b, lam=w.lam, haario_k=w.haario_k)
    else:
        eng.add_gaussian_rw_update(np.arange(w.D), w.rw_sigma)
    if not cfg3:
        eng.set_gsn_target(w.mu_true, w.t_sigma, w.obs, ll_mode=ll_mode)
    eng.set_state(np.ascontiguousarray(np.broadcast_to(np.asarray(w.theta_init, dtype=np.float64), (Cg, w.D))))
    eng.synchronize(allow_faults=True)  # setup done before the clock starts to settle
    times, it, t0 = [], 1, time.perf_counter()
    while time.perf_counter() - t0 < a.settle_ms / 1e3:
        t1 = time.perf_counter()
        eng.run_iters(it, spl)
        eng.synchronize(allow_faults=True)
        times.append(time.perf_counter() - t1)
        it += spl
    # the handle is closed after the timed region: freeing it now would idle the GPU
    return eng, {"ms": (time.perf_counter() - t0) * 1e3, "launches": len(times), "steps_per_launch": spl,
                 "first_launch_ms": times[0] * 1e3 if times else None,
                 "last_launch_ms": times[-1] * 1e3 if times else None,
                 "note": "throwaway handle, same kernel and shape, between the warm-up steps and the timed "
                         "steps; not in the timed region"}


def _free_port():
    import socket

    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def launch_ranks(n: int) -> int:
    """--gpus n > 1 with no launcher: run this command line as n ranks of a fresh
    `torch.distributed.run` child (one rank per GPU, rendezvous on 127.0.0.1) and
    return its exit code.  A child process, never an exec; nothing in this process
    has imported torch or initialised a GPU.  The ranks inherit stdout, so the one
    JSON line rank 0 prints is this command's output."""
    import subprocess

    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}",
           "--master-addr=127.0.0.1", f"--master-port={_free_port()}", str(Path(__file__).resolve()), *sys.argv[1:]]
    env = dict(os.environ, HSA_ENABLE_IPC_MODE_LEGACY="0")  # dmabuf IPC only on this host driver (RCCL)
    sys.stdout.flush()
    return subprocess.run(cmd, env=env).returncode


def world_size(a) -> int:
    """The rank count this process belongs to; exits when --gpus and the launcher disagree."""
    env = os.environ.get("WORLD_SIZE")
    if env is None:
        return 1
    if a.gpus is not None and int(env) != a.gpus:
        sys.exit(f"bench.py: --gpus {a.gpus} but WORLD_SIZE={env}: the line would report "
                 f"{env} GPU(s); launch {a.gpus} ranks or pass --gpus {env}")
    return int(env)


def main():
    a = parse()
    if os.environ.get("WORLD_SIZE") is None and (a.gpus or 1) > 1:
        sys.exit(launch_ranks(a.gpus))
    world = world_size(a)
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    # EMCMC_BENCH_SHARED_DEVICE=1: every rank on device 0 with gloo (a rehearsal of
    # the torchrun path on a one-GPU box; RCCL needs one GPU per rank)
    stub = os.environ.get(STUB_ENV) == "1"
    shared = os.environ.get("EMCMC_BENCH_SHARED_DEVICE") == "1" or stub
    # EMCMC_BENCH_FORCE_NCCL=1: the RCCL process group even at world size 1 (RCCL init, the
    # device all-gather of the diagnostics and libemcmc beside torch's HIP context in one process)
    force_nccl = os.environ.get("EMCMC_BENCH_FORCE_NCCL") == "1" and not shared
    device = 0 if shared else local
    dist = None
    dev = None  # where the diagnostics all-gather runs
    if world > 1 or force_nccl:
        import torch
        import torch.distributed as dist

        if shared:
            dist.init_process_group("gloo")
        else:
            if torch.cuda.device_count() < world:  # one GPU per rank: never two ranks silently on one device
                sys.exit(f"bench.py: {world} ranks but {torch.cuda.device_count()} visible GPU(s)")
            torch.cuda.set_device(local)
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))
            dev = f"cuda:{local}"

    from extensible_mcmc import _lib as L
    from extensible_mcmc import diagnostics as DG
    from extensible_mcmc import workloads as W

    Engine, EngineConfig = engine_classes()
    cfg4 = a.workload == "cfg4"
    cfg3 = a.workload == "cfg3"
    # cfg 5 (131,072 chains per GPU, 1,048,576 over 8, overdispersed θinit) only when asked for:
    # the default line keeps cfg 2's 65,536 chains per GPU at every N
    cfg5 = a.workload == "cfg5"
    Cg = chains_per_gpu(a.workload, a.chains_per_gpu)
    first = (a.shard if a.shard >= 0 else rank) * Cg  # global id of this process's chain 0
    if cfg4:
        w = W.cfg4(Cg, k=a.haario_k)
    elif cfg3:
        w = W.cfg3(Cg)
    elif cfg5:
        w = W.cfg5(first + Cg)  # rows [first, first + Cg) are this shard's θinit whatever the world size
        w.theta_init = w.theta_init[first:]
        w.num_chains = Cg
    else:
        w = W.cfg2(Cg)
    if a.steps_per_launch is None:  # cfg 4: one launch group per readjust period
        a.steps_per_launch = w.haario_k if cfg4 else 100
    theta0 = np.broadcast_to(np.asarray(w.theta_init, dtype=np.float64), (Cg, w.D))
    ll_mode = L.LL_PER_OBS if a.ll_mode == "per_obs" else L.LL_SUFFSTAT
    hist = L.HIST_FULL if a.history == "full" else L.HIST_ACCEPT_ONLY
    reps = a.reps
    # every value rep is followed by a kernel-timing rep of the same launches (below), and
    # every timed step keeps its history slot: the repetitions' histories must fit in HBM
    rep_factor = 1 if a.no_kernel_timing else 2
    if reps <= 0:  # median of 5 value repetitions when all the histories fit in 96 GB of HBM
        per_iter = Cg * (16 * w.D + 8.125) if (hist == L.HIST_FULL and not a.history_ring) else 0
        reps = 5 if (a.warmup + rep_factor * 5 * a.steps) * per_iter <= 96e9 else 1
    timing_reps = 0 if a.no_kernel_timing else reps
    M = a.warmup + a.steps * (reps + timing_reps)
    eng = Engine(EngineConfig(dim=w.D, num_chains=Cg, num_mcmc_steps=M, seed=w.seed, first_chain_id=first,
                              device=device, history_mode=hist, lanes_per_chain=a.lpc,
                              steps_per_launch=a.steps_per_launch, history_ring=a.history_ring,
                              kernel_variant=a.variant))
    stream_bufs = None
    if a.stream_thin:
        assert a.history_ring > 0 and a.history_ring % a.stream_thin == 0 and a.steps % a.history_ring == 0
        from extensible_mcmc.engine import PinnedArray
        stream_bufs = PinnedArray((a.steps // a.stream_thin, 1, Cg, w.D), np.float64)
    if cfg3:
        eng.add_mala_update(np.arange(w.D), w.eps)
        eng.set_logistic_target(w.X, w.y)
    elif cfg4:
        eng.add_gaussian_rw_mix_update(np.arange(w.D), w.rw_sigma, w.sigma_b, lam=w.lam, haario_k=w.haario_k)
    else:
        eng.add_gaussian_rw_update(np.arange(w.D), w.rw_sigma)
    if not cfg3:
        eng.set_gsn_target(w.mu_true, w.t_sigma, w.obs, ll_mode=ll_mode)
    eng.set_state(np.ascontiguousarray(theta0))
    if a.warmup:
        eng.run_iters(1, a.warmup)
    eng.synchronize(allow_faults=cfg4)  # cfg 4: PosDef faults are counted and reported
    # the clock settles under load right before the timed steps (no idle gap in between)
    settle_eng, settle = settle_clock(w, Cg, device, a, first, cfg3, cfg4, ll_mode) if a.settle_ms > 0 \
        else (None, None)

    def barrier():
        if dist is not None:
            if shared:
                dist.barrier()
            else:
                dist.barrier(device_ids=[local])

    class _Sync:  # the engine's synchronize for timed_rep (cfg 4: PosDef faults are counted, not raised)
        def synchronize(self):
            eng.synchronize(allow_faults=cfg4)  # hipStreamSynchronize of the engine's stream (+ a 4-byte fault flag)

    # Timed repetitions alternate: a value rep (the launches alone, no dispatch events:
    # `value` and `ms_per_step` are the median of these walls) and a kernel-timing rep of
    # the same launches, each carrying its own start/stop dispatch events (hipExtLaunchKernel),
    # whose kernel time feeds roofline.achieved.  The events cost the 20-step window ≈ 5%
    # of its wall (8.35–8.42e9 without vs 7.71–8.03e9 with, profiles/r4_s10/), so they
    # stay out of the value reps.
    times, kern, barrier_s, kwall = [], [], [], []
    it = a.warmup + 1
    for r in range(reps + timing_reps):
        value_rep = a.no_kernel_timing or r % 2 == 0
        # the rep's (mcmciter, pidx) schedule is built before the clock starts
        steps = np.stack([np.arange(it, it + a.steps, dtype=np.uint32), np.ones(a.steps, dtype=np.uint32)], axis=1)
        eng.set_timing(not value_rep)

        def run(steps, it=it):
            if stream_bufs is None:
                eng.run(steps)
                return
            # half a ring per chunk: a chunk's thinned θ history leaves while the next chunk runs
            ch = a.history_ring // 2 if a.history_ring >= 2 * a.stream_thin else a.history_ring
            for c0 in range(0, a.steps, ch):
                eng.run(steps[c0:c0 + ch])
                k0 = c0 // a.stream_thin
                eng.stream_history(L.H_STATE, it + c0 + a.stream_thin - 1, ch // a.stream_thin, thin=a.stream_thin,
                                   out=stream_bufs[k0:k0 + ch // a.stream_thin])
            eng.stream_wait()

        dt, bs = timed_rep(_Sync(), steps, barrier, run)
        ms, launches, nbytes = eng.get_timing(reset=True)
        eng.set_timing(False)
        if value_rep:
            if a.no_kernel_timing:  # placeholders: the wall clock stands in for the kernel time
                kern.append((dt * 1e3, 1, 1.0))
            times.append(reduce_over_ranks(dt, dist, dev, "max"))  # the slowest rank's window
            barrier_s.append(bs)
        else:
            kern.append((ms, launches, nbytes))
            kwall.append(reduce_over_ranks(dt, dist, dev, "max"))
        it += a.steps
    if settle_eng is not None:
        settle_eng.close()
    order = np.argsort(times)
    mid = int(order[len(order) // 2])
    dt = times[mid]
    korder = np.argsort([k[0] for k in kern])
    ms, launches, nbytes = kern[int(korder[len(korder) // 2])]  # the median kernel-timing rep

    # diagnostics over the first timed window, through the C ABI (emcmc_diagnostics): one
    # all-gather of 3·D+3 doubles per rank — ncclAllGather inside libemcmc on an RCCL comm
    # (nccl process group), the host-callback comm over gloo — Chan-merged in rank order
    diag, diag_via, diag_stuck = None, None, False
    if hist == L.HIST_FULL and not a.history_ring and a.steps >= 4:
        if dist is None:
            diag = eng.diagnostics(a.warmup + 1, a.steps, split=True)
            diag_via = "emcmc_diagnostics, this rank alone"
        else:
            def gathered(make, label):
                comm = make()
                try:
                    d = eng.diagnostics(a.warmup + 1, a.steps, split=True, comm=comm)
                finally:
                    comm.close()
                return d, f"emcmc_diagnostics over {label}, {d['nranks']} ranks"

            def agree(ok):
                """every rank's verdict on its last diagnostics collective (MIN over the ranks), so
                that no rank takes the fallback collective while another moves on to the parity
                reduction; None when the agreement itself does not complete"""
                v, e = watchdog(lambda: reduce_over_ranks(1.0 if ok else 0.0, dist, dev, "min"), 60.0)
                return None if e is not None else v == 1.0

            if shared:
                res, err = watchdog(lambda: gathered(DG.Comm.torch_host, "a host all-gather (gloo)"), 120.0)
            else:
                res, err = watchdog(lambda: gathered(lambda: DG.Comm.from_process_group(local),
                                                     "RCCL (ncclAllGather inside libemcmc)"), 120.0)
                if err != "timeout":
                    all_ok = agree(err is None)
                    if all_ok is None:
                        err = "timeout"
                    elif not all_ok:  # a rank's RCCL comm failed: every rank merges through torch's all-gather
                        why = (err or "on another rank")[:160]
                        res, err = watchdog(lambda: gathered(lambda: DG.Comm.torch_host(device=dev),
                                                             f"torch's all-gather (RCCL comm failed: {why})"), 120.0)
                        if err != "timeout" and not agree(err is None):
                            err = err or "the fallback all-gather failed on another rank"
            if err is None:
                diag, diag_via = res
            else:  # measured already; report without diagnostics and do not wait on a stuck collective
                diag_via, diag_stuck = f"diagnostics failed: {err[:200]}", True

    # parity on every rank: its first 4,096 chains (all of them within the replay budget)
    # replayed on the oracle after the timed region, AND-reduced over the ranks
    par = None
    if not a.history_ring and not a.no_parity and not diag_stuck:
        try:
            par = parity_replay(eng, w, a, ll_mode, first, reps + timing_reps)
            nbad = par["mismatched_chains"]
        except Exception as e:
            par, nbad = {"error": repr(e)}, -1
        if dist is not None:
            par["ranks"] = world
            worst = reduce_over_ranks(1.0 if nbad == 0 else 0.0, dist, dev, "min")
            par["all_ranks_bitwise"] = worst == 1.0

    if rank != 0:
        if diag_stuck:
            os._exit(0)  # a collective may still be pending on the stream: no teardown
        dist.destroy_process_group()
        return

    total_chains = Cg * world
    value = total_chains * a.steps / dt
    avg_launch_s = ms / 1e3 / launches
    bytes_per_launch = nbytes / launches
    achieved = bytes_per_launch / avg_launch_s / 1e9
    traffic = None
    pmc = ROOT / "profiles" / "pmc_traffic.json"
    kname = eng.kernel_name()
    traffic_src = None
    if pmc.exists():  # measured HBM bytes per launch of this kernel at this launch length and chain count
        try:
            tb = json.loads(pmc.read_text()).get(kname, {}).get("by_steps_per_launch", {})
            e = tb.get(str(int(round(a.steps / launches))))
            if e and e.get("chains") == Cg:
                traffic, traffic_src = e["traffic_per_launch"], e["source"]
        except Exception:
            traffic = None

    out = {
        "metric": "MCMC steps×chains/sec on D=32 Gaussian, 1/2/4/8 MI355X; accept-rate parity",
        "value": value,
        "unit": "chain-steps/s",
        "n_gpus": world,
        "steps": a.steps,
        "warmup": a.warmup,
        "ms_per_step": dt / a.steps * 1e3,
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "f64",
        "data": ("synthetic (X ~ N(0, 1/D), θ* ~ N(0, I), y ~ Bernoulli(σ(Xθ*)), numpy default_rng(20261018)), "
                 "θinit = 0" if cfg3 else
                 "synthetic (GsnTargetLaw(μ*, I32), 10 obs from numpy default_rng(20261015)), " +
                 ("θinit = x̄ + 3z/√n overdispersed (z from default_rng(20261016), row = global chain id)" if cfg5
                  else "θinit = 0")),
        "config": {
            "workload": (f"BASELINE cfg 3: {Cg} MALA chains per GPU on a logistic-regression log-likelihood, "
                         f"N={w.nobs}, D={w.D}, fp64" if cfg3 else
                         f"BASELINE cfg 4: {Cg} adaptive RWM chains per GPU (GaussianRandomWalkMix + "
                         f"HaarioTypeAdaptation, per-chain running mean/cov on device), D=32 Gaussian target, fp64"
                         if cfg4 else
                         (f"BASELINE cfg 5: chains sharded over MI355X GPUs, {Cg} per GPU (1,048,576 at 8 GPUs), "
                          f"here {world} GPU(s) = {Cg * world} chains, D=32 Gaussian target, fp64; cross-chain "
                          "split-R̂ moments all-gathered once after the timed region" if cfg5 else
                          f"BASELINE cfg 2: {Cg} independent RWM chains per GPU at every GPU count (weak "
                          f"scaling of one per-GPU shape), here {world} GPU(s) = {Cg * world} chains, D=32 "
                          "Gaussian target, fp64")),
            "chains_per_gpu": Cg,
            "total_chains": total_chains, "first_chain_id": first,
            "dim": w.D,
            "num_obs": w.nobs,
            "proposal": (f"MALA(ϵ={w.eps:.4g})" if cfg3 else
                         f"GaussianRandomWalkMix(σ²I32, σ²I32, λ={w.lam}) + HaarioTypeAdaptation(k={w.haario_k})"
                         if cfg4 else "GaussianRandomWalk(σ²I32), σ=2.38/√(D·n)"),
            "prior": "ImproperPrior",
            "history": a.history,
            "ll_mode": a.ll_mode,
            "chain_stats": ("rolling acceptance (chain_statistics.jl:51-65)" if cfg3 else
                            "rolling acceptance + running mean/cov (chain_statistics.jl:41-66)" if cfg4
                            else "rolling acceptance (chain_statistics.jl:51-65)"),
            "steps_per_launch": a.steps_per_launch,
            "clock_settle": settle,
            "kernel": kname,
            "parallelism": f"chain-sharded x{world}",
            "process_group": None if dist is None else ("gloo" if shared else "nccl"),
        },
        "roofline": {
            "bound": "hbm",
            "achieved": achieved,
            "peak": HBM_PEAK_GBS,
            "unit": "GB/s",
            "frac": achieved / HBM_PEAK_GBS,
            "traffic": traffic,
            "traffic_source": traffic_src,
            "kernel": kname,
            "algorithmic_bytes_per_launch": bytes_per_launch,
            "avg_launch_ms": avg_launch_s * 1e3,
            "launches": launches,
            "bytes_per_chain_step": bytes_per_launch / (Cg * a.steps / launches),
        },
        "kernel_chain_steps_per_s": Cg * a.steps / (ms / 1e3),
        "reps": reps,
        "times_s": times,
        "kernel_timing_reps": {"n": timing_reps, "wall_s": kwall,
                               "kernel_ms": [k[0] for k in kern] if timing_reps else None,
                               "note": "each value rep is followed by one rep of the same launches with dispatch "
                                       "events (hipExtLaunchKernel start/stop); roofline.achieved and "
                                       "kernel_chain_steps_per_s come from their median kernel time, value from "
                                       "the event-free reps"},
        "timing": {"window": "between the engine synchronizes after the opening barrier and before the closing "
                             "one; max over ranks (barriers outside the window)",
                   "closing_barrier_ms_rank0": [b * 1e3 for b in barrier_s]},
    }
    out["roofline"]["achievable"] = {"peak": HBM_ACHIEVABLE_GBS, "frac": achieved / HBM_ACHIEVABLE_GBS,
                                     "source": "MI355X_MICROARCH.md:36 (6.29 TB/s measured, float4 copy)"}
    # the same bytes on the wall clock of the timed region (host launch + synchronize included)
    e2e = bytes_per_launch * launches / dt / 1e9
    out["roofline"]["end_to_end"] = {"achieved": e2e, "frac": e2e / HBM_PEAK_GBS,
                                     "note": "this rank's algorithmic bytes over the timed region's wall clock"}
    if cfg4:  # HIP events bracket the launch group, and its bytes cover all three kernels
        out["roofline"]["timed_region"] = ("per launch group: mix_gsn_kernel (steps) + mix_moments_kernel (batched "
                                           "GenericChainStats mean/cov) + mix_readjust_kernel when Haario is due")
    if cfg4:  # the group is VALU-issue bound, not HBM-bound: fp64 rate and VALU busy next to the HBM figure
        pc = ROOT / "profiles" / "pmc_compute.json"
        try:
            ent = json.loads(pc.read_text()).get(kname) if pc.exists() else None
        except Exception:
            ent = None
        if ent:
            ks = ent["kernels"]
            # measured fp64 flop of one launch group (step + moments, readjust when due) at this shape,
            # per step of the PMC pass's launch length, times this run's steps per launch
            grp = sum(k["fp64_tflops"] * k["avg_ns"] * 1e3 * (k.get("per_group", 1.0)) for k in ks.values())
            grp *= (a.steps / launches) / float(ent.get("steps_per_launch", 100))
            step_k = next((v for n, v in ks.items() if n.startswith("mix_res") or n.startswith("mix_gsn")), None)
            mom_k = next((v for n, v in ks.items() if n.startswith("mix_moments")), None)
            live = grp / avg_launch_s / 1e12
            out["roofline"]["compute"] = {
                "bound": "valu issue (fp64)", "unit": "TFLOP/s", "peak": FP64_VALU_PEAK_TFS,
                "achieved": live, "frac": live / FP64_VALU_PEAK_TFS,
                "note": "fp64 flop per launch group from the PMC pass (64 lanes x (2 FMA + MUL + ADD) per "
                        "wave-instruction) over this run's HIP-event group time; a fp64 mul or add issues like "
                        "an fma, so the flop fraction understates the issue fraction: valu_busy is that",
                "valu_busy": {"step_kernel": step_k and step_k["valu_busy"],
                              "moments_kernel": mom_k and mom_k["valu_busy"]},
                "fp64_share_of_valu": {"step_kernel": step_k and step_k["f64_share_of_valu"],
                                       "moments_kernel": mom_k and mom_k["f64_share_of_valu"]},
                "measured_valu_ceiling": {
                    "value": FP64_VALU_MEASURED_TFS, "frac": live / FP64_VALU_MEASURED_TFS,
                    "source": "profiles/r3_valu_f64_ubench.txt (scripts/ubench/valu_f64_rate.hip: v_fma_f64, 8 "
                              "independent chains per lane, 2 waves/SIMD as these kernels run; 59.5 at 4)"},
                "source": ent["source"]}
            # the binding limit is VALU issue (both kernels; the HBM fraction is ≈ 0.17): the
            # compute roofline is the line's primary figure, the HBM one its secondary
            hbm = out["roofline"]
            comp = hbm.pop("compute")
            out["roofline"] = {"bound": "valu", "achieved": comp["achieved"], "peak": comp["peak"],
                               "unit": comp["unit"], "frac": comp["frac"], "traffic": hbm["traffic"],
                               "kernel": kname, "valu_busy": comp["valu_busy"],
                               "fp64_share_of_valu": comp["fp64_share_of_valu"],
                               "measured_valu_ceiling": comp["measured_valu_ceiling"], "note": comp["note"],
                               "source": comp["source"], "secondary_hbm": hbm}
    if cfg3:  # MFMA-bound: the two contractions, 4·N·D flop per chain-step
        flops = 4.0 * w.nobs * w.D * Cg * (a.steps / launches)
        tfs = flops / avg_launch_s / 1e12
        out["roofline"] = {"bound": "mfma", "achieved": tfs, "peak": FP64_MFMA_PEAK_TFS, "unit": "TFLOP/s",
                           "frac": tfs / FP64_MFMA_PEAK_TFS, "traffic": traffic, "kernel": kname,
                           "measured_mfma_ceiling": {
                               "value": FP64_MFMA_MEASURED_TFS, "frac": tfs / FP64_MFMA_MEASURED_TFS,
                               "source": "profiles/r3_mfma_f64_ubench.txt (scripts/ubench/mfma_f64_chain.hip: "
                                         "back-to-back v_mfma_f64_16x16x4f64, 8 independent accumulators, "
                                         "4 waves/SIMD)"},
                           "algorithmic_flops_per_launch": flops, "avg_launch_ms": avg_launch_s * 1e3,
                           "launches": launches, "flops_per_chain_step": 4.0 * w.nobs * w.D}
    if stream_bufs is not None:
        sb = stream_bufs.nbytes
        out["streaming"] = {"history_ring": a.history_ring, "thin": a.stream_thin, "host_bytes": sb,
                            "d2h_gb_per_s": sb / dt / 1e9,
                            "note": "value here includes the D2H stream of every thin-th θ history slot (PCIe)"}
    if cfg4:
        out["posdef_faulted_chains"] = int(np.count_nonzero(eng.get_faults() & L.FAULT_POSDEF))
    if diag is not None:
        w0, w1 = a.warmup + 1, a.warmup + a.steps
        # D = 32 RWM from θinit needs ≈ 1,000 iterations of burn-in (tests/test_gpu_fullsize.py
        # test_posterior_matches_analytic): a window that starts earlier is a plumbing check of
        # the on-device reduction and the all-gather, not convergence evidence
        burn_in = w0 <= BURN_IN_ITERS
        out["diagnostics"] = {
            "window_iterations": [w0, w1], "chains_merged": diag["num_chains"], "via": diag_via,
            "accept_rate": diag["accept_rate"],
            ("plumbing_check_split_rhat_max" if burn_in else "max_split_rhat"): float(np.max(diag["rhat"])),
            "purpose": ("plumbing check, burn-in window: these moments exercise the device reduction and the "
                        "rank merge (emcmc_diagnostics); chains started at θinit %s are still in burn-in over "
                        "iterations %d–%d, so R̂ > 1 here is expected and is not a convergence result (that is "
                        "tests/test_gpu_fullsize.py::test_posterior_matches_analytic, iterations 2001–4000)"
                        % ("= 0" if not cfg5 else "overdispersed", w0, w1)) if burn_in else
                       "convergence diagnostic over a post-burn-in window"}
        if not cfg3:
            key = "plumbing_check_max_abs_mean_minus_xbar" if burn_in else "max_abs_mean_minus_xbar"
            out["diagnostics"][key] = float(np.max(np.abs(diag["mean"] - w.obs.mean(0))))
    elif diag_via is not None:
        out["diagnostics"] = {"error": diag_via}
    if world == 1 and not a.no_cpu:
        try:
            out["cpu_baseline"] = cpu_baseline(w, a.cpu_seconds, ll_mode)
            out["gpu_over_cpu"] = value / out["cpu_baseline"]["value"]
        except Exception as e:  # the oracle is a reported baseline, never the measured path
            out["cpu_baseline"] = {"error": repr(e)}
    if par is not None:
        out["parity"] = par
    if stub:
        out["stub_engine"] = True
        out["data"] = "STUB ENGINE (tests/bench_stub.py): launcher and rank plumbing only, nothing measured"
    print(json.dumps(out), flush=True)
    if diag_stuck:
        os._exit(0)  # a collective may still be pending on the engine's stream: no teardown
    eng.close()
    if dist is not None:
        dist.destroy_process_group()


def watchdog(fn, seconds):
    """(fn(), None), or (None, "timeout") when fn has not returned after `seconds`, or
    (None, repr(exception)): the diagnostics collective runs after the timed region, and a
    rank that never joins it must not turn a finished measurement into a hung job."""
    import threading

    box = {}

    def run():
        try:
            box["v"] = fn()
        except BaseException as e:  # noqa: BLE001 — reported in the line
            box["e"] = repr(e)

    t = threading.Thread(target=run, daemon=True)
    t.start()
    t.join(seconds)
    if t.is_alive():
        return None, "timeout"
    return box.get("v"), box.get("e")


BURN_IN_ITERS = 2000  # diagnostics windows starting at or before this iteration are labelled burn-in
# the oracle's accept-only replay after the timed region: ~REPLAY_SECONDS of its measured rate on
# 16 threads (profiles/r6_bench: 2.3e7 chain-steps/s on cfg 2 / 5, 1.0e7 on cfg 4), so the
# driver's 20-step line and the 1000-step default replay every chain, cfg 4 / cfg 5 ≥ 4,096
REPLAY_SECONDS = 10.0
REPLAY_RATE_16T = {"gsn": 2.0e7, "mix": 0.9e7}


def parity_replay(eng, w, a, ll_mode, first=0, reps=1, n=4096):
    """the accept bitstream of the rank's first chains (global ids first + c)
    over EVERY iteration this handle ran (warm-up and all timed repetitions), replayed on the
    oracle in its accept-only mode, plus each chain's final θ and ll; the count of chains
    whose stream or state differs is reported.  As many chains as the replay budget holds
    (REPLAY_SECONDS at the oracle's rate; all of them for the driver's 20-step line and the
    1000-step default), at least n.  cfg 3 (MALA: 4·N·D flop per oracle chain-step) replays
    the first 20 iterations of 2 chains."""
    from extensible_mcmc import _lib as L
    from oracle import oracle as O

    S = a.warmup + a.steps * reps
    threads = int(os.environ.get("OMP_NUM_THREADS", "0") or 0) or (host_info()["affinity_cores"] or 1)
    threads = max(1, min(threads, 16))
    t0 = time.perf_counter()
    if hasattr(w, "X"):  # MALA: the first 20 iterations of 2 chains, θ at the last replayed iteration
        S = min(S, 20)
        acc = eng.get_history(L.H_ACCEPT, 1, S)[:, 0]
        hist_theta = eng.get_history(L.H_STATE, S, 1)[0, 0]
        bad = 0
        for c in (0, w.num_chains - 1):
            st = O.MALAState(np.zeros((1, w.D)), w.X, w.y, nthreads=threads)
            h = O.run_mala(st, seed=w.seed, eps=w.eps, X=w.X, y=w.y, iter0=1, nsteps=S, chain0=first + int(c),
                           nthreads=threads)
            bad += int(not (np.array_equal(acc[:, c], h["acc"][:, 0]) and np.array_equal(hist_theta[c], st.theta[0])))
        return {"chains_replayed": 2, "iterations": int(S), "mismatched_chains": bad,
                "accept_stream_bitwise": bad == 0, "theta_at_last_replayed_iteration_bitwise": bad == 0,
                "replay_s": time.perf_counter() - t0, "oracle_threads": threads}
    rate = REPLAY_RATE_16T["mix" if w.haario_k is not None else "gsn"] * threads / 16.0
    fit = int(rate * REPLAY_SECONDS / S) // 64 * 64  # chains whose whole run fits the replay budget
    C = min(w.num_chains, max(n, fit))
    C -= C % 64 if C > 64 else 0  # whole accept words
    init = np.ascontiguousarray(np.broadcast_to(np.asarray(w.theta_init, dtype=np.float64), (w.num_chains, w.D))[:C])
    if w.haario_k is not None:
        st = O.MixState(np.zeros((C, w.D)), sigma_b=w.sigma_b)
        h = O.run_mix(st, seed=w.seed, sigma_a=w.rw_sigma, t_sigma=w.t_sigma, obs=w.obs, iter0=1, nsteps=S,
                      lam=w.lam, haario_k=w.haario_k, chain0=first, ll_mode=ll_mode, accept_only=True, nthreads=threads)
    else:
        st = O.OracleState(init)
        h = O.run_gsn(st, seed=w.seed, rw_sigma=w.rw_sigma, t_sigma=w.t_sigma, obs=w.obs, iter0=1, nsteps=S,
                      chain0=first, ll_mode=ll_mode, accept_only=True, nthreads=threads)
    got = eng.get_history_bits(1, S)[:, 0, :(C + 63) // 64]
    bad_acc = O.accept_mismatch_chains(got, O.pack_accept(h["acc"]), C)
    theta, ll = eng.get_state()
    bad_th = np.flatnonzero((theta[:C] != st.theta).any(axis=1) | (ll[:C] != st.ll))
    bad = np.union1d(bad_acc, bad_th)
    return {"chains_replayed": int(C), "chain_ids": [int(first), int(first + C - 1)], "iterations": int(S),
            "mismatched_chains": int(bad.size), "accept_stream_mismatched_chains": int(bad_acc.size),
            "final_theta_ll_mismatched_chains": int(bad_th.size),
            "accept_stream_bitwise": bad_acc.size == 0, "final_theta_ll_bitwise": bad_th.size == 0,
            "replay_s": time.perf_counter() - t0, "oracle_threads": threads,
            "note": "every iteration this handle ran (warm-up + value and kernel-timing reps), oracle/liboracle.so "
                    "accept-only mode, compared after the timed region"}


if __name__ == "__main__":
    main()
