"""Multi-process chain sharding on CPU (torch.distributed gloo, world_size 2).

The N>1 path of bench.py/extensible_mcmc shards chains by global id with no
data-path collective and all-gathers the cross-chain diagnostics once.  Here
each rank advances its shard with the oracle (no GPU in this container; the
engine's shards are exercised by tests/test_gpu_cfg5.py), reduces its shard's
split-chain moments and all-gathers them through
extensible_mcmc.diagnostics.allgather_moments (Chan merge in rank order); the
result must equal the single-process reduction, and per-chain states must equal
the unsharded run (RNG keyed by global chain id)."""
import os
import socket
import sys
from pathlib import Path

import numpy as np
import pytest

ROOT = Path(__file__).resolve().parent.parent


def shard_moments(hist_theta, split=True):
    """Per-(half-)chain mean/var over the window, reduced over chains — the
    host restatement of chain_moments_kernel + moments_reduce_kernel."""
    from extensible_mcmc import diagnostics as DG

    S, C, D = hist_theta.shape
    halves = 2 if split else 1
    ln = S // halves
    parts = [hist_theta[h * ln:(h + 1) * ln] for h in range(halves)]
    means = np.concatenate([p.mean(axis=0) for p in parts])  # [halves*C][D]
    vars_ = np.concatenate([p.var(axis=0, ddof=1) for p in parts])
    return DG.from_chain_moments(means, vars_, ln)


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, out_dir):
    sys.path[:0] = [str(ROOT), str(ROOT / "extensiblemcmc.jl_amd")]
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    import torch.distributed as dist

    from extensible_mcmc import diagnostics as DG
    from extensible_mcmc import workloads as W
    from oracle import oracle as O

    dist.init_process_group("gloo", rank=rank, world_size=world)
    w = W.cfg5(256, D=8)
    per = 256 // world
    lo = rank * per
    st = O.OracleState(w.theta_init[lo:lo + per])
    h = O.run_gsn(st, seed=w.seed, rw_sigma=w.rw_sigma, t_sigma=w.t_sigma, obs=w.obs, iter0=1, nsteps=120,
                  chain0=lo)
    m = shard_moments(h["theta"][20:])
    m["accepted"] = int(h["acc"][20:].sum())
    m["proposed"] = int(h["acc"][20:].size)
    tot = DG.allgather_moments(m, w.D)
    np.save(os.path.join(out_dir, f"theta_{rank}.npy"), st.theta)
    if rank == 0:
        np.save(os.path.join(out_dir, "reduced.npy"), DG.pack(tot))
    dist.barrier()
    dist.destroy_process_group()


def test_two_rank_sharding_and_diagnostics(tmp_path, oracle):
    import torch.multiprocessing as mp

    from extensible_mcmc import diagnostics as DG
    from extensible_mcmc import workloads as W

    mp.spawn(_worker, args=(2, _free_port(), str(tmp_path)), nprocs=2, join=True)
    w = W.cfg5(256, D=8)
    st = oracle.OracleState(w.theta_init[:256])
    h = oracle.run_gsn(st, seed=w.seed, rw_sigma=w.rw_sigma, t_sigma=w.t_sigma, obs=w.obs, iter0=1, nsteps=120)
    # per-chain results do not depend on the sharding
    sharded = np.concatenate([np.load(tmp_path / "theta_0.npy"), np.load(tmp_path / "theta_1.npy")])
    assert np.array_equal(sharded, st.theta)
    # the all-gathered, merged diagnostics equal the single-process reduction
    ref = shard_moments(h["theta"][20:])
    ref["accepted"], ref["proposed"] = int(h["acc"][20:].sum()), int(h["acc"][20:].size)
    got = DG.unpack(np.load(tmp_path / "reduced.npy"), w.D, ref["num_draws"])
    for k in ("mean", "sum_var"):
        np.testing.assert_allclose(got[k], ref[k], rtol=1e-12)
    np.testing.assert_allclose(got["m2"], ref["m2"], rtol=1e-10)
    assert got["num_chains"] == ref["num_chains"] and got["accepted"] == ref["accepted"]
    r_got, r_ref = DG.rhat_from_moments(got), DG.rhat_from_moments(ref)
    np.testing.assert_allclose(r_got["rhat"], r_ref["rhat"], rtol=1e-10)
    assert r_got["accept_rate"] == r_ref["accept_rate"]


def test_chan_merge_does_not_cancel():
    """1M chain means at 1e8 ± 1e-3: Σm² − (Σm)²/m loses every digit of M2, the
    Chan merge of 8 shards keeps it (the cfg 5 shape)."""
    from extensible_mcmc import diagnostics as DG

    rng = np.random.default_rng(5)
    means = 1e8 + 1e-3 * rng.standard_normal((1 << 20, 2))
    vars_ = np.ones_like(means)
    exact = ((means - means.mean(0)) ** 2).sum(0)
    shards = [DG.from_chain_moments(m, v, 100) for m, v in zip(np.split(means, 8), np.split(vars_, 8))]
    got = DG.merge(shards)
    np.testing.assert_allclose(got["m2"], exact, rtol=1e-5)
    naive = (means * means).sum(0) - means.sum(0) ** 2 / means.shape[0]
    assert np.all(np.abs(naive - exact) > 1e3 * np.abs(got["m2"] - exact))
    assert got["num_chains"] == 1 << 20


class _SleepEngine:
    """A stand-in for one rank's engine: run() takes a fixed time."""

    def __init__(self, secs):
        self.secs = secs

    def synchronize(self):
        pass

    def run(self, steps):
        import time

        time.sleep(self.secs)


def _bench_worker(rank, world, port, out_dir):
    sys.path[:0] = [str(ROOT), str(ROOT / "extensiblemcmc.jl_amd")]
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    import json

    import torch.distributed as dist

    import bench

    dist.init_process_group("gloo", rank=rank, world_size=world)
    eng = _SleepEngine(0.02 if rank == 0 else 0.4)
    dt, bs = bench.timed_rep(eng, None, dist.barrier)
    dmax = bench.reduce_over_ranks(dt, dist, None, "max")
    # rank 1's replay disagrees: the AND over ranks is false on every rank
    all_ok = bench.reduce_over_ranks(0.0 if rank == 1 else 1.0, dist, None, "min") == 1.0
    with open(os.path.join(out_dir, f"bench_{rank}.json"), "w") as f:
        json.dump({"dt": dt, "barrier": bs, "dmax": dmax, "all_ok": all_ok,
                   "cg": [bench.chains_per_gpu(wl) for wl in ("cfg2", "cfg3", "cfg4", "cfg5")]}, f)
    dist.barrier()
    dist.destroy_process_group()


def test_bench_scaling_line_two_ranks(tmp_path):
    """bench.py's N > 1 path on 2 gloo ranks: the timed window holds no barrier (a
    fast rank's own window is its own run, the wait for the slow rank shows up in
    the closing barrier), the line's time is the max over ranks, the per-GPU chain
    count does not depend on the world size, and parity is AND-reduced over ranks."""
    import json

    import torch.multiprocessing as mp

    mp.spawn(_bench_worker, args=(2, _free_port(), str(tmp_path)), nprocs=2, join=True)
    r0, r1 = (json.loads((tmp_path / f"bench_{r}.json").read_text()) for r in (0, 1))
    assert r0["dt"] < 0.2, r0  # rank 0 did not wait for rank 1 inside its window
    assert r0["barrier"] > 0.2, r0  # it waited in the closing barrier instead
    assert r1["dt"] >= 0.4
    assert r0["dmax"] == r1["dmax"] == max(r0["dt"], r1["dt"])
    assert r0["all_ok"] is False and r1["all_ok"] is False
    assert r0["cg"] == r1["cg"] == [65536, 32768, 131072, 131072]


def _diag_c_worker(rank, world, port, out_dir):
    """Each rank: its shard's record through the library's host-callback comm
    (emcmc_comm_init_host + emcmc_diagnostics_merge, over gloo) and through the
    Python all-gather + merge; both results saved for the parent to compare."""
    sys.path[:0] = [str(ROOT), str(ROOT / "extensiblemcmc.jl_amd")]
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    import torch.distributed as dist

    from extensible_mcmc import diagnostics as DG
    from extensible_mcmc import workloads as W
    from oracle import oracle as O

    dist.init_process_group("gloo", rank=rank, world_size=world)
    w = W.cfg5(192, D=6)
    per = 192 // world
    lo = rank * per
    st = O.OracleState(w.theta_init[lo:lo + per])
    h = O.run_gsn(st, seed=w.seed, rw_sigma=w.rw_sigma, t_sigma=w.t_sigma, obs=w.obs, iter0=1, nsteps=80, chain0=lo)
    m = shard_moments(h["theta"][16:])
    m["accepted"] = int(h["acc"][16:].sum())
    m["proposed"] = int(h["acc"][16:].size)
    comm = DG.Comm.torch_host()
    c = DG.merge_c(DG.pack(m), w.D, m["num_draws"], comm)
    py = DG.rhat_from_moments(DG.allgather_moments(m, w.D))
    # an all-gather that raises: the exception comes back through the C ABI, not a crash
    bad = DG.Comm.host(world, rank, lambda s: (_ for _ in ()).throw(KeyError("boom")))
    try:
        DG.merge_c(DG.pack(m), w.D, m["num_draws"], bad)
        raised = None
    except KeyError as e:
        raised = str(e)
    np.savez(os.path.join(out_dir, f"diag_{rank}.npz"), c_rhat=c["rhat"], c_mean=c["mean"], c_W=c["W"], c_B=c["B"],
             py_rhat=py["rhat"], py_mean=py["mean"], py_W=py["W"], py_B=py["B"],
             scal=np.array([c["accept_rate"], py["accept_rate"], c["num_chains"], c["nranks"], c["max_rhat"]]),
             raised=np.array([raised or ""]))
    comm.close()
    bad.close()
    dist.barrier()
    dist.destroy_process_group()


def test_two_rank_diagnostics_through_the_c_abi(tmp_path, oracle):
    """emcmc_diagnostics_merge over a host all-gather (the callback form an MPI or gloo
    caller passes through the C ABI): every rank gets the Python reduction's bits."""
    import torch.multiprocessing as mp

    mp.spawn(_diag_c_worker, args=(2, _free_port(), str(tmp_path)), nprocs=2, join=True)
    r0, r1 = (np.load(tmp_path / f"diag_{r}.npz") for r in (0, 1))
    for r in (r0, r1):
        for k in ("rhat", "mean", "W", "B"):
            assert np.array_equal(r[f"c_{k}"], r[f"py_{k}"]), k
        acc_c, acc_py, nch, nranks, mx = r["scal"]
        assert acc_c == acc_py and nch == 2 * 192 and nranks == 2 and mx == np.max(r["py_rhat"])
        assert "boom" in str(r["raised"][0])
    for k in ("c_rhat", "c_mean"):
        assert np.array_equal(r0[k], r1[k])
