"""The N>1 path with the ENGINE on every rank (tests/test_distributed_cpu.py
covers it with the oracle): two processes (torch.distributed gloo, both ranks on
cuda:0 of the one-GPU box — the 8-GPU run uses "nccl"), each advancing its
shard of a cfg 5-shaped job keyed by global chain id through libemcmc, reducing
its shard's split-chain moments on device (emcmc_moments_window) and
all-gathering them (extensible_mcmc.diagnostics.allgather_moments, Chan merge
in rank order).  Bar: every chain's final state and accept stream equal the
unsharded single-handle run bit for bit, the merged moments equal the
one-handle moments (Chan merge vs. one device reduction: fp64 rounding only),
and rank 0 spot-checks chains of rank 1's shard against the oracle."""
import os
import socket
import sys
from pathlib import Path

import numpy as np
import pytest

ROOT = Path(__file__).resolve().parent.parent
pytestmark = pytest.mark.gpu

C_PER, S, WARM = 2048, 120, 20


@pytest.fixture(autouse=True)
def _gpu(require_gpu):
    pass


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _run(w, C, chain0, theta0):
    from extensible_mcmc import _lib as L
    from extensible_mcmc.engine import Engine, EngineConfig

    eng = Engine(EngineConfig(dim=w.D, num_chains=C, num_mcmc_steps=S, seed=w.seed, first_chain_id=chain0))
    eng.add_gaussian_rw_update(np.arange(w.D), w.rw_sigma)
    eng.set_gsn_target(w.mu_true, w.t_sigma, w.obs)
    eng.set_state(theta0)
    eng.run_iters(1, S)
    eng.synchronize()
    th, ll = eng.get_state()
    acc = eng.get_history(L.H_ACCEPT, 1, S)[:, 0]
    mom = eng.moments_window(WARM + 1, S - WARM, split=True)
    eng.close()
    return th, ll, acc, mom


def _worker(rank, world, port, out_dir):
    sys.path[:0] = [str(ROOT), str(ROOT / "extensiblemcmc.jl_amd")]
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    import torch.distributed as dist

    from extensible_mcmc import diagnostics as DG
    from extensible_mcmc import workloads as W

    dist.init_process_group("gloo", rank=rank, world_size=world)
    w = W.cfg5(world * C_PER)
    lo = rank * C_PER
    th, ll, acc, mom = _run(w, C_PER, lo, w.theta_init[lo:lo + C_PER])
    tot = DG.allgather_moments(mom, w.D)
    np.savez(os.path.join(out_dir, f"rank{rank}.npz"), theta=th, ll=ll, acc=acc, moments=DG.pack(tot))
    dist.barrier()
    dist.destroy_process_group()


def test_two_rank_engine_shards_and_allgathered_diagnostics(tmp_path, oracle):
    import torch.multiprocessing as mp

    from extensible_mcmc import diagnostics as DG
    from extensible_mcmc import workloads as W

    world = 2
    mp.spawn(_worker, args=(world, _free_port(), str(tmp_path)), nprocs=world, join=True)
    w = W.cfg5(world * C_PER)
    th, ll, acc, mom = _run(w, world * C_PER, 0, w.theta_init[:world * C_PER])
    r = [np.load(tmp_path / f"rank{k}.npz") for k in range(world)]
    assert np.array_equal(np.concatenate([x["theta"] for x in r]), th)
    assert np.array_equal(np.concatenate([x["ll"] for x in r]), ll)
    assert np.array_equal(np.concatenate([x["acc"] for x in r], axis=1), acc)
    got = [DG.unpack(x["moments"], w.D, mom["num_draws"]) for x in r]
    for g in got[1:]:  # every rank merged the same thing
        assert np.array_equal(DG.pack(g), DG.pack(got[0]))
    g = got[0]
    assert g["num_chains"] == mom["num_chains"] and g["accepted"] == mom["accepted"]
    np.testing.assert_allclose(g["mean"], mom["mean"], rtol=1e-12, atol=1e-14)
    np.testing.assert_allclose(g["m2"], mom["m2"], rtol=1e-10)
    np.testing.assert_allclose(g["sum_var"], mom["sum_var"], rtol=1e-12)
    # rank 1's chains against the oracle (keyed by global id C_PER + i)
    st = oracle.OracleState(w.theta_init[C_PER:C_PER + 64])
    oracle.run_gsn(st, seed=w.seed, rw_sigma=w.rw_sigma, t_sigma=w.t_sigma, obs=w.obs, iter0=1, nsteps=S,
                   chain0=C_PER, history=False)
    assert np.array_equal(r[1]["theta"][:64], st.theta)
