"""RCCL on hardware at one rank: a fresh `torchrun --nproc-per-node 1` child runs
bench.py with the nccl process group forced at world size 1 (RCCL init, the device
all_gather_into_tensor of the split-R̂ moments, libemcmc beside torch's HIP context),
and its diagnostics equal those of the plain single-process line bit for bit."""
import json
import os
import socket
import subprocess
import sys
from pathlib import Path

import pytest

pytestmark = pytest.mark.gpu
ROOT = Path(__file__).resolve().parents[1]
ARGS = ["--gpus", "1", "--steps", "20", "--warmup", "5", "--no-cpu", "--settle-ms", "0", "--reps", "1"]


@pytest.fixture(autouse=True)
def _gpu(require_gpu):
    pass


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _line(cmd, env):
    r = subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=240)
    assert r.returncode == 0, r.stderr[-3000:]
    return json.loads([x for x in r.stdout.splitlines() if x.startswith("{")][-1])


def test_nccl_process_group_at_one_rank_matches_the_single_process_line():
    env = dict(os.environ, HSA_ENABLE_IPC_MODE_LEGACY="0")
    env.pop("WORLD_SIZE", None)
    single = _line([sys.executable, "bench.py", *ARGS], env)
    env_n = dict(env, EMCMC_BENCH_FORCE_NCCL="1")
    rccl = _line([sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "1",
                  "--master-addr", "127.0.0.1", "--master-port", str(_free_port()), "bench.py", *ARGS], env_n)
    assert single["config"]["process_group"] is None
    assert rccl["config"]["process_group"] == "nccl" and rccl["n_gpus"] == 1
    assert rccl["config"]["workload"] == single["config"]["workload"]
    via = rccl["diagnostics"].pop("via")
    assert "RCCL (ncclAllGather inside libemcmc), 1 ranks" in via and single["diagnostics"].pop("via").endswith("this rank alone")
    assert rccl["diagnostics"] == single["diagnostics"]
    assert rccl["parity"]["all_ranks_bitwise"] is True and single["parity"]["accept_stream_bitwise"] is True


RCCL_CHILD = r"""
import sys
sys.path[:0] = [sys.argv[1], sys.argv[1] + "/extensiblemcmc.jl_amd"]
import numpy as np
from extensible_mcmc import _lib as L
from extensible_mcmc import diagnostics as DG
from extensible_mcmc import workloads as W
from extensible_mcmc.engine import Engine, EngineConfig

assert len(L.hip_runtime_images()) == 1, L.hip_runtime_images()
w = W.cfg2(4096)
eng = Engine(EngineConfig(dim=w.D, num_chains=4096, num_mcmc_steps=40, seed=w.seed, device=0))
eng.add_gaussian_rw_update(np.arange(w.D), w.rw_sigma)
eng.set_gsn_target(w.mu_true, w.t_sigma, w.obs)
eng.set_state(np.zeros((4096, w.D)))
eng.run_iters(1, 40)
eng.synchronize()
mom = eng.moments_window(9, 32, split=True)
py = DG.rhat_from_moments(mom)
comm = DG.Comm.rccl(1, 0, 0, DG.Comm.unique_id())
try:
    for got in (eng.diagnostics(9, 32, comm=comm), eng.diagnostics(9, 32),
                DG.merge_c(DG.pack(mom), w.D, mom["num_draws"], comm)):
        for k in ("rhat", "mean", "W", "B"):
            assert np.array_equal(got[k], py[k]), k
        assert got["accept_rate"] == py["accept_rate"] and got["num_chains"] == 2 * 4096
        assert got["max_rhat"] == float(np.max(py["rhat"]))
finally:
    comm.close()
    eng.close()
print("rccl child ok")
"""


def test_emcmc_diagnostics_on_an_rccl_comm_equals_the_python_reduction():
    """emcmc_diagnostics at world size 1 on a real RCCL communicator:
    the library's all-gather (ncclAllGather on the comm's stream), Chan merge and
    split-R̂ give the bits of extensible_mcmc.diagnostics on the same moments, as do
    the no-comm call and emcmc_diagnostics_merge over the RCCL comm.  In a fresh process with
    one HIP runtime: the suite's own process may hold torch's beside the library's, which
    emcmc_comm_init refuses (tests/test_hip_runtimes_cpu.py; such a process also crashes in
    its teardown on a GPU box, so the refusal is exercised on the CPU only)."""
    r = subprocess.run([sys.executable, "-c", RCCL_CHILD, str(ROOT)], cwd=ROOT, capture_output=True, text=True,
                       timeout=240, env=dict(os.environ, HSA_ENABLE_IPC_MODE_LEGACY="0"))
    assert r.returncode == 0 and "rccl child ok" in r.stdout, r.stderr[-3000:]


def test_two_ranks_on_one_device_carry_parity_and_the_same_per_gpu_shape():
    """`python bench.py --gpus 2` with no outer launcher (bench.py starts the
    torch.distributed.run child itself) at world size 2, both ranks on device 0 with
    gloo (one GPU on this box): each rank replays all of its chains on the oracle
    (bench.py parity_replay), AND-reduced; the per-GPU chain count is the N = 1 line's; the barriers sit
    outside the timed window."""
    env = dict(os.environ, HSA_ENABLE_IPC_MODE_LEGACY="0", EMCMC_BENCH_SHARED_DEVICE="1")
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK"):
        env.pop(k, None)
    two = _line([sys.executable, "bench.py", *[x if x != "1" or i != 1 else "2" for i, x in enumerate(ARGS)]], env)
    assert two["n_gpus"] == 2 and two["config"]["process_group"] == "gloo"
    assert two["config"]["chains_per_gpu"] == 65536 and two["config"]["total_chains"] == 131072
    assert two["parity"]["ranks"] == 2 and two["parity"]["all_ranks_bitwise"] is True
    assert "closing_barrier_ms_rank0" in two["timing"]
