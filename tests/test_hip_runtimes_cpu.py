"""Two HIP runtimes in one process: torch's wheel bundles its own
libamdhip64, and when libemcmc.so is loaded first, importing torch maps a second runtime
beside the library's.  emcmc_hip_runtime_images reports them; emcmc_comm_init and
emcmc_comm_unique_id refuse such a process with EMCMC_HIP_ERROR and say why (before any
device check, so this runs on CPU); the Python layer warns once."""
import subprocess
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]

CHILD = r"""
import sys, warnings
sys.path[:0] = [sys.argv[1], sys.argv[1] + "/extensiblemcmc.jl_amd"]
from extensible_mcmc import _lib as L
from extensible_mcmc import diagnostics as DG
torch_first = sys.argv[2] == "torch_first"
if torch_first:
    import torch  # noqa: F401  (the library then binds to torch's runtime by its SONAME)
L.lib()
if not torch_first:
    assert len(L.hip_runtime_images()) == 1, L.hip_runtime_images()
    import torch  # noqa: F401
imgs = L.hip_runtime_images()
print("images", len(imgs))
try:
    DG.Comm.rccl(1, 0, 0, bytes(L.COMM_ID_BYTES))
    print("status", 0)
except L.EMCMCError as e:
    print("status", e.status)
    print("msg", str(e).replace("\n", " "))
try:
    DG.Comm.unique_id()
except L.EMCMCError as e:
    print("uid_status", e.status)
with warnings.catch_warnings(record=True) as w:
    warnings.simplefilter("always")
    ok = L.check_single_hip_runtime()
    L.check_single_hip_runtime()
print("single", ok, "warnings", len(w))
"""


def _child(order):
    r = subprocess.run([sys.executable, "-c", CHILD, str(ROOT), order], capture_output=True, text=True, timeout=240)
    assert r.returncode == 0, r.stderr[-3000:]
    return dict(line.split(" ", 1) for line in r.stdout.splitlines() if " " in line)


def test_library_first_then_torch_is_refused_with_the_reason():
    from extensible_mcmc import _lib as L

    out = _child("library_first")
    assert out["images"] == "2"
    assert int(out["status"]) == L.HIP_ERROR and int(out["uid_status"]) == L.HIP_ERROR
    assert "2 HIP runtimes" in out["msg"] and "import torch" in out["msg"]
    assert out["single"] == "False warnings 1"  # warned once


def test_torch_first_shares_one_runtime():
    from extensible_mcmc import _lib as L

    out = _child("torch_first")
    assert out["images"] == "1"
    assert int(out["status"]) != L.HIP_ERROR  # no device here: NO_DEVICE / RCCL_ERROR, not the refusal
    assert out["single"] == "True warnings 0"
