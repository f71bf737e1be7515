"""ctypes binding of the C ABI in include/emcmc.h (libemcmc.so).

This is the Python-side twin of the Julia ``ccall`` shim in
``extensiblemcmc.jl_amd/julia/ExtensibleMCMCHip.jl``.  The library is built
in-tree by ``make -C extensiblemcmc.jl_amd`` (``__graft_entry__.build()``).
There is no fallback: if the shared object is missing this module raises.
"""
from __future__ import annotations

import ctypes as C
import os
from pathlib import Path

import numpy as np

ABI_VERSION = 2

OK = 0
INVALID_ARG = 1
HIP_ERROR = 2
RCCL_ERROR = 3
UNSUPPORTED_PLUGIN = 4
CHAIN_FAULT = 5
OUT_OF_MEMORY = 6
NO_DEVICE = 7
STATE_ERROR = 8

STATUS_NAMES = {
    0: "EMCMC_OK",
    1: "EMCMC_INVALID_ARG",
    2: "EMCMC_HIP_ERROR",
    3: "EMCMC_RCCL_ERROR",
    4: "EMCMC_UNSUPPORTED_PLUGIN",
    5: "EMCMC_CHAIN_FAULT",
    6: "EMCMC_OUT_OF_MEMORY",
    7: "EMCMC_NO_DEVICE",
    8: "EMCMC_STATE_ERROR",
}

RW_UNIFORM, RW_GAUSSIAN, RW_GAUSSIAN_MIX, MALA, USER_UPDATE = 1, 2, 3, 4, 5
PRIOR_IMPROPER, PRIOR_IMPROPER_POS, PRIOR_PRODUCT, PRIOR_STANDARD = 0, 1, 2, 3
DIST_NORMAL, DIST_UNIFORM, DIST_EXPONENTIAL, DIST_GAMMA = 1, 2, 3, 4
DIST_LOGNORMAL, DIST_BETA, DIST_INVERSE_GAMMA, DIST_CAUCHY, DIST_LAPLACE, DIST_TDIST = 5, 6, 7, 8, 9, 10
DIST_PRODUCT, DIST_MVNORMAL = 32, 33
ADPT_NONE, ADPT_UNIF_RW, ADPT_HAARIO, ADPT_UNIF_RW_VEC = 0, 1, 2, 3
TARGET_GSN, TARGET_LOGISTIC, TARGET_USER = 1, 2, 3
LL_PER_OBS, LL_SUFFSTAT = 0, 1
HIST_FULL, HIST_ACCEPT_ONLY = 0, 1
H_STATE, H_PROPOSAL, H_LL, H_ACCEPT = 0, 1, 2, 3
FAULT_NONFINITE_LL = 1
FAULT_RNG_RETRIES = 2
FAULT_POSDEF = 4
FAULT_PRIOR_RESAMPLES = 8
VARIANT_SCALAR_OBS = 4
VARIANT_MIX_STREAM = 8
VARIANT_NO_XCD_ORDER = 16
VARIANT_NO_RTC_CHOL = 32
VARIANT_NO_MIX_CHOL = 64
VARIANT_UNCAPPED = 128  # diag kernel without the 2-waves-per-SIMD register cap
VARIANT_NO_BLOCK = 256  # MALA / user updates over all D > 16 coordinates and random-walk schedules at D > 16: the wide kernel
VARIANT_NO_FUSED_PRIOR = 512  # joint diagonal GaussianRandomWalk with a Product of univariates: not the fused kernel


class EmcmcConfig(C.Structure):
    _fields_ = [
        ("abi_version", C.c_uint32),
        ("dim", C.c_uint32),
        ("num_chains", C.c_uint64),
        ("first_chain_id", C.c_uint64),
        ("num_mcmc_steps", C.c_uint64),
        ("seed", C.c_uint64),
        ("device", C.c_int32),
        ("history_mode", C.c_uint32),
        ("roll_window", C.c_uint32),
        ("lanes_per_chain", C.c_uint32),
        ("steps_per_launch", C.c_uint32),
        ("kernel_variant", C.c_uint32),
        ("chain_moments", C.c_uint32),
        ("history_ring", C.c_uint32),
        ("reserved", C.c_uint32 * 4),
    ]


class EmcmcUpdateDesc(C.Structure):
    _fields_ = [
        ("kernel", C.c_uint32),
        ("prior", C.c_uint32),
        ("adaptation", C.c_uint32),
        ("num_coords", C.c_uint32),
        ("coords", C.POINTER(C.c_uint32)),
        ("sigma", C.POINTER(C.c_double)),
        ("epsilon", C.POINTER(C.c_double)),
        ("pos", C.POINTER(C.c_uint8)),
        ("adaptation_params", C.c_void_p),
        ("sigma_b", C.POINTER(C.c_double)),
        ("prior_params", C.c_void_p),
        ("user_update", C.c_void_p),
        ("mix_lambda", C.c_double),
        ("reserved_f64", C.c_double * 3),
    ]


class EmcmcPriorFactor(C.Structure):
    """One ProductPrior / StandardPrior factor (include/emcmc.h emcmc_prior_factor)."""


EmcmcPriorFactor._fields_ = [("family", C.c_uint32), ("count", C.c_uint32), ("a", C.c_double), ("b", C.c_double),
                             ("components", C.POINTER(EmcmcPriorFactor)), ("mu", C.POINTER(C.c_double)),
                             ("sigma", C.POINTER(C.c_double))]


class EmcmcPriorDesc(C.Structure):
    """emcmc_update_desc.prior_params (include/emcmc.h emcmc_prior_desc)."""
    _fields_ = [("num_factors", C.c_uint32), ("reserved", C.c_uint32),
                ("factors", C.POINTER(EmcmcPriorFactor))]


class EmcmcHaarioAdaptation(C.Structure):
    """HaarioTypeAdaptation parameters (include/emcmc.h emcmc_haario_adaptation)."""
    _fields_ = [
        ("adapt_every_k_steps", C.c_uint32),
        ("reserved", C.c_uint32),
        ("scale", C.c_double),
    ]


class EmcmcUnifRWAdaptation(C.Structure):
    """AdaptationUnifRW parameters (include/emcmc.h emcmc_unifrw_adaptation)."""
    _fields_ = [
        ("adapt_every_k_steps", C.c_uint32),
        ("reserved", C.c_uint32),
        ("target_accpt_rate", C.c_double),
        ("scale", C.c_double),
        ("min", C.c_double),
        ("max", C.c_double),
        ("offset", C.c_double),
    ]


class EmcmcUnifRWAdaptationVec(C.Structure):
    """AdaptationUnifRW per-coordinate form (include/emcmc.h emcmc_unifrw_adaptation_vec)."""
    _fields_ = [
        ("adapt_every_k_steps", C.c_uint32),
        ("reserved", C.c_uint32),
        ("target_accpt_rate", C.c_double),
        ("scale", C.POINTER(C.c_double)),
        ("min", C.POINTER(C.c_double)),
        ("max", C.POINTER(C.c_double)),
        ("offset", C.POINTER(C.c_double)),
    ]


class EmcmcTargetDesc(C.Structure):
    _fields_ = [
        ("kind", C.c_uint32),
        ("dim", C.c_uint32),
        ("mu", C.POINTER(C.c_double)),
        ("sigma", C.POINTER(C.c_double)),
        ("num_obs", C.c_uint64),
        ("obs", C.POINTER(C.c_double)),
        ("ll_mode", C.c_uint32),
        ("reserved", C.c_uint32),
        ("labels", C.POINTER(C.c_double)),
    ]


class EmcmcUserUpdateDesc(C.Structure):
    """A user update compiled at run time (include/emcmc.h emcmc_user_update_desc)."""
    _fields_ = [("source", C.c_char_p), ("options", C.c_char_p), ("num_params", C.c_uint64),
                ("params", C.POINTER(C.c_double))]


class EmcmcUserTargetDesc(C.Structure):
    """A user law compiled at run time (include/emcmc.h emcmc_user_target_desc)."""
    _fields_ = [
        ("dim", C.c_uint32),
        ("obs_dim", C.c_uint32),
        ("theta0", C.POINTER(C.c_double)),
        ("num_obs", C.c_uint64),
        ("obs", C.POINTER(C.c_double)),
        ("num_params", C.c_uint64),
        ("params", C.POINTER(C.c_double)),
        ("source", C.c_char_p),
        ("options", C.c_char_p),
    ]


class EmcmcStep(C.Structure):
    _fields_ = [("mcmciter", C.c_uint32), ("pidx", C.c_uint32)]


class EmcmcMoments(C.Structure):
    _fields_ = [
        ("num_chains", C.c_uint64),
        ("num_draws", C.c_uint64),
        ("accepted", C.c_uint64),
        ("proposed", C.c_uint64),
    ]


class EmcmcDiag(C.Structure):
    _fields_ = [
        ("num_chains", C.c_uint64),
        ("num_draws", C.c_uint64),
        ("accepted", C.c_uint64),
        ("proposed", C.c_uint64),
        ("accept_rate", C.c_double),
        ("max_rhat", C.c_double),
        ("dim", C.c_uint32),
        ("nranks", C.c_uint32),
        ("mean", C.POINTER(C.c_double)),
        ("m2", C.POINTER(C.c_double)),
        ("sum_var", C.POINTER(C.c_double)),
        ("W", C.POINTER(C.c_double)),
        ("B", C.POINTER(C.c_double)),
        ("rhat", C.POINTER(C.c_double)),
    ]


COMM_ID_BYTES = 128
# emcmc_allgather_fn: (send, recv, count, ctx) -> 0 on success
ALLGATHER_FN = C.CFUNCTYPE(C.c_int, C.POINTER(C.c_double), C.POINTER(C.c_double), C.c_uint64, C.c_void_p)

LAMBDA_FN = C.CFUNCTYPE(C.c_double, C.c_double, C.c_int64, C.c_int64, C.c_void_p)  # emcmc_lambda_fn

# every symbol declared in include/emcmc.h, with its ctypes signature
_H = C.c_void_p
_ST = C.c_int
SIGNATURES = {
    "emcmc_device_count": (_ST, [C.POINTER(C.c_int)]),
    "emcmc_create": (_ST, [C.POINTER(_H), C.POINTER(EmcmcConfig)]),
    "emcmc_add_update": (_ST, [_H, C.POINTER(EmcmcUpdateDesc)]),
    "emcmc_set_target": (_ST, [_H, C.POINTER(EmcmcTargetDesc)]),
    "emcmc_set_user_target": (_ST, [_H, C.POINTER(EmcmcUserTargetDesc)]),
    "emcmc_check_user_target": (_ST, [C.c_char_p, C.c_uint32, C.c_char_p, C.c_char_p, C.c_size_t]),
    "emcmc_check_user_update": (_ST, [C.c_char_p, C.c_uint32, C.c_char_p, C.c_char_p, C.c_size_t]),
    "emcmc_set_state": (_ST, [_H, C.POINTER(C.c_double), C.POINTER(C.c_double)]),
    # const emcmc_step * passed as an address: the step list's numpy buffer, without a
    # per-call ctypes pointer object (≈ 3 µs of the 20-step window's host path)
    "emcmc_run": (_ST, [_H, C.c_void_p, C.c_uint64]),
    "emcmc_synchronize": (_ST, [_H]),
    "emcmc_destroy": (None, [_H]),
    "emcmc_last_error": (C.c_char_p, [_H]),
    "emcmc_get_state": (_ST, [_H, C.POINTER(C.c_double), C.POINTER(C.c_double)]),
    "emcmc_get_chain_stats": (_ST, [_H, C.POINTER(C.c_double), C.POINTER(C.c_uint64)]),
    "emcmc_get_update_state": (
        _ST, [_H, C.c_uint32, C.POINTER(C.c_double), C.POINTER(C.c_uint32), C.POINTER(C.c_uint32)]
    ),
    "emcmc_get_faults": (_ST, [_H, C.POINTER(C.c_uint32)]),
    "emcmc_set_mix_lambda_fn": (_ST, [_H, C.c_uint32, LAMBDA_FN, C.c_void_p]),
    "emcmc_get_mix_lambda": (_ST, [_H, C.c_uint32, C.POINTER(C.c_double)]),
    "emcmc_get_proposal_ll": (_ST, [_H, C.POINTER(C.c_double)]),
    "emcmc_get_chain_moments": (_ST, [_H, C.POINTER(C.c_double), C.POINTER(C.c_double)]),
    "emcmc_get_mix_state": (_ST, [_H, C.c_uint32, C.POINTER(C.c_double), C.POINTER(C.c_uint32)]),
    "emcmc_get_adaptation_moments": (_ST, [_H, C.c_uint32, C.POINTER(C.c_double), C.POINTER(C.c_double)]),
    "emcmc_get_history": (_ST, [_H, C.c_uint32, C.c_uint64, C.c_uint64, C.c_void_p, C.c_size_t]),
    "emcmc_get_history_chains": (
        _ST, [_H, C.c_uint32, C.c_uint64, C.c_uint64, C.c_uint64, C.c_uint64, C.c_void_p, C.c_size_t]
    ),
    "emcmc_history_device_ptr": (_ST, [_H, C.c_uint32, C.POINTER(C.c_void_p), C.POINTER(C.c_size_t)]),
    "emcmc_stream_history": (_ST, [_H, C.c_uint32, C.c_uint64, C.c_uint64, C.c_uint64, C.c_void_p, C.c_size_t]),
    "emcmc_stream_wait": (_ST, [_H]),
    "emcmc_host_alloc": (_ST, [C.c_size_t, C.POINTER(C.c_void_p)]),
    "emcmc_host_free": (_ST, [C.c_void_p]),
    "emcmc_moments_window": (
        _ST,
        [_H, C.c_uint64, C.c_uint64, C.c_int, C.POINTER(C.c_double), C.POINTER(EmcmcMoments)],
    ),
    "emcmc_comm_unique_id": (_ST, [C.POINTER(C.c_uint8)]),
    "emcmc_comm_init": (_ST, [C.POINTER(_H), C.c_int, C.c_int, C.c_int, C.POINTER(C.c_uint8)]),
    "emcmc_comm_init_host": (_ST, [C.POINTER(_H), C.c_int, C.c_int, ALLGATHER_FN, C.c_void_p]),
    "emcmc_comm_destroy": (None, [_H]),
    "emcmc_comm_last_error": (C.c_char_p, [_H]),
    "emcmc_hip_runtime_images": (C.c_int, [C.c_char_p, C.c_size_t]),
    "emcmc_diagnostics": (_ST, [_H, _H, C.c_uint64, C.c_uint64, C.c_int, C.POINTER(EmcmcDiag)]),
    "emcmc_diagnostics_merge": (_ST, [_H, C.POINTER(C.c_double), C.c_uint32, C.c_uint64, C.POINTER(EmcmcDiag)]),
    "emcmc_set_timing": (_ST, [_H, C.c_int]),
    "emcmc_get_timing": (
        _ST,
        [_H, C.POINTER(C.c_double), C.POINTER(C.c_uint64), C.POINTER(C.c_double), C.c_int],
    ),
    "emcmc_kernel_name": (_ST, [_H, C.c_char_p, C.c_size_t]),
    "emcmc_rtc_info": (_ST, [_H, C.POINTER(C.c_uint32), C.POINTER(C.c_double)]),
    "emcmc_prebuild_chol_kernel": (_ST, [C.c_uint32, C.c_uint32, C.c_uint32, C.c_char_p, C.c_size_t]),
    "emcmc_prebuild_block_kernel": (
        _ST, [C.c_uint32, C.c_uint32, C.c_uint32, C.c_int, C.c_char_p, C.c_char_p, C.c_char_p, C.c_char_p, C.c_char_p,
              C.c_size_t]),
    "emcmc_prebuild_rw_block_kernel": (
        _ST, [C.c_uint32, C.c_uint32, C.c_uint32, C.c_int, C.c_void_p, C.c_uint32, C.c_char_p, C.c_char_p,
              C.c_char_p, C.c_size_t]),
    "emcmc_prebuild_fused_prior_kernel": (
        _ST, [C.c_uint32, C.c_uint32, C.c_uint32, C.c_uint32, C.c_int, C.c_void_p, C.c_char_p, C.c_size_t]),
    "emcmc_probe_variates": (
        _ST,
        [C.c_int, C.c_uint64, C.c_uint32, C.c_uint32, C.c_uint64, C.POINTER(C.c_uint32), C.POINTER(C.c_uint32),
         C.POINTER(C.c_double), C.POINTER(C.c_double)],
    ),
    "emcmc_probe_log": (_ST, [C.c_int, C.POINTER(C.c_double), C.POINTER(C.c_double), C.c_uint64]),
}

PKG_ROOT = Path(__file__).resolve().parent.parent  # extensiblemcmc.jl_amd/
LIB_PATH = Path(os.environ.get("EMCMC_LIB", PKG_ROOT / "lib" / "libemcmc.so"))


class EMCMCError(RuntimeError):
    """A non-OK emcmc_status, with the library's last error message."""

    def __init__(self, status: int, where: str, message: str = ""):
        self.status = status
        super().__init__(f"{where}: {STATUS_NAMES.get(status, status)}" + (f" — {message}" if message else ""))


class UnsupportedPlugin(NotImplementedError):
    """A plugin (update, transition kernel, prior, target) with no device
    implementation: raised instead of any CPU fallback."""


class UnsupportedPluginError(EMCMCError, UnsupportedPlugin):
    """EMCMC_UNSUPPORTED_PLUGIN from the library: both an EMCMCError (with the
    status and message) and an UnsupportedPlugin."""


_lib = None


def lib() -> C.CDLL:
    """Load libemcmc.so (raises if it was not built: there is no CPU fallback)."""
    global _lib
    if _lib is None:
        if not LIB_PATH.exists():
            raise ImportError(
                f"libemcmc.so not found at {LIB_PATH}; build it with `make -C {PKG_ROOT}` "
                "or `python -c 'import __graft_entry__ as g; g.build()'`"
            )
        L = C.CDLL(str(LIB_PATH))
        for name, (res, args) in SIGNATURES.items():
            fn = getattr(L, name)
            fn.restype = res
            fn.argtypes = args
        _lib = L
    return _lib


def hip_runtime_images() -> list[str]:
    """Paths of the HIP runtime images (libamdhip64.so*) mapped into this process."""
    buf = C.create_string_buffer(1 << 14)
    n = lib().emcmc_hip_runtime_images(buf, len(buf))
    paths = [p for p in buf.value.decode(errors="replace").split("\n") if p]
    return paths if len(paths) == n else paths + ["?"] * (n - len(paths))


_warned_runtimes = False


def check_single_hip_runtime() -> bool:
    """Warn (once per process) when more than one HIP runtime is mapped: torch's wheel bundles
    its own, and when libemcmc.so is loaded before torch both end up in the process — the
    library's streams and device pointers then mean nothing to torch's runtime (and RCCL
    refuses, emcmc_comm_init).  Returns True when one runtime (or none) is mapped."""
    global _warned_runtimes
    imgs = hip_runtime_images()
    if len(imgs) > 1 and not _warned_runtimes:
        import warnings

        _warned_runtimes = True
        warnings.warn("this process holds %d HIP runtimes (%s): import torch before extensible_mcmc (or run "
                      "without torch) so that one runtime serves both; RCCL communicators refuse to start"
                      % (len(imgs), ", ".join(imgs)), RuntimeWarning, stacklevel=2)
    return len(imgs) <= 1


def dptr(a: np.ndarray):
    assert a.dtype == np.float64 and a.flags.c_contiguous
    return a.ctypes.data_as(C.POINTER(C.c_double))


def u32ptr(a: np.ndarray):
    assert a.dtype == np.uint32 and a.flags.c_contiguous
    return a.ctypes.data_as(C.POINTER(C.c_uint32))


def probe_variates(seed: int, chains, iters, dim: int, pidx0: int = 0, device: int = 0):
    ch = np.ascontiguousarray(chains, dtype=np.uint32)
    it = np.ascontiguousarray(iters, dtype=np.uint32)
    n = ch.size
    z = np.empty((n, dim))
    E = np.empty(n)
    st = lib().emcmc_probe_variates(device, seed & 0xFFFFFFFFFFFFFFFF, pidx0, dim, n, u32ptr(ch), u32ptr(it),
                                    dptr(z), dptr(E))
    if st != OK:
        raise EMCMCError(st, "emcmc_probe_variates")
    return z, E


def probe_log(x, device: int = 0):
    x = np.ascontiguousarray(x, dtype=np.float64)
    y = np.empty_like(x)
    st = lib().emcmc_probe_log(device, dptr(x), dptr(y), x.size)
    if st != OK:
        raise EMCMCError(st, "emcmc_probe_log")
    return y


def check_user_target(source: str, dim: int, options: str = "") -> None:
    """Compile-only check of a user log-likelihood (hiprtc; no device needed).
    Raises EMCMCError(INVALID_ARG) carrying the compiler log."""
    buf = C.create_string_buffer(1 << 16)
    st = lib().emcmc_check_user_target(source.encode(), dim, options.encode(), buf, len(buf))
    if st != OK:
        raise EMCMCError(st, "emcmc_check_user_target", buf.value.decode(errors="replace"))


def check_user_update(source: str, dim: int, options: str = "") -> None:
    """Compile-only check of a user update's proposal! / log_transition_density source."""
    buf = C.create_string_buffer(1 << 16)
    st = lib().emcmc_check_user_update(source.encode(), dim, options.encode(), buf, len(buf))
    if st != OK:
        raise EMCMCError(st, "emcmc_check_user_update", buf.value.decode(errors="replace"))


def prebuild_chol_kernel(dim: int, history_mode: int = 0, ll_mode: int = 0) -> None:
    """Compile the run-time chol kernel at dim into the on-disk code-object cache
    (no device needed), so a handle at that D loads it instead of compiling."""
    buf = C.create_string_buffer(1 << 16)
    st = lib().emcmc_prebuild_chol_kernel(dim, history_mode, ll_mode, buf, len(buf))
    if st != OK:
        raise EMCMCError(st, "emcmc_prebuild_chol_kernel", buf.value.decode(errors="replace"))


def prebuild_block_kernel(dim: int, history_mode: int = 0, ll_mode: int = 0, dense_target: bool = True,
                          target_source: str = "", target_options: str = "", update_source: str = "",
                          update_options: str = "") -> None:
    """Compile mwg_block_kernel (one MALA or user update over all 17 ≤ dim ≤ 64 coordinates)
    into the on-disk code-object cache (no device needed)."""
    buf = C.create_string_buffer(1 << 16)
    enc = lambda x: x.encode() if x else None  # noqa: E731
    st = lib().emcmc_prebuild_block_kernel(dim, history_mode, ll_mode, int(bool(dense_target)), enc(target_source),
                                           enc(target_options), enc(update_source), enc(update_options), buf, len(buf))
    if st != OK:
        raise EMCMCError(st, "emcmc_prebuild_block_kernel", buf.value.decode(errors="replace"))


def prebuild_rw_block_kernel(dim: int, update_descs, history_mode: int = 0, ll_mode: int = 0,
                             dense_target: bool = False, target_source: str = "", target_options: str = "") -> None:
    """Compile mwg_rw_block_kernel for the schedule of `update_descs` (EmcmcUpdateDesc objects, in
    update order, e.g. [Engine.uniform_rw_desc(...)[0]]; a single desc is accepted too) into the
    on-disk code-object cache (no device needed)."""
    if isinstance(update_descs, EmcmcUpdateDesc):
        update_descs = [update_descs]
    arr = (EmcmcUpdateDesc * len(update_descs))(*update_descs)
    buf = C.create_string_buffer(1 << 16)
    enc = lambda x: x.encode() if x else None  # noqa: E731
    st = lib().emcmc_prebuild_rw_block_kernel(dim, history_mode, ll_mode, int(bool(dense_target)),
                                              C.cast(arr, C.c_void_p), len(update_descs), enc(target_source),
                                              enc(target_options), buf, len(buf))
    if st != OK:
        raise EMCMCError(st, "emcmc_prebuild_rw_block_kernel", buf.value.decode(errors="replace"))



def prebuild_fused_prior_kernel(dim: int, update_desc, lanes_per_chain: int = 0, history_mode: int = 0,
                                ll_mode: int = 0, unit_target: bool = True) -> None:
    """Compile the fused diagonal step with the update's separable prior (rwm_gsn_diag_kernel +
    FusedPrior) into the on-disk code-object cache (no device needed)."""
    buf = C.create_string_buffer(1 << 16)
    st = lib().emcmc_prebuild_fused_prior_kernel(dim, lanes_per_chain, history_mode, ll_mode, int(bool(unit_target)),
                                                 C.cast(C.byref(update_desc), C.c_void_p), buf, len(buf))
    if st != OK:
        raise EMCMCError(st, "emcmc_prebuild_fused_prior_kernel", buf.value.decode(errors="replace"))
def device_count() -> int:
    n = C.c_int(0)
    lib().emcmc_device_count(C.byref(n))
    return int(n.value)
