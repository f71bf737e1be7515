"""C-ABI boundary checks that need no GPU: the library loads, exports every
symbol include/emcmc.h declares, the ctypes struct layouts match the header's
C layout, and on a GPU-less host the engine refuses to run (no CPU fallback)."""
import ctypes as C
import re
import subprocess
import textwrap
from pathlib import Path

import numpy as np
import pytest

from extensible_mcmc import _lib as L

ROOT = Path(__file__).resolve().parent.parent
HEADER = ROOT / "include" / "emcmc.h"


def declared_functions():
    txt = HEADER.read_text()
    txt = re.sub(r"/\*.*?\*/", "", txt, flags=re.S)
    return sorted(set(re.findall(r"\b(emcmc_[a-z_]+)\s*\(", txt)))


def test_header_and_binding_agree():
    assert declared_functions() == sorted(L.SIGNATURES)


def test_library_exports_every_declared_symbol():
    lib = L.lib()
    out = subprocess.run(["nm", "-D", "--defined-only", str(L.LIB_PATH)], capture_output=True, text=True,
                         check=True).stdout
    exported = set(re.findall(r" T (emcmc_\w+)", out))
    for name in declared_functions():
        assert name in exported, name
        assert getattr(lib, name) is not None


def test_julia_shim_binds_only_declared_symbols():
    """Every ccall of the Julia MI355XBackend shim names a function the header
    declares (the shim is not executed here: no Julia in the image)."""
    jl = (ROOT / "extensiblemcmc.jl_amd" / "julia" / "ExtensibleMCMCHip.jl").read_text()
    called = set(re.findall(r"ccall\(\(:(emcmc_\w+), LIB\)", jl))
    assert called and called <= set(declared_functions()), called - set(declared_functions())
    for name in ("emcmc_create", "emcmc_run", "emcmc_get_history", "emcmc_get_chain_stats", "emcmc_moments_window"):
        assert name in called


def test_struct_layout_matches_header(tmp_path):
    src = textwrap.dedent(
        """
        #include <stdio.h>
        #include <stddef.h>
        #include "emcmc.h"
        int main(void) {
          printf("%zu %zu %zu %zu %zu\\n", sizeof(emcmc_config), sizeof(emcmc_update_desc),
                 sizeof(emcmc_target_desc), sizeof(emcmc_step), sizeof(emcmc_moments));
          printf("%zu %zu %zu %zu %zu\\n", offsetof(emcmc_config, device), offsetof(emcmc_update_desc, pos),
                 offsetof(emcmc_target_desc, ll_mode), sizeof(emcmc_unifrw_adaptation),
                 offsetof(emcmc_unifrw_adaptation, offset));
          printf("%zu %zu %zu %zu %zu %zu\\n", offsetof(emcmc_config, history_ring), offsetof(emcmc_config, chain_moments),
                 offsetof(emcmc_update_desc, adaptation_params), offsetof(emcmc_update_desc, sigma_b),
                 offsetof(emcmc_update_desc, mix_lambda), sizeof(emcmc_haario_adaptation));
          return 0;
        }
        """
    )
    c = tmp_path / "layout.c"
    c.write_text(src)
    exe = tmp_path / "layout"
    subprocess.run(["gcc", "-std=c11", "-I", str(HEADER.parent), str(c), "-o", str(exe)], check=True)
    sizes, offs, offs2 = subprocess.run([str(exe)], capture_output=True, text=True, check=True).stdout.split("\n")[:3]
    assert [int(x) for x in sizes.split()] == [C.sizeof(L.EmcmcConfig), C.sizeof(L.EmcmcUpdateDesc),
                                               C.sizeof(L.EmcmcTargetDesc), C.sizeof(L.EmcmcStep),
                                               C.sizeof(L.EmcmcMoments)]
    assert [int(x) for x in offs.split()] == [L.EmcmcConfig.device.offset, L.EmcmcUpdateDesc.pos.offset,
                                              L.EmcmcTargetDesc.ll_mode.offset, C.sizeof(L.EmcmcUnifRWAdaptation),
                                              L.EmcmcUnifRWAdaptation.offset.offset]
    assert [int(x) for x in offs2.split()] == [L.EmcmcConfig.history_ring.offset, L.EmcmcConfig.chain_moments.offset,
                                               L.EmcmcUpdateDesc.adaptation_params.offset,
                                               L.EmcmcUpdateDesc.sigma_b.offset, L.EmcmcUpdateDesc.mix_lambda.offset,
                                               C.sizeof(L.EmcmcHaarioAdaptation)]


def test_no_device_means_no_run():
    """With no GPU the engine refuses (EMCMC_NO_DEVICE) instead of computing on the CPU."""
    if L.device_count() > 0:
        pytest.skip("a GPU is visible; covered by the gpu tests")
    from extensible_mcmc import Engine, EngineConfig

    with pytest.raises(L.EMCMCError) as e:
        Engine(EngineConfig(dim=2, num_chains=4, num_mcmc_steps=10))
    assert e.value.status == L.NO_DEVICE


def test_invalid_config_rejected_without_device():
    cfg = L.EmcmcConfig()
    cfg.abi_version = 999
    h = C.c_void_p()
    assert L.lib().emcmc_create(C.byref(h), C.byref(cfg)) == L.INVALID_ARG
    n = C.c_int(-1)
    assert L.lib().emcmc_device_count(C.byref(n)) == L.OK and n.value >= 0


@pytest.mark.parametrize("hist", [L.HIST_FULL, L.HIST_ACCEPT_ONLY])
def test_state_beyond_32bit_offsets_rejected(hist):
    """C·D·8 bytes above 4 GiB − 1 is refused in every history mode: the state and a
    history slot are addressed with 32-bit per-lane offsets."""
    cfg = L.EmcmcConfig()
    cfg.abi_version = L.ABI_VERSION
    cfg.dim, cfg.num_mcmc_steps, cfg.history_mode = 32, 10, hist
    cfg.num_chains = (1 << 32) // (32 * 8)  # exactly 4 GiB of state
    cfg.roll_window = 10
    h = C.c_void_p()
    assert L.lib().emcmc_create(C.byref(h), C.byref(cfg)) == L.INVALID_ARG


def test_runtime_kernels_share_the_soa_tile_width():
    """The state_pos tile width (emcmc_kernels.h EMCMC_SOA_TILE) is passed to every run-time
    compile by emcmc_rtc.hip from its own default: the two defaults must agree, or the
    run-time kernels would lay out θ and the histories differently from the ahead-of-time
    ones (text-level)."""
    csrc = ROOT / "extensiblemcmc.jl_amd" / "csrc"
    pat = re.compile(r"#define\s+EMCMC_SOA_TILE\s+(\d+)")
    k = pat.findall((csrc / "emcmc_kernels.h").read_text())
    r = pat.findall((csrc / "emcmc_rtc.hip").read_text())
    assert k and r and k == r, (k, r)
    t = int(k[0])
    assert t > 0 and t & (t - 1) == 0  # a power of two: tile starts are c & ~(T - 1)


def test_state_pos_tiling_matches_the_documented_formula():
    """state_pos as include/emcmc.h documents it for emcmc_history_device_ptr: tiles of
    T = 32 chains when 32 | C (else one tile of C), pair-interleaved inside a tile; a
    bijection of the D·C slot positions (restated here; the device gathers through the
    same function, tests/test_gpu_* compare every history bitwise)."""
    def pos(d, c, C, D):
        T = 32 if C % 32 == 0 else C
        c0 = c - c % T
        return c0 * D + (((d // 2) * T + (c - c0)) * 2 + d % 2 if D % 2 == 0 else d * T + (c - c0))

    for C, D in ((64, 32), (96, 5), (1000, 32), (37, 7), (32, 64)):
        seen = {pos(d, c, C, D) for c in range(C) for d in range(D)}
        assert seen == set(range(C * D)), (C, D)
    # a wave's 32 chains (one tile at LPC = 2) write pair k of all its chains contiguously
    C, D = 65536, 32
    base = pos(0, 32 * 7, C, D)
    assert [pos(2 * 3, 32 * 7 + c, C, D) for c in range(32)] == [base + 2 * (3 * 32 + c) for c in range(32)]
