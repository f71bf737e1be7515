"""The inline-asm v_fmac_f64_dpp of mix_res_kernel (csrc/emcmc_mixres.h) is invisible to the
compiler's hazard recognizer: scripts/check_dpp_hazards.py disassembles the built gfx950 code
object and fails when a DPP source VGPR was written by a VALU instruction fewer than two wait
states before.  The checker is exercised on synthetic listings, then on the build."""
import sys
from pathlib import Path

import pytest

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT / "scripts"))
import check_dpp_hazards as H  # noqa: E402

HEAD = "0000000000001000 <_ZN5emcmc14mix_res_kernelILi32ELb1ELi0ELb1EEEvNS_9MixParamsE>:\n"


def test_checker_flags_a_fresh_write():
    asm = HEAD + "\tv_mov_b64 v[20:21], v[40:41]\n\tv_fmac_f64_dpp v[10:11], v[20:21], v[30:31] row_newbcast:1\n"
    n, bad = H.check(asm)
    assert n == 1 and len(bad) == 1


def test_checker_accepts_waits():
    for gap in ("\ts_nop 1\n", "\tv_add_f64 v[50:51], v[52:53], v[54:55]\n\ts_nop 0\n"):
        asm = HEAD + "\tv_mov_b64 v[20:21], v[40:41]\n" + gap + \
            "\tv_fmac_f64_dpp v[10:11], v[20:21], v[30:31] row_newbcast:1\n"
        n, bad = H.check(asm)
        assert n == 1 and not bad, (gap, bad)


def test_checker_ignores_other_kernels():
    asm = "0000000000002000 <other_kernel>:\n\tv_mov_b64 v[20:21], v[40:41]\n" \
          "\tv_fmac_f64_dpp v[10:11], v[20:21], v[30:31] row_newbcast:1\n"
    assert H.check(asm) == (0, [])


def test_built_mix_res_kernel_has_no_dpp_hazard():
    obj = ROOT / "extensiblemcmc.jl_amd" / "build" / "obj" / "inst_mix.o"
    if not obj.exists():
        pytest.skip("library not built (make -C extensiblemcmc.jl_amd)")
    n, bad = H.check(H.disassemble(obj))
    assert n > 0, "no v_fmac_f64_dpp found: the checker no longer sees the sweep"
    assert not bad, "\n".join(bad)
