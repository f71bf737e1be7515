#!/usr/bin/env python3
"""Check the inline-asm v_fmac_f64_dpp of mix_res_kernel (csrc/emcmc_mixres.h fmac_bcast)
for the VALU-write → DPP-read hazard the compiler does not see inside inline asm: a VGPR
written by a VALU instruction needs two wait states before a DPP instruction reads it.
The gfx950 code object is unbundled from the built object (build/obj/inst_mix.o), the
kernels are disassembled, and for every v_fmac_f64_dpp the two preceding slots are
inspected (an s_nop N provides N + 1 wait states; any other instruction one).  Exit 1
with the offending lines if a DPP source was written too recently.

  python3 scripts/check_dpp_hazards.py [path/to/inst_mix.o]
"""
import re
import subprocess
import sys
import tempfile
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
LLVM = Path("/opt/rocm/lib/llvm/bin")


def disassemble(obj: Path) -> str:
    with tempfile.TemporaryDirectory() as t:
        fat = Path(t) / "fatbin"
        co = Path(t) / "gfx950.co"
        subprocess.run([str(LLVM / "llvm-objcopy"), f"--dump-section=.hip_fatbin={fat}", str(obj), str(Path(t) / "x")],
                       check=True, capture_output=True)
        subprocess.run([str(LLVM / "clang-offload-bundler"), "--unbundle", "--type=o", f"--input={fat}",
                        "--targets=hipv4-amdgcn-amd-amdhsa--gfx950", f"--output={co}"], check=True, capture_output=True)
        return subprocess.run([str(LLVM / "llvm-objdump"), "-d", "--mcpu=gfx950", "--no-show-raw-insn", str(co)],
                              check=True, capture_output=True, text=True).stdout


def regs(op: str):
    """VGPR numbers named by one operand (v5, v[4:5])."""
    m = re.fullmatch(r"v(\d+)", op)
    if m:
        return {int(m.group(1))}
    m = re.fullmatch(r"v\[(\d+):(\d+)\]", op)
    if m:
        return set(range(int(m.group(1)), int(m.group(2)) + 1))
    return set()


def parse(line: str):
    line = line.split("//")[0].split(";")[0].strip()
    if not line or line.endswith(":"):
        return None
    parts = line.split(None, 1)
    ops = [o.strip() for o in parts[1].split(",")] if len(parts) > 1 else []
    return parts[0], ops


def check(asm: str):
    bad, n = [], 0
    in_kernel = False
    window = []  # (mnemonic, written VGPRs, wait states it provides), most recent last
    for raw in asm.splitlines():
        if raw.strip().endswith(">:"):  # a symbol
            in_kernel = "mix_res_kernel" in raw
            window = []
            continue
        if not in_kernel:
            continue
        p = parse(raw)
        if p is None:
            continue
        mn, ops = p
        if mn == "v_fmac_f64_dpp":
            n += 1
            src = regs(ops[1]) if len(ops) > 1 else set()
            waits = 0
            for pm, pw, pws in reversed(window):
                if waits >= 2:
                    break
                if pm.startswith("v_") and (pw & src):
                    bad.append(f"{raw.strip()}  ← {pm} wrote v{sorted(pw & src)} {waits} wait state(s) before")
                    break
                waits += pws
        written = regs(ops[0]) if (mn.startswith("v_") and ops and not mn.startswith("v_cmp")) else set()
        ws = int(ops[0], 0) + 1 if (mn == "s_nop" and ops) else 1
        window.append((mn, written, ws))
        window = window[-4:]
    return n, bad


def main():
    obj = Path(sys.argv[1]) if len(sys.argv) > 1 else ROOT / "extensiblemcmc.jl_amd" / "build" / "obj" / "inst_mix.o"
    n, bad = check(disassemble(obj))
    if n == 0:
        print("no v_fmac_f64_dpp found in mix_res_kernel", file=sys.stderr)
        sys.exit(2)
    if bad:
        print("\n".join(bad))
        sys.exit(1)
    print(f"{n} v_fmac_f64_dpp in mix_res_kernel: every DPP source written ≥ 2 wait states before")


if __name__ == "__main__":
    main()
