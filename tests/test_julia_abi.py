"""The Julia MI355XBackend shim and the Python ctypes mirror bind the same C
structs as include/emcmc.h: every `struct Emcmc*` of ExtensibleMCMCHip.jl and
every ctypes Structure of _lib.py is laid out with C rules and compared field by
field (name, offset) and in size against offsetof/sizeof from a gcc-compiled
probe of the header.  (There is no Julia in the image, so the shim cannot be
executed; its struct layouts and ccall names are what can be checked.)"""
import ctypes as C
import re
import subprocess
from pathlib import Path

import pytest

from extensible_mcmc import _lib as L

ROOT = Path(__file__).resolve().parent.parent
HEADER = ROOT / "include" / "emcmc.h"
SHIM = ROOT / "extensiblemcmc.jl_amd" / "julia" / "ExtensibleMCMCHip.jl"

C_NAME = {"EmcmcConfig": "emcmc_config", "EmcmcUpdateDesc": "emcmc_update_desc",
          "EmcmcHaarioAdaptation": "emcmc_haario_adaptation", "EmcmcUnifRWAdaptation": "emcmc_unifrw_adaptation",
          "EmcmcUnifRWAdaptationVec": "emcmc_unifrw_adaptation_vec",
          "EmcmcTargetDesc": "emcmc_target_desc", "EmcmcStep": "emcmc_step", "EmcmcMoments": "emcmc_moments",
          "EmcmcPriorFactor": "emcmc_prior_factor", "EmcmcPriorDesc": "emcmc_prior_desc",
          "EmcmcUserTargetDesc": "emcmc_user_target_desc", "EmcmcUserUpdateDesc": "emcmc_user_update_desc",
          "EmcmcDiag": "emcmc_diag"}

JL_SCALAR = {"UInt8": 1, "Int8": 1, "UInt16": 2, "Int16": 2, "UInt32": 4, "Int32": 4, "Cint": 4, "Float32": 4,
             "UInt64": 8, "Int64": 8, "Float64": 8, "Csize_t": 8, "Cstring": 8}


def jl_type(t):
    """(size, alignment) of a Julia isbits field type as laid out in a C-compatible struct."""
    t = t.strip()
    if t.startswith("Ptr{") or t == "Ptr":
        return 8, 8
    m = re.fullmatch(r"NTuple\{(\d+),\s*(.+)\}", t)
    if m:
        n, (sz, al) = int(m.group(1)), jl_type(m.group(2))
        return n * sz, al
    return JL_SCALAR[t], JL_SCALAR[t]


def julia_structs():
    src = SHIM.read_text()
    out = {}
    for m in re.finditer(r"^struct (Emcmc\w+)\n(.*?)^end", src, flags=re.S | re.M):
        fields = []
        for line in m.group(2).split("\n"):
            line = line.split("#")[0].strip()
            if "::" in line:
                name, typ = line.split("::", 1)
                fields.append((name.strip(), typ.strip()))
        out[m.group(1)] = fields
    return out


def c_layout(fields):
    off, al_max, offs = 0, 1, []
    for name, (sz, al) in fields:
        off = (off + al - 1) // al * al
        offs.append((name, off))
        off += sz
        al_max = max(al_max, al)
    return offs, (off + al_max - 1) // al_max * al_max


def probe(tmp_path, queries):
    """queries: [(c_struct, [field, ...])] → {c_struct: (sizeof, [offsetof...])}"""
    lines = ['#include <stdio.h>', '#include <stddef.h>', '#include "emcmc.h"', "int main(void) {"]
    for cs, fs in queries:
        lines.append(f'  printf("%zu", sizeof({cs}));')
        for f in fs:
            lines.append(f'  printf(" %zu", offsetof({cs}, {f}));')
        lines.append('  printf("\\n");')
    lines += ["  return 0;", "}"]
    c = tmp_path / "probe.c"
    c.write_text("\n".join(lines))
    exe = tmp_path / "probe"
    subprocess.run(["gcc", "-std=c11", "-I", str(HEADER.parent), str(c), "-o", str(exe)], check=True)
    rows = subprocess.run([str(exe)], capture_output=True, text=True, check=True).stdout.strip().split("\n")
    res = {}
    for (cs, _), row in zip(queries, rows):
        v = [int(x) for x in row.split()]
        res[cs] = (v[0], v[1:])
    return res


def header_structs():
    txt = re.sub(r"/\*.*?\*/", "", HEADER.read_text(), flags=re.S)
    return set(re.findall(r"typedef struct (emcmc_\w+)\s*\{", txt))


def test_julia_structs_match_the_header(tmp_path):
    js = julia_structs()
    assert set(C_NAME) <= set(js), set(C_NAME) - set(js)
    queries = [(C_NAME[n], [f for f, _ in js[n]]) for n in C_NAME]
    got = probe(tmp_path, queries)
    for n in C_NAME:
        offs, size = c_layout([(f, jl_type(t)) for f, t in js[n]])
        csize, coffs = got[C_NAME[n]]
        assert size == csize, f"{n}: Julia {size} B vs C {csize} B"
        assert [o for _, o in offs] == coffs, f"{n}: field offsets differ"
    # every public struct of the header has a Julia twin
    assert header_structs() == set(C_NAME.values())


def test_ctypes_structs_match_the_header(tmp_path):
    classes = {n: getattr(L, n) for n in C_NAME if hasattr(L, n)}
    assert set(classes) == set(C_NAME), set(C_NAME) - set(classes)
    queries = [(C_NAME[n], [f for f, _ in cls._fields_]) for n, cls in classes.items()]
    got = probe(tmp_path, queries)
    for n, cls in classes.items():
        csize, coffs = got[C_NAME[n]]
        assert C.sizeof(cls) == csize, n
        assert [getattr(cls, f).offset for f, _ in cls._fields_] == coffs, n


@pytest.mark.parametrize("fn", ["emcmc_get_proposal_ll", "emcmc_get_history_chains", "emcmc_get_state"])
def test_callback_accessors_bind_declared_functions(fn):
    """The views REPLCallback/SavingCallback read through (callbacks.jl:246-319) call these."""
    assert f"ccall((:{fn}, LIB)" in SHIM.read_text()


def test_reference_accessors_are_defined():
    src = SHIM.read_text()
    for f in ("num_mcmc_steps", "num_updt", "estim_mean", "estim_cov", "accepted", "ll", "ll°", "state",
              "state°", "name_of_update"):
        assert re.search(rf"^(function )?eMCMC\.{re.escape(f)}\(", src, flags=re.M), f
    for prop in (":sub_ws", ":sub_ws°", ":acceptance_history", ":state_history", ":state_proposal_history",
                 ":ll_history"):
        assert prop in src, prop


# The fields only a RandomWalkUpdate carries (updates.jl:163-170): the plugin
# updates HipUpdate / HipMALAUpdate have neither `rw` nor a Haario `adpt`.
_RW_ONLY = re.compile(r"\b(?:u|updt)\.(?:rw|adpt)\b")
_ALLOWED_DEF = re.compile(r"^(function _update_desc\(updt::eMCMC\.RandomWalkUpdate|_mix\(u\) =|_haario_mix\(u\) =)")
_GUARD = re.compile(r"^\s*(?:if|elseif)\s+(?:_mix\(u\)|_haario_mix\(u\)|u isa eMCMC\.RandomWalkUpdate)")


def _indent(line):
    return len(line) - len(line.lstrip(" "))


def test_rw_field_reads_are_guarded():
    """Every read of `.rw` / `.adpt` on an update sits inside
    `_update_desc(::RandomWalkUpdate)`, the `_mix` / `_haario_mix` predicates, or an
    `if` on one of them: init_global_workspace and __run! loop over every update,
    user plugins included (round-3 defect: a FieldError on `u.rw` before the first
    ccall of a HipUpdate / HipMALAUpdate run)."""
    lines = SHIM.read_text().split("\n")
    bad = []
    for i, line in enumerate(lines):
        code = line.split("#")[0]
        if not _RW_ONLY.search(code):
            continue
        if _ALLOWED_DEF.match(code):
            continue
        ok, level = False, _indent(line)
        for j in range(i - 1, -1, -1):  # the enclosing lines, innermost first
            up = lines[j]
            if not up.strip() or _indent(up) >= level:
                continue
            level = _indent(up)
            if _GUARD.match(up) or _ALLOWED_DEF.match(up):
                ok = True
                break
            if level == 0:
                break
        if not ok:
            bad.append(f"{i + 1}: {line.strip()}")
    assert not bad, "unguarded RandomWalkUpdate field reads:\n" + "\n".join(bad)


def test_plugin_updates_reach_emcmc_add_update():
    """HipUpdate and HipMALAUpdate have a `_update_desc` method, and the loop that
    passes each update to emcmc_add_update reads no RandomWalkUpdate field before
    the ccall."""
    src = SHIM.read_text()
    for t in ("HipUpdate", "HipMALAUpdate"):
        assert re.search(rf"^function _update_desc\(updt::{t}, keep\)", src, flags=re.M), t
    loop = src[src.index("for (i, u) in enumerate(updates)"):src.index(":emcmc_add_update")]
    assert not _RW_ONLY.search(loop), loop


def test_diagnostics_collective_is_bound():
    """The cross-rank diagnostics (SURVEY §8(b) emcmc_diagnostics) reach the Julia caller:
    the RCCL and host-callback communicators and the diagnostics call itself."""
    src = SHIM.read_text()
    for fn in ("emcmc_comm_unique_id", "emcmc_comm_init", "emcmc_comm_init_host", "emcmc_comm_destroy",
               "emcmc_comm_last_error", "emcmc_diagnostics"):
        assert f"ccall((:{fn}, LIB)" in src, fn
    assert re.search(r"@cfunction\(_allgather_trampoline, Cint, \(Ptr\{Float64\}, Ptr\{Float64\}, UInt64, "
                     r"Ptr\{Cvoid\}\)\)", src)
