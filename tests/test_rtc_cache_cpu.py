"""The on-disk code-object cache of the run-time compiler (csrc/emcmc_rtc.hip; ADVICE r4
medium): entries are written only into a private directory of this user (created 0700),
through a private temporary renamed into place, and an entry is loaded only when its
payload digest checks out — a torn, truncated or altered file is recompiled and rewritten,
never run.  hiprtc needs no device, so each case compiles the D = 9 chol kernel
(`emcmc_prebuild_chol_kernel`) in a child process (the process-wide cache would otherwise
answer the second call) and reads EMCMC_RTC_LOG's "compiled" line to tell a compile from
a load."""
import os
import stat
import subprocess
import sys
from pathlib import Path

import pytest

ROOT = Path(__file__).resolve().parents[1]
PKG = ROOT / "extensiblemcmc.jl_amd"
MAGIC = b"EMCRTC2\n"


def prebuild(cache: Path, D: int = 9) -> str:
    """stderr of a child that prebuilds the chol kernel at D into `cache`"""
    code = (f"import sys; sys.path[:0] = [{str(ROOT)!r}, {str(PKG)!r}]; "
            f"from extensible_mcmc import _lib as L; L.prebuild_chol_kernel({D}, 0, 0)")
    env = dict(os.environ, EMCMC_RTC_CACHE=str(cache), EMCMC_RTC_LOG="1")
    r = subprocess.run([sys.executable, "-c", code], env=env, capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stderr[-2000:]
    return r.stderr


def entries(cache: Path):
    return sorted(p for p in cache.iterdir() if p.suffix == ".co")


@pytest.fixture(scope="module")
def built(tmp_path_factory):
    """a cache directory the first compile created, and that compile's entry bytes"""
    if not (PKG / "lib" / "libemcmc.so").exists():
        pytest.skip("libemcmc.so not built")
    cache = tmp_path_factory.mktemp("rtc") / "cache"
    log = prebuild(cache)
    assert "compiled" in log
    (co,) = entries(cache)
    return cache, co, co.read_bytes()


def test_first_compile_creates_a_private_directory_and_a_checked_entry(built):
    cache, co, data = built
    assert stat.S_IMODE(cache.stat().st_mode) == 0o700
    assert stat.S_IMODE(co.stat().st_mode) & 0o077 == 0  # mkstemp: 0600
    assert data.startswith(MAGIC) and len(data) > 1000
    assert not [p for p in cache.iterdir() if ".tmp." in p.name]  # renamed into place


def test_a_second_process_loads_the_entry(built):
    cache, co, data = built
    assert "compiled" not in prebuild(cache)
    assert co.read_bytes() == data


@pytest.mark.parametrize("damage", ["flip", "truncate", "pad", "zero"])
def test_a_damaged_entry_is_recompiled_not_loaded(built, damage):
    cache, co, data = built
    b = bytearray(data)
    if damage == "flip":
        b[len(b) // 2] ^= 0x40  # inside the code object
    elif damage == "truncate":
        b = b[:-100]
    elif damage == "pad":
        b += b"\0" * 16
    else:
        b = bytearray(MAGIC) + bytearray(len(data) - len(MAGIC))  # right length, zero-filled
    co.write_bytes(bytes(b))
    assert "compiled" in prebuild(cache)
    assert co.read_bytes() == data  # rewritten with the compile's own bytes


def test_a_group_writable_directory_is_not_used(tmp_path):
    if not (PKG / "lib" / "libemcmc.so").exists():
        pytest.skip("libemcmc.so not built")
    cache = tmp_path / "shared"
    cache.mkdir()
    os.chmod(cache, 0o775)
    log = prebuild(cache)
    # said without EMCMC_RTC_LOG too: the refusal costs a compile in every process
    assert "warning" in log and "not a private directory" in log and "mode 775" in log and "compiled" in log
    assert log.count("not a private directory") == 1  # once per process
    assert entries(cache) == []
    assert "compiled" in prebuild(cache)  # and nothing was loaded from it either
