"""The CPU restatement under AddressSanitizer + UndefinedBehaviorSanitizer
("race detection / sanitizers": the host-side counterpart; the
device has no shared mutable state on the hot path).  oracle/Makefile's
`sanitize` target builds liboracle_san.so; a child process preloads the
sanitizer runtimes and drives every oracle entry point (tests/sanitized_oracle_run.py)."""
import os
import subprocess
import sys
from pathlib import Path

import pytest

ROOT = Path(__file__).resolve().parent.parent


def _runtime(name):
    p = subprocess.run(["gcc", f"-print-file-name={name}"], capture_output=True, text=True).stdout.strip()
    return p if p and os.path.isabs(p) and os.path.exists(p) else None


def test_oracle_under_asan_and_ubsan():
    asan, ubsan = _runtime("libasan.so"), _runtime("libubsan.so")
    if not asan or not ubsan:
        pytest.skip("gcc sanitizer runtimes not installed")
    subprocess.run(["make", "-C", str(ROOT / "oracle"), "sanitize"], check=True, capture_output=True)
    env = dict(os.environ)
    env.update(LD_PRELOAD=f"{asan}:{ubsan}", EMCMC_ORACLE_LIB=str(ROOT / "oracle" / "lib" / "liboracle_san.so"),
               ASAN_OPTIONS="detect_leaks=0:abort_on_error=0:halt_on_error=1",
               UBSAN_OPTIONS="print_stacktrace=1:halt_on_error=1", OMP_NUM_THREADS="1")
    r = subprocess.run([sys.executable, str(ROOT / "tests" / "sanitized_oracle_run.py")], env=env,
                       capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stderr[-4000:]
    assert "sanitized oracle run: ok liboracle_san.so" in r.stdout
    assert "AddressSanitizer" not in r.stderr and "runtime error" not in r.stderr, r.stderr[-4000:]
