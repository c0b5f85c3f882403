"""Host code under AddressSanitizer + UndefinedBehaviorSanitizer (CPU only).

`make -C quadruped-pympc-tamols_amd asan` (run by __graft_entry__.build()) builds
libsrbd_hip_asan.so: the C-ABI and host merge (srbd_api.hip, host side) and the host producers /
SHM transport (srbd_host.cpp) instrumented, the device code as usual.  This test runs the host-logic,
C-ABI and SHM test files in a child process against that library with the sanitizer runtime
preloaded (Python itself is not instrumented); any report aborts the child and fails the test.
"""
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "quadruped-pympc-tamols_amd")
ASAN_LIB = os.path.join(PKG, "quadruped_pympc_amd", "libsrbd_hip_asan.so")


def runtime_path():
    try:
        out = subprocess.run(["/opt/rocm/bin/hipcc", "-print-file-name=libclang_rt.asan-x86_64.so"],
                             capture_output=True, text=True, timeout=60).stdout.strip()
    except (OSError, subprocess.TimeoutExpired):
        return None
    return out if out and os.path.isfile(out) else None


def test_host_code_clean_under_asan_ubsan():
    if not os.path.isfile(ASAN_LIB):
        pytest.fail("libsrbd_hip_asan.so missing: run `make -C quadruped-pympc-tamols_amd asan` (build() does)")
    rt = runtime_path()
    if rt is None:
        pytest.skip("clang ASan runtime not found (ROCm LLVM)")
    env = dict(os.environ)
    env.update(SRBD_LIB_PATH=ASAN_LIB, LD_PRELOAD=rt,
               ASAN_OPTIONS="detect_leaks=0:halt_on_error=1:abort_on_error=1",
               UBSAN_OPTIONS="halt_on_error=1:print_stacktrace=1")
    files = [os.path.join(ROOT, "tests", f) for f in ("test_host_logic.py", "test_capi.py", "test_shm_transport.py")]
    r = subprocess.run([sys.executable, "-m", "pytest", "-q", "-x", "-m", "not gpu", "-p", "no:cacheprovider",
                        *files], cwd=ROOT, env=env, capture_output=True, text=True, timeout=900)
    tail = (r.stdout + r.stderr)[-4000:]
    assert r.returncode == 0, tail
    assert "ERROR: AddressSanitizer" not in r.stderr and "runtime error:" not in r.stderr, tail
    assert " passed" in r.stdout, tail
