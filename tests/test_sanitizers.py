"""Host-compiled pieces under AddressSanitizer + UndefinedBehaviorSanitizer
(SURVEY.md §5): the kernel's headers np_math.h (the reference NumPy's
transcendentals) and nproots.h (np.roots restated), built for the host as the
bitwise tests build them, run over random, edge and special inputs
(oracle/asan_host.cpp, ``make -C oracle asan``).  Any out-of-bounds table
read, signed overflow or bad shift aborts the run."""
import os
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_np_math_and_nproots_clean_under_asan_ubsan():
    if shutil.which("g++") is None:
        pytest.skip("g++ not available")
    b = subprocess.run(["make", "-C", os.path.join(ROOT, "oracle"), "asan"], capture_output=True, text=True)
    if b.returncode != 0 and "sanitize" in b.stderr:
        pytest.skip("this toolchain has no sanitizer runtime: " + b.stderr[-300:])
    assert b.returncode == 0, b.stderr[-2000:]
    # (verify_asan_link_order=0: the environment may preload a library of its own)
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=1:abort_on_error=1:verify_asan_link_order=0",
               UBSAN_OPTIONS="print_stacktrace=1:halt_on_error=1")
    r = subprocess.run([os.path.join(ROOT, "oracle", "_devmath", "asan_host"), "300000"],
                       capture_output=True, text=True, env=env, timeout=300)
    assert r.returncode == 0, (r.stdout + r.stderr)[-3000:]
    assert "asan_host ok" in r.stdout
    assert "runtime error" not in r.stderr and "AddressSanitizer" not in r.stderr
