"""Host AddressSanitizer + UndefinedBehaviorSanitizer run of the host code: the
symbolic plan (orderings, supernodes, partition, per-rank layouts, projection) and the CPU oracle
(fixed-pivot LU, solves, multifrontal pivot-choosing LU) built with -fsanitize=address,undefined
and driven over several matrices (tools/sanitize/host_asan.cpp).  Device code is not part of it:
GPU sanitizers are not available on this pool."""
import os
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.skipif(shutil.which("g++") is None, reason="needs g++ with libasan/libubsan")
def test_host_code_under_asan_ubsan():
    r = subprocess.run(["make", "-s", "-j8", "-C", os.path.join(ROOT, "tools", "sanitize"), "run"],
                       capture_output=True, text=True, timeout=600)
    out = r.stdout + r.stderr
    assert r.returncode == 0, out[-4000:]
    assert "HOST SANITIZER RUN OK" in out
    assert "ERROR: AddressSanitizer" not in out and "runtime error" not in out, out[-4000:]
