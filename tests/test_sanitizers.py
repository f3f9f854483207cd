"""The host C++ under AddressSanitizer + UndefinedBehaviorSanitizer (VERDICT r04 "Next round" 9).

tests/native/sanitize_main.cpp and tests/native/host_ops.cpp (the kernels' per-lane arithmetic compiled for x86, the
same source the GPU runs) are built as one executable with -fsanitize=address,undefined -fno-sanitize-recover=all and
run: the batch split planner of the host runtime (charon_amd/csrc/ranges.h), sign/verify round trips in both
Miller-loop forms, Shamir threshold aggregation on both Lagrange paths, the RLC windows pipeline and the batch-wide
Pippenger check with invalid items, and the binary-GCD inversion.  Any memory error or undefined behaviour aborts the
run.  No GPU: the sanitizers cover host code only (GPU AddressSanitizer is not available on the pool).
"""
import os
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
NATIVE = os.path.join(ROOT, "tests", "native")


@pytest.mark.skipif(shutil.which("g++") is None, reason="no g++")
def test_host_code_clean_under_asan_ubsan(tmp_path):
    exe = str(tmp_path / "sanitize_main")
    subprocess.run(["g++", "-std=c++17", "-O1", "-g", "-fsanitize=address,undefined", "-fno-sanitize-recover=all",
                    "-fno-omit-frame-pointer", "-o", exe, os.path.join(NATIVE, "sanitize_main.cpp"),
                    os.path.join(NATIVE, "host_ops.cpp")], check=True, timeout=600)
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=1:abort_on_error=1", UBSAN_OPTIONS="print_stacktrace=1")
    env.pop("LD_PRELOAD", None)
    r = subprocess.run([exe], capture_output=True, text=True, timeout=600, env=env)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "sanitize OK" in r.stdout
