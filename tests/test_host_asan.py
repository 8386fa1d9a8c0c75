"""Host C++ under AddressSanitizer + UBSan: `make asan` builds
tests/native/host_fuzz.cpp against range_coder.cpp and host_util.cpp with
-fsanitize=address,undefined and runs it (known-answer stream, multi-table round trips,
random / truncated / bit-flipped / empty .encoded streams, error contract, CRC-32C).
CPU only; any sanitizer report or failed check fails the test."""
import os
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.skipif(shutil.which("g++") is None, reason="needs g++")
def test_host_code_under_asan(tmp_path):
    build = subprocess.run(["make", "-C", ROOT, "build/host_fuzz_asan"], capture_output=True, text=True)
    assert build.returncode == 0, build.stderr[-2000:]
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=1:abort_on_error=0",
               UBSAN_OPTIONS="print_stacktrace=1:halt_on_error=1")
    env.pop("LD_PRELOAD", None)
    run = subprocess.run([os.path.join(ROOT, "build", "host_fuzz_asan"), str(tmp_path)], capture_output=True,
                         text=True, env=env, timeout=300)
    assert run.returncode == 0, (run.stdout[-2000:], run.stderr[-4000:])
    assert "host_fuzz ok" in run.stdout
