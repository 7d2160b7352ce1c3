"""The engine's host-side C++ under AddressSanitizer + UndefinedBehaviorSanitizer
(and the staging copy pool under ThreadSanitizer).

tests/cpp/fuzz_host.cpp links table_walker.cpp, log_reader.cpp, log_writer.cpp
and host_crc.cpp (and the oracle) with -fsanitize=address,undefined and feeds
them mutated SSTable images, random log-writer plans and corrupted logs, checking
each against the oracle (see its header).  Any sanitizer report aborts the run
(-fno-sanitize-recover=all).  CPU only: the GPU kernels cannot run under ASan on
this pool, and their inputs are range-checked on the device instead
(tests/test_gpu_robust.py).
"""
import os
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CPP = os.path.join(ROOT, "tests", "cpp")


@pytest.fixture(scope="module")
def harness():
    if not shutil.which("g++"):
        pytest.skip("no g++")
    subprocess.run(["make", "-s", "-C", CPP], check=True)
    return os.path.join(CPP, "_build", "fuzz_host")


def test_host_code_under_asan_ubsan(harness):
    golden = os.path.join(ROOT, "tests", "golden")
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=1", UBSAN_OPTIONS="print_stacktrace=1")
    r = subprocess.run([harness, "2000", os.path.join(golden, "sstable.bin"), os.path.join(golden, "table.bin")],
                       capture_output=True, text=True, env=env, timeout=600)
    assert r.returncode == 0, r.stderr[-4000:]
    assert r.stdout.strip() == "OK 2000"


@pytest.mark.parametrize("san", ["tsan", "asan"])
def test_copy_pool_under_sanitizers(harness, san):
    """The staging copy pool (jleveldb_amd/csrc/copy_pool.hpp) of the host-memory
    entry points: 4 concurrent callers, copies around the piece sizes, every
    result compared (tests/cpp/copy_pool_test.cpp) — under ThreadSanitizer (data
    races on the job queue / cursors) and ASan/UBSan (a worker touching a job
    after its caller returned)."""
    exe = os.path.join(CPP, "_build", f"copy_pool_{san}")
    env = dict(os.environ, TSAN_OPTIONS="halt_on_error=1", ASAN_OPTIONS="detect_leaks=1")
    r = subprocess.run([exe, "100"], capture_output=True, text=True, env=env, timeout=300)
    assert r.returncode == 0, r.stderr[-4000:]
    assert r.stdout.strip() == "OK"
