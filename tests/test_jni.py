"""The JNI adapter (jleveldb_amd/jni/jlcrc_jni.c) driven through a fake JVM.

This image has no JDK, so the adapter is compiled against a test-only JNIEnv
function table (tests/cpp/jni_stub/jni.h) and exercised by tests/cpp/jni_harness.c:
Crc32C.value / extend / update (J/util/Crc32C.java:43-48,85-93,119-162) against
the C-ABI scalars, out-of-range (offset, n) -> ArrayIndexOutOfBoundsException
with no array access, the block-handle walk's grow-and-retry protocol
(Crc32CShims.verifyTable) at every capacity, bad arguments ->
IllegalArgumentException, and the JNI rules (no call with an exception pending
or inside a critical region, region copies in bounds and of the right type,
JNI_ABORT releases).  CPU suite: under ASan/UBSan, the device entry points
failing cleanly with JL_ERR_NO_DEVICE.  GPU suite: tableVerify / logVerify on
direct buffers equal jl_table_verify / jl_log_verify (the call sites
TableFormat.java:211-212 and LogReader.java:357-358), flips seen.
"""
import os
import shutil
import subprocess

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CPP = os.path.join(ROOT, "tests", "cpp")
SST = os.path.join(ROOT, "tests", "golden", "sstable.bin")


@pytest.fixture(scope="module")
def harness(jl):
    if not shutil.which("gcc"):
        pytest.skip("no gcc")
    if not os.path.exists(os.path.join(CPP, "_build", "jni_harness")):  # built in-tree before a GPU run
        subprocess.run(["make", "-s", "-C", CPP], check=True)
    return os.path.join(CPP, "_build")


def test_jni_adapter_cpu_asan(harness):
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=0", UBSAN_OPTIONS="print_stacktrace=1")
    r = subprocess.run([os.path.join(harness, "jni_harness_san"), "cpu", SST], capture_output=True, text=True,
                       env=env, timeout=300)
    assert r.returncode == 0, r.stderr[-4000:]
    assert r.stdout.startswith("OK ") and int(r.stdout.split()[1]) > 40000


@pytest.mark.gpu
def test_jni_adapter_gpu(harness, oracle, tmp_path):
    rng = np.random.default_rng(77)
    log = bytearray(oracle.log_write([rng.integers(0, 256, int(n), dtype=np.uint8).tobytes()
                                      for n in rng.integers(0, 3000, 400)]))
    log[len(log) // 2] ^= 0x08
    p = tmp_path / "wal.log"
    p.write_bytes(bytes(log))
    r = subprocess.run([os.path.join(harness, "jni_harness"), "gpu", SST, str(p)], capture_output=True, text=True,
                       timeout=300)
    assert r.returncode == 0, r.stderr[-4000:]
    assert r.stdout.startswith("OK ")
