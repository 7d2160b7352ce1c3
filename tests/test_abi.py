"""CPU-side checks of the product boundary: libjlcrc.so loads, exports every
entry point include/jlcrc.h declares, its host scalar statics and the Crc32C
mirror behave as the reference's T/TestCrc32C.java requires, and the batch
entry points refuse to run without a GPU (no CPU fallback)."""
import os
import re
import subprocess

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def declared_symbols():
    text = open(os.path.join(ROOT, "include", "jlcrc.h")).read()
    return sorted(set(re.findall(r"\b(jl_[a-z0-9_]+)\s*\(", text)))


def test_library_exports_every_declared_symbol(jl):
    out = subprocess.run(["nm", "-D", "--defined-only", jl.LIB_PATH], capture_output=True, text=True, check=True).stdout
    exported = {line.split()[-1] for line in out.splitlines() if " T " in line}
    missing = [s for s in declared_symbols() if s not in exported]
    assert not missing, missing
    lib = jl.lib()
    for s in declared_symbols():
        assert hasattr(lib, s)


def test_library_has_gfx950_code_object(jl, tmp_path):
    # llvm-objdump --offloading extracts the bundles next to its input: work on a copy
    import shutil

    lib_copy = tmp_path / "libjlcrc.so"
    shutil.copy(jl.LIB_PATH, lib_copy)
    out = subprocess.run(["/opt/rocm/lib/llvm/bin/llvm-objdump", "--offloading", str(lib_copy)],
                         capture_output=True, text=True, cwd=tmp_path).stdout
    assert "gfx950" in out


# --- T/TestCrc32C.java re-expressed against the Crc32C mirror -------------
def test01_resume(jl):
    data = bytes(range(127))
    c = jl.Crc32C()
    c.update(data, 0, len(data))
    ret1 = c.getValue()
    c2 = jl.Crc32C()
    c2.update(data, 0, 50)
    c3 = jl.Crc32C()
    c3.setValue(c2.getValue())
    c3.update(data, 50, len(data) - 50)
    assert ret1 == c3.getValue()


def test_standard_results(jl, golden):
    for k in golden("golden.json")["kats"]:
        assert jl.Crc32C.value(bytes.fromhex(k["hex"])) == k["value"], k["name"]


def test_values(jl):
    assert jl.Crc32C.value(b"a") != jl.Crc32C.value(b"foo")


def test_extend(jl):
    assert jl.Crc32C.value(b"hello world") == jl.Crc32C.extend(jl.Crc32C.value(b"hello "), b"world")


def test_mask(jl):
    C = jl.Crc32C
    crc = C.value(b"foo")
    assert crc != C.mask(crc)
    assert crc != C.mask(C.mask(crc))
    assert crc == C.unmask(C.mask(crc))
    assert crc == C.unmask(C.unmask(C.mask(C.mask(crc))))


def test_update_int_and_offsets(jl, oracle):
    c = jl.Crc32C()
    for b in b"jleveldb":
        c.update(b)
    assert c.getValue() == oracle.value(b"jleveldb")
    buf = b"0123456789"
    assert jl.Crc32C.value(buf, 2, 5) == oracle.value(buf[2:7])
    with pytest.raises(IndexError):
        jl.Crc32C.value(buf, 8, 5)


def test_host_scalar_matches_oracle(jl, oracle):
    rng = np.random.default_rng(7)
    buf = rng.integers(0, 256, 20000, dtype=np.uint8)
    for n in list(range(0, 40)) + [63, 64, 65, 4096, 4101, 19999]:
        o = int(rng.integers(0, 8))
        seg = buf[o:o + n]
        assert jl.Crc32C.value(seg) == oracle.value(seg)
        init = int(rng.integers(0, 2**32))
        assert jl.Crc32C.extend(init, seg) == oracle.extend(init, seg)
    for v in [0, 1, 0xFFFFFFFF, 0x12345678, 0xA282EAD8]:
        assert jl.Crc32C.mask(v) == oracle.mask(v)
        assert jl.Crc32C.unmask(v) == oracle.unmask(v)


def test_derived_goldens_host(jl, golden):
    d = golden("golden.json")["derived"]
    assert [jl.Crc32C.value(bytes([t])) for t in range(5)] == d["type_crc"]
    assert jl.Crc32C.mask(0) == d["mask0"]


@pytest.mark.skipif(os.path.exists("/dev/kfd") and os.access("/dev/kfd", os.R_OK), reason="a GPU is present")
def test_batch_fails_loudly_without_gpu(jl):
    arena = np.zeros(64, dtype=np.uint8)
    with pytest.raises(jl.JLError):
        jl.crc32c_batch(arena, np.array([0], np.uint64), np.array([64], np.uint32))
    with pytest.raises(jl.JLError):
        jl.log_verify(b"\0" * 64)


def test_engine_math_emulation():
    """Host emulation of the device lane algorithm (LDS image, gap tables,
    z^-(4l) re-alignment, front injection) against a byte-serial CRC."""
    exe = "/tmp/jlcrc_emulate_engine"
    subprocess.run(["g++", "-O2", "-std=c++17", os.path.join(ROOT, "tests", "cpp", "emulate_engine.cpp"), "-o", exe],
                   check=True)
    r = subprocess.run([exe], capture_output=True, text=True)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "0 mismatches" in r.stdout


# --- LogWriter.addRecord framing plan (host C++, no device work) -----------
def _records(seed, n):
    rng = np.random.default_rng(seed)
    lens = rng.choice([0, 1, 6, 7, 100, 1056, 32761, 32762, 40000, 100000], size=n).astype(np.uint32)
    payloads = [rng.integers(0, 256, int(k), dtype=np.uint8).tobytes() for k in lens]
    return payloads, lens


@pytest.mark.parametrize("dest_length", [0, 32768 - 7, 32768 - 3, 5000])
def test_log_layout_matches_logwriter(jl, oracle, dest_length):
    payloads, lens = _records(dest_length + 1, 60)
    offs = np.zeros(lens.size, np.uint64)
    offs[1:] = np.cumsum(lens[:-1], dtype=np.uint64)
    plan = jl.log_layout(offs, lens, dest_length)
    ref = oracle.log_write(payloads, dest_length)
    assert plan["log_bytes"] == len(ref)
    src = b"".join(payloads)
    img = bytearray(len(ref))
    for h, so, n, t in zip(plan["hdr_off"], plan["src_off"], plan["len"], plan["type"]):
        h, so, n = int(h), int(so), int(n)
        assert ref[h + 4] | (ref[h + 5] << 8) == n and ref[h + 6] == t
        img[h:h + 7] = ref[h:h + 7]  # CRC bytes are the device's job; framing is checked here
        img[h + 7:h + 7 + n] = src[so:so + n]
    assert bytes(img) == ref  # everything outside the fragments is zero trailer


def test_options_round_trip_and_ranges(jl):
    """jl_set_option / jl_get_option: every option keeps a valid value and refuses
    out-of-range ones (JL_ERR_INVALID, the previous value kept); no device needed."""
    cases = [  # option, valid values, invalid values
        (jl.OPT_HOST_REGISTER, [0, 1], [2, -1]),
        (jl.OPT_STAGE_THREADS, [1, 8, 64], [0, 65]),
        (jl.OPT_HOST_THRESHOLD, [0, 2 << 20, jl.HOST_THRESHOLD_AUTO], [-2]),
        (jl.OPT_LOG_HOST_THRESHOLD, [0, 8 << 20, jl.HOST_THRESHOLD_AUTO], [-2]),
        (jl.OPT_LOG_SMALL_MAX, [0, 64 << 20, 16 << 20], [-1, (64 << 20) + 1]),
        (jl.OPT_STAGE_PIECE, [0, 1 << 20, 16 << 20], [-1, 4096]),
    ]
    for opt, good, bad in cases:
        prev = jl.get_option(opt)
        try:
            for v in good:
                jl.set_option(opt, v)
                assert jl.get_option(opt) == v
            for v in bad:
                with pytest.raises(Exception):
                    jl.set_option(opt, v)
                assert jl.get_option(opt) == good[-1]
        finally:
            jl.set_option(opt, prev)
    assert jl.get_option(jl.OPT_STAGE_PIECE) == 16 << 20
