"""The CPU oracle (test infrastructure) pinned against the reference's own
vectors: T/TestCrc32C.java KATs, the SHA-256 of the reference's literal table
(J/util/Crc32C.java:173-334), an independent bit-serial CRC, and the LogWriter /
LogReader / TableBuilder framing behaviour the reference tests pin."""
import hashlib
import struct

import numpy as np
import pytest


def test_table_matches_reference_literal_table(oracle, golden):
    t = oracle.tables()
    assert hashlib.sha256(t.astype("<u4").tobytes()).hexdigest() == golden("golden.json")["reference_table_sha256"]


def test_rfc3720_kats(oracle, golden):  # T/TestCrc32C.java:60-93
    for k in golden("golden.json")["kats"]:
        data = bytes.fromhex(k["hex"])
        assert oracle.value(data) == k["value"], k["name"]
        assert oracle.bitwise(data) == k["value"], k["name"]


def test_test01_resume(oracle):  # T/TestCrc32C.java:36-57
    data = bytes(range(127))
    whole = oracle.value(data)
    first = oracle.value(data[:50])
    assert oracle.extend(first, data[50:]) == whole


def test_values_and_extend(oracle):  # :96-109
    assert oracle.value(b"a") != oracle.value(b"foo")
    assert oracle.value(b"hello world") == oracle.extend(oracle.value(b"hello "), b"world")


def test_mask(oracle):  # :112-119
    crc = oracle.value(b"foo")
    assert crc != oracle.mask(crc)
    assert crc != oracle.mask(oracle.mask(crc))
    assert crc == oracle.unmask(oracle.mask(crc))
    assert crc == oracle.unmask(oracle.unmask(oracle.mask(oracle.mask(crc))))


def test_slicing_vs_bitwise_random(oracle):
    rng = np.random.default_rng(1)
    buf = rng.integers(0, 256, 70000, dtype=np.uint8).tobytes()
    for n in list(range(0, 70)) + [255, 256, 257, 4095, 4096, 4097, 4101, 32768, 65536]:
        o = int(rng.integers(0, 8))
        assert oracle.value(buf[o:o + n]) == oracle.bitwise(buf[o:o + n]), n


def test_update_byte_matches_update(oracle):  # update(int), Crc32C.java:165-167
    s = 0xFFFFFFFF
    data = b"jleveldb"
    for b in data:
        s = oracle.update_byte(s, b)
    assert s == oracle.update(0xFFFFFFFF, data)


def test_derived_goldens(oracle, golden):
    d = golden("golden.json")["derived"]
    assert [oracle.value(bytes([t])) for t in range(5)] == d["type_crc"]
    assert oracle.value(b"x" * 4096) == d["dbbench_4k_x"]
    assert oracle.table_trailer(b"x" * 4096).hex() == d["trailer_4096x"]


def test_block_fixture(oracle, golden):
    arena = np.frombuffer(golden("blocks.bin"), dtype=np.uint8)
    b = golden("blocks.json")
    off = np.array(b["off"], dtype=np.uint64)
    ln = np.array(b["len"], dtype=np.uint32)
    assert list(oracle.batch(arena, off, ln, flags=0)) == b["crc"]
    assert list(oracle.batch(arena, off, ln)) == b["masked"]
    assert list(oracle.batch(arena, off, ln, init=np.array(b["init"], dtype=np.uint32), flags=0)) == b["extend"]
    assert list(oracle.batch(arena, off, ln, suffix=np.zeros(len(ln), np.uint8), flags=0)) == b["suffix_crc_type0"]


def test_log_fixture_and_framing(oracle, golden):
    log = golden("log.bin")
    meta = golden("log.json")
    ev = oracle.log_events(log)
    assert [[int(e["offset"]), int(e["length"]), int(e["type"]), int(e["kind"])] for e in ev] == meta["events"]
    recs, reps = oracle.log_read(log)
    assert reps == []
    assert [r[0] for r in recs] == meta["record_offsets"]
    assert [hashlib.sha256(r[1]).hexdigest() for r in recs] == meta["payload_sha256"]
    # no record header ever leaves fewer than 7 bytes in a block (LogWriter.java:101-107)
    for e in ev:
        assert e["offset"] % 32768 <= 32768 - 7


def test_table_fixture(oracle, golden):
    f = golden("table.bin")
    meta = golden("table.json")
    for (off, n), tr in zip(meta["handles"], meta["trailers"]):
        assert f[off + n:off + n + 5].hex() == tr
        assert oracle.table_verify(f, off, n)
        bad = bytearray(f)
        bad[off + (n // 2 if n else 0)] ^= 0x80  # TestCorruption.corrupt flips 0x80
        assert not oracle.table_verify(bytes(bad), off, n)


def _batch_payload(i: int, value_len: int = 1000) -> bytes:
    """A WriteBatch with one Put (WriteBatchInternal header 12 B, tag, varint key/value).
    Key "%016d" and a 1000-byte value, the shape of TestCorruption.build (T/TestCorruption.java:125-140)."""
    key = b"%016d" % i
    val = bytes((i * 7 + j) & 0xFF for j in range(value_len))
    def varint(n):
        out = b""
        while n >= 0x80:
            out += bytes([(n & 0x7F) | 0x80])
            n >>= 7
        return out + bytes([n])
    return struct.pack("<QI", i + 1, 1) + b"\x01" + varint(len(key)) + key + varint(len(val)) + val


def test_corruption_recovery_semantics(oracle):
    """TestCorruption.testRecovery (T/TestCorruption.java:250-270): flipping log byte 19
    and byte 32768+1000 loses the 64 records of the first two blocks; 36 survive."""
    payloads = [_batch_payload(i) for i in range(100)]
    log = bytearray(oracle.log_write(payloads))
    for pos in (19, 32768 + 1000):
        log[pos] ^= 0x80
    recs, reps = oracle.log_read(bytes(log))
    assert len(recs) == 36
    assert [r[1] for r in recs] == payloads[64:]
    # checksum mismatch drops the rest of each block; the orphaned Last fragments
    # that begin blocks 1 and 2 report "missing start of fragmented record(2)"
    assert reps == [(32768, 2, 0), (480, 6, 0), (32281, 2, 0), (967, 6, 0)]
