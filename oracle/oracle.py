"""ctypes wrapper for the CPU oracle (oracle/crc32c_oracle.c) — TEST INFRASTRUCTURE ONLY.

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may import
this module, and only as the checker / the timed CPU baseline.  Every function
restates the reference cited in crc32c_oracle.c
(J = src/main/java/com/tchaicatkovsky/jleveldb):

* value/extend/mask/unmask/update       -> J/util/Crc32C.java:43-167
* table_trailer / table_verify           -> J/table/TableBuilder.java:305-323,
                                           J/table/TableFormat.java:207-218
* log_write                              -> J/db/LogWriter.java:88-161
* log_events / log_read                  -> J/db/LogReader.java:146-383
"""
from __future__ import annotations

import ctypes
import os
import subprocess

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB_PATH = os.path.join(_HERE, "_build", "liboracle.so")
_lib = None

FLAG_MASK = 1

# readRecord corruption reasons (J/db/LogReader.java:181-250, 334-369)
REASONS = {
    1: "bad record length",
    2: "checksum mismatch",
    3: "partial record without end(1)",
    4: "partial record without end(2)",
    5: "missing start of fragmented record(1)",
    6: "missing start of fragmented record(2)",
    7: "error in middle of record",
    8: "unknown record type",
}

EVENT_DTYPE = np.dtype([("offset", "<u8"), ("length", "<u4"), ("type", "u1"), ("kind", "u1"), ("pad", "<u2")])
RECORD_DTYPE = np.dtype([("offset", "<u8"), ("data_off", "<u8"), ("size", "<u8")])
REPORT_DTYPE = np.dtype([("bytes", "<u8"), ("reason", "<u4"), ("aux", "<u4")])


def build() -> str:
    subprocess.run(["make", "-s", "-C", _HERE], check=True)
    return _LIB_PATH


def lib() -> ctypes.CDLL:
    global _lib
    if _lib is None:
        if not os.path.exists(_LIB_PATH):
            build()
        L = ctypes.CDLL(_LIB_PATH)
        u8p = ctypes.c_void_p
        L.orc_update.argtypes = [ctypes.c_uint32, u8p, ctypes.c_size_t]
        L.orc_update.restype = ctypes.c_uint32
        L.orc_update_byte.argtypes = [ctypes.c_uint32, ctypes.c_uint32]
        L.orc_update_byte.restype = ctypes.c_uint32
        for name in ("orc_value", "orc_bitwise"):
            getattr(L, name).argtypes = [u8p, ctypes.c_size_t]
            getattr(L, name).restype = ctypes.c_uint32
        L.orc_extend.argtypes = [ctypes.c_uint32, u8p, ctypes.c_size_t]
        L.orc_extend.restype = ctypes.c_uint32
        for name in ("orc_mask", "orc_unmask"):
            getattr(L, name).argtypes = [ctypes.c_uint32]
            getattr(L, name).restype = ctypes.c_uint32
        L.orc_tables.argtypes = [u8p]
        L.orc_batch.argtypes = [u8p, u8p, u8p, u8p, u8p, ctypes.c_uint64, ctypes.c_uint32, u8p, ctypes.c_int]
        L.orc_fixed.argtypes = [u8p, ctypes.c_uint64, ctypes.c_uint64, ctypes.c_uint32, u8p, ctypes.c_int]
        L.orc_table_trailer.argtypes = [u8p, ctypes.c_uint64, ctypes.c_uint8, u8p]
        L.orc_table_verify.argtypes = [u8p, ctypes.c_uint64, ctypes.c_uint64]
        L.orc_table_verify.restype = ctypes.c_int
        L.orc_log_write.argtypes = [u8p, u8p, u8p, ctypes.c_uint64, ctypes.c_uint64, u8p, ctypes.c_uint64]
        L.orc_log_write.restype = ctypes.c_uint64
        L.orc_log_events.argtypes = [u8p, ctypes.c_uint64, ctypes.c_int, u8p, ctypes.c_uint64]
        L.orc_log_events.restype = ctypes.c_uint64
        L.orc_log_read.argtypes = [u8p, ctypes.c_uint64, ctypes.c_int, ctypes.c_uint64, u8p, ctypes.c_uint64,
                                   u8p, ctypes.c_uint64, u8p, ctypes.c_uint64, ctypes.POINTER(ctypes.c_uint64)]
        L.orc_log_read.restype = ctypes.c_uint64
        L.orc_fill_splitmix.argtypes = [u8p, ctypes.c_uint64, ctypes.c_uint64, ctypes.c_uint64]
        _lib = L
    return _lib


def _buf(data) -> tuple[np.ndarray, int]:
    a = np.frombuffer(bytes(data), dtype=np.uint8) if isinstance(data, (bytes, bytearray, memoryview)) else data
    a = np.ascontiguousarray(a, dtype=np.uint8)
    return a, a.ctypes.data


def _ptr(a) -> int | None:
    return None if a is None else a.ctypes.data


def value(data) -> int:
    a, p = _buf(data)
    return lib().orc_value(p, a.size)


def extend(init_crc: int, data) -> int:
    a, p = _buf(data)
    return lib().orc_extend(init_crc & 0xFFFFFFFF, p, a.size)


def update(state: int, data) -> int:
    a, p = _buf(data)
    return lib().orc_update(state & 0xFFFFFFFF, p, a.size)


def update_byte(state: int, b: int) -> int:
    return lib().orc_update_byte(state & 0xFFFFFFFF, b & 0xFFFFFFFF)


def bitwise(data) -> int:
    a, p = _buf(data)
    return lib().orc_bitwise(p, a.size)


def mask(crc: int) -> int:
    return lib().orc_mask(crc & 0xFFFFFFFF)


def unmask(m: int) -> int:
    return lib().orc_unmask(m & 0xFFFFFFFF)


def tables() -> np.ndarray:
    out = np.zeros(8 * 256, dtype=np.uint32)
    lib().orc_tables(out.ctypes.data)
    return out


def batch(base: np.ndarray, off: np.ndarray, length: np.ndarray, init=None, suffix=None, flags: int = FLAG_MASK,
          threads: int = 1) -> np.ndarray:
    base = np.ascontiguousarray(base, dtype=np.uint8)
    off = np.ascontiguousarray(off, dtype=np.uint64)
    length = np.ascontiguousarray(length, dtype=np.uint32)
    init = None if init is None else np.ascontiguousarray(init, dtype=np.uint32)
    suffix = None if suffix is None else np.ascontiguousarray(suffix, dtype=np.uint8)
    n = off.size
    assert length.size == n
    if n:
        assert int((off + length.astype(np.uint64)).max()) <= base.size
    out = np.zeros(n, dtype=np.uint32)
    lib().orc_batch(base.ctypes.data, off.ctypes.data, length.ctypes.data, _ptr(init), _ptr(suffix), n, flags,
                    out.ctypes.data, threads)
    return out


def fixed(base: np.ndarray, block_bytes: int, n_blocks: int, flags: int = FLAG_MASK, threads: int = 1) -> np.ndarray:
    base = np.ascontiguousarray(base, dtype=np.uint8)
    assert block_bytes * n_blocks <= base.size
    out = np.zeros(n_blocks, dtype=np.uint32)
    lib().orc_fixed(base.ctypes.data, block_bytes, n_blocks, flags, out.ctypes.data, threads)
    return out


def table_trailer(block, type_byte: int = 0) -> bytes:
    a, p = _buf(block)
    out = np.zeros(5, dtype=np.uint8)
    lib().orc_table_trailer(p, a.size, type_byte, out.ctypes.data)
    return out.tobytes()


def table_verify(file, off: int, n: int) -> bool:
    a, p = _buf(file)
    assert off + n + 5 <= a.size
    return bool(lib().orc_table_verify(p, off, n))


def log_write(payloads, dest_length: int = 0) -> bytes:
    """LogWriter.addRecord over each payload (list of bytes) into a fresh file."""
    lens = np.array([len(x) for x in payloads], dtype=np.uint32)
    offs = np.zeros(len(payloads), dtype=np.uint64)
    if len(payloads):
        offs[1:] = np.cumsum(lens[:-1], dtype=np.uint64)
    src = np.frombuffer(b"".join(bytes(x) for x in payloads) or b"\0", dtype=np.uint8).copy()
    cap = int(lens.sum()) + 7 * (len(payloads) + int(lens.sum()) // 32000 + 2) + 32768
    out = np.zeros(cap, dtype=np.uint8)
    w = lib().orc_log_write(src.ctypes.data, offs.ctypes.data, lens.ctypes.data, len(payloads), dest_length,
                            out.ctypes.data, cap)
    assert w != 2**64 - 1
    return out[:w].tobytes()


def log_events(log, checksum: bool = True) -> np.ndarray:
    a, p = _buf(log)
    cap = a.size // 7 + 2
    ev = np.zeros(cap, dtype=EVENT_DTYPE)
    n = lib().orc_log_events(p, a.size, int(checksum), ev.ctypes.data, cap)
    assert n <= cap
    return ev[:n]


def log_read(log, checksum: bool = True, initial_offset: int = 0):
    """Returns (records, reports): records = [(offset, bytes)], reports = [(bytes, reason_code, aux)]."""
    a, p = _buf(log)
    arena = np.zeros(max(a.size, 1), dtype=np.uint8)
    rcap = a.size // 7 + 2
    recs = np.zeros(rcap, dtype=RECORD_DTYPE)
    reps = np.zeros(rcap, dtype=REPORT_DTYPE)
    nrep = ctypes.c_uint64(0)
    n = lib().orc_log_read(p, a.size, int(checksum), initial_offset, arena.ctypes.data, arena.size,
                           recs.ctypes.data, rcap, reps.ctypes.data, rcap, ctypes.byref(nrep))
    assert n != 2**64 - 1
    records = [(int(r["offset"]), arena[int(r["data_off"]):int(r["data_off"]) + int(r["size"])].tobytes())
               for r in recs[:n]]
    reports = [(int(r["bytes"]), int(r["reason"]), int(r["aux"])) for r in reps[:nrep.value]]
    return records, reports


def fill_splitmix(nbytes: int, seed: int, first_word: int = 0) -> np.ndarray:
    out = np.empty(nbytes, dtype=np.uint8)
    lib().orc_fill_splitmix(out.ctypes.data, nbytes, seed & (2**64 - 1), first_word)
    return out
