"""jleveldb_amd — MI355X-native masked-CRC32C engine for jleveldb's checksum path.

Python host layer over the C-ABI in ``include/jlcrc.h`` (``libjlcrc.so``, built
in-tree from ``jleveldb_amd/csrc``).  It mirrors the reference's checksum
surface, ``com.tchaicatkovsky.jleveldb.util.Crc32C``
(src/main/java/com/tchaicatkovsky/jleveldb/util/Crc32C.java:29-167), and adds the
batched device entry points used by the table/log shims.

PyTorch is used only as device-memory / stream plumbing for the ``*_dev``
helpers; the computation is the HIP engine.  There is no CPU fallback: if the
shared library or a GPU is missing, the batch functions raise.
"""
from __future__ import annotations

import ctypes
import os

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("JLCRC_STUDY_LIB") or os.path.join(_HERE, "libjlcrc.so")  # study builds (tools/)

FLAG_MASK = 1

# jl_log_event kinds (include/jlcrc.h)
LOG_OK, LOG_BAD_CRC, LOG_BAD_LENGTH, LOG_ZERO_SKIP, LOG_EOF_BAD_LENGTH, LOG_EOF_TRUNC = 1, 2, 3, 4, 5, 6
# checksum argument of the log entry points (include/jlcrc.h): False/0, True/1 (= 2, two-pass), 3 (fused single pass)
LOG_NO_CHECKSUM, LOG_CHECKSUM, LOG_CHECKSUM_TWO_PASS, LOG_CHECKSUM_FUSED = 0, 1, 2, 3
LOG_EVENT_DTYPE = np.dtype([("offset", "<u8"), ("length", "<u4"), ("type", "u1"), ("kind", "u1"), ("pad", "<u2")])
LOG_RECORD_DTYPE = np.dtype([("offset", "<u8"), ("arena_off", "<u8"), ("size", "<u8")])
LOG_REPORT_DTYPE = np.dtype([("bytes", "<u8"), ("reason", "<u4"), ("aux", "<u4")])

# JL_REASON_* (include/jlcrc.h) -> the reference's Status messages (J/db/LogReader.java)
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


class JLError(RuntimeError):
    pass


_lib = None


def build(force: bool = False) -> str:
    """Compiles libjlcrc.so in-tree (hipcc, gfx950)."""
    import subprocess

    if force or not os.path.exists(LIB_PATH):
        subprocess.run(["make", "-s", "-C", os.path.join(_HERE, "csrc"), "-j8"], check=True)
    return LIB_PATH


def lib() -> ctypes.CDLL:
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise JLError(f"{LIB_PATH} is missing: build it with `make -C jleveldb_amd/csrc` (no CPU fallback)")
    L = ctypes.CDLL(LIB_PATH)
    vp, u8, u32, u64, i32, sz = (ctypes.c_void_p, ctypes.c_uint8, ctypes.c_uint32, ctypes.c_uint64, ctypes.c_int,
                                 ctypes.c_size_t)
    sig = {
        "jl_crc32c_value": (u32, [vp, sz]),
        "jl_crc32c_extend": (u32, [u32, vp, sz]),
        "jl_crc32c_update": (u32, [u32, vp, sz]),
        "jl_crc32c_mask": (u32, [u32]),
        "jl_crc32c_unmask": (u32, [u32]),
        "jl_init": (i32, [i32]),
        "jl_shutdown": (i32, []),
        "jl_last_error": (ctypes.c_char_p, []),
        "jl_device_count": (i32, []),
        "jl_version": (ctypes.c_char_p, []),
        "jl_set_option": (i32, [i32, ctypes.c_int64]),
        "jl_get_option": (ctypes.c_int64, [i32]),
        "jl_crc32c_fixed_dev": (i32, [vp, u64, u64, u32, vp, vp]),
        "jl_crc32c_batch_dev": (i32, [vp, u64, vp, vp, vp, vp, u64, u32, vp, vp]),
        "jl_crc32c_fixed": (i32, [vp, u64, u64, u32, vp]),
        "jl_crc32c_batch": (i32, [vp, u64, vp, vp, vp, vp, u64, u32, vp]),
        "jl_table_trailers_dev": (i32, [vp, vp, vp, vp, u64, vp, vp]),
        "jl_table_verify_dev": (i32, [vp, u64, vp, vp, u64, vp, vp]),
        "jl_table_verify": (i32, [vp, u64, vp, vp, u64, vp]),
        "jl_tables_verify": (i32, [u64, vp, vp, vp, vp, vp, vp]),
        "jl_table_block_handles": (i32, [vp, u64, vp, vp, vp, u64, ctypes.POINTER(u64)]),
        "jl_log_verify_dev": (i32, [vp, u64, i32, vp, u64, ctypes.POINTER(u64), vp]),
        "jl_log_verify_dev_async": (i32, [vp, u64, i32, vp, u64, vp, vp]),
        "jl_log_verify": (i32, [vp, u64, i32, vp, u64, ctypes.POINTER(u64)]),
        "jl_log_read_records": (i32, [vp, u64, i32, u64, vp, u64, vp, u64, ctypes.POINTER(u64), vp, u64,
                                      ctypes.POINTER(u64)]),
        "jl_log_headers_dev": (i32, [vp, vp, vp, vp, u64, vp, vp]),
        "jl_log_layout": (i32, [vp, vp, u64, u64, vp, vp, vp, vp, u64, vp, vp]),
        "jl_log_emit_dev": (i32, [vp, vp, vp, vp, vp, u64, u64, vp, vp]),
        "jl_fill_random_dev": (i32, [vp, u64, u64, u64, vp]),
        "jl_read_stream_dev": (i32, [vp, u64, vp, vp]),
    }
    for name, (res, args) in sig.items():
        f = getattr(L, name)
        f.restype = res
        f.argtypes = args
    del u8
    _lib = L
    return L


def _check(rc: int, what: str) -> None:
    if rc != 0:
        msg = lib().jl_last_error()
        raise JLError(f"{what} failed ({rc}): {msg.decode() if msg else ''}")


def _host(data) -> np.ndarray:
    if isinstance(data, np.ndarray):
        return np.ascontiguousarray(data, dtype=np.uint8).reshape(-1)
    return np.frombuffer(bytes(data), dtype=np.uint8)


def _host_bytes(data):
    """(pointer, size, keep-alive) of host input: a numpy array, bytes, or a
    contiguous CPU torch tensor (pinned ones are DMA'd without staging)."""
    if hasattr(data, "data_ptr"):
        if data.is_cuda or not data.is_contiguous():
            raise JLError("host entry point needs a contiguous CPU tensor")
        return data.data_ptr(), data.numel() * data.element_size(), data
    a = _host(data)
    return a.ctypes.data, a.size, a


# --------------------------------------------------------------------------
# Crc32C mirror (J/util/Crc32C.java)
# --------------------------------------------------------------------------
class Crc32C:
    """Mirror of ``com.tchaicatkovsky.jleveldb.util.Crc32C``.

    Statics ``value``/``extend``/``mask``/``unmask`` (Crc32C.java:43-93) and the
    ``java.util.zip.Checksum`` instance API (:96-167) map onto the C-ABI's host
    scalar entry points; batched work goes through the ``*_dev`` / batch
    functions of this module.
    """

    kMaskDelta = 0xA282EAD8

    def __init__(self) -> None:
        self.reset()

    # -- statics
    @staticmethod
    def value(data, offset: int = 0, n: int | None = None) -> int:
        a = _host(data)
        n = a.size - offset if n is None else n
        if offset < 0 or n < 0 or offset + n > a.size:
            raise IndexError("ArrayIndexOutOfBoundsException")
        return lib().jl_crc32c_value(a.ctypes.data + offset, n)

    @staticmethod
    def extend(init_crc: int, data, offset: int = 0, n: int | None = None) -> int:
        a = _host(data)
        n = a.size - offset if n is None else n
        if offset < 0 or n < 0 or offset + n > a.size:
            raise IndexError("ArrayIndexOutOfBoundsException")
        return lib().jl_crc32c_extend(init_crc & 0xFFFFFFFF, a.ctypes.data + offset, n)

    @staticmethod
    def mask(crc: int) -> int:
        return lib().jl_crc32c_mask(crc & 0xFFFFFFFF)

    @staticmethod
    def unmask(masked_crc: int) -> int:
        return lib().jl_crc32c_unmask(masked_crc & 0xFFFFFFFF)

    # -- java.util.zip.Checksum
    def reset(self) -> None:
        self._crc = 0xFFFFFFFF

    def setValue(self, v: int) -> None:  # noqa: N802 (reference name)
        self._crc = (~v) & 0xFFFFFFFF

    def getValue(self) -> int:  # noqa: N802
        return (~self._crc) & 0xFFFFFFFF

    def update(self, b, off: int | None = None, length: int | None = None) -> None:
        if isinstance(b, int) and off is None:  # update(int b), Crc32C.java:165-167
            one = np.array([b & 0xFF], dtype=np.uint8)
            self._crc = lib().jl_crc32c_update(self._crc, one.ctypes.data, 1)
            return
        a = _host(b)
        off = 0 if off is None else off
        length = a.size - off if length is None else length
        if off < 0 or length < 0 or off + length > a.size:
            raise IndexError("ArrayIndexOutOfBoundsException")
        self._crc = lib().jl_crc32c_update(self._crc, a.ctypes.data + off, length)


# --------------------------------------------------------------------------
# device engine
# --------------------------------------------------------------------------
def init(device: int = 0) -> None:
    _check(lib().jl_init(device), "jl_init")


def shutdown() -> None:
    _check(lib().jl_shutdown(), "jl_shutdown")


OPT_GENERAL_PATH, OPT_STREAM_DEPTH, OPT_STREAM_PARTITION, OPT_SPLIT_CAP = 1, 2, 3, 4
OPT_HOST_REGISTER, OPT_STAGE_THREADS, OPT_HOST_THRESHOLD, OPT_LOG_HOST_THRESHOLD = 5, 6, 7, 8
OPT_STAGE_PIECE = 9
OPT_FAILPOINT = 10  # tests only
OPT_LOG_SMALL_MAX = 11
HOST_THRESHOLD_AUTO = -1
INFO_STAGE_WORKERS, INFO_STAGE_SPAWN_FAILURES, INFO_LAST_PATH, INFO_LAST_CALL_NS, INFO_LAST_STAGE_NS = 201, 202, 203, 204, 205
PATH_AUTO, PATH_STREAM, PATH_GV4 = 0, 1, 2


def set_option(option: int, value: int) -> int:
    """jl_set_option: forces a kernel choice / tuning value; returns the previous value."""
    prev = int(lib().jl_get_option(option))
    _check(lib().jl_set_option(option, int(value)), "jl_set_option")
    return prev


def get_option(option: int) -> int:
    return int(lib().jl_get_option(option))


def version() -> str:
    return lib().jl_version().decode()


def _dptr(t) -> int:
    if t is None:
        return None
    if not t.is_cuda:
        raise JLError("expected a device tensor")
    if not t.is_contiguous():
        raise JLError("expected a contiguous tensor")
    return t.data_ptr()


def _nbytes(t) -> int:
    """Size in bytes of a device tensor (the arena / file bound the device range
    checks use: numel() alone undercounts any dtype wider than a byte)."""
    return t.numel() * t.element_size()


def _stream(stream=None):
    import torch

    s = stream if stream is not None else torch.cuda.current_stream()
    return ctypes.c_void_p(s.cuda_stream)


def crc32c_fixed_dev(data, block_bytes: int, n_blocks: int | None = None, flags: int = FLAG_MASK, out=None,
                     stream=None):
    """Per-block (masked) CRC32C of contiguous blocks in a uint8 device tensor."""
    import torch

    n_blocks = _nbytes(data) // block_bytes if n_blocks is None else n_blocks
    if n_blocks * block_bytes > _nbytes(data):
        raise JLError("blocks exceed the tensor")
    if out is None:
        out = torch.empty(n_blocks, dtype=torch.int32, device=data.device)
    _check(lib().jl_crc32c_fixed_dev(_dptr(data), block_bytes, n_blocks, flags, _dptr(out), _stream(stream)),
           "jl_crc32c_fixed_dev")
    return out


def crc32c_fixed(data, block_bytes: int, n_blocks: int | None = None, flags: int = FLAG_MASK) -> np.ndarray:
    """Host-memory blocks (numpy array, bytes, or a pinned CPU tensor), streamed
    through the engine with overlapped H2D copies (jl_crc32c_fixed)."""
    ptr, nbytes, _keep = _host_bytes(data)
    if n_blocks is None:
        n_blocks = nbytes // block_bytes
    if n_blocks * block_bytes > nbytes:
        raise JLError("crc32c_fixed: buffer smaller than n_blocks * block_bytes")
    out = np.zeros(n_blocks, dtype=np.uint32)
    _check(lib().jl_crc32c_fixed(ptr, block_bytes, n_blocks, flags, out.ctypes.data), "jl_crc32c_fixed")
    return out


def crc32c_batch_dev(base, off, length, init=None, suffix=None, flags: int = FLAG_MASK, out=None, stream=None):
    """Per-block (masked) CRC32C of arena ranges (device tensors: u8 base, i64 off, i32 len)."""
    import torch

    n = off.numel()
    if out is None:
        out = torch.empty(n, dtype=torch.int32, device=base.device)
    _check(lib().jl_crc32c_batch_dev(_dptr(base), _nbytes(base), _dptr(off), _dptr(length), _dptr(init), _dptr(suffix),
                                     n, flags,
                                     _dptr(out), _stream(stream)), "jl_crc32c_batch_dev")
    return out


def crc32c_batch(base, off, length, init=None, suffix=None, flags: int = FLAG_MASK) -> np.ndarray:
    """Host-memory batch (numpy / bytes / CPU tensor arena): streamed to the
    device in chunks (jl_crc32c_batch), returns uint32 results."""
    b_ptr, b_size, _keep = _host_bytes(base)
    off = np.ascontiguousarray(off, dtype=np.uint64)
    length = np.ascontiguousarray(length, dtype=np.uint32)
    init_a = None if init is None else np.ascontiguousarray(init, dtype=np.uint32)
    sfx_a = None if suffix is None else np.ascontiguousarray(suffix, dtype=np.uint8)
    out = np.zeros(off.size, dtype=np.uint32)
    _check(lib().jl_crc32c_batch(b_ptr, b_size, off.ctypes.data, length.ctypes.data,
                                 None if init_a is None else init_a.ctypes.data,
                                 None if sfx_a is None else sfx_a.ctypes.data, off.size, flags, out.ctypes.data),
           "jl_crc32c_batch")
    return out


def table_verify(file, off, size) -> np.ndarray:
    """Batched TableFormat.readBlock checksum test over a host file image (1 = ok)."""
    f_ptr, f_size, _keep = _host_bytes(file)
    off = np.ascontiguousarray(off, dtype=np.uint64)
    size = np.ascontiguousarray(size, dtype=np.uint32)
    st = np.zeros(off.size, dtype=np.uint8)
    _check(lib().jl_table_verify(f_ptr, f_size, off.ctypes.data, size.ctypes.data, off.size, st.ctypes.data),
           "jl_table_verify")
    return st


def tables_verify(tables):
    """Several tables at once (a compaction's inputs, jl_tables_verify): `tables`
    = [(file bytes, offsets, sizes), ...]; returns one status array per table."""
    keep, ptrs, nbytes, offs, sizes, first = [], [], [], [], [], [0]
    for f, o, z in tables:
        p, n, k = _host_bytes(f)
        keep.append(k)
        ptrs.append(p)
        nbytes.append(n)
        offs.append(np.ascontiguousarray(o, dtype=np.uint64))
        sizes.append(np.ascontiguousarray(z, dtype=np.uint32))
        first.append(first[-1] + offs[-1].size)
    P = (ctypes.c_void_p * max(1, len(ptrs)))(*ptrs)
    fb = np.array(nbytes, dtype=np.uint64)
    fi = np.array(first, dtype=np.uint64)
    off = np.concatenate(offs) if offs else np.zeros(0, np.uint64)
    size = np.concatenate(sizes) if sizes else np.zeros(0, np.uint32)
    st = np.zeros(max(1, off.size), dtype=np.uint8)
    _check(lib().jl_tables_verify(len(tables), ctypes.cast(P, ctypes.c_void_p), fb.ctypes.data, fi.ctypes.data,
                                  off.ctypes.data, size.ctypes.data, st.ctypes.data), "jl_tables_verify")
    return [st[first[i]:first[i + 1]] for i in range(len(tables))]


BLOCK_DATA, BLOCK_INDEX, BLOCK_METAINDEX, BLOCK_META = 0, 1, 2, 3


def table_block_handles(file):
    """Every block handle of an SSTable image (data blocks in index order, then the
    meta/filter blocks, the metaindex, the index): (offset u64[], size u32[],
    kind u8[]).  Host parse of the footer and index/metaindex blocks; raises
    JLError with the reference's Status message on a malformed table."""
    f = _host(file)
    cap = 64
    while True:
        off = np.zeros(cap, dtype=np.uint64)
        size = np.zeros(cap, dtype=np.uint32)
        kind = np.zeros(cap, dtype=np.uint8)
        n = ctypes.c_uint64(0)
        rc = lib().jl_table_block_handles(f.ctypes.data if f.size else None, f.size, off.ctypes.data,
                                          size.ctypes.data, kind.ctypes.data, cap, ctypes.byref(n))
        if rc == -5 and n.value > cap:  # JL_ERR_CAPACITY: grow and retry
            cap = int(n.value)
            continue
        _check(rc, "jl_table_block_handles")
        return off[: n.value], size[: n.value], kind[: n.value]


def table_verify_file(file) -> tuple:
    """Whole-table verification from the file bytes: the block handles of the table,
    then the batched TableFormat.readBlock checksum test over all of them.
    Returns (status u8[] per handle, off, size, kind)."""
    off, size, kind = table_block_handles(file)
    return table_verify(file, off, size), off, size, kind


def table_verify_dev(file, off, size, out=None, stream=None):
    import torch

    n = off.numel()
    if out is None:
        out = torch.empty(n, dtype=torch.uint8, device=file.device)
    _check(lib().jl_table_verify_dev(_dptr(file), _nbytes(file), _dptr(off), _dptr(size), n, _dptr(out),
                                     _stream(stream)),
           "jl_table_verify_dev")
    return out


def table_trailers_dev(file, off, size, types=None, out=None, stream=None):
    import torch

    n = off.numel()
    if out is None:
        out = torch.empty(5 * n, dtype=torch.uint8, device=file.device)
    _check(lib().jl_table_trailers_dev(_dptr(file), _dptr(off), _dptr(size), _dptr(types), n, _dptr(out),
                                       _stream(stream)), "jl_table_trailers_dev")
    return out


def log_headers_dev(base, off, length, types, out=None, stream=None):
    import torch

    n = off.numel()
    if out is None:
        out = torch.empty(7 * n, dtype=torch.uint8, device=base.device)
    _check(lib().jl_log_headers_dev(_dptr(base), _dptr(off), _dptr(length), _dptr(types), n, _dptr(out),
                                    _stream(stream)), "jl_log_headers_dev")
    return out


def log_layout(rec_src_off, rec_len, dest_length: int = 0):
    """LogWriter.addRecord framing plan (jl_log_layout): dict of numpy arrays
    hdr_off / src_off / len / type per physical fragment, plus log_bytes."""
    so = np.ascontiguousarray(rec_src_off, dtype=np.uint64)
    ln = np.ascontiguousarray(rec_len, dtype=np.uint32)
    n = ln.size
    # a record of L bytes spans at most L // 32761 + 2 fragments
    cap = int((ln.astype(np.uint64) // 32761).sum()) + 2 * n + 1
    hdr = np.zeros(cap, np.uint64)
    src = np.zeros(cap, np.uint64)
    fl = np.zeros(cap, np.uint32)
    ft = np.zeros(cap, np.uint8)
    nf, lb = ctypes.c_uint64(0), ctypes.c_uint64(0)
    _check(lib().jl_log_layout(so.ctypes.data, ln.ctypes.data, n, dest_length, hdr.ctypes.data, src.ctypes.data,
                               fl.ctypes.data, ft.ctypes.data, cap, ctypes.byref(nf), ctypes.byref(lb)),
           "jl_log_layout")
    k = nf.value
    return {"hdr_off": hdr[:k], "src_off": src[:k], "len": fl[:k], "type": ft[:k], "log_bytes": lb.value}


def log_emit_dev(src, plan, out=None, stream=None):
    """Batched LogWriter on the device (jl_log_emit_dev): the log image (uint8
    tensor) of a log_layout plan over the device arena `src`."""
    import torch

    dev = src.device
    t = {k: torch.from_numpy(np.ascontiguousarray(plan[k]).view(
        {"hdr_off": np.int64, "src_off": np.int64, "len": np.int32, "type": np.uint8}[k])).to(dev)
        for k in ("hdr_off", "src_off", "len", "type")}
    nb = plan["log_bytes"]
    if out is None:
        out = torch.empty(max(nb, 1), dtype=torch.uint8, device=dev)
    _check(lib().jl_log_emit_dev(_dptr(src), _dptr(t["hdr_off"]), _dptr(t["src_off"]), _dptr(t["len"]),
                                 _dptr(t["type"]), plan["len"].size, nb, _dptr(out), _stream(stream)),
           "jl_log_emit_dev")
    return out[:nb]


def log_verify(log, checksum: bool = True, out=None) -> np.ndarray:
    """Device verification of a host log image (numpy / bytes / CPU tensor) ->
    physical-record events (LOG_EVENT_DTYPE).  `checksum`: bool or a LOG_* mode.
    `out`: an event array (LOG_EVENT_DTYPE) to fill, reused across calls; its
    size is the capacity (a log has at most size / 7 + 2 physical records)."""
    ptr, size, _keep = _host_bytes(log)
    if out is None:
        cap = size // 7 + 2
        ev = np.zeros(cap, dtype=LOG_EVENT_DTYPE)
    else:
        # checked here, not by assert (python -O): the engine writes through out's pointer
        if not isinstance(out, np.ndarray) or out.dtype != LOG_EVENT_DTYPE:
            raise TypeError("log_verify: out must be a numpy array of LOG_EVENT_DTYPE")
        if not out.flags.c_contiguous or not out.flags.writeable:
            raise ValueError("log_verify: out must be C-contiguous and writeable")
        ev, cap = out, out.size
    n = ctypes.c_uint64(0)
    _check(lib().jl_log_verify(ptr if size else None, size, int(checksum), ev.ctypes.data, cap,
                               ctypes.byref(n)), "jl_log_verify")
    return ev[: n.value]


def log_verify_dev(log, checksum: bool = True, events=None, stream=None):
    """Device-resident verification; returns (events tensor view, count)."""
    import torch

    n = ctypes.c_uint64(0)
    cap = 0 if events is None else _nbytes(events) // LOG_EVENT_DTYPE.itemsize
    rc = lib().jl_log_verify_dev(_dptr(log), _nbytes(log), int(checksum), _dptr(events), cap, ctypes.byref(n),
                                 _stream(stream))
    if rc == -5:  # JL_ERR_CAPACITY: allocate and retry
        events = torch.empty(max(1, n.value) * LOG_EVENT_DTYPE.itemsize, dtype=torch.uint8, device=log.device)
        rc = lib().jl_log_verify_dev(_dptr(log), _nbytes(log), int(checksum), _dptr(events), n.value, ctypes.byref(n),
                                     _stream(stream))
    _check(rc, "jl_log_verify_dev")
    return events, n.value


def log_verify_dev_async(log, checksum: bool = True, events=None, result=None, stream=None):
    """Asynchronous device-resident verification (jl_log_verify_dev_async): enqueues
    the kernels and returns (events, result) at once; result (3 x int64 on the
    device, filled in stream order) = [events, dense blocks of the chunked path
    (informational; 0 on the one-launch small-log path), internal-capacity flag]; the events are complete for any log when [0] <= the
    events capacity."""
    import torch

    if result is None:
        result = torch.empty(3, dtype=torch.int64, device=log.device)
    cap = 0 if events is None else _nbytes(events) // LOG_EVENT_DTYPE.itemsize
    _check(lib().jl_log_verify_dev_async(_dptr(log), _nbytes(log), int(checksum), _dptr(events), cap, _dptr(result),
                                         _stream(stream)), "jl_log_verify_dev_async")
    return events, result


def log_read_records(log, checksum: bool = True, initial_offset: int = 0):
    """LogReader.readRecord over a whole log image: ([(offset, bytes)], [(bytes, reason, aux)])."""
    a = _host(log)
    arena = np.zeros(max(a.size, 1), dtype=np.uint8)
    cap = a.size // 7 + 2
    recs = np.zeros(cap, dtype=LOG_RECORD_DTYPE)
    reps = np.zeros(cap, dtype=LOG_REPORT_DTYPE)
    nr, np_ = ctypes.c_uint64(0), ctypes.c_uint64(0)
    _check(lib().jl_log_read_records(a.ctypes.data if a.size else None, a.size, int(checksum), initial_offset,
                                     arena.ctypes.data, arena.size, recs.ctypes.data, cap, ctypes.byref(nr),
                                     reps.ctypes.data, cap, ctypes.byref(np_)), "jl_log_read_records")
    records = [(int(r["offset"]), arena[int(r["arena_off"]):int(r["arena_off"]) + int(r["size"])].tobytes())
               for r in recs[: nr.value]]
    reports = [(int(r["bytes"]), int(r["reason"]), int(r["aux"])) for r in reps[: np_.value]]
    return records, reports


def fill_random_dev(t, seed: int, first_word: int = 0, stream=None) -> None:
    _check(lib().jl_fill_random_dev(_dptr(t), t.numel() * t.element_size(), seed & (2**64 - 1), first_word,
                                    _stream(stream)), "jl_fill_random_dev")


def read_stream_dev(t, sink, stream=None) -> None:
    """Read-only HBM stream over a device tensor (roofline calibration)."""
    _check(lib().jl_read_stream_dev(_dptr(t), t.numel() * t.element_size(), _dptr(sink), _stream(stream)),
           "jl_read_stream_dev")
