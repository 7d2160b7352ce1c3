"""Whole-table verification: jl_table_block_handles
walks an SSTable image (footer, index, metaindex) and hands every block handle
to the batched readBlock checksum test.

CPU: the walker (host code in libjlcrc.so) against oracle/sstable.py — the
committed golden table, seeded random tables, every error path with the
reference's Status text, and a byte-flip fuzz where walker and oracle must agree
on the outcome.  GPU: TestCorruption.testTableFile / testTableFileIndexData
(T/TestCorruption.java:318-388) restated on one table.
"""
import struct

import numpy as np
import pytest

from oracle import sstable


def _table(n_pairs, seed=0, value_size=1000, filt=True, **kw):
    rng = np.random.default_rng(seed)
    pairs = [(b"%016d" % i + struct.pack("<Q", (i + 1) << 8 | 1),
              rng.integers(0, 256, value_size, dtype=np.uint8).tobytes()) for i in range(n_pairs)]
    fb = rng.integers(0, 256, 300, dtype=np.uint8).tobytes() if filt else None
    return sstable.build_table(pairs, filter_block=fb, **kw)


def _walk(jl, buf):
    off, size, kind = jl.table_block_handles(buf)
    return [(int(o), int(s), int(k)) for o, s, k in zip(off, size, kind)]


def _oracle_outcome(buf):
    try:
        return sstable.walk(buf)
    except ValueError as e:
        return str(e)


def _product_outcome(jl, buf):
    try:
        return _walk(jl, buf)
    except jl.JLError as e:
        return str(e).split(": ", 1)[1]


def _patch_crc(buf, off, size):
    """Re-seal the trailer of the block at (off, size) after editing it."""
    from oracle import oracle

    b = bytearray(buf)
    b[off + size + 1:off + size + 5] = struct.pack("<I", oracle.mask(oracle.value(bytes(b[off:off + size + 1]))))
    return bytes(b)


def test_golden_table(jl, golden):
    buf = golden("sstable.bin")
    want = [tuple(h) for h in golden("sstable.json")["handles"]]
    assert sstable.walk(buf) == want
    assert _walk(jl, buf) == want
    kinds = [k for _, _, k in want]
    assert kinds.count(jl.BLOCK_DATA) == 20 and kinds[-3:] == [jl.BLOCK_META, jl.BLOCK_METAINDEX, jl.BLOCK_INDEX]


@pytest.mark.parametrize("n_pairs,value_size,block_size,restart,filt", [
    (0, 10, 4096, 16, False),      # empty table: no data blocks, empty index
    (1, 0, 4096, 16, False),
    (100, 1000, 4096, 16, True),
    (700, 100, 4096, 16, True),   # more than 64 handles: capacity regrowth
    (300, 37, 1024, 1, False),
    (50, 5000, 4096, 4, True),    # values larger than a block
    (2000, 20, 65536, 16, True),
])
def test_random_tables(jl, n_pairs, value_size, block_size, restart, filt):
    buf, handles = _table(n_pairs, seed=n_pairs, value_size=value_size, filt=filt, block_size=block_size,
                          restart_interval=restart)
    assert sstable.walk(buf) == handles
    assert _walk(jl, buf) == handles


def test_capacity_contract(jl):
    import ctypes

    buf, handles = _table(700, value_size=100)
    f = np.frombuffer(buf, dtype=np.uint8)
    off = np.zeros(4, np.uint64)
    size = np.zeros(4, np.uint32)
    n = ctypes.c_uint64(0)
    rc = jl.lib().jl_table_block_handles(f.ctypes.data, f.size, off.ctypes.data, size.ctypes.data, None, 4,
                                         ctypes.byref(n))
    assert rc == -5 and n.value == len(handles)
    assert [int(o) for o in off] == [h[0] for h in handles[:4]]  # the first cap handles are written
    n.value = 7
    assert jl.lib().jl_table_block_handles(None, 0, None, None, None, 0, ctypes.byref(n)) == -6 and n.value == 0


def test_error_messages(jl):
    buf, handles = _table(100)
    ioff, isize, _ = handles[-1]
    moff, msize, _ = handles[-2]
    cases = {
        "file is too short to be an sstable": buf[-47:],
        "not an sstable (bad magic number)": buf[:-1] + bytes([buf[-1] ^ 1]),
        "block checksum mismatch": buf[:ioff + 3] + bytes([buf[ioff + 3] ^ 0x40]) + buf[ioff + 4:],
    }
    t = bytearray(buf)
    t[ioff + isize] = 1
    cases["corrupted compressed block contents"] = _patch_crc(bytes(t), ioff, isize)
    t[ioff + isize] = 0xFE
    cases["bad compress type -2"] = _patch_crc(bytes(t), ioff, isize)
    t = bytearray(buf)  # restart count larger than the block
    t[ioff + isize - 4:ioff + isize] = struct.pack("<I", 1 << 20)
    cases["bad block contents"] = _patch_crc(bytes(t), ioff, isize)
    small, sh = _table(1, filt=False)  # one ~1 KiB data block at offset 0: handle bytes 00 xx 08
    so, ss, _ = sh[-1]
    hs = so + 3 + small[so + 1] + 1  # the index entry's handle: after 3 varints, the key, offset varint 0
    t = bytearray(small)  # its size becomes 16383: past the end of the file
    t[hs:hs + 2] = b"\xff\x7f"
    cases["truncated block read"] = _patch_crc(bytes(t), so, ss)
    t = bytearray(small)  # the handle's size varint never terminates inside the value
    t[hs:hs + 2] = b"\xff\xff"
    cases["bad block handle"] = _patch_crc(bytes(t), so, ss)
    t = bytearray(buf)  # first entry's key length runs past the restart array
    t[ioff + 1] = 0x7F
    cases["bad entry in block"] = _patch_crc(bytes(t), ioff, isize)
    for msg, b in cases.items():
        assert _oracle_outcome(b) == msg, msg
        with pytest.raises(jl.JLError, match=msg.replace("(", r"\(").replace(")", r"\)")):
            jl.table_block_handles(b)


def test_bad_metaindex_drops_meta_handles(jl):
    """Table.readMeta (Table.java:287-310) returns without a filter when the
    metaindex cannot be read; the table still opens."""
    buf, handles = _table(100)
    moff = handles[-2][0]
    bad = buf[:moff] + bytes([buf[moff] ^ 1]) + buf[moff + 1:]
    want = [h for h in handles if h[2] != jl.BLOCK_META]
    assert sstable.walk(bad) == want
    assert _walk(jl, bad) == want


def test_byte_flip_fuzz_agrees_with_oracle(jl):
    buf, _ = _table(60, value_size=300)
    rng = np.random.default_rng(7)
    tail = len(buf) - 1200  # index, metaindex, filter and footer live at the end
    positions = list(rng.integers(0, len(buf), 100)) + list(rng.integers(tail, len(buf), 400))
    for p in positions:
        b = bytearray(buf)
        b[p] ^= int(rng.integers(1, 256))
        b = bytes(b)
        assert _product_outcome(jl, b) == _oracle_outcome(b), p
    for cut in list(rng.integers(0, len(buf), 60)):  # truncated files
        b = buf[:cut]
        assert _product_outcome(jl, b) == _oracle_outcome(b), cut


def test_index_data_corruption_fails_open(jl):
    """TestCorruption.testTableFileIndexData (T/TestCorruption.java:371-388):
    500 bytes corrupted 2000 bytes before the end land in the index block, and
    the table cannot be opened (its keys are lost to check(5000, 9999))."""
    buf, handles = _table(2000, value_size=1000)
    ioff, isize, _ = handles[-1]
    lo = len(buf) - 2000
    assert ioff <= lo and lo + 500 <= ioff + isize
    bad = buf[:lo] + bytes(500) + buf[lo + 500:]
    assert _oracle_outcome(bad) == "block checksum mismatch"
    with pytest.raises(jl.JLError, match="block checksum mismatch"):
        jl.table_block_handles(bad)


@pytest.mark.gpu
def test_table_file_corruption(gpu, jl, oracle):
    """TestCorruption.testTableFile (T/TestCorruption.java:318-338): one byte
    flipped at offset 100 — exactly the first data block fails verification."""
    import torch

    buf, handles = _table(100)
    st, off, size, kind = jl.table_verify_file(buf)
    assert list(st) == [1] * len(handles)
    bad = buf[:100] + bytes([buf[100] ^ 0x80]) + buf[101:]
    st, off, size, kind = jl.table_verify_file(bad)
    assert list(st) == [0] + [1] * (len(handles) - 1)
    assert [oracle.table_verify(bad, int(o), int(n)) for o, n in zip(off, size)] == [bool(x) for x in st]
    d_f = torch.from_numpy(np.frombuffer(bad, dtype=np.uint8).copy()).to(gpu)
    d_off = torch.from_numpy(off.astype(np.int64)).to(gpu)
    d_size = torch.from_numpy(size.astype(np.int32)).to(gpu)
    assert list(jl.table_verify_dev(d_f, d_off, d_size).cpu().numpy()) == list(st)


@pytest.mark.gpu
def test_whole_table_random_corruption(gpu, jl, oracle):
    """Every block of a 2000-entry table (data, filter, metaindex, index) through the
    walker + batched verify, with a third of the data blocks corrupted."""
    buf, handles = _table(2000, value_size=1000, seed=3)
    rng = np.random.default_rng(11)
    b = bytearray(buf)
    for o, s, k in handles:
        if k == jl.BLOCK_DATA and rng.random() < 0.33:
            p = o + int(rng.integers(0, s + 5))
            b[p] ^= 1 << int(rng.integers(0, 8))
    b = bytes(b)
    st, off, size, kind = jl.table_verify_file(b)
    assert [(int(o), int(s), int(k)) for o, s, k in zip(off, size, kind)] == handles
    assert [bool(x) for x in st] == [oracle.table_verify(b, int(o), int(n)) for o, n in zip(off, size)]
    assert 0 < int((st == 0).sum()) < len(handles)


def test_index_key_shortening(jl):
    """The restated comparators (BytewiseComparatorImpl.java:60-94,
    InternalKeyComparator.java:77-109): the index keys TableBuilder writes
    (TableBuilder.java:138-145, 221-228) are what the restatement writes."""
    sep, suc = sstable.bytewise_shortest_separator, sstable.bytewise_short_successor
    assert sep(b"abcdefg", b"abzzz") == b"abd"
    assert sep(b"abc", b"abcd") == b"abc"  # a prefix: not shortened
    assert sep(b"ab\xff", b"ac") == b"ab\xff" and sep(b"a4", b"a5") == b"a4"  # no room between
    assert suc(b"\xff\xffabc") == b"\xff\xffb" and suc(b"\xff\xff") == b"\xff\xff"
    tag = struct.pack("<Q", 5 << 8 | 1)
    assert sstable.internal_shortest_separator(b"abcdefg" + tag, b"abzzz" + tag) == b"abd" + sstable.SEEK_TAG
    assert sstable.internal_short_successor(b"abc" + tag) == b"b" + sstable.SEEK_TAG
    assert sstable.SEEK_TAG == bytes.fromhex("01ffffffffffff7f")  # (Long.MAX_VALUE >> 8) << 8 | Value
    # a table whose keys leave room between blocks: shortened index keys, same handles
    pairs = [(b"key%05d-%s" % (i, b"x" * (i % 7)), bytes(300)) for i in range(0, 4000, 7)]
    for cmp in ("bytewise", "internal"):
        kv = pairs if cmp == "bytewise" else [(k + struct.pack("<Q", (i + 1) << 8 | 1), v)
                                              for i, (k, v) in enumerate(pairs)]
        buf, handles = sstable.build_table(kv, comparator=cmp)
        assert sstable.walk(buf) == handles
        assert _walk(jl, buf) == handles
        # the index keys are the separators, not the blocks' last keys
        ioff, isize, _ = [h for h in handles if h[2] == sstable.KIND_INDEX][0]
        nres = struct.unpack_from("<I", buf, ioff + isize - 4)[0]
        lim, pos, key, ikeys = ioff + isize - 4 * (1 + nres), ioff, b"", []
        while pos < lim:
            sh, pos = sstable.get_varint(buf, pos, lim)
            ns, pos = sstable.get_varint(buf, pos, lim)
            vl, pos = sstable.get_varint(buf, pos, lim)
            key = key[:sh] + buf[pos:pos + ns]
            ikeys.append(key)
            pos += ns + vl
        data_keys = {k for k, _ in kv}
        assert len(ikeys) == sum(h[2] == sstable.KIND_DATA for h in handles)
        assert sum(k not in data_keys for k in ikeys) >= 5  # shortened separators (not data keys)
        assert ikeys == sorted(ikeys)
