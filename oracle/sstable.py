"""TEST INFRASTRUCTURE ONLY — never imported by the product (jleveldb_amd/).

A plain-Python restatement of jleveldb's SSTable writer and of the block-handle
walk over its index / metaindex blocks, used to build SSTable images for the
parity tests of the product's table walker (jl_table_block_handles) and
whole-table verification.  Follows:

  BlockBuilder.add / finish        J/table/BlockBuilder.java:69-114
  TableBuilder.add / flush / finish / writeBlock / writeRawBlock
                                   J/table/TableBuilder.java:127-186, 188-245, 269-323
  index keys: findShortestSeparator / findShortSuccessor of the table's comparator,
    bytewise  J/util/BytewiseComparatorImpl.java:60-94
    internal  J/db/format/InternalKeyComparator.java:77-109 (user key shortened,
              then the tag packSequenceAndType(kMaxSequenceNumber, kValueTypeForSeek),
              J/db/format/DBFormat.java:74-76,97-100)
  BlockHandle.encodeTo / decodeFrom J/table/TableFormat.java:66-78
  Footer.encodeTo / decodeFrom     J/table/TableFormat.java:116-146  (magic :161)
  Block (restart array) / decodeEntry  J/table/Block.java:44-84, 312-342
  Table.readMeta ("filter." key)   J/table/Table.java:287-310
  TableFormat.readBlock            J/table/TableFormat.java:195-258 (paranoid: checksum,
                                   then type byte; util/Snappy.java is a stub)

(J = src/main/java/com/tchaicatkovsky/jleveldb in the reference.)  The
reference is Java and no JVM exists here, so the images are produced by this
restatement; the walker parity is therefore pinned to the restated format, not
to files written by the reference.  For a given key/value
sequence, options (block size, restart interval, comparator) and filter block,
the image is byte for byte what TableBuilder writes, index keys included.
"""
from __future__ import annotations

import struct

from oracle import oracle

MAGIC = 0xDB4775248B80FB57  # TableFormat.kTableMagicNumber
FOOTER_LEN = 48              # 2 * BlockHandle.MaxEncodedLength + 8
KIND_DATA, KIND_INDEX, KIND_METAINDEX, KIND_META = 0, 1, 2, 3


def varint(v: int) -> bytes:
    out = bytearray()
    while v >= 0x80:
        out.append((v & 0x7F) | 0x80)
        v >>= 7
    out.append(v)
    return bytes(out)


def get_varint(buf: bytes, pos: int, limit: int) -> tuple[int, int]:
    v, shift = 0, 0
    while pos < limit and shift <= 63:
        b = buf[pos]
        pos += 1
        v |= (b & 0x7F) << shift
        if not b & 0x80:
            return v, pos
        shift += 7
    raise ValueError("bad varint")


K_MAX_SEQUENCE = (2**63 - 1) >> 8  # DBFormat.kMaxSequenceNumber = Long.MAX_VALUE >> 8 (DBFormat.java:76)
SEEK_TAG = struct.pack("<Q", (K_MAX_SEQUENCE << 8) | 1)  # packSequenceAndType(.., kValueTypeForSeek = Value)


def bytewise_shortest_separator(start: bytes, limit: bytes) -> bytes:
    """BytewiseComparatorImpl.findShortestSeparator (:60-79)."""
    m = min(len(start), len(limit))
    i = 0
    while i < m and start[i] == limit[i]:
        i += 1
    if i >= m:
        return start  # one is a prefix of the other: not shortened
    b = start[i]
    if b < 0xFF and b + 1 < limit[i]:
        return start[:i] + bytes([b + 1])
    return start


def bytewise_short_successor(key: bytes) -> bytes:
    """BytewiseComparatorImpl.findShortSuccessor (:82-94)."""
    for i, b in enumerate(key):
        if b != 0xFF:
            return key[:i] + bytes([b + 1])
    return key  # a run of 0xff: left alone


def internal_shortest_separator(start: bytes, limit: bytes) -> bytes:
    """InternalKeyComparator.findShortestSeparator (:77-92): on the user keys."""
    us, ul = start[:-8], limit[:-8]
    t = bytewise_shortest_separator(us, ul)
    if len(t) < len(us) and us < t:
        return t + SEEK_TAG
    return start


def internal_short_successor(key: bytes) -> bytes:
    """InternalKeyComparator.findShortSuccessor (:97-109)."""
    uk = key[:-8]
    t = bytewise_short_successor(uk)
    if len(t) < len(uk) and uk < t:
        return t + SEEK_TAG
    return key


COMPARATORS = {
    "bytewise": (bytewise_shortest_separator, bytewise_short_successor),
    "internal": (internal_shortest_separator, internal_short_successor),
}


class BlockBuilder:
    """BlockBuilder.java:69-114 (prefix-compressed entries, restart array)."""

    def __init__(self, restart_interval: int):
        self.interval = restart_interval
        self.buf = bytearray()
        self.restarts = [0]
        self.counter = 0
        self.last = b""

    def add(self, key: bytes, value: bytes) -> None:
        shared = 0
        if self.counter < self.interval:
            m = min(len(self.last), len(key))
            while shared < m and self.last[shared] == key[shared]:
                shared += 1
        else:
            self.restarts.append(len(self.buf))
            self.counter = 0
        non_shared = len(key) - shared
        self.buf += varint(shared) + varint(non_shared) + varint(len(value))
        self.buf += key[shared:] + value
        self.last = key
        self.counter += 1

    def size_estimate(self) -> int:
        return len(self.buf) + 4 * len(self.restarts) + 4

    def finish(self) -> bytes:
        return bytes(self.buf) + b"".join(struct.pack("<I", r) for r in self.restarts) + struct.pack("<I", len(self.restarts))

    def empty(self) -> bool:
        return not self.buf


def build_table(pairs, block_size: int = 4096, restart_interval: int = 16, filter_block: bytes | None = None,
                type_byte: int = 0, comparator: str = "bytewise"):
    """SSTable image from sorted (key, value) pairs.  Returns (bytes, handles)
    with handles = [(offset, size, kind)] of every block the walker must find:
    data blocks in index order, the filter block, the metaindex, the index.
    `comparator`: "bytewise" (Options' default) or "internal" (the DB's tables:
    keys are internal keys, user key || 8-byte tag)."""
    separator, successor = COMPARATORS[comparator]
    out = bytearray()
    handles = []

    def write_raw(contents: bytes, kind: int):  # writeRawBlock: block || [type][LE32 mask(crc)]
        off = len(out)
        out.extend(contents)
        out.extend(oracle.table_trailer(contents, type_byte))
        handles.append((off, len(contents), kind))
        return off, len(contents)

    data = BlockBuilder(restart_interval)
    index = BlockBuilder(1)  # index blocks restart at every entry (TableBuilder.java:84)
    last_key = b""
    pending = None  # handle of the last flushed data block, indexed at the next add / finish
    for key, value in pairs:
        if pending is not None:  # TableBuilder.add :138-145: separator between the blocks
            index.add(separator(last_key, key), varint(pending[0]) + varint(pending[1]))
            pending = None
        data.add(key, value)
        last_key = key
        if data.size_estimate() >= block_size:  # TableBuilder.add -> flush
            pending = write_raw(data.finish(), KIND_DATA)
            data = BlockBuilder(restart_interval)
    if not data.empty():  # finish -> flush
        pending = write_raw(data.finish(), KIND_DATA)
    meta = BlockBuilder(restart_interval)
    if filter_block is not None:
        foff, fsize = write_raw(filter_block, KIND_META)
        meta.add(b"filter.leveldb.BuiltinBloomFilter2", varint(foff) + varint(fsize))
    moff, msize = write_raw(meta.finish(), KIND_METAINDEX)
    if pending is not None:  # TableBuilder.finish :221-228: the last block under a short successor
        index.add(successor(last_key), varint(pending[0]) + varint(pending[1]))
    ioff, isize = write_raw(index.finish(), KIND_INDEX)
    footer = varint(moff) + varint(msize) + varint(ioff) + varint(isize)
    footer += b"\0" * (40 - len(footer)) + struct.pack("<II", MAGIC & 0xFFFFFFFF, MAGIC >> 32)
    out.extend(footer)
    order = {KIND_DATA: 0, KIND_META: 1, KIND_METAINDEX: 2, KIND_INDEX: 3}
    handles.sort(key=lambda h: (order[h[2]], h[0]))
    return bytes(out), handles


def block_entries(buf: bytes, off: int, size: int):
    """Values of the entries of the block at [off, off+size) (Block.java:44-84, 312-342)."""
    if size < 4:
        raise ValueError("bad block contents")
    nres = struct.unpack_from("<I", buf, off + size - 4)[0]
    if nres > (size - 4) // 4:
        raise ValueError("bad block contents")
    limit = off + size - (1 + nres) * 4
    pos, vals = off, []
    while pos < limit:
        try:
            shared, pos = get_varint(buf, pos, limit)
            non_shared, pos = get_varint(buf, pos, limit)
            vlen, pos = get_varint(buf, pos, limit)
        except ValueError:
            raise ValueError("bad entry in block") from None
        pos += non_shared
        if pos + vlen > limit:
            raise ValueError("bad entry in block")
        vals.append(buf[pos:pos + vlen])
        pos += vlen
    return vals


def read_block(buf: bytes, off: int, size: int) -> None:
    """TableFormat.readBlock with verifyChecksums (raises with the reference's Status text)."""
    if off + size + 5 > len(buf):
        raise ValueError("truncated block read")
    stored = struct.unpack_from("<I", buf, off + size + 1)[0]
    if oracle.unmask(stored) != oracle.value(buf[off:off + size + 1]):
        raise ValueError("block checksum mismatch")
    t = buf[off + size]
    if t == 1:
        raise ValueError("corrupted compressed block contents")
    if t != 0:
        raise ValueError(f"bad compress type {t - 256 if t > 127 else t}")


def _handles(buf: bytes, off: int, size: int, kind: int):
    out = []
    for v in block_entries(buf, off, size):
        try:  # BlockHandle.decodeFrom (TableFormat.java:74-78)
            o, q = get_varint(v, 0, len(v))
            s, _ = get_varint(v, q, len(v))
        except ValueError:
            raise ValueError("bad block handle") from None
        if o + s + 5 > len(buf):
            raise ValueError("truncated block read")
        out.append((o, s, kind))
    return out


def walk(buf: bytes):
    """Block handles of an SSTable image, in the product walker's order: the index
    read paranoidly (a failure fails the walk), the metaindex likewise but a
    failure there only drops the meta handles (Table.readMeta returns)."""
    if len(buf) < FOOTER_LEN:
        raise ValueError("file is too short to be an sstable")
    f = len(buf) - FOOTER_LEN
    lo, hi = struct.unpack_from("<II", buf, f + 40)
    if (hi << 32 | lo) != MAGIC:
        raise ValueError("not an sstable (bad magic number)")
    try:  # Footer.decodeFrom (TableFormat.java:126-146)
        moff, p = get_varint(buf, f, f + 40)
        msize, p = get_varint(buf, p, f + 40)
        ioff, p = get_varint(buf, p, f + 40)
        isize, p = get_varint(buf, p, f + 40)
    except ValueError:
        raise ValueError("bad block handle") from None
    if ioff + isize + 5 > len(buf):
        raise ValueError("truncated block read")
    read_block(buf, ioff, isize)
    out = _handles(buf, ioff, isize, KIND_DATA)
    if moff + msize + 5 > len(buf):
        raise ValueError("truncated block read")
    try:
        read_block(buf, moff, msize)
        out += _handles(buf, moff, msize, KIND_META)
    except ValueError:
        pass
    out.append((moff, msize, KIND_METAINDEX))
    out.append((ioff, isize, KIND_INDEX))
    return out
