#!/usr/bin/env python3
"""Generates the committed golden fixtures under tests/golden/ (run in the build
container; the GPU box only reads the outputs).

What is pinned and where it comes from:

* ``reference_table_sha256`` — SHA-256 of the 2048 literal ``int`` values of
  ``T8_0..T8_7`` parsed as text from the reference
  ``src/main/java/com/tchaicatkovsky/jleveldb/util/Crc32C.java:173-334``,
  serialised little-endian.  Only the hash is stored (the table text is not
  copied).  The oracle's generated table must hash to the same value.
* ``kats`` — the reference's own known-answer tests,
  ``src/test/java/com/tchaicatkovsky/jleveldb/test/TestCrc32C.java:60-93``
  (RFC 3720 §B.4 vectors), as inputs and expected values.
* ``derived`` — values computed with the oracle *after* it passes the two pins
  above, and cross-checked against the numbers SURVEY.md §8(c) recorded from an
  independent restatement: typeCrc[0..4] (LogWriter.initTypeCrc), the DBBench
  4 KiB 'x' buffer, log headers, table trailers.
* ``blocks.bin``/``blocks.json`` — 64 seeded random blocks (0..9000 B) with raw
  and masked CRC32C, plus 8 ``extend``/suffix cases.
* ``log.bin``/``log.json`` — a LogWriter-framed file (LogWriter.java:88-161) of
  mixed-size records, its physical-record events and readRecord output.
* ``table.bin``/``table.json`` — blocks with 5-byte trailers
  (TableBuilder.writeRawBlock, TableBuilder.java:305-323).
* ``sstable.bin``/``sstable.json`` — a whole table written by the
  oracle/sstable.py restatement of TableBuilder (TestCorruption.build(100)
  shape, plus a filter block) and every block handle the walker must find.
  No JVM here: parity of the walker is pinned to the restated writer.
"""
from __future__ import annotations

import hashlib
import json
import os
import re
import struct
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, ROOT)
from oracle import oracle  # noqa: E402

REF_CRC = "/root/reference/src/main/java/com/tchaicatkovsky/jleveldb/util/Crc32C.java"

ISCSI_PDU = bytes([
    0x01, 0xc0, 0x00, 0x00, 0x00, 0x00, 0x00, 0x00, 0x00, 0x00, 0x00, 0x00, 0x00, 0x00, 0x00, 0x00,
    0x14, 0x00, 0x00, 0x00, 0x00, 0x00, 0x04, 0x00, 0x00, 0x00, 0x00, 0x14, 0x00, 0x00, 0x00, 0x18,
    0x28, 0x00, 0x00, 0x00, 0x00, 0x00, 0x00, 0x00, 0x02, 0x00, 0x00, 0x00, 0x00, 0x00, 0x00, 0x00,
])

# T/TestCrc32C.java:60-93 — (name, input hex, expected value)
KATS = [
    ("zeros32", bytes(32), 0x8a9136aa),
    ("ones32", bytes([0xff] * 32), 0x62a8ab43),
    ("ramp32", bytes(range(32)), 0x46dd794e),
    ("rramp32", bytes(31 - i for i in range(32)), 0x113fdb5c),
    ("iscsi48", ISCSI_PDU, 0xd9963a56),
]

# SURVEY.md §8(c) "Derived goldens" (recorded by an independent restatement)
SURVEY_DERIVED = {
    "type_crc": [0x527d5351, 0xa016d052, 0xb34623a6, 0x412da0a5, 0x95e7c44e],
    "dbbench_4k_x": 0xa46ab21f,
    "mask0": 0xa282ead8,
    "log_hdr_full_empty": "052b2843000001",
    "log_hdr_full_foo": "dd5fb37a030001",
    "log_hdr_first_100x": "ee53a01a640002",
    "log_hdr_last_hello_world": "9c0622100b0004",
    "trailer_empty": "00d28f2549",
    "trailer_4096x": "000124d327",
    "trailer_16x_ramp256": "004af155da",
}


def reference_table_sha256() -> str | None:
    if not os.path.exists(REF_CRC):
        return None
    text = open(REF_CRC).read()
    body = text[text.index("private static final int[] T"):]
    body = body[body.index("{") + 1: body.index("};")]
    vals = [int(v, 16) for v in re.findall(r"0x([0-9A-Fa-f]{8})", body)]
    assert len(vals) == 2048, len(vals)
    return hashlib.sha256(struct.pack("<2048I", *vals)).hexdigest()


def log_header(payload: bytes, type_byte: int) -> str:
    crc = oracle.mask(oracle.extend(oracle.value(bytes([type_byte])), payload))
    return (struct.pack("<I", crc) + struct.pack("<H", len(payload)) + bytes([type_byte])).hex()


def main() -> None:
    gen_table = oracle.tables()
    gen_sha = hashlib.sha256(gen_table.astype("<u4").tobytes()).hexdigest()
    ref_sha = reference_table_sha256()
    if ref_sha is not None and ref_sha != gen_sha:
        raise SystemExit(f"oracle table does not match reference table: {gen_sha} vs {ref_sha}")
    for name, data, want in KATS:
        got = oracle.value(data)
        assert got == want, (name, hex(got), hex(want))
        assert oracle.bitwise(data) == want

    derived = {
        "type_crc": [oracle.value(bytes([t])) for t in range(5)],
        "dbbench_4k_x": oracle.value(b"x" * 4096),
        "mask0": oracle.mask(0),
        "log_hdr_full_empty": log_header(b"", 1),
        "log_hdr_full_foo": log_header(b"foo", 1),
        "log_hdr_first_100x": log_header(b"x" * 100, 2),
        "log_hdr_last_hello_world": log_header(b"hello world", 4),
        "trailer_empty": oracle.table_trailer(b"", 0).hex(),
        "trailer_4096x": oracle.table_trailer(b"x" * 4096, 0).hex(),
        "trailer_16x_ramp256": oracle.table_trailer(bytes(range(256)) * 16, 0).hex(),
    }
    for k, v in SURVEY_DERIVED.items():
        assert derived[k] == v, (k, derived[k], v)

    golden = {
        "reference_table_sha256": ref_sha or gen_sha,
        "kats": [{"name": n, "hex": d.hex(), "value": v} for n, d, v in KATS],
        "derived": derived,
    }
    with open(os.path.join(HERE, "golden.json"), "w") as f:
        json.dump(golden, f, indent=1, sort_keys=True)

    # ---- random blocks
    rng = np.random.default_rng(0x4A4C4442)
    lens = [0, 1, 2, 3, 4, 5, 7, 8, 9, 15, 16, 17, 31, 63, 64, 65, 255, 256, 257, 1023, 1024, 1025, 1057,
            4095, 4096, 4097, 4101, 8191, 8192, 9000]
    lens += [int(x) for x in rng.integers(0, 9000, 64 - len(lens))]
    blobs = [rng.integers(0, 256, n, dtype=np.uint8).tobytes() for n in lens]
    offs, pos = [], 0
    for b in blobs:
        pos += int(rng.integers(0, 4))  # unaligned starts
        offs.append(pos)
        pos += len(b)
    arena = bytearray(pos + 3)
    for o, b in zip(offs, blobs):
        arena[o:o + len(b)] = b
    inits = [int(x) for x in rng.integers(0, 2**32, len(lens), dtype=np.uint64)]
    blocks = {
        "off": offs,
        "len": lens,
        "crc": [oracle.value(b) for b in blobs],
        "masked": [oracle.mask(oracle.value(b)) for b in blobs],
        "init": inits,
        "extend": [oracle.extend(i, b) for i, b in zip(inits, blobs)],
        "suffix_crc_type0": [oracle.extend(oracle.value(b), b"\0") for b in blobs],
    }
    with open(os.path.join(HERE, "blocks.bin"), "wb") as f:
        f.write(bytes(arena))
    with open(os.path.join(HERE, "blocks.json"), "w") as f:
        json.dump(blocks, f)

    # ---- log file: mixed sizes incl. fragments across 32 KiB blocks
    sizes = [0, 1, 10, 1000, 32761, 32762, 40000, 5, 100000, 7, 3, 1056, 1056, 1056, 65535, 2]
    payloads = [rng.integers(0, 256, n, dtype=np.uint8).tobytes() for n in sizes]
    log = oracle.log_write(payloads)
    ev = oracle.log_events(log)
    recs, reps = oracle.log_read(log)
    assert [r[1] for r in recs] == payloads and reps == []
    with open(os.path.join(HERE, "log.bin"), "wb") as f:
        f.write(log)
    with open(os.path.join(HERE, "log.json"), "w") as f:
        json.dump({
            "payload_sizes": sizes,
            "payload_sha256": [hashlib.sha256(p).hexdigest() for p in payloads],
            "events": [[int(e["offset"]), int(e["length"]), int(e["type"]), int(e["kind"])] for e in ev],
            "record_offsets": [r[0] for r in recs],
        }, f)

    # ---- table blocks with trailers
    tsizes = [0, 1, 100, 4096, 4100, 4163, 256, 17]
    tblocks = [rng.integers(0, 256, n, dtype=np.uint8).tobytes() for n in tsizes]
    tfile, handles = b"", []
    for b in tblocks:
        handles.append([len(tfile), len(b)])
        tfile += b + oracle.table_trailer(b, 0)
    with open(os.path.join(HERE, "table.bin"), "wb") as f:
        f.write(tfile)
    with open(os.path.join(HERE, "table.json"), "w") as f:
        json.dump({"handles": handles, "trailers": [oracle.table_trailer(b, 0).hex() for b in tblocks]}, f)

    # ---- a whole SSTable (oracle/sstable.py restatement of TableBuilder), shaped
    # like TestCorruption.build(100): keys "%016d" + 8-byte internal-key tag,
    # 1000-byte values (TestCorruption.java:68, 125-143, 574-584), 4 KiB blocks,
    # plus a filter block behind the metaindex, index keys shortened by the
    # InternalKeyComparator as the DB's TableBuilder does (TableBuilder.java:138-145,
    # 221-228).  Handles = the walker's expected output.
    from oracle import sstable

    srng = np.random.default_rng(0x53535442)
    pairs = [(b"%016d" % i + struct.pack("<Q", (i + 1) << 8 | 1), srng.integers(0, 256, 1000, dtype=np.uint8).tobytes())
             for i in range(100)]
    sst, sh = sstable.build_table(pairs, filter_block=srng.integers(0, 256, 300, dtype=np.uint8).tobytes(),
                                  comparator="internal")  # a DB table: internal keys, InternalKeyComparator
    assert sstable.walk(sst) == sh
    with open(os.path.join(HERE, "sstable.bin"), "wb") as f:
        f.write(sst)
    with open(os.path.join(HERE, "sstable.json"), "w") as f:
        json.dump({"handles": [list(h) for h in sh], "n_pairs": len(pairs),
                   "sha256": hashlib.sha256(sst).hexdigest()}, f)
    print("golden fixtures written; reference table sha256", ref_sha)


if __name__ == "__main__":
    main()
