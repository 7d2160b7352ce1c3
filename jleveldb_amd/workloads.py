"""Synthetic inputs of the BASELINE.json configs, shared by bench.py and the
tests so that the full-size parity tests check exactly the sets the bench
reports.

All generators are seeded and deterministic; the bytes themselves come from
jl_fill_random_dev's splitmix64 stream (device) or its oracle twin (host).
"""
from __future__ import annotations

import numpy as np

SEED = 0x4A4C4442
LOG_BLOCK = 32768  # J/db/LogFormat.java:52
C5_LOG_BYTES = (1 << 17) * LOG_BLOCK  # 2^17 x 32 KiB = 4 GiB
C1_PAYLOAD = 12 + 1 + 1 + 16 + 2 + 1024  # WriteBatch header + tag + varint + 16-B key + varint + 1 KiB value
# DBBench's default write (J/benchmark/DBBench.java:80 FLAGS_value_size = 100, 16-B keys):
# one Put per WriteBatch = 12-B header + tag + varint + 16-B key + varint + 100-B value
DBBENCH_PAYLOAD = 12 + 1 + 1 + 16 + 1 + 100
# a WAL of variable small values: payloads of 0-200 B, uniform random lengths
# (~306 records per 32 KiB block, every block dense, almost no two neighbours
# equal: lc_dense's walk cannot join records into runs)
RANDOM_MAX = 200
C5_SETS = ("c1_1056", "mixed_1b_100k", "dbbench_131", "random_0_200")


def c3_lengths(n: int = 1 << 20, seed: int = SEED) -> np.ndarray:
    """Config C3 block sizes: k ~ Zipf(1.1) on {1..64}, len = 1024(k-1) + 1 + U[0,1023]
    (1 B - 64 KiB)."""
    rng = np.random.default_rng(seed)
    ks = np.empty(0, dtype=np.int64)
    while ks.size < n:
        k = rng.zipf(1.1, 2 * n)
        ks = np.concatenate([ks, k[k <= 64]])
    ks = ks[:n]
    return (1024 * (ks - 1) + 1 + rng.integers(0, 1024, n)).astype(np.uint32)


def packed_offsets(lens: np.ndarray) -> np.ndarray:
    """Offsets of blocks packed back-to-back (unaligned starts)."""
    offs = np.zeros(lens.size, np.uint64)
    if lens.size > 1:
        offs[1:] = np.cumsum(lens[:-1], dtype=np.uint64)
    return offs


def _frag_bytes(lens: np.ndarray) -> np.ndarray:
    """Upper bound on the log bytes of each record: payload + one 7-B header per
    started block-sized fragment."""
    lens = lens.astype(np.uint64)
    return lens + 7 * (lens // (LOG_BLOCK - 7) + 1)


def c5_lengths(mixed, target: int = C5_LOG_BYTES, seed: int = SEED) -> np.ndarray:
    """Config C5 payload lengths whose LogWriter framing fills about `target`
    bytes.  `mixed` names the set (C5_SETS; a bool picks the first two): C1-shaped
    records (1 056-B payloads), a mixed 1 B - 100 KiB set whose records fragment
    FIRST/MIDDLE/LAST across 32 KiB blocks, or DBBench-default records (131-B
    payloads, ~237 per 32 KiB block: every block dense), or 0-200-B payloads of
    uniform random lengths (~306 per block, every block dense, runs of one)."""
    name = mixed if isinstance(mixed, str) else C5_SETS[1 if mixed else 0]
    if name == "random_0_200":
        rng = np.random.default_rng(seed + 13)
        lens = rng.integers(0, RANDOM_MAX + 1, target // (RANDOM_MAX // 2 + 7) + 4096).astype(np.uint32)
        keep = int(np.searchsorted(np.cumsum(_frag_bytes(lens)), target))
        return lens[:keep]
    if name == "dbbench_131":
        return np.full(target // (DBBENCH_PAYLOAD + 7), DBBENCH_PAYLOAD, np.uint32)
    if name == "c1_1056":
        return np.full(target // (C1_PAYLOAD + 7), C1_PAYLOAD, np.uint32)
    assert name == "mixed_1b_100k", name
    rng = np.random.default_rng(seed + 7)
    lens = rng.integers(1, 100 * 1024 + 1, target // (50 * 1024) + 1).astype(np.uint32)
    keep = int(np.searchsorted(np.cumsum(_frag_bytes(lens)), target))
    return lens[:keep]
