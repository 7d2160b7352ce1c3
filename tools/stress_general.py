#!/usr/bin/env python3
"""Randomised parity stress of the general path (gv4 rounds pipeline, split
blocks, descriptor prefetch, half turns, stream kernel for small verify
batches): random batch shapes, length distributions, alignments, init / suffix
/ mask flags and table-verify corruption, each checked against the CPU oracle.
Runs for SECONDS (default 60) or ITERS iterations; prints one line per batch
and exits non-zero on the first mismatch."""
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import jleveldb_amd as jl  # noqa: E402
from oracle import oracle  # noqa: E402

oracle.build()
torch.cuda.set_device(0)
jl.init(0)
dev = torch.device("cuda:0")
seed = int(os.environ.get("SEED", 7))
rng = np.random.default_rng(seed)
t_end = time.time() + float(os.environ.get("SECONDS", 60))
iters = int(os.environ.get("ITERS", 10**9))
THREADS = 16


def lengths(n):
    kind = rng.integers(0, 6)
    if kind == 0:
        return rng.integers(0, 200, n)                       # tiny
    if kind == 1:
        return rng.integers(0, 70000, n)                     # C3-like range
    if kind == 2:
        k = np.minimum(rng.zipf(1.1, n), 64)
        return 1024 * (k - 1) + 1 + rng.integers(0, 1024, n)  # C3 shape
    if kind == 3:
        return np.full(n, int(rng.integers(1, 9000)))        # one K bin
    if kind == 4:
        base = rng.integers(0, 3000, n)
        big = rng.random(n) < 0.02
        return np.where(big, rng.integers(512 << 10, 3 << 20, n), base)  # some split blocks
    return 128 * rng.integers(0, 80, n) + rng.integers(-1, 2, n).clip(0)  # around the step grid


it = 0
while time.time() < t_end and it < iters:
    it += 1
    n = int(rng.choice([1, 7, 8, 9, 100, 4095, 4096, 5000, 20000]))
    lens = lengths(n).astype(np.uint64).astype(np.uint32)
    gaps = rng.integers(0, 130, n).astype(np.uint64)
    offs = np.cumsum(gaps + np.concatenate([[0], lens[:-1].astype(np.uint64)])).astype(np.uint64)
    total = int(offs[-1] + lens[-1]) + 16
    if total > (600 << 20):
        continue
    arena = rng.integers(0, 256, total, dtype=np.uint8)
    d = (torch.from_numpy(arena).to(dev), torch.from_numpy(offs.view(np.int64)).to(dev),
         torch.from_numpy(lens.view(np.int32)).to(dev))
    use_init, use_sfx, flags = bool(rng.integers(0, 2)), bool(rng.integers(0, 2)), int(rng.integers(0, 2))
    init = rng.integers(0, 2**32, n, dtype=np.uint64).astype(np.uint32) if use_init else None
    sfx = rng.integers(0, 256, n, dtype=np.uint8) if use_sfx else None
    got = jl.crc32c_batch_dev(*d, init=None if init is None else torch.from_numpy(init.view(np.int32)).to(dev),
                              suffix=None if sfx is None else torch.from_numpy(sfx).to(dev), flags=flags)
    want = oracle.batch(arena, offs, lens, init=init, suffix=sfx, flags=flags, threads=THREADS)
    ok = np.array_equal(got.cpu().numpy().view(np.uint32), want)
    print(f"iter {it} n={n} bytes={int(lens.sum())} init={use_init} sfx={use_sfx} flags={flags} ok={ok}", flush=True)
    if not ok:
        sys.exit(1)
    if it % 3 == 0 and n > 1:  # table verify over the same blocks with trailers appended
        tb = bytearray()
        toff, tsz = [], []
        for i in range(min(n, 3000)):
            b = arena[offs[i]:offs[i] + lens[i]].tobytes()
            toff.append(len(tb))
            tsz.append(len(b))
            tb += b + oracle.table_trailer(b, 0)
        for _ in range(5):
            tb[int(rng.integers(0, len(tb)))] ^= 1
        f = np.frombuffer(bytes(tb), dtype=np.uint8)
        st = jl.table_verify(f, np.array(toff, np.uint64), np.array(tsz, np.uint32))
        want_st = [oracle.table_verify(bytes(tb), o, s) for o, s in zip(toff, tsz)]
        ok = [bool(x) for x in st] == want_st
        print(f"iter {it} table verify blocks={len(toff)} ok={ok}", flush=True)
        if not ok:
            sys.exit(1)
print("stress done", it, "iterations")
