#!/usr/bin/env python3
"""Driver for PMC passes over the general-path kernels: C3 batch with the r1
chunked kernel and the stream kernel (depth 16 / 32), a few launches each."""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import jleveldb_amd as jl  # noqa: E402

SEED = 0x4A4C4442
torch.cuda.set_device(0)
jl.init(0)
dev = torch.device("cuda:0")
rng = np.random.default_rng(SEED)
n = 1 << 20
ks = np.empty(0, dtype=np.int64)
while ks.size < n:
    k = rng.zipf(1.1, 2 * n)
    ks = np.concatenate([ks, k[k <= 64]])
lens = (1024 * (ks[:n] - 1) + 1 + rng.integers(0, 1024, n)).astype(np.uint32)
offs = np.zeros(n, np.uint64)
offs[1:] = np.cumsum(lens[:-1], dtype=np.uint64)
arena = torch.empty(int(lens.sum(dtype=np.uint64)) + 16, dtype=torch.uint8, device=dev)
jl.fill_random_dev(arena, SEED + 3)
d_off = torch.from_numpy(offs.view(np.int64)).to(dev)
d_len = torch.from_numpy(lens.view(np.int32)).to(dev)
out = torch.empty(n, dtype=torch.int32, device=dev)
for v in os.environ.get("VARIANTS", "chunk s16 s32").split():
    os.environ["JL_GENERAL"] = "chunk" if v == "chunk" else "stream"
    if v != "chunk":
        os.environ["JL_STREAM_DEPTH"] = v[1:]
    for _ in range(3):
        jl.crc32c_batch_dev(arena, d_off, d_len, out=out)
    torch.cuda.synchronize()
