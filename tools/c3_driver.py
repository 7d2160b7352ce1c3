#!/usr/bin/env python3
"""C3 (1M mixed Zipf blocks, 1 B-64 KiB, one arena) through the general path,
LAUNCHES times: a short driver for rocprofv3 PMC passes (C3_PATH picks the
kernel: auto / stream / gv4, through jl_set_option)."""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import jleveldb_amd as jl  # noqa: E402

SEED = 0x4A4C4442
torch.cuda.set_device(0)
jl.init(0)
jl.set_option(jl.OPT_GENERAL_PATH, {"auto": jl.PATH_AUTO, "stream": jl.PATH_STREAM,
                                    "gv4": jl.PATH_GV4}[os.environ.get("C3_PATH", "auto")])
dev = torch.device("cuda:0")
rng = np.random.default_rng(SEED)
n = int(os.environ.get("C3_N", 1 << 20))
ks = np.empty(0, dtype=np.int64)
while ks.size < n:
    k = rng.zipf(1.1, 2 * n)
    ks = np.concatenate([ks, k[k <= 64]])
lens = (1024 * (ks[:n] - 1) + 1 + rng.integers(0, 1024, n)).astype(np.uint32)
if os.environ.get("C3_ROUND"):  # study: lengths rounded up to C3_ROUND bytes (aligned grid)
    r_ = int(os.environ["C3_ROUND"])
    lens = (((lens.astype(np.uint64) + r_ - 1) // r_) * r_).astype(np.uint32)
if os.environ.get("C3_ALIGN"):  # study: every block C3_ALIGN-byte aligned (lengths kept)
    al = int(os.environ["C3_ALIGN"])
    offs = np.zeros(n, np.uint64)
    offs[1:] = np.cumsum(((lens[:-1].astype(np.uint64) + al - 1) // al) * al, dtype=np.uint64)
    total = int(offs[-1] + lens[-1])
elif os.environ.get("C3_SORTED"):  # study: blocks laid out in the arena in order of their step count
    order = np.argsort((lens.astype(np.int64) + 127) // 128, kind="stable")
    pos = np.zeros(n, np.uint64)
    pos[1:] = np.cumsum(lens[order][:-1], dtype=np.uint64)
    offs = np.zeros(n, np.uint64)
    offs[order] = pos
    total = int(lens.sum(dtype=np.uint64))
else:
    offs = np.zeros(n, np.uint64)
    offs[1:] = np.cumsum(lens[:-1], dtype=np.uint64)
    total = int(lens.sum(dtype=np.uint64))
arena = torch.empty(total + 16, dtype=torch.uint8, device=dev)
jl.fill_random_dev(arena, SEED + 3)
d_off = torch.from_numpy(offs.view(np.int64)).to(dev)
d_len = torch.from_numpy(lens.view(np.int32)).to(dev)
out = torch.empty(n, dtype=torch.int32, device=dev)
L = int(os.environ.get("LAUNCHES", 5))
ev = [torch.cuda.Event(enable_timing=True) for _ in range(L + 1)]
ev[0].record()
for i in range(L):
    jl.crc32c_batch_dev(arena, d_off, d_len, out=out)
    ev[i + 1].record()
torch.cuda.synchronize()
t = [ev[i].elapsed_time(ev[i + 1]) for i in range(L)]
print(os.environ.get("C3_PATH", "auto"), "C3 bytes", int(lens.sum(dtype=np.uint64)), "ms", [round(x, 3) for x in t])
if os.environ.get("C3_STREAM"):  # read ceiling over the same arena
    sink = torch.zeros(1, dtype=torch.int32, device=dev)
    view = arena[: (total // 4096) * 4096]
    for _ in range(2):
        jl.read_stream_dev(view, sink)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(5):
        jl.read_stream_dev(view, sink)
    e1.record()
    torch.cuda.synchronize()
    ms = e0.elapsed_time(e1) / 5
    print("read_stream bytes", view.numel(), "ms", round(ms, 3), "GB/s", round(view.numel() / ms / 1e6, 1))
