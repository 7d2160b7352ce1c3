#!/usr/bin/env python3
"""Study: what holds crc_gv4_kernel back on short rounds (the C5 1 056-B log
path runs rounds of K = 9-10 windows at ~6.0 TB/s, C2-shaped rounds of K = 32
at ~6.7).  Same 4 GiB arena, blocks of ~1 KiB, one leg per layout:
  implicit_1152  1152-B blocks at a 1152-B stride (128-B aligned: implicit rounds of K = 9, no descriptors)
  sorted_1152    the same blocks through offsets (rounds pipeline, descriptors, ascending order)
  shuffled_1152  the same blocks in a random order (rounds of 8 scattered blocks)
  log_1057       1057-B blocks at a 1063-B stride (the C5 record crc ranges: K = 9/10, every tail pad)
  implicit_4224  4224-B blocks at a 4224-B stride (implicit rounds of K = 33)
  fixed4k        1M x 4 KiB through the 4 KiB kernel (reference)
LEGS=a,b selects legs (the gv4 study variants it ran in r3 live on the branch
study-r5-gv4-switches).
Run under rocprofv3 --kernel-trace --stats: the gv4 kernel's own time per leg
is in the trace (legs run in this order, 20 launches each)."""
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import jleveldb_amd as jl  # noqa: E402

torch.cuda.set_device(0)
jl.init(0)
dev = torch.device("cuda:0")
size = 4 << 30
data = torch.empty(size + 8192, dtype=torch.uint8, device=dev)
jl.fill_random_dev(data, 0x4A4C4442)
n9 = size // 1152
nl = size // 1063
out = torch.empty(max(n9, nl, 1 << 20), dtype=torch.int32, device=dev)
rng = np.random.default_rng(7)


def offs_t(o):
    return torch.from_numpy(o.astype(np.uint64).view(np.int64)).to(dev)


o9 = np.arange(n9, dtype=np.uint64) * 1152
o9s = o9[rng.permutation(n9)]
ol = np.arange(nl, dtype=np.uint64) * 1063 + 6
t9, t9s, tl = offs_t(o9), offs_t(o9s), offs_t(ol)
l9 = torch.full((n9,), 1152, dtype=torch.int32, device=dev)
ll = torch.full((nl,), 1057, dtype=torch.int32, device=dev)
legs = {
    "implicit_1152": (lambda: jl.crc32c_fixed_dev(data, 1152, n9, out=out), n9 * 1152),
    "sorted_1152": (lambda: jl.crc32c_batch_dev(data, t9, l9, out=out), n9 * 1152),
    "shuffled_1152": (lambda: jl.crc32c_batch_dev(data, t9s, l9, out=out), n9 * 1152),
    "log_1057": (lambda: jl.crc32c_batch_dev(data, tl, ll, out=out), nl * 1057),
    "implicit_4224": (lambda: jl.crc32c_fixed_dev(data, 4224, size // 4224, out=out), (size // 4224) * 4224),
    "fixed4k": (lambda: jl.crc32c_fixed_dev(data, 4096, 1 << 20, out=out), 1 << 32),
}
if os.environ.get("LEGS"):
    legs = {k: v for k, v in legs.items() if k in os.environ["LEGS"].split(",")}
res = {}
for name, (fn, nbytes) in legs.items():
    for _ in range(10):
        fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(20):
        fn()
    e1.record()
    torch.cuda.synchronize()
    ms = e0.elapsed_time(e1) / 20
    res[name] = {"ms_call": round(ms, 4), "bytes": nbytes, "TB_per_s_call": round(nbytes / ms / 1e9, 3)}
    print(name, res[name], flush=True)
print(json.dumps(res), flush=True)
