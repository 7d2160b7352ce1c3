#!/usr/bin/env python3
"""Cost of the gv4 round descriptors: the same blocks (4 GiB of BLOCK-byte
blocks, 128-B aligned) as implicit fixed-stride rounds (no descriptor loads)
and as an offset/length batch (rounds pipeline + scalar descriptor loads)."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import jleveldb_amd as jl  # noqa: E402

os.environ["JL_GENERAL"] = "gv4"
torch.cuda.set_device(0)
jl.init(0)
dev = torch.device("cuda:0")


def t_of(fn, reps=10):
    fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps


for bb in [int(x) for x in os.environ.get("BLOCKS", "1024 2048 8192").split()]:
    n = (4 << 30) // bb
    data = torch.empty(n * bb, dtype=torch.uint8, device=dev)
    jl.fill_random_dev(data, 7)
    off = torch.arange(n, dtype=torch.int64, device=dev) * bb
    ln = torch.full((n,), bb, dtype=torch.int32, device=dev)
    out1 = torch.empty(n, dtype=torch.int32, device=dev)
    out2 = torch.empty(n, dtype=torch.int32, device=dev)
    a = t_of(lambda: jl.crc32c_fixed_dev(data, bb, n, out=out1))
    b = t_of(lambda: jl.crc32c_batch_dev(data, off, ln, out=out2))
    assert torch.equal(out1, out2)
    print(json.dumps({"block": bb, "implicit_ms": round(a, 4), "desc_ms": round(b, 4)}), flush=True)
    del data, off, ln, out1, out2
