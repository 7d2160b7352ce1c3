#!/usr/bin/env python3
"""Short-round driver for PMC passes: 4 GiB of BLOCK-byte blocks (default 1024,
C5-like rounds of ~8 steps) through gv4 as implicit fixed-stride rounds."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import jleveldb_amd as jl  # noqa: E402

os.environ["JL_GENERAL"] = "gv4"
torch.cuda.set_device(0)
jl.init(0)
bb = int(os.environ.get("BLOCK", 1024))
n = (4 << 30) // bb
data = torch.empty(n * bb, dtype=torch.uint8, device="cuda")
jl.fill_random_dev(data, 7)
out = torch.empty(n, dtype=torch.int32, device="cuda")
L = int(os.environ.get("LAUNCHES", 3))
ev = [torch.cuda.Event(enable_timing=True) for _ in range(L + 1)]
ev[0].record()
for i in range(L):
    jl.crc32c_fixed_dev(data, bb, n, out=out)
    ev[i + 1].record()
torch.cuda.synchronize()
print("block", bb, "ms", [round(ev[i].elapsed_time(ev[i + 1]), 4) for i in range(L)])
