#!/usr/bin/env python3
"""Per-call latency of small general batches (device-resident, synchronised per
call) through gv4 and the stream kernel: n blocks of 4 KiB, crc mode."""
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import jleveldb_amd as jl  # noqa: E402

torch.cuda.set_device(0)
jl.init(0)
dev = torch.device("cuda:0")
for n in (1, 16, 256, 4096):
    data = torch.empty(n * 4096 + 64, dtype=torch.uint8, device=dev)
    jl.fill_random_dev(data, 1)
    off = torch.arange(n, dtype=torch.int64, device=dev) * 4096 + 3
    ln = torch.full((n,), 4096, dtype=torch.int32, device=dev)
    out = torch.empty(n, dtype=torch.int32, device=dev)
    row = {"n": n}
    for v in ("gv4", "stream"):
        os.environ["JL_GENERAL"] = v
        for _ in range(20):
            jl.crc32c_batch_dev(data, off, ln, out=out)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(200):
            jl.crc32c_batch_dev(data, off, ln, out=out)
            torch.cuda.synchronize()
        row[v + "_us"] = round((time.perf_counter() - t0) / 200 * 1e6, 1)
    print(json.dumps(row), flush=True)
