#!/usr/bin/env python3
"""Sustained-rate check: LAUNCHES back-to-back launches of each kernel (C2
shape), per-launch HIP-event times; prints the first-5 and last-20 averages so
short-burst and steady-state (power/thermal-limited) rates can be told apart."""
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import jleveldb_amd as jl  # noqa: E402

n = 1 << 20
L = int(os.environ.get("LAUNCHES", 60))
torch.cuda.set_device(0)
jl.init(0)
data = torch.empty(n * 4096, dtype=torch.uint8, device="cuda")
jl.fill_random_dev(data, 0x4A4C4442)
out = torch.empty(n, dtype=torch.int32, device="cuda")
sink = torch.zeros(1, dtype=torch.int32, device="cuda")
kinds = os.environ.get("KINDS", "crc7 stream").split()
for kind in kinds:
    if kind.startswith("crc"):  # crc7 = the product kernel (the r1 variants: branch study-superseded-kernels)
        fn = lambda: jl.crc32c_fixed_dev(data, 4096, out=out)  # noqa: E731
    else:
        fn = lambda: jl.read_stream_dev(data, sink)  # noqa: E731
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(L + 1)]
    torch.cuda.synchronize()
    ev[0].record()
    for i in range(L):
        fn()
        ev[i + 1].record()
    torch.cuda.synchronize()
    t = np.array([ev[i].elapsed_time(ev[i + 1]) for i in range(L)])
    gbs = lambda ms: round(n * 4096 / (ms / 1e3) / 1e9, 1)  # noqa: E731
    print(json.dumps({"kind": kind, "first5_ms": round(t[:5].mean(), 4), "last20_ms": round(t[-20:].mean(), 4),
                      "first5_GBps": gbs(t[:5].mean()), "last20_GBps": gbs(t[-20:].mean()),
                      "min_ms": round(t.min(), 4)}), flush=True)
