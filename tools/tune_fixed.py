#!/usr/bin/env python3
"""A/B of crc_fixed4k_kernel variants (nt loads x prefetch depth) and of the
read-stream ceiling, interleaved in one process (cdna_hip_programming.md §5.4
rule 24).  Prints one JSON line per variant: median / min kernel time over
rounds and GB/s of algorithmic bytes."""
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import jleveldb_amd as jl  # noqa: E402

n = int(os.environ.get("BLOCKS", 1 << 20))
rounds = int(os.environ.get("ROUNDS", 7))
torch.cuda.set_device(0)
jl.init(0)
data = torch.empty(n * 4096, dtype=torch.uint8, device="cuda")
jl.fill_random_dev(data, 0x4A4C4442)
out = torch.empty(n, dtype=torch.int32, device="cuda")
sink = torch.zeros(1, dtype=torch.int32, device="cuda")
variants = [tuple(int(x) for x in v.split(",")) for v in os.environ.get("VARIANTS", "1,1,2 1,1,3 1,1,103").split()]
ref = None
times = {v: [] for v in variants}
times["read_stream"] = []
for r in range(rounds):
    for v in variants:
        os.environ["JL_FIXED_NT"], os.environ["JL_FIXED_DEPTH"], os.environ["JL_FIXED_CHAINS"] = map(str, v)
        jl.crc32c_fixed_dev(data, 4096, out=out)
        torch.cuda.synchronize()
        res = out.cpu().numpy()
        if ref is None:
            ref = res
        assert v[2] > 100 or np.array_equal(ref, res), v
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(5):
            jl.crc32c_fixed_dev(data, 4096, out=out)
        e1.record()
        torch.cuda.synchronize()
        times[v].append(e0.elapsed_time(e1) / 5)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(5):
        jl.read_stream_dev(data, sink)
    e1.record()
    torch.cuda.synchronize()
    times["read_stream"].append(e0.elapsed_time(e1) / 5)
for k, t in times.items():
    t = np.array(t)
    byts = n * 4096 + (0 if k == "read_stream" else n * 4)
    print(json.dumps({"variant": str(k), "median_ms": round(float(np.median(t)), 4), "min_ms": round(float(t.min()), 4),
                      "GBps_median": round(byts / (np.median(t) / 1e3) / 1e9, 1),
                      "GBps_best": round(byts / (t.min() / 1e3) / 1e9, 1)}))
