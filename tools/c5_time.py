#!/usr/bin/env python3
"""Times config C5 (device-resident WAL verification, both payload sets) through
the fused and the default (walk + chunked rounds) log paths — bench.py's secondary_c5 without the CPU
leg.  Usage: python tools/c5_time.py [steps] [sets: both | c1 | mixed] [device: skip the copy-inclusive leg]"""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402
import jleveldb_amd as jl  # noqa: E402

steps = int(sys.argv[1]) if len(sys.argv) > 1 else 10
torch.cuda.set_device(0)
jl.init(0)
dev = torch.device("cuda:0")
stream = torch.cuda.current_stream()
which = sys.argv[2] if len(sys.argv) > 2 else "both"
for mixed in {"both": (False, True), "c1": (False,), "mixed": (True,)}[which]:
    print(json.dumps(bench.secondary_c5(dev, stream, steps, 3, mixed=mixed, cpu=False,
                                             host_copy=len(sys.argv) < 4)), flush=True)
    torch.cuda.empty_cache()
