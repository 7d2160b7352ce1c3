#!/usr/bin/env python3
"""Device-resident timings of the general-path configs without CPU legs:
C3 (bench.secondary_c3) and the C5 sets (bench.secondary_c5).
Usage: [JL_OPTS="option=value,..."] python tools/sec_time.py [steps] [which: all | c3 | c5 | dispatch | <C5 set name>[,<set>...]]"""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402
import jleveldb_amd as jl  # noqa: E402
from jleveldb_amd import workloads as wl  # noqa: E402

steps = int(sys.argv[1]) if len(sys.argv) > 1 else 10
which = sys.argv[2] if len(sys.argv) > 2 else "all"
torch.cuda.set_device(0)
jl.init(0)
for kv in filter(None, os.environ.get("JL_OPTS", "").split(",")):  # engine options for A/Bs: "option=value,..."
    k, v = kv.split("=")
    jl.set_option(int(k), int(v))
dev = torch.device("cuda:0")
stream = torch.cuda.current_stream()
if which == "all" or "c3" in which.split(","):
    print(json.dumps(bench.secondary_c3(dev, stream, steps, 3, cpu=False)), flush=True)
    torch.cuda.empty_cache()
if which in ("all", "dispatch"):
    print(json.dumps(bench.dispatch_latency()), flush=True)
ws = which.split(",")
sets = wl.C5_SETS if which == "all" or "c5" in ws else [x for x in ws if x in wl.C5_SETS]
for s in sets:
    r = bench.secondary_c5(dev, stream, steps, 3, which=s, cpu=False, host_copy=False)
    print(json.dumps({k: r[k] for k in ("config", "GiB_per_s", "achieved_GBps", "achieved_frac_of_peak", "ms_per_step",
                                        "records_ok", "dense_blocks", "sync_call", "async_events_equal_sync", "fused")
                      if k in r}), flush=True)
    torch.cuda.empty_cache()
