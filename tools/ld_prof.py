#!/usr/bin/env python3
"""Per-phase shader clocks of lc_dense (study build with -DJL_LD_PROF=1).

Usage: JLCRC_STUDY_LIB=tools/libjlcrc_<name>.so python tools/ld_prof.py [steps] [set]
Runs bench.secondary_c5 on one C5 set and prints, per dense block a workgroup
processed, the clocks thread 0 saw in each phase: stage (wait for the previous
block's readers, prefetched bytes to LDS), issue (the next block's prefetch
loads), walk (wave 0), walk_barrier (waiting for the other waves), crc (one
thread per record), stash (events out).  Analysis tool only."""
import ctypes
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402
import jleveldb_amd as jl  # noqa: E402

steps = int(sys.argv[1]) if len(sys.argv) > 1 else 10
which = sys.argv[2] if len(sys.argv) > 2 else "dbbench_131"
torch.cuda.set_device(0)
jl.init(0)
lib = ctypes.CDLL(jl.LIB_PATH)
prof = lib.jl_study_ld_prof
out = (ctypes.c_ulonglong * 8)()
assert prof(out) == 0
dev = torch.device("cuda:0")
r = bench.secondary_c5(dev, torch.cuda.current_stream(), steps, 3, which=which, cpu=False, host_copy=False)
assert prof(out) == 0
blocks = max(out[4], 1)
names = {0: "stage", 5: "issue", 1: "walk", 6: "walk_barrier", 2: "crc", 3: "stash"}
per = {n: round(out[i] / blocks, 1) for i, n in names.items()}
print(json.dumps({"set": which, "ms_per_step": r["ms_per_step"], "dense_block_iterations": out[4],
                  "clocks_per_block": per, "sum": round(sum(per.values()), 1)}), flush=True)
