#!/usr/bin/env python3
"""Per-workgroup phase clocks of lc_dense (study build with -DJL_LD_PROF=1).

Usage: JLCRC_STUDY_LIB=tools/libjlcrc_<name>.so python tools/ld_prof.py [set]
Verifies one C5 set once (after warm-up calls) and prints, averaged over the
blocks, the shader clocks thread 0 of a workgroup saw in each phase: stage
(waiting for the previous block's readers, storing the prefetched bytes), walk
(the runs, with their barriers), crc, stash (runs out, next pass) — and the
spread of the workgroups' start and end times (s_memrealtime, 100 MHz): a wide
end spread means the persistent grid's static block dealing leaves a tail.
Analysis tool only."""
import ctypes
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import jleveldb_amd as jl  # noqa: E402
from jleveldb_amd import workloads as wl  # noqa: E402

which = sys.argv[1] if len(sys.argv) > 1 else "dbbench_131"
torch.cuda.set_device(0)
jl.init(0)
prof = jl.lib().jl_study_ld_prof
prof.argtypes = [ctypes.c_void_p]
buf = np.zeros(4096 * 8, np.uint64)
dev = torch.device("cuda:0")
# random_0_200: a WAL of variable small values (tools/cliff_probe.py), ~1 GiB
lens = (np.random.default_rng(5).integers(0, 201, (1 << 30) // 107).astype(np.uint32) if which == "random_0_200"
        else wl.c5_lengths(which))
plan = jl.log_layout(wl.packed_offsets(lens), lens)
src = torch.empty(int(lens.sum(dtype=np.uint64)), dtype=torch.uint8, device=dev)
jl.fill_random_dev(src, wl.SEED + 3)
log = jl.log_emit_dev(src, plan)
del src
ev = torch.empty((log.numel() // 7 + 2) * 16, dtype=torch.uint8, device=dev)
for _ in range(3):
    jl.log_verify_dev(log, 1, events=ev)
torch.cuda.synchronize()
assert prof(buf.ctypes.data) == 0
jl.log_verify_dev(log, 1, events=ev)
torch.cuda.synchronize()
assert prof(buf.ctypes.data) == 0
w = buf.reshape(-1, 8)
w = w[w[:, 6] > 0].astype(np.float64)
blocks = w[:, 4].sum()
per = {n: round(float(w[:, i].sum() / blocks), 1) for i, n in enumerate(("stage", "walk", "crc", "stash"))}
t0 = w[:, 5].min()
end = (w[:, 6] - t0) / 100.0
print(json.dumps({"set": which, "workgroups": int(w.shape[0]), "blocks": int(blocks),
                  "clocks_per_block": per, "clocks_sum": round(sum(per.values()), 1),
                  "blocks_per_wg": {"min": int(w[:, 4].min()), "max": int(w[:, 4].max())},
                  "start_spread_us": round(float((w[:, 5].max() - t0) / 100.0), 1),
                  "end_us_percentiles": {p: round(float(np.percentile(end, p)), 1) for p in (1, 10, 50, 90, 99, 100)}}),
      flush=True)
