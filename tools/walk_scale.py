#!/usr/bin/env python3
"""Does lc_walk scale with the log (random-line throughput) or stay put (one
hop latency per record, fewer chains in flight)?  Verifies prefixes of the C5
1 056-B log (whole 32 KiB blocks) REPS times each, largest first; run it under
`rocprofv3 --kernel-trace --stats` and read the per-size kernel durations with
`python tools/walk_scale.py --parse <kernel_trace.csv>`.
Usage: python tools/walk_scale.py [set]"""
import csv
import os
import sys

FRACS = (1.0, 0.5, 0.25, 0.125, 0.0625)
REPS = 20

if len(sys.argv) > 2 and sys.argv[1] == "--parse":
    rows = list(csv.DictReader(open(sys.argv[2])))
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    for name in ("lc_walk_kernel", "lc_build_kernel", "crc_gv4_kernel", "lc_dense_kernel"):
        d = [(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3 for r in rows if name in r["Kernel_Name"]]
        d = d[-len(FRACS) * REPS:]  # the timed calls (the first verification is a warm-up)
        if len(d) == len(FRACS) * REPS:
            med = [sorted(d[i * REPS:(i + 1) * REPS])[REPS // 2] for i in range(len(FRACS))]
            print(name, " ".join(f"{f:g}:{m:.1f}us" for f, m in zip(FRACS, med)))
    sys.exit(0)

import numpy as np  # noqa: E402
import torch  # noqa: E402

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import jleveldb_amd as jl  # noqa: E402
from jleveldb_amd import workloads as wl  # noqa: E402

which = sys.argv[1] if len(sys.argv) > 1 else "c1_1056"
torch.cuda.set_device(0)
jl.init(0)
lens = wl.c5_lengths(which, seed=0x4A4C4442)
plan = jl.log_layout(wl.packed_offsets(lens), lens)
src = torch.empty(int(lens.sum(dtype=np.uint64)), dtype=torch.uint8, device="cuda")
jl.fill_random_dev(src, 0x4A4C4447)
log = jl.log_emit_dev(src, plan)
del src
nb = plan["log_bytes"]
events = torch.empty((nb // 7 + 2) * 16, dtype=torch.uint8, device="cuda")
result = torch.empty(3, dtype=torch.int64, device="cuda")
jl.log_verify_dev_async(log, jl.LOG_CHECKSUM, events=events, result=result)  # warm-up
for f in FRACS:
    n = int(nb * f) // 32768 * 32768
    part = log[:n]
    for _ in range(REPS):
        jl.log_verify_dev_async(part, jl.LOG_CHECKSUM, events=events, result=result)
    torch.cuda.synchronize()
    print(f"{f:g}: {n} bytes, {int(result[0])} events", flush=True)
