#!/usr/bin/env python3
"""Study: staged (pageable, not registered) copy-inclusive C2 rate against the
staging piece size (JL_OPT_STAGE_PIECE) and copy threads (JL_OPT_STAGE_THREADS),
interleaved repetitions on one box.  Usage: staged_probe.py [GiB] [reps]"""
import json
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import jleveldb_amd as jl  # noqa: E402

gib = float(sys.argv[1]) if len(sys.argv) > 1 else 4.0
reps = int(sys.argv[2]) if len(sys.argv) > 2 else 3
n = int(gib * (1 << 30)) // 4096 * 4096
data = np.random.default_rng(7).integers(0, 256, n, dtype=np.uint8)
ref = jl.crc32c_fixed(data[: 64 << 20], 4096)
jl.set_option(jl.OPT_HOST_REGISTER, 0)
variants = [(p, t) for p in (4 << 20, 16 << 20, 0) for t in (8, 12)]
res = {f"piece={p >> 20}MiB threads={t}": [] for p, t in variants}
for r in range(reps):
    for p, t in variants:
        jl.set_option(jl.OPT_STAGE_PIECE, p)
        jl.set_option(jl.OPT_STAGE_THREADS, t)
        t0 = time.perf_counter()
        got = jl.crc32c_fixed(data, 4096)
        dt = time.perf_counter() - t0
        assert np.array_equal(got[: len(ref)], ref)
        res[f"piece={p >> 20}MiB threads={t}"].append(round(n / dt / (1 << 30), 2))
        print(json.dumps({"rep": r, "piece": p, "threads": t, "GiB_per_s": round(n / dt / (1 << 30), 2)}), flush=True)
print(json.dumps({"staged_c2_GiB_per_s": res, "bytes": n}))
