#!/usr/bin/env python3
"""Study: a WAL whose 32 KiB blocks each hold 10 short records and then one
~31 KiB record.  lc_walk sees 8 short records within 4 KiB and marks every block
dense, so lc_dense checks the long record with ONE thread (a 7 900-dword chain)
while the workgroup's other threads wait.  Times it against a log of the same
size with one ~32 KiB record per block (the chunked rounds), ms per call.
Usage: python tools/cliff_probe.py [GiB]"""
import json
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import jleveldb_amd as jl  # noqa: E402
from jleveldb_amd import workloads as wl  # noqa: E402

gib = float(sys.argv[1]) if len(sys.argv) > 1 else 1.0
torch.cuda.set_device(0)
jl.init(0)
dev = torch.device("cuda:0")
nblk = int(gib * (1 << 30)) // 32768
big = 32768 - 7 - 10 * 107  # fills the block after 10 records of 100 B
mixed = np.tile(np.array([100] * 10 + [big], np.uint32), nblk)
single = np.full(nblk, 32768 - 7, np.uint32)


def run(lens, reps=10):
    plan = jl.log_layout(wl.packed_offsets(lens), lens)
    src = torch.empty(int(lens.sum(dtype=np.uint64)), dtype=torch.uint8, device=dev)
    jl.fill_random_dev(src, 11)
    log = jl.log_emit_dev(src, plan)
    del src
    ev = torch.empty((log.numel() // 7 + 2) * 16, dtype=torch.uint8, device=dev)
    _, n = jl.log_verify_dev(log, 1, events=ev)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(reps):
        jl.log_verify_dev(log, 1, events=ev)
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / reps * 1e3, int(n), log.numel()


ms_m, n_m, b_m = run(mixed)
ms_s, n_s, b_s = run(single)
# short records of random lengths (a WAL of variable small values): every block
# dense, its runs one record long, so lc_dense walks it one header at a time
rnd = np.random.default_rng(5).integers(0, 201, int(gib * (1 << 30)) // 107).astype(np.uint32)
ms_r, n_r, b_r = run(rnd)
dbb = np.full(int(gib * (1 << 30)) // 138, 131, np.uint32)
ms_d, n_d, b_d = run(dbb)
print(json.dumps({"blocks": nblk, "short_then_long": {"ms": round(ms_m, 3), "events": n_m, "bytes": b_m},
                  "one_record_per_block": {"ms": round(ms_s, 3), "events": n_s, "bytes": b_s},
                  "random_0_200": {"ms": round(ms_r, 3), "events": n_r, "bytes": b_r},
                  "dbbench_131": {"ms": round(ms_d, 3), "events": n_d, "bytes": b_d}}))
