#!/usr/bin/env python3
"""gv4 per-entry path cost: the same batches with fast ring turns allowed and
disabled (JL_GV4_NOFAST).  Workloads: 4M blocks of 1057 B at 1064-B spacing
(C5 record shape), 4M x 1 KiB implicit rounds, 512 x 8 MiB blocks (long rounds)."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import jleveldb_amd as jl  # noqa: E402

os.environ["JL_GENERAL"] = "gv4"
torch.cuda.set_device(0)
jl.init(0)
dev = torch.device("cuda:0")
n = 4 << 20
arena = torch.empty(n * 1064 + 64, dtype=torch.uint8, device=dev)
jl.fill_random_dev(arena, 9)
off = torch.arange(n, dtype=torch.int64, device=dev) * 1064 + 7
ln = torch.full((n,), 1057, dtype=torch.int32, device=dev)
out = torch.empty(n, dtype=torch.int32, device=dev)


def t_of(fn, reps=10):
    fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps


res = {}
big = 8 << 20
nbig = arena.numel() // big
for rnd in range(2):
    for v in ["", "nofast", "fullturn"]:
        os.environ.pop("JL_GV4_NOFAST", None)
        os.environ.pop("JL_GV4_FULLTURN", None)
        if v == "nofast":
            os.environ["JL_GV4_NOFAST"] = "1"
        if v == "fullturn":
            os.environ["JL_GV4_FULLTURN"] = "1"
        a = t_of(lambda: jl.crc32c_batch_dev(arena, off, ln, out=out))
        b = t_of(lambda: jl.crc32c_fixed_dev(arena, 1024, n, out=out))
        c = t_of(lambda: jl.crc32c_fixed_dev(arena, big, nbig, out=out))
        res.setdefault(v or "base", []).append((round(a, 4), round(b, 4), round(c, 4)))
for k, v in res.items():
    print(json.dumps({"variant": k, "c5shape_ms": [x[0] for x in v], "implicit1k_ms": [x[1] for x in v],
                      "blocks8M_ms": [x[2] for x in v]}))
