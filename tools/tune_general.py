#!/usr/bin/env python3
"""A/B of the general-path kernels (r1 chunked kernel vs the stream kernel at
ring depths 16/32/48) on configs C3 (mixed Zipf sizes) and C5 (WAL verify),
interleaved in one process; results must agree across variants."""
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import jleveldb_amd as jl  # noqa: E402

SEED = 0x4A4C4442
torch.cuda.set_device(0)
jl.init(0)
dev = torch.device("cuda:0")
rounds = int(os.environ.get("ROUNDS", 3))
variants = os.environ.get("VARIANTS", "s16 gv4").split()

# C3
rng = np.random.default_rng(SEED)
n = 1 << 20
ks = np.empty(0, dtype=np.int64)
while ks.size < n:
    k = rng.zipf(1.1, 2 * n)
    ks = np.concatenate([ks, k[k <= 64]])
lens = (1024 * (ks[:n] - 1) + 1 + rng.integers(0, 1024, n)).astype(np.uint32)
offs = np.zeros(n, np.uint64)
offs[1:] = np.cumsum(lens[:-1], dtype=np.uint64)
total = int(lens.sum(dtype=np.uint64))
arena = torch.empty(total + 16, dtype=torch.uint8, device=dev)
jl.fill_random_dev(arena, SEED + 3)
d_off = torch.from_numpy(offs.view(np.int64)).to(dev)
d_len = torch.from_numpy(lens.view(np.int32)).to(dev)
out = torch.empty(n, dtype=torch.int32, device=dev)

# C5 (smaller: 1 GiB log)
rec = 1056
n_rec = (1 << 30) // (rec + 7)
plan = jl.log_layout(np.arange(n_rec, dtype=np.uint64) * rec, np.full(n_rec, rec, np.uint32))
src = torch.empty(n_rec * rec, dtype=torch.uint8, device=dev)
jl.fill_random_dev(src, SEED + 5)
log = jl.log_emit_dev(src, plan)
del src
events = torch.empty((log.numel() // 7 + 2) * 16, dtype=torch.uint8, device=dev)

# C2 through the general path (1M x 4 KiB blocks described by off/len arrays)
n2 = 1 << 20
arena2 = torch.empty(n2 * 4096, dtype=torch.uint8, device=dev)
jl.fill_random_dev(arena2, SEED)
off2 = torch.arange(n2, dtype=torch.int64, device=dev) * 4096
len2 = torch.full((n2,), 4096, dtype=torch.int32, device=dev)
out2 = torch.empty(n2, dtype=torch.int32, device=dev)


def setv(v):
    os.environ["JL_GENERAL"] = v if v in ("chunk", "gv4") else ("gv4" if v.startswith("gv4") else "stream")
    for knob, name in (("JL_GV4_NONT", "gv4nont"), ("JL_GV4_FULLTURN", "gv4full")):
        if v == name:
            os.environ[knob] = "1"
        else:
            os.environ.pop(knob, None)
    os.environ.pop("JL_NO_PARTITION", None)
    if v not in ("chunk",) and not v.startswith("gv4"):
        os.environ["JL_STREAM_DEPTH"] = v[1:].replace("np", "")
        if v.endswith("np"):
            os.environ["JL_NO_PARTITION"] = "1"


def t_of(fn, reps=5):
    fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps


ref3 = ref5 = None
times = {v: {"c3": [], "c5": [], "c2": []} for v in variants}
for r in range(rounds):
    for v in variants:
        setv(v)
        jl.crc32c_batch_dev(arena, d_off, d_len, out=out)
        got3 = out.cpu().numpy().copy()
        ev, ne = jl.log_verify_dev(log, events=events)
        got5 = ev[: ne * 16].cpu().numpy().copy()
        if ref3 is None:
            ref3, ref5 = got3, got5
        assert np.array_equal(ref3, got3), ("C3 mismatch", v)
        assert np.array_equal(ref5, got5), ("C5 mismatch", v)
        times[v]["c3"].append(t_of(lambda: jl.crc32c_batch_dev(arena, d_off, d_len, out=out)))
        times[v]["c5"].append(t_of(lambda: jl.log_verify_dev(log, events=events)))
        times[v]["c2"].append(t_of(lambda: jl.crc32c_batch_dev(arena2, off2, len2, out=out2)))
kinds5 = ref5.reshape(-1, 16)[:, 13]
print(json.dumps({"c5_records": int(ne), "c5_ok": int((kinds5 == 1).sum())}))
for v in variants:
    c3 = float(np.median(times[v]["c3"]))
    c5 = float(np.median(times[v]["c5"]))
    print(json.dumps({"variant": v, "c3_ms": round(c3, 3), "c3_GBps": round((total + 16 * n) / (c3 / 1e3) / 1e9, 1),
                      "c5_ms": round(c5, 3), "c5_GiBps": round(log.numel() / (c5 / 1e3) / 2**30, 1),
                      "c2_general_ms": round(float(np.median(times[v]["c2"])), 3)}))
