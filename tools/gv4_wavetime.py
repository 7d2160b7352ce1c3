#!/usr/bin/env python3
"""Study (JLCRC_STUDY_LIB = a build with -DJL_GV4_WAVETIME=1): the end-time
distribution of crc_gv4_kernel's waves on C3 (MODE_CRC) and the C5 1 056-B set
(MODE_LOG_CHUNK): if the last waves run long after the median one, the grid's
tail (per-wave work imbalance) holds the kernel back.
Usage: JLCRC_STUDY_LIB=tools/libjlcrc_wt.so python tools/gv4_wavetime.py"""
import ctypes
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402
import jleveldb_amd as jl  # noqa: E402
from jleveldb_amd import workloads as wl  # noqa: E402

torch.cuda.set_device(0)
jl.init(0)
L = jl.lib()


def read(mode):
    buf = np.zeros(2 * 16384, np.uint64)
    fn = getattr(L, f"jl_study_gv4_wavetime_m{mode}" if mode != "fx" else "jl_study_fx_wavetime")
    fn.argtypes = [ctypes.c_void_p]
    assert fn(buf.ctypes.data) == 0
    t = buf.reshape(-1, 2)
    np.save(os.path.join("gpurun_out", f"wavetime_m{mode}_{len(os.listdir('gpurun_out')) if os.path.isdir('gpurun_out') else 0}.npy"), t)
    t = t[t[:, 1] > 0].astype(np.float64) / 100.0  # us
    t0 = t[:, 0].min()
    end = t[:, 1] - t0
    return {"waves": int(t.shape[0]), "first_start_to_last_end_us": round(float(end.max()), 1),
            "start_spread_us": round(float(t[:, 0].max() - t0), 1),
            "end_us_percentiles": {p: round(float(np.percentile(end, p)), 1) for p in (1, 10, 50, 90, 99, 100)}}


dev = torch.device("cuda:0")
c2 = torch.empty(1 << 32, dtype=torch.uint8, device=dev)
jl.fill_random_dev(c2, wl.SEED)
out = torch.empty(1 << 20, dtype=torch.int32, device=dev)
for _ in range(20):
    jl.crc32c_fixed_dev(c2, 4096, out=out)
torch.cuda.synchronize()
read("fx")
jl.crc32c_fixed_dev(c2, 4096, out=out)
torch.cuda.synchronize()
print(json.dumps({"C2 crc_fixed4k_v4_kernel": read("fx")}), flush=True)
del c2
torch.cuda.empty_cache()
lens = wl.c3_lengths()
offs = wl.packed_offsets(lens)
total = int(offs[-1]) + int(lens[-1])
arena = torch.empty(total + 4096, dtype=torch.uint8, device=dev)
jl.fill_random_dev(arena, wl.SEED)
o = torch.from_numpy(offs.view(np.int64)).to(dev)
n = torch.from_numpy(lens.view(np.int32)).to(dev)
for _ in range(5):
    jl.crc32c_batch_dev(arena, o, n)
torch.cuda.synchronize()
read(0)
jl.crc32c_batch_dev(arena, o, n)
torch.cuda.synchronize()
print(json.dumps({"C3 crc_gv4_kernel<MODE_CRC>": read(0)}), flush=True)
del arena
torch.cuda.empty_cache()
for which in ("c1_1056", "mixed_1b_100k"):
    lens = wl.c5_lengths(which)
    plan = jl.log_layout(wl.packed_offsets(lens), lens)
    src = torch.empty(int(lens.sum(dtype=np.uint64)), dtype=torch.uint8, device=dev)
    jl.fill_random_dev(src, wl.SEED + 3)
    log = jl.log_emit_dev(src, plan)
    del src
    for _ in range(3):
        jl.log_verify_dev(log, 1)
    torch.cuda.synchronize()
    read(5)
    jl.log_verify_dev(log, 1)
    torch.cuda.synchronize()
    print(json.dumps({f"C5 {which} crc_gv4_kernel<MODE_LOG_CHUNK>": read(5)}), flush=True)
    del log
    torch.cuda.empty_cache()
