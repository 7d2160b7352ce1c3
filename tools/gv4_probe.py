#!/usr/bin/env python3
"""Study: where the general v4 kernel (crc_gv4_kernel<MODE_CRC>) loses against
the 4 KiB kernel (fixed_v4) on the same bytes.  Times, on one 4 GiB arena:
  fixed4k   1M x 4 KiB through jl_crc32c_fixed_dev (crc_fixed4k_v4_kernel)
  implicit  the same bytes as 4224-B blocks (fixed stride, 128-B multiple: gv4
            implicit rounds, no descriptors)
  sorted    1M x 4 KiB through jl_crc32c_batch_dev (offsets: gv4 rounds pipeline,
            round descriptors)
  ceiling   jl_read_stream_dev over the arena
(The gv4 bound-study variants this probe drove in r3, GV4_VARIANT=6 / 7, live on
the branch study-r5-gv4-switches.)"""
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import jleveldb_amd as jl  # noqa: E402

torch.cuda.set_device(0)
jl.init(0)
dev = torch.device("cuda:0")
n = 1 << 20
data = torch.empty(n * 4096 + 4096, dtype=torch.uint8, device=dev)
jl.fill_random_dev(data, 0x4A4C4442)
out = torch.empty(n, dtype=torch.int32, device=dev)
offs = torch.from_numpy((np.arange(n, dtype=np.uint64) * 4096).view(np.int64)).to(dev)
lens = torch.full((n,), 4096, dtype=torch.int32, device=dev)
sink = torch.zeros(1, dtype=torch.int32, device=dev)
n2 = (n * 4096) // 4224
legs = {
    "fixed4k": lambda: jl.crc32c_fixed_dev(data, 4096, n, out=out),
    "implicit": lambda: jl.crc32c_fixed_dev(data, 4224, n2, out=out),
    "sorted": lambda: jl.crc32c_batch_dev(data, offs, lens, out=out),
    "ceiling": lambda: jl.read_stream_dev(data[: n * 4096], sink),
}
res = {}
for name, fn in legs.items():
    for _ in range(30):
        fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(10):
        fn()
    e1.record()
    torch.cuda.synchronize()
    ms = e0.elapsed_time(e1) / 10
    res[name] = {"ms": round(ms, 4), "TB_per_s": round(n * 4096 / ms / 1e9, 3)}
print(json.dumps(res), flush=True)
