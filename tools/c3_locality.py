#!/usr/bin/env python3
"""Study: does address locality bound the C3 gv4 kernel?  Times the C3 set
(bench.secondary_c3's lengths) twice through jl_crc32c_batch_dev: packed in
index order (the bench's arena: a round's blocks of one K lie far apart), and
the same lengths packed in ascending-length order (the blocks of a K bin are
neighbours, so concurrently active rounds cover a narrow address window)."""
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402
import jleveldb_amd as jl  # noqa: E402
from jleveldb_amd import workloads as wl  # noqa: E402

steps = int(sys.argv[1]) if len(sys.argv) > 1 else 10
torch.cuda.set_device(0)
jl.init(0)
dev = torch.device("cuda:0")
stream = torch.cuda.current_stream()
lens = wl.c3_lengths(1 << 20, bench.SEED)
total = int(lens.sum(dtype=np.uint64))
arena = torch.empty(total + 16, dtype=torch.uint8, device=dev)
jl.fill_random_dev(arena, bench.SEED + 3)
d_len = torch.from_numpy(lens.view(np.int32)).to(dev)
out = torch.empty(lens.size, dtype=torch.int32, device=dev)
order = np.argsort(lens, kind="stable")
sorted_offs = np.empty(lens.size, np.uint64)
sorted_offs[order] = wl.packed_offsets(lens[order])
for name, offs in (("index order", wl.packed_offsets(lens)), ("length order", sorted_offs)):
    d_off = torch.from_numpy(offs.view(np.int64)).to(dev)
    wall, ms = bench.timed(lambda: jl.crc32c_batch_dev(arena, d_off, d_len, out=out), steps, 3, stream)
    print(json.dumps({"layout": name, "ms_per_step": round(ms / steps, 3),
                      "GiB_per_s": round(total / (ms / steps / 1e3) / 2**30, 1)}), flush=True)
