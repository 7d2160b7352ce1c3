#!/usr/bin/env python3
"""Study: the engine clock while C2 (1M x 4 KiB) and C3 (1M Zipf blocks) launches
run back to back for ~3 s each, sampled with rocm-smi from a child process."""
import os
import subprocess
import sys
import threading
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402
import jleveldb_amd as jl  # noqa: E402
from jleveldb_amd import workloads as wl  # noqa: E402

torch.cuda.set_device(0)
jl.init(0)
dev = torch.device("cuda:0")


def sample(out, stop):
    while not stop.is_set():
        r = subprocess.run(["rocm-smi", "--showclocks", "--showpower"], capture_output=True, text=True)
        out.append(" | ".join(l.strip() for l in r.stdout.splitlines() if "sclk" in l.lower() or "power" in l.lower()))
        time.sleep(0.4)


def run(name, fn, secs=3.0):
    fn()
    torch.cuda.synchronize()
    out, stop = [], threading.Event()
    th = threading.Thread(target=sample, args=(out, stop))
    th.start()
    t0, n = time.perf_counter(), 0
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    while time.perf_counter() - t0 < secs:
        for _ in range(20):
            fn()
        n += 20
        torch.cuda.synchronize()
    e1.record()
    torch.cuda.synchronize()
    stop.set()
    th.join()
    print(name, "ms/launch %.4f" % (e0.elapsed_time(e1) / n), flush=True)
    for o in out[1:-1]:
        print("   ", o[:300], flush=True)


blocks = torch.empty(1 << 32, dtype=torch.uint8, device=dev)
jl.fill_random_dev(blocks, bench.SEED)
out = torch.empty(1 << 20, dtype=torch.int32, device=dev)
run("C2", lambda: jl.crc32c_fixed_dev(blocks, 4096, out=out))
del blocks
torch.cuda.empty_cache()
lens = wl.c3_lengths(1 << 20, bench.SEED)
arena = torch.empty(int(lens.sum(dtype=np.uint64)) + 16, dtype=torch.uint8, device=dev)
jl.fill_random_dev(arena, bench.SEED + 3)
d_off = torch.from_numpy(wl.packed_offsets(lens).view(np.int64)).to(dev)
d_len = torch.from_numpy(lens.view(np.int32)).to(dev)
run("C3", lambda: jl.crc32c_batch_dev(arena, d_off, d_len, out=out))
