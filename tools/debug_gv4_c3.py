"""Debug: the C3 workload through gv4 with load-address validation
(JL_GV4_DEBUG=lo:hi = the arena); repeated calls; parity vs the stream kernel."""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import jleveldb_amd as jl  # noqa: E402

SEED = 0x4A4C4442
jl.init(0)
dev = torch.device("cuda:0")
rng = np.random.default_rng(SEED)
n = int(os.environ.get("N", 1 << 20))
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
os.environ["JL_GENERAL"] = "stream"
ref = jl.crc32c_batch_dev(arena, d_off, d_len).cpu().numpy()
os.environ["JL_GENERAL"] = "gv4"
lo = arena.data_ptr()
os.environ["JL_GV4_DEBUG"] = f"{lo:x}:{lo + arena.numel():x}"
for it in range(int(os.environ.get("ITERS", 3))):
    got = jl.crc32c_batch_dev(arena, d_off, d_len).cpu().numpy()
    print("iter", it, "mismatches", int((got != ref).sum()), flush=True)
