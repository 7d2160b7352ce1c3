"""Debug: which step counts K fail on the gv4 path (prints K -> mismatches)."""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import jleveldb_amd as jl  # noqa: E402
from oracle import oracle  # noqa: E402

os.environ["JL_GENERAL"] = "gv4"
jl.init(0)
rng = np.random.default_rng(1)
Ks = [int(x) for x in os.environ.get("KS", "1 8 15 16 17 24 31 32 33 40 47 48 49 54 64 65 100 128 129 300").split()]
reps = int(os.environ.get("REPS", "9"))
lens = np.array([128 * k - int(rng.integers(0, 128)) for k in Ks for _ in range(reps)], np.uint32)
offs = np.zeros(lens.size, np.uint64)
align = int(os.environ.get("ALIGN", "0"))  # 1: virtual starts p - f 16-B aligned (aligned plain-step loads)
pos = int(os.environ.get("BASE", "0"))
for i, n in enumerate(lens):
    if align:
        f = (-int(n)) % 128
        pos += (f - pos) % 16
    offs[i] = pos
    pos += int(n) + int(os.environ.get("GAP", "0"))
arena = rng.integers(0, 256, pos + 8, dtype=np.uint8)
d = torch.from_numpy(arena).cuda()
got = jl.crc32c_batch_dev(d, torch.from_numpy(offs.view(np.int64)).cuda(),
                          torch.from_numpy(lens.view(np.int32)).cuda()).cpu().numpy().view(np.uint32)
want = oracle.batch(arena, offs, lens)
bad = got != want
for i, k in enumerate(Ks):
    b = bad[i * reps:(i + 1) * reps]
    print(k, int(b.sum()), "".join("x" if v else "." for v in b))
