import sys, os
sys.path.insert(0, os.getcwd())
sys.path.insert(0, os.path.join(os.getcwd(), "tests"))
import numpy as np, torch
import jleveldb_amd as jl
from oracle import oracle
import test_gpu_handoffs as T

jl.init(0)
jl.set_option(jl.OPT_LOG_SMALL_MAX, 0)
gpu = torch.device("cuda:0")
for shape in sys.argv[1:]:
    rng = np.random.default_rng(T.SEED + len(shape))
    log = T._log(jl, gpu, T._segments(rng, shape))
    host = log.cpu().numpy().copy()
    flip = "noflip" not in os.environ.get("DBG", "")
    if flip:
        for b in rng.choice(host.size // 32768, 24, replace=False):
            host[int(b) * 32768 + int(rng.integers(0, 32768))] ^= 0x10
    log = torch.from_numpy(host).to(gpu)
    want = oracle.log_events(host)
    want = want[want["kind"] != 0]
    wb = np.bincount((want["offset"] >> 15).astype(np.int64), minlength=host.size // 32768 + 1)
    for it in range(3):
        ev, n = jl.log_verify_dev(log)
        got = ev[: n * 16].cpu().numpy().view(jl.LOG_EVENT_DTYPE)
        gl = got[got["kind"] != 0]
        gb = np.bincount((gl["offset"] >> 15).astype(np.int64), minlength=wb.size)[: wb.size]
        bad = np.nonzero(gb != wb)[0]
        g, w = T._live(got), T._live(want)
        same = g.shape == w.shape and np.array_equal(g, w)
        print(shape, "flip" if flip else "noflip", "iter", it, "n", n, "want", want.size, "equal", same,
              "blocks differing", bad.size, bad[:8].tolist(), (gb[bad[:4]] if bad.size else []), (wb[bad[:4]] if bad.size else []), flush=True)
