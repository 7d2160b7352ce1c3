"""Copy-inclusive log verify from pinned vs pageable (registered per call) input,
timed alternately into one reused event array, plus plain H2D rates of 64 MiB
pieces from each kind (r5q: profiles/r5q_copy_pinned_vs_registered.log).
Usage (GPU box): python tools/copy_probe.py [set ...]  (C5 set names, workloads.C5_SETS)"""
import json, os, sys, time
sys.path.insert(0, os.getcwd())
import numpy as np, torch
import jleveldb_amd as jl
from jleveldb_amd import workloads as wl
torch.cuda.set_device(0); jl.init(0)
dev = torch.device("cuda:0")
for which in sys.argv[1:] or ["random_0_200", "mixed_1b_100k"]:
    lens = wl.c5_lengths(which, seed=0x4A4C4442)
    plan = jl.log_layout(wl.packed_offsets(lens), lens)
    src = torch.empty(int(lens.sum(dtype=np.uint64)), dtype=torch.uint8, device=dev)
    jl.fill_random_dev(src, 7)
    log = jl.log_emit_dev(src, plan); del src
    nb = log.numel()
    host = torch.empty(nb, dtype=torch.uint8, pin_memory=True); host.copy_(log)
    d = torch.empty(64 << 20, dtype=torch.uint8, device=dev)
    del log; torch.cuda.empty_cache()
    hn = host.numpy(); pg = hn.copy()
    out = np.zeros(int(plan["len"].size) + 64, dtype=jl.LOG_EVENT_DTYPE)
    jl.log_verify(hn, out=out); jl.log_verify(pg, out=out)
    res = {"set": which, "pinned": [], "pageable": [], "h2d_pinned_64MiB_GiBps": [], "h2d_registered_64MiB_GiBps": []}
    for r in range(3):
        order = (("pinned", hn), ("pageable", pg)) if r % 2 == 0 else (("pageable", pg), ("pinned", hn))
        for name, a in order:
            t0 = time.perf_counter(); jl.log_verify(a, out=out); el = time.perf_counter() - t0
            res[name].append(round(nb / el / 2**30, 2))
    # plain copies: 64 pieces of 64 MiB from the pinned tensor
    torch.cuda.synchronize(); t0 = time.perf_counter()
    for i in range(64):
        d.copy_(host[i << 26:(i + 1) << 26], non_blocking=True)
    torch.cuda.synchronize(); res["h2d_pinned_64MiB_GiBps"].append(round(4 / (time.perf_counter() - t0), 2))
    cudart = torch.cuda.cudart()
    pt = torch.from_numpy(pg)
    rc = cudart.cudaHostRegister(pt.data_ptr(), pt.numel(), 0)
    torch.cuda.synchronize(); t0 = time.perf_counter()
    for i in range(64):
        d.copy_(pt[i << 26:(i + 1) << 26], non_blocking=True)
    torch.cuda.synchronize(); res["h2d_registered_64MiB_GiBps"].append(round(4 / (time.perf_counter() - t0), 2))
    cudart.cudaHostUnregister(pt.data_ptr())
    res["register_rc"] = int(rc)
    print(json.dumps(res), flush=True)
    del host, hn, pg, out, d
