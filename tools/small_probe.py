"""Small-log paths side by side (r6): per C5 shape and size, the device-resident
verification time of the one-launch path (lc_small, JL_OPT_LOG_SMALL_MAX) and of
the chunked path, and the per-call latency of jl_log_verify from pageable host
memory through each device path and the host SSE4.2 path.  Medians.
Usage (GPU box): python tools/small_probe.py [sizes MiB, comma-separated]"""
import json
import os
import sys
import time

sys.path.insert(0, os.getcwd())
import numpy as np  # noqa: E402
import torch  # noqa: E402

import jleveldb_amd as jl  # noqa: E402
from jleveldb_amd import workloads as wl  # noqa: E402

torch.cuda.set_device(0)
jl.init(0)
dev = torch.device("cuda:0")
sizes = [float(x) for x in (sys.argv[1] if len(sys.argv) > 1 else "0.25,1,2,4,8,16,32,64").split(",")]


def med(fn, reps):
    fn()
    ts = []
    for _ in range(reps):
        t0 = time.perf_counter()
        fn()
        ts.append(time.perf_counter() - t0)
    return round(float(np.median(ts)) * 1e6, 1)


def dev_time(log, ev, res, reps=30, checksum=True):
    """Back-to-back asynchronous verifications on one stream, HIP events around them."""
    st = torch.cuda.current_stream()
    for _ in range(3):
        jl.log_verify_dev_async(log, checksum, events=ev, result=res)
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record(st)
    for _ in range(reps):
        jl.log_verify_dev_async(log, checksum, events=ev, result=res)
    b.record(st)
    torch.cuda.synchronize()
    return round(a.elapsed_time(b) / reps * 1e3, 1)


for which in wl.C5_SETS:
    for mib in sizes:
        lens = wl.c5_lengths(which, target=int(mib * (1 << 20)), seed=wl.SEED)
        plan = jl.log_layout(wl.packed_offsets(lens), lens)
        src = torch.empty(max(1, int(lens.sum(dtype=np.uint64))), dtype=torch.uint8, device=dev)
        jl.fill_random_dev(src, 5)
        log = jl.log_emit_dev(src, plan)
        del src
        ev = torch.empty((log.numel() // 7 + 2) * 16, dtype=torch.uint8, device=dev)
        res = torch.zeros(3, dtype=torch.int64, device=dev)
        host = log.cpu().numpy().copy()
        out = np.zeros(host.size // 7 + 2, dtype=jl.LOG_EVENT_DTYPE)
        row = {"set": which, "MiB": mib}
        reps = 30 if mib <= 8 else 10
        for path, small in (("small", 64 << 20), ("chunked", 0)):
            jl.set_option(jl.OPT_LOG_SMALL_MAX, small)
            row[f"dev_{path}_us"] = dev_time(log, ev, res)
            if path == "small":
                row["dev_small_nocrc_us"] = dev_time(log, ev, res, checksum=False)
            jl.set_option(jl.OPT_LOG_HOST_THRESHOLD, 0)
            row[f"call_{path}_us"] = med(lambda: jl.log_verify(host, out=out), reps)
        jl.set_option(jl.OPT_LOG_HOST_THRESHOLD, 1 << 40)
        row["call_host_us"] = med(lambda: jl.log_verify(host, out=out), reps)
        jl.set_option(jl.OPT_LOG_HOST_THRESHOLD, -1)
        jl.set_option(jl.OPT_LOG_SMALL_MAX, 16 << 20)
        print(json.dumps(row), flush=True)
        del log, ev, host
        torch.cuda.empty_cache()
