#!/usr/bin/env python3
"""Headline benchmark: device-resident masked CRC32C over 4 KiB blocks.

BASELINE.json metric "GiB/s CRC32C over 4 KiB blocks (device-resident); % of HBM
read roofline", workload = config C2 (1M x 4 KiB random blocks per GPU, bit-exact
vs the reference algorithm).  One step = one pass of the engine over the whole
1M-block batch (jl_crc32c_fixed_dev), inputs resident in HBM.  With N GPUs
(torchrun, one process per GPU) every rank holds its own 1M-block shard of the
C4 8M-block set, generated in place (weak scaling, no data-path collective);
value = all ranks' bytes / max-over-ranks time.

Also reported on the same JSON line:
  roofline     — dominant kernel (crc_fixed4k_v4_kernel) timed with HIP events on
                 its launch stream; algorithmic bytes = 4096 B read + 4 B
                 written per block; peak = 8.0 TB/s (MI355X spec);
                 measured read-stream ceiling beside it; traffic from the
                 committed rocprofv3 PMC summary (profiles/) when present.
  cpu_baseline — rank 0 at N=1: the CPU oracle (restatement of the reference's
                 slicing-by-8 Crc32C.update) on a 1 GiB sample of the same
                 blocks, looped for ~10 s; parity of that sample checked.
  secondary    — configs C3 (mixed Zipf sizes) and C5 (WAL verify), N=1 only.
"""
from __future__ import annotations

import argparse
import glob
import json
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)
import jleveldb_amd as jl  # noqa: E402
from jleveldb_amd import shard as shd  # noqa: E402
from jleveldb_amd import workloads as wl  # noqa: E402

SEED = 0x4A4C4442
PEAK_GBS = 8000.0  # MI355X HBM3E spec, /opt/skills/guides/MI355X_MICROARCH.md:36
GIB = float(1 << 30)


def timed(fn, steps, warmup, stream):
    """Runs fn() warmup+steps times; returns (wall_s, event_ms) of the timed steps."""
    for _ in range(warmup):
        fn()
    torch.cuda.synchronize()
    e0 = torch.cuda.Event(enable_timing=True)
    e1 = torch.cuda.Event(enable_timing=True)
    t0 = time.perf_counter()
    e0.record(stream)
    for _ in range(steps):
        fn()
    e1.record(stream)
    torch.cuda.synchronize()
    return time.perf_counter() - t0, e0.elapsed_time(e1)


def read_stream_ceiling(data, stream) -> float:
    sink = torch.zeros(1, dtype=torch.int32, device=data.device)
    _, ms = timed(lambda: jl.read_stream_dev(data, sink), 10, 3, stream)
    return data.numel() / (ms / 10 / 1e3) / 1e9


def pmc_traffic():
    """HBM bytes per launch of the 4 KiB kernel from the committed PMC summary."""
    files = sorted(glob.glob(os.path.join(ROOT, "profiles", "*pmc*fixed4k*.json")))
    if not files:
        return None, None
    with open(files[-1]) as f:
        d = json.load(f)
    return d.get("hbm_bytes_per_launch"), os.path.relpath(files[-1], ROOT)


def cpu_model() -> str:
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def cpu_quota():
    """CPUs the cgroup's CFS quota allows (cpu.max / cpu.cfs_quota_us), or None."""
    for path, parse in (("/sys/fs/cgroup/cpu.max", lambda t: t.split()),
                        ("/sys/fs/cgroup/cpu/cpu.cfs_quota_us", lambda t: [t.strip(), open(
                            "/sys/fs/cgroup/cpu/cpu.cfs_period_us").read().strip()])):
        try:
            with open(path) as f:
                q, per = parse(f.read())[:2]
            if q not in ("max", "-1") and int(per) > 0:
                return max(1, int(q) // int(per))
        except (OSError, ValueError, IndexError):
            continue
    return None


def cpu_threads() -> int:
    """Threads of the all-cores CPU legs: the CPUs this process may run on
    (sched_getaffinity), bounded by the cgroup's CPU quota when it sets one (more
    threads than the quota only time-slice the same cores)."""
    n = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else (os.cpu_count() or 1)
    q = cpu_quota()
    return max(1, min(n, q) if q else n)


def cpu_context() -> dict:
    aff = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else None
    return {"cpu_model": cpu_model(), "affinity_cpus": aff, "cgroup_cpu_quota": cpu_quota(),
            "os_cpu_count": os.cpu_count()}


def best_host_rate(host: np.ndarray, seconds: float = 3.0) -> dict:
    """Context line (not the baseline): the product's host scalar path
    (jl_crc32c_value: x86 SSE4.2 crc32, host_crc.cpp) over 64 MiB pieces of the
    same bytes on all the threads used for the CPU baseline."""
    from concurrent.futures import ThreadPoolExecutor

    threads = cpu_threads()
    piece = 64 << 20
    pieces = [host[i:i + piece] for i in range(0, host.size - piece + 1, piece)] or [host]
    L = jl.lib()

    def one(a):
        return L.jl_crc32c_value(a.ctypes.data, a.size)

    done = 0
    t0 = time.perf_counter()
    with ThreadPoolExecutor(threads) as ex:
        while time.perf_counter() - t0 < seconds:
            list(ex.map(one, pieces))
            done += sum(a.size for a in pieces)
    el = time.perf_counter() - t0
    return {"value": round(done / el / GIB, 2), "unit": "GiB/s", "cores": threads,
            "kind": "host sse4.2 crc32 (jl_crc32c_value, the product's scalar host path)"}


def cpu_baseline(data, n_blocks, gpu_out, seconds):
    from oracle import oracle  # cpu_baseline leg only (test infrastructure)

    sample_blocks = min(n_blocks, 1 << 18)  # 1 GiB
    host = data[: sample_blocks * 4096].cpu().numpy()
    threads = cpu_threads()
    want = oracle.fixed(host, 4096, sample_blocks, threads=threads)
    parity = bool(np.array_equal(want, gpu_out[:sample_blocks]))
    done = 0
    t0 = time.perf_counter()
    while True:
        oracle.fixed(host, 4096, sample_blocks, threads=threads)
        done += 1
        el = time.perf_counter() - t0
        if el >= seconds:
            break
    t1 = time.perf_counter()
    oracle.fixed(host[: 1 << 26], 4096, 1 << 14, threads=1)
    one = (1 << 26) / (time.perf_counter() - t1) / GIB
    return {
        "value": round(done * sample_blocks * 4096 / el / GIB, 3),
        "unit": "GiB/s",
        "cores": threads,
        "kind": "port",
        **cpu_context(),
        "sample": f"{sample_blocks} x 4 KiB blocks (1 GiB) of the same data, {done} passes in {el:.1f} s; "
                  f"oracle/crc32c_oracle.c slicing-by-8 restatement of Crc32C.update; 1-thread rate {one:.2f} GiB/s",
        "one_thread_GiB_per_s": round(one, 3),
        "parity_with_gpu": parity,
        "best_host": best_host_rate(host),
    }


def secondary_c3(dev, stream, steps, warmup, cpu=True):
    """Config C3: 1M blocks, k~Zipf(1.1) on 1..64, len = 1024(k-1)+1+U[0,1023], packed, unaligned."""
    lens = wl.c3_lengths(1 << 20, SEED)
    n = lens.size
    offs = wl.packed_offsets(lens)
    total = int(lens.sum(dtype=np.uint64))
    arena = torch.empty(total + 16, dtype=torch.uint8, device=dev)
    jl.fill_random_dev(arena, SEED + 3)
    d_off = torch.from_numpy(offs.view(np.int64)).to(dev)
    d_len = torch.from_numpy(lens.view(np.int32)).to(dev)
    out = torch.empty(n, dtype=torch.int32, device=dev)
    for _ in range(50):  # ~0.1 s of untimed calls: clocks settle after the host-side set-up
        jl.crc32c_batch_dev(arena, d_off, d_len, out=out)
    wall, ms = timed(lambda: jl.crc32c_batch_dev(arena, d_off, d_len, out=out), steps, warmup, stream)
    alg = total + n * (4 + 12)
    res = {"config": "C3 1M mixed Zipf 1 B-64 KiB blocks, one arena, unaligned", "bytes": total,
           "GiB_per_s": round(total / (ms / steps / 1e3) / GIB, 1),
           "achieved_GBps": round(alg / (ms / steps / 1e3) / 1e9, 1), "ms_per_step": round(ms / steps, 3)}
    if cpu:  # the oracle on the blocks of the arena's first ~1 GiB, all threads and one
        from oracle import oracle  # cpu_baseline leg only (test infrastructure)

        k = int(np.searchsorted(offs + lens, 1 << 30))
        sub = arena[: int(offs[k - 1] + lens[k - 1])].cpu().numpy()
        want = oracle.batch(sub, offs[:k], lens[:k], threads=cpu_threads())
        parity = bool(np.array_equal(want, out[:k].cpu().numpy().view(np.uint32)))
        legs = {}
        for th in (cpu_threads(), 1):
            t0 = time.perf_counter()
            oracle.batch(sub, offs[:k], lens[:k], threads=th)
            legs[th] = sub.size / (time.perf_counter() - t0) / GIB
        res["cpu_baseline"] = {"GiB_per_s": round(legs[cpu_threads()], 3), "cores": cpu_threads(),
                               "one_thread_GiB_per_s": round(legs[1], 3), "kind": "port", **cpu_context(),
                               "sample": f"the first {k} blocks ({sub.size / GIB:.2f} GiB) of the same arena, "
                                         "oracle slicing-by-8 batch", "parity_with_gpu": parity}
    del arena
    return res


C5_LABELS = {
    "c1_1056": "C5 WAL verify, 2^17 x 32 KiB blocks, 1 056-B records, device-resident",
    "mixed_1b_100k": "C5 WAL verify, 2^17 x 32 KiB blocks, mixed 1 B-100 KiB records (fragmented), device-resident",
    "dbbench_131": "C5 WAL verify, 2^17 x 32 KiB blocks, DBBench-default 131-B records (16-B key + 100-B value, "
                   "DBBench.java:80; ~237 per block, every block dense), device-resident",
    "random_0_200": "C5 WAL verify, 2^17 x 32 KiB blocks, 0-200-B records of random lengths (a WAL of variable "
                    "small values; ~306 per block, every block dense, no runs), device-resident",
}


def secondary_c5(dev, stream, steps, warmup, which="c1_1056", cpu=True, host_copy=True):
    """Config C5: streaming WAL verification over 2^17 x 32 KiB log blocks (4 GiB).

    The log is produced on the device by the product's batched LogWriter
    (jl_log_layout + jl_log_emit_dev), then verified with jl_log_verify_dev
    (header walk + per-record masked-CRC check with
    LogReader.readPhysicalRecord semantics).  Three payload sets: C1-shaped
    records (1 056-B payload = 12-B batch header + 16-B key + 1 KiB value) and a
    mixed 1 B-100 KiB set whose records fragment into FIRST/MIDDLE/LAST across
    log blocks, and DBBench's default write (16-B key,
    100-B value: 131-B payloads, every 32 KiB block dense).  Timed
    device-resident, and copy-inclusive from pinned and pageable host memory
    through jl_log_verify; the CPU legs time the oracle's readPhysicalRecord
    walk on the first 1 GiB of the same log (1 thread and all threads)."""
    lens = wl.c5_lengths(which, seed=SEED)
    label = C5_LABELS[which]
    offs = wl.packed_offsets(lens)
    plan = jl.log_layout(offs, lens)
    src = torch.empty(int(lens.sum(dtype=np.uint64)), dtype=torch.uint8, device=dev)
    jl.fill_random_dev(src, SEED + 5)
    log = jl.log_emit_dev(src, plan)
    del src
    nb = plan["log_bytes"]
    crc_bytes = int(plan["len"].sum(dtype=np.uint64)) + plan["len"].size  # type byte || payload
    events = torch.empty((nb // 7 + 2) * 16, dtype=torch.uint8, device=dev)
    fn = lambda: jl.log_verify_dev(log, jl.LOG_CHECKSUM, events=events)  # noqa: E731
    ev, n_ev = fn()
    kinds = ev[: n_ev * 16].view(-1, 16)[:, 13].cpu().numpy()
    ok = int((kinds == jl.LOG_OK).sum())
    # the timed steps: the asynchronous form (back-to-back verifications, no host
    # round trip per log); the synchronous call's rate is reported beside it
    result = torch.empty(3, dtype=torch.int64, device=dev)
    fa = lambda: jl.log_verify_dev_async(log, jl.LOG_CHECKSUM, events=events, result=result)  # noqa: E731
    for _ in range(100):  # ~0.1 s of untimed calls: clocks settle after the host-side log generation
        fa()
    wall, ms = timed(fa, steps, warmup, stream)
    r = result.cpu().numpy()
    same_async = int(r[0]) == n_ev and int(r[2]) == 0 and torch.equal(
        events[: n_ev * 16].view(-1, 16)[:, 13].cpu(), torch.from_numpy(kinds))
    _, ms_sync = timed(fn, steps, warmup, stream)
    alg = crc_bytes + 7 * plan["len"].size
    res = {"config": label, "log_bytes": nb, "payload_records": int(lens.size),
           "physical_records": int(plan["len"].size), "records_ok": ok, "dense_blocks": int(r[1]),
           "path": "header walk + record chunks in exact (K, d) rounds through general v4 + fold/apply, dense blocks "
                   "(> 64 records) whole from LDS (JL_LOG_CHECKSUM), jl_log_verify_dev_async back to back",
           "achieved_frac_of_peak": round(alg / (ms / steps / 1e3) / 1e9 / PEAK_GBS, 4),
           "GiB_per_s": round(nb / (ms / steps / 1e3) / GIB, 1),
           "achieved_GBps": round(alg / (ms / steps / 1e3) / 1e9, 1),
           "ms_per_step": round(ms / steps, 3), "wall_ms_per_step": round(wall / steps * 1e3, 3),
           "async_events_equal_sync": bool(same_async),
           "sync_call": {"GiB_per_s": round(nb / (ms_sync / steps / 1e3) / GIB, 1),
                         "ms_per_step": round(ms_sync / steps, 3)}}
    fn2 = lambda: jl.log_verify_dev(log, jl.LOG_CHECKSUM_FUSED, events=events)  # noqa: E731
    ev2, n2 = fn2()
    same = n2 == n_ev and torch.equal(ev2[: n2 * 16], ev[: n_ev * 16])
    _, ms2 = timed(fn2, steps, warmup, stream)
    res["fused"] = {"GiB_per_s": round(nb / (ms2 / steps / 1e3) / GIB, 1), "ms_per_step": round(ms2 / steps, 3),
                    "events_equal": bool(same)}
    if not host_copy:
        return res
    host = torch.empty(nb, dtype=torch.uint8, pin_memory=True)
    host.copy_(log)
    del log, events
    torch.cuda.empty_cache()
    hn = host.numpy()
    # the event array is allocated and touched once and reused (a caller's buffer):
    # a fresh multi-GB array per call times the kernel's page faults on its first
    # writes, not the engine (r4: pinned 38 < pageable 47 GiB/s on the DBBench set)
    out = np.zeros(int(plan["len"].size) + 64, dtype=jl.LOG_EVENT_DTYPE)
    pageable = hn.copy()  # the same log in pageable memory (an mmap'd file's case): pinned for each call
    jl.log_verify(hn, out=out)
    jl.log_verify(pageable, out=out)
    # pinned (64 MiB chunks double-buffered) and pageable sources timed alternately,
    # median of 3 each: r5k timed the two legs one after the other and saw pinned
    # 2-6 % below pageable on two sets; alternated on one box they are equal (r5q:
    # 50.0 / 50.0 GiB/s on the random set, 50.5 / 50.5 mixed, H2D ceiling 52.7)
    ts = {"pinned": [], "pageable": []}
    for r in range(3):
        for name in (("pinned", "pageable") if r % 2 == 0 else ("pageable", "pinned")):
            t0 = time.perf_counter()
            jl.log_verify(hn if name == "pinned" else pageable, out=out)
            ts[name].append(time.perf_counter() - t0)
    res["copy_inclusive_GiB_per_s"] = round(nb / float(np.median(ts["pinned"])) / GIB, 2)
    hev = jl.log_verify(hn, out=out)
    res["copy_inclusive_records_ok"] = int((hev["kind"] == jl.LOG_OK).sum())
    del host, hev
    res["copy_inclusive_pageable_GiB_per_s"] = round(nb / float(np.median(ts["pageable"])) / GIB, 2)
    hn = pageable
    if cpu:  # the oracle's readPhysicalRecord walk + crc on the log's first 1 GiB: one thread, and
        # all threads over block-aligned pieces (readPhysicalRecord decides within a 32 KiB block)
        from concurrent.futures import ThreadPoolExecutor

        from oracle import oracle  # cpu_baseline leg only (test infrastructure)

        sample = hn[: 1 << 30]
        want = oracle.log_events(sample)
        t0 = time.perf_counter()
        oracle.log_events(sample)
        one = sample.size / (time.perf_counter() - t0) / GIB
        th = cpu_threads()
        step = -(-sample.size // th // 32768) * 32768
        pieces = [sample[i:i + step] for i in range(0, sample.size, step)]
        with ThreadPoolExecutor(th) as ex:
            t0 = time.perf_counter()
            parts = list(ex.map(oracle.log_events, pieces))
            allc = sample.size / (time.perf_counter() - t0) / GIB
        ok_all = sum(int((p["kind"] == jl.LOG_OK).sum()) for p in parts)
        res["cpu_baseline"] = {"GiB_per_s": round(allc, 3), "cores": th, "one_thread_GiB_per_s": round(one, 3),
                               "kind": "port", **cpu_context(),
                               "sample": "first 1 GiB of the same log, oracle readPhysicalRecord walk + CRC "
                                         f"({th} threads over 32 KiB-block-aligned pieces, and 1 thread)",
                               "records_ok": int((want["kind"] == jl.LOG_OK).sum()),
                               "records_ok_threaded": ok_all}
    return res


def dispatch_latency(oracle_free=True):
    """Per-call latency at the reference's call granularity (host memory, as an
    mmap'd file): one table of ~4.2 KB blocks (Options.java:206,208: 4 KiB blocks,
    2 MiB tables) and one WAL of 1 056-B records (Options.java:203: 4 MiB write
    buffer), at several sizes, through the device path (threshold 0), the host
    SSE4.2 path (threshold above the size) and the engine's default, the auto
    dispatch (JL_HOST_THRESHOLD_AUTO: both paths measured per size class, then
    the faster one; timed after its six probe calls per size class).  Medians of repeated calls; the crossover is the smallest
    size from which the device is faster.  Per size also the device call's
    staging-copy rate (pageable -> pinned, JL_INFO_LAST_STAGE_NS) and the share of
    the auto calls that ran on the device; the copy pool's threads at the end."""
    rng = np.random.default_rng(SEED + 17)
    prev = (jl.get_option(jl.OPT_HOST_THRESHOLD), jl.get_option(jl.OPT_LOG_HOST_THRESHOLD))

    def med(fn, reps, path_log=None, warm=1):
        for _ in range(warm):
            fn()
        ts = []
        for _ in range(reps):
            t0 = time.perf_counter()
            fn()
            ts.append(time.perf_counter() - t0)
            if path_log is not None:
                path_log.append(jl.get_option(jl.INFO_LAST_PATH))
        return float(np.median(ts)) * 1e6

    def stage_rate(fn, nbytes):
        fn()
        ns = jl.get_option(jl.INFO_LAST_STAGE_NS)
        return round(nbytes / ns, 2) if ns > 0 else None  # GB/s

    res = {"table": [], "log": []}
    for mib in (0.25, 1, 2, 4, 8, 16, 64):
        nbytes = int(mib * (1 << 20))
        sizes = rng.integers(3900, 4400, max(1, nbytes // 4150)).astype(np.uint32)
        offs = wl.packed_offsets(sizes + 5)
        table = rng.integers(0, 256, int(offs[-1]) + int(sizes[-1]) + 5, dtype=np.uint8)
        lens = np.full(max(1, nbytes // (wl.C1_PAYLOAD + 7)), wl.C1_PAYLOAD, np.uint32)
        plan = jl.log_layout(wl.packed_offsets(lens), lens)
        src = torch.empty(int(lens.sum(dtype=np.uint64)), dtype=torch.uint8, device="cuda")
        jl.fill_random_dev(src, SEED + 19)
        log = jl.log_emit_dev(src, plan).cpu().numpy().copy()
        reps = 30 if mib <= 4 else 12
        row_t, row_l = {"MiB": mib}, {"MiB": mib}
        run_t = lambda: jl.table_verify(table, offs, sizes)  # noqa: E731
        run_l = lambda: jl.log_verify(log)  # noqa: E731
        for path, thr in (("device_us", 0), ("host_us", 1 << 40), ("auto_us", jl.HOST_THRESHOLD_AUTO)):
            jl.set_option(jl.OPT_HOST_THRESHOLD, thr)
            jl.set_option(jl.OPT_LOG_HOST_THRESHOLD, thr)
            pt, pl = [], []
            # auto: the size class's six probe calls (three per path) untimed, the
            # steady state timed (the probes cost each size class once per process)
            warm = 7 if path == "auto_us" else 1
            row_t[path] = round(med(run_t, reps, pt, warm), 1)
            row_l[path] = round(med(run_l, reps, pl, warm), 1)
            if path == "device_us":
                row_t["device_stage_GBps"] = stage_rate(run_t, table.size)
                row_l["device_stage_GBps"] = stage_rate(run_l, log.size)
            if path == "auto_us":
                row_t["auto_device_share"] = round(pt.count(1) / len(pt), 2)
                row_l["auto_device_share"] = round(pl.count(1) / len(pl), 2)
        res["table"].append(row_t)
        res["log"].append(row_l)
    jl.set_option(jl.OPT_HOST_THRESHOLD, prev[0])
    jl.set_option(jl.OPT_LOG_HOST_THRESHOLD, prev[1])
    for k in ("table", "log"):
        faster = [r["MiB"] for r in res[k] if r["device_us"] < r["host_us"]]
        res[f"{k}_crossover_MiB"] = min(faster) if faster else None
        # the default (auto) against the better of the two fixed paths, worst size
        res[f"{k}_auto_vs_best"] = round(max(r["auto_us"] / min(r["device_us"], r["host_us"]) for r in res[k]), 3)
    res["config"] = ("per-call latency, host-memory input (pageable), device path vs the host SSE4.2 path vs the "
                     "default auto dispatch: one table of ~4.2 KB blocks and one WAL of 1 056-B records per call, "
                     "1 calling thread")
    res["host_threshold_default_bytes"] = {"tables_batches": prev[0], "logs": prev[1]}
    res["stage_pool"] = {"workers": jl.get_option(jl.INFO_STAGE_WORKERS),
                         "spawn_failures": jl.get_option(jl.INFO_STAGE_SPAWN_FAILURES),
                         "threads_option": jl.get_option(jl.OPT_STAGE_THREADS)}
    return res


def copy_inclusive_c2(data):
    """C2 bytes starting in host memory: jl_crc32c_fixed (H2D overlapped with the
    kernel on two streams), pinned and pageable sources."""
    nbytes = data.numel()
    pinned = torch.empty(nbytes, dtype=torch.uint8, pin_memory=True)
    pinned.copy_(data)
    ref = jl.crc32c_fixed(pinned, 4096)
    t0 = time.perf_counter()
    jl.crc32c_fixed(pinned, 4096)
    pin_s = time.perf_counter() - t0
    # the link's own ceiling on this box: one plain pinned H2D copy of the same bytes
    dev_buf = torch.empty(nbytes, dtype=torch.uint8, device=data.device)
    dev_buf[: 64 << 20].copy_(pinned[: 64 << 20])  # warm the DMA path
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    dev_buf.copy_(pinned, non_blocking=True)
    torch.cuda.synchronize()
    h2d_s = time.perf_counter() - t0
    del dev_buf
    pageable = pinned.numpy().copy()
    del pinned
    res = {"config": "C2 from host memory (H2D + kernel + D2H, 64 MiB chunks, double-buffered)",
           "pinned_GiB_per_s": round(nbytes / pin_s / GIB, 2),
           "h2d_copy_ceiling_GiB_per_s": round(nbytes / h2d_s / GIB, 2)}
    same = True
    prev = jl.get_option(jl.OPT_HOST_REGISTER)
    for reg, key in ((1, "pageable_registered_GiB_per_s"), (0, "pageable_staged_GiB_per_s")):
        jl.set_option(jl.OPT_HOST_REGISTER, reg)  # pin the input for the call / stage it through pinned buffers
        jl.crc32c_fixed(pageable[: 64 << 20], 4096)
        t0 = time.perf_counter()
        got = jl.crc32c_fixed(pageable, 4096)
        res[key] = round(nbytes / (time.perf_counter() - t0) / GIB, 2)
        if not reg:  # the host side of the staged leg: pageable -> pinned copies (the copy pool)
            ns = jl.get_option(jl.INFO_LAST_STAGE_NS)
            res["pageable_staged_copy_GBps"] = round(nbytes / ns, 2) if ns > 0 else None
        same = same and bool(np.array_equal(ref, got))
    jl.set_option(jl.OPT_HOST_REGISTER, prev)
    res["parity_with_device_resident"] = same
    return res


def visible_gpus() -> int:
    """GPUs this process would see, counted WITHOUT initialising HIP (the parent
    of the ranks must not touch the GPU): the *_VISIBLE_DEVICES lists when set,
    else the GPU nodes of the KFD topology (nodes with SIMDs)."""
    for var in ("HIP_VISIBLE_DEVICES", "ROCR_VISIBLE_DEVICES", "CUDA_VISIBLE_DEVICES"):
        v = os.environ.get(var)
        if v is not None:
            return len([x for x in v.split(",") if x.strip() != ""])
    n = 0
    for props in glob.glob("/sys/class/kfd/kfd/topology/nodes/*/properties"):
        try:
            with open(props) as f:
                for line in f:
                    k, _, val = line.partition(" ")
                    if k == "simd_count" and int(val) > 0:
                        n += 1
        except (OSError, ValueError):
            continue
    return n


def spawn_ranks(gpus: int, same_device: bool) -> None:
    """`bench.py --gpus N` (N > 1) outside torch.distributed.run: launch N ranks,
    one process per GPU, through torch.distributed.run as a CHILD process (this
    process never initialises HIP: the devices are counted from the environment /
    KFD topology) and exit with its status.  Refuses to run on fewer than N
    visible GPUs unless --same-device (every rank on GPU 0: the rank path's
    rehearsal on a one-GPU box)."""
    import socket
    import subprocess

    have = visible_gpus()
    if have < (1 if same_device else gpus):
        print(f"bench.py: --gpus {gpus} but only {have} GPU(s) visible", file=sys.stderr, flush=True)
        sys.exit(2)
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={gpus}",
           "--master-addr", "127.0.0.1", f"--master-port={port}", os.path.abspath(__file__)] + sys.argv[1:]
    sys.exit(subprocess.call(cmd, env=env))


def gathered_parity(out, world, args, dev) -> bool:
    """Outside the timed region: every rank's results gathered in rank order
    (padded all-gather, unequal strong shards included) equal ONE launch over
    the whole set on this GPU (regenerated from splitmix64 word 0)."""
    allres = shd.gather_results(out, world)
    if int(os.environ.get("RANK", "0")) != 0:
        return True
    total = args.strong_total if args.strong_total else world * args.blocks
    whole = torch.empty(total * 4096, dtype=torch.uint8, device=dev)
    jl.fill_random_dev(whole, SEED)
    ref = jl.crc32c_fixed_dev(whole, 4096, total)
    ok = bool(torch.equal(allres.to(ref.device), ref))
    del whole, ref
    torch.cuda.empty_cache()
    return ok


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=20)
    ap.add_argument("--settle-ms", type=float, default=200.0,
                    help="untimed launches for this long before the warmup steps (clocks ramp up from idle)")
    ap.add_argument("--blocks", type=int, default=1 << 20, help="4 KiB blocks per GPU (C2: 1M)")
    ap.add_argument("--strong-total", type=int, default=0,
                    help="strong scaling: split this many 4 KiB blocks over the ranks (C4: 8388608) instead of "
                         "--blocks per rank")
    ap.add_argument("--cpu-seconds", type=float, default=10.0)
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--no-secondary", action="store_true")
    ap.add_argument("--same-device", action="store_true",
                    help="rehearsal of the N-rank path on one GPU: every rank on GPU 0, gloo collectives "
                         "(the timing then measures N ranks sharing one GPU)")
    args = ap.parse_args()

    if "WORLD_SIZE" not in os.environ and args.gpus > 1:
        spawn_ranks(args.gpus, args.same_device)
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = 0 if args.same_device else int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus and rank == 0:
        print(f"bench.py: --gpus {args.gpus} but WORLD_SIZE={world}; reporting the process group's size",
              file=sys.stderr, flush=True)
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    if world > 1:
        import torch.distributed as dist

        if args.same_device:  # RCCL refuses two ranks on one GPU: gloo carries the same collectives
            dist.init_process_group("gloo")
        else:
            dist.init_process_group("nccl", device_id=dev)
        world = dist.get_world_size()
    jl.init(local)
    stream = torch.cuda.current_stream()

    if args.strong_total:  # C4 strong: a fixed set split into contiguous ranges
        sh = shd.strong_shard(rank, world, args.strong_total)
    else:  # weak: rank r holds blocks [r*n, (r+1)*n) of the C4 set
        sh = shd.weak_shard(rank, world, args.blocks)
    n = sh.n_blocks
    data = torch.empty(n * 4096, dtype=torch.uint8, device=dev)
    jl.fill_random_dev(data, SEED, first_word=sh.first_word)  # generated in place
    out = torch.empty(n, dtype=torch.int32, device=dev)
    step = lambda: jl.crc32c_fixed_dev(data, 4096, n, out=out)  # noqa: E731

    settle = 0  # clock settling: the GPU ramps its clocks up from idle over ~100 ms of load
    t_settle = time.perf_counter()
    while (time.perf_counter() - t_settle) * 1e3 < args.settle_ms:
        for _ in range(10):
            step()
        settle += 10
        torch.cuda.synchronize()
    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(args.steps + 1)]
    t0 = time.perf_counter()
    ev[0].record(stream)
    for i in range(args.steps):
        step()
        ev[i + 1].record(stream)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    wall = time.perf_counter() - t0
    per_launch = [ev[i].elapsed_time(ev[i + 1]) for i in range(args.steps)]
    kern_ms = sum(per_launch) / args.steps
    wall = shd.job_wall_time(wall, dev)  # max over ranks (no-op at N=1)
    rank_kern = shd.per_rank(kern_ms, dev)  # every rank's kernel ms (HIP events), beside the MAX
    if args.strong_total:
        value = args.strong_total * 4096 * args.steps / wall / GIB
    else:
        value = shd.aggregate_rate(n * 4096, world, wall, args.steps)
    gather_ms = parity = None
    if world > 1:  # result all-gather (unequal strong shards padded): reported beside, not part of the checksum path
        dist.barrier()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        shd.gather_results(out, world)
        torch.cuda.synchronize()
        gather_ms = shd.job_wall_time(time.perf_counter() - t0, dev) * 1e3
        parity = gathered_parity(out, world, args, dev)
    alg_launch = n * (4096 + 4)
    achieved = alg_launch / (kern_ms / 1e3) / 1e9
    result = None
    if rank == 0:
        gpu_out = out.cpu().numpy().view(np.uint32)
        traffic, traffic_src = pmc_traffic()
        ceiling = read_stream_ceiling(data, stream)
        result = {
            "metric": "GiB/s CRC32C over 4 KiB blocks (device-resident); % of HBM read roofline",
            "value": round(value, 1),
            "unit": "GiB/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "settle_launches": settle,
            "ms_per_step": round(wall / args.steps * 1e3, 4),
            "higher_is_better": True,
            "scaling": "strong" if args.strong_total else "weak",
            "vs_baseline": None,
            "dtype": "u8",
            "data": "synthetic (device splitmix64, seed 0x4A4C4442; rank r = blocks "
                    f"[{sh.first_block}, {sh.first_block + n}) of the C4 set)",
            "config": {"workload": (f"C4 strong: {args.strong_total} x 4 KiB blocks split over {world} GPUs"
                                    if args.strong_total else "C2: 1M x 4 KiB random blocks per GPU")
                       + ", masked CRC32C, device-resident",
                       "blocks_per_gpu": n, "block_bytes": 4096,
                       "parallelism": f"shard{world}" + (" (same-device rehearsal, gloo)" if args.same_device else "")},
            "result_allgather_ms": None if gather_ms is None else round(gather_ms, 3),
            "rank_kernel_ms": [round(x, 4) for x in rank_kern],
            "rank_kernel_ms_spread": round(max(rank_kern) - min(rank_kern), 4),
            "parity_gathered_vs_single_launch": parity,
            "roofline": {
                "bound": "hbm",
                "kernel": "crc_fixed4k_v4_kernel<8 lanes/block, nt, 8-slot ring, 1024 threads>",
                "achieved": round(achieved, 1),
                "peak": PEAK_GBS,
                "unit": "GB/s",
                "frac": round(achieved / PEAK_GBS, 4),
                # PMC was collected on 1M-block launches; scale to this launch's blocks
                "traffic": None if traffic is None else round(traffic * n / (1 << 20)),
                "traffic_source": traffic_src if n == 1 << 20 else f"{traffic_src} x {n}/1048576 blocks",
                "kernel_ms": round(kern_ms, 4),
                "kernel_ms_min": round(min(per_launch), 4),
                "kernel_ms_median": round(float(np.median(per_launch)), 4),
                "alg_bytes_per_launch": alg_launch,
                "read_stream_ceiling_GBps": round(ceiling, 1),
                "frac_of_read_ceiling": round(achieved / ceiling, 4),
            },
        }
        if world == 1 and not args.no_cpu:
            result["cpu_baseline"] = cpu_baseline(data, n, gpu_out, args.cpu_seconds)
    if world == 1 and not args.no_secondary and not args.strong_total:  # secondaries describe the 1M-block C2 box
        sec = [copy_inclusive_c2(data), dispatch_latency()]
        sec[0]["parity_with_device_resident"] &= bool(np.array_equal(gpu_out, out.cpu().numpy().view(np.uint32)))
        del data
        torch.cuda.empty_cache()
        sec.append(secondary_c3(dev, stream, 5, 2, cpu=not args.no_cpu))
        torch.cuda.empty_cache()
        for which in wl.C5_SETS:
            sec.append(secondary_c5(dev, stream, 5, 2, which=which, cpu=not args.no_cpu))
            torch.cuda.empty_cache()
        result["secondary"] = sec
    if rank == 0:
        print(json.dumps(result), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
