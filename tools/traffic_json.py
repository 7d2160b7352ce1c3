#!/usr/bin/env python3
"""Turns a gpu_pmc.sh summary (FETCH_SIZE / WRITE_SIZE / TCC_EA0_RDREQ_sum passes)
into the per-launch HBM-traffic record bench.py reports as roofline.traffic.

  python tools/traffic_json.py gpurun_out/<tag>_pmc.json <kernel-substring> <round> > profiles/<round>_pmc_fixed4k_<x>.json

Corrections (MI355X_MICROARCH.md, HBM/rocprofv3 section): FETCH_SIZE is in KiB
and reports half of a wide coalesced streaming read on gfx950 -> read bytes =
FETCH_SIZE*1024*2, cross-checked with TCC_EA0_RDREQ_sum*128; WRITE_SIZE in KiB."""
import json
import sys

pmc = json.load(open(sys.argv[1]))
sub, rnd = sys.argv[2], sys.argv[3]
k = [n for n in pmc if sub in n]
assert len(k) == 1, (sub, list(pmc))
d = pmc[k[0]]
rd = d["FETCH_SIZE"] * 1024 * 2
wr = d["WRITE_SIZE"] * 1024
n = 1 << 20
print(json.dumps({
    "kernel": k[0], "workload": "C2 1M x 4 KiB", "round": rnd,
    "command": "tools/gpu_pmc.sh (rocprofv3 --pmc, one counter per pass) over tools/sustain.py",
    "FETCH_SIZE_KB_median": d["FETCH_SIZE"], "WRITE_SIZE_KB_median": d["WRITE_SIZE"],
    "TCC_EA0_RDREQ_sum_median": d.get("TCC_EA0_RDREQ_sum"),
    "correction": "gfx950: read bytes = FETCH_SIZE*1024*2 (MI355X_MICROARCH.md HBM section); cross-check TCC_EA0_RDREQ_sum*128 B",
    "hbm_read_bytes_per_launch": rd, "hbm_write_bytes_per_launch": wr, "hbm_bytes_per_launch": rd + wr,
    "rdreq_x128_bytes": d["TCC_EA0_RDREQ_sum"] * 128 if d.get("TCC_EA0_RDREQ_sum") else None,
    "algorithmic_bytes_per_launch": n * (4096 + 4),
    "pmc_pass_kernel_ns_median": d.get("_dur_ns"),
}, indent=1))
