#!/usr/bin/env python3
"""Per-kernel split of the chunked log verification from a rocprofv3 kernel trace.

Usage: c5_split.py TRACE.csv [OUT.json]

Reads a `--kernel-trace` CSV of `tools/sec_time.py ... c5` (or bench.py's C5
legs), cuts it into verifications (each starts at `lc_walk_kernel`), names the
set each verification belongs to from its own kernel times (dense blocks ->
the DBBench 131-B set, a long walk -> the 1 056-B set, else the mixed set) and
prints the median microseconds per kernel and set.  Analysis tool only.
"""
import csv
import json
import statistics
import sys


def short(name):
    if "rocprim" in name or "lc_scan_kernel" in name:
        return "scans"
    if "crc_gv4_kernel<5" in name:
        return "crc_gv4_kernel<LOG_CHUNK>"
    for k in ("lc_walk", "lc_dwalk", "lc_dense", "lc_dense_inplace", "lc_build", "lc_setup", "lc_combine", "lc_apply"):
        if k + "_kernel" in name:
            return k
    return None


def main():
    rows = list(csv.DictReader(open(sys.argv[1])))
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    runs, cur = [], None
    for r in rows:
        k = short(r["Kernel_Name"])
        if k is None:
            continue
        if k == "lc_walk":
            cur = {}
            runs.append(cur)
        if cur is None:
            continue
        us = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
        cur[k] = cur.get(k, 0.0) + us
    sets = {}
    for v in runs:
        if "crc_gv4_kernel<LOG_CHUNK>" not in v:
            continue
        if v.get("lc_dwalk", 0) > 100:
            name = "random_0_200"
        elif v.get("lc_dense", 0) > 200:
            name = "dbbench_131"
        elif v.get("lc_walk", 0) > 80:
            name = "c1_1056"
        elif v["crc_gv4_kernel<LOG_CHUNK>"] > 300:
            name = "mixed_1b_100k"
        else:
            name = "small (settling / dispatch calls)"
        sets.setdefault(name, []).append(v)
    out = {"source": sys.argv[1], "unit": "us, median per verification", "sets": {}}
    for name, vs in sets.items():
        keys = sorted({k for v in vs for k in v})
        d = {"verifications": len(vs)}
        for k in keys:
            d[k] = round(statistics.median(v.get(k, 0.0) for v in vs), 1)
        d["sum_of_medians"] = round(sum(d[k] for k in keys), 1)
        out["sets"][name] = d
    text = json.dumps(out, indent=1)
    print(text)
    if len(sys.argv) > 2:
        open(sys.argv[2], "w").write(text + "\n")


if __name__ == "__main__":
    main()
