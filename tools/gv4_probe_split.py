#!/usr/bin/env python3
"""Kernel-trace split of tools/gv4_probe.py (run under rocprofv3 --kernel-trace):
per leg, the median duration of each kernel of one call, so the 'sorted' leg's
gv4 kernel is compared with the 'implicit' leg's on its own (the leg's wall time
also holds the rounds pipeline: memset, hist, scan, place).
Usage: gv4_probe_split.py <run_kernel_trace.csv> [calls per leg, default 40]"""
import csv
import json
import sys
from collections import defaultdict

import numpy as np

rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: int(r["Start_Timestamp"]))
per = int(sys.argv[2]) if len(sys.argv) > 2 else 40


def short(n):
    for k in ("crc_fixed4k_v4", "crc_gv4_kernel", "gv4_hist", "gv4_scan", "gv4_place", "read_stream", "fill_random",
              "fillBuffer"):
        if k in n:
            return k
    return n.split("(")[0][-40:]


# legs in gv4_probe.py order; a leg starts at its first characteristic kernel
legs, cur = defaultdict(lambda: defaultdict(list)), None
seen_gv4 = 0
for r in rows:
    k = short(r["Kernel_Name"])
    us = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
    if k == "crc_fixed4k_v4":
        cur = "fixed4k"
    elif k == "crc_gv4_kernel":
        seen_gv4 += 1
        cur = "implicit" if seen_gv4 <= per else "sorted"
    elif k == "read_stream":
        cur = "ceiling"
    elif k in ("gv4_hist", "gv4_scan", "gv4_place") and cur == "implicit" and seen_gv4 >= per:
        cur = "sorted"
    if cur:
        legs[cur][k].append(us)
out = {leg: {k: round(float(np.median(v)), 1) for k, v in ks.items() if k not in ("fill_random",)}
       for leg, ks in legs.items()}
for leg, ks in out.items():
    ks["sum_of_medians_us"] = round(sum(v for k, v in ks.items()), 1)
print(json.dumps({"source": sys.argv[1], "unit": "us, median per call", "legs": out}, indent=1))
