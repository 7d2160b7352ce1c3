#!/usr/bin/env python3
"""Summarises rocprofv3 --pmc CSV passes: per kernel, the median per-dispatch
value of every counter, plus the kernel's median duration."""
import csv
import glob
import json
import statistics
import sys
from collections import defaultdict

vals = defaultdict(lambda: defaultdict(list))
for d in sys.argv[1:]:
    for f in glob.glob(f"{d}/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            k = r["Kernel_Name"].split("(")[0].replace("void ", "")
            vals[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
            if "End_Timestamp" in r and "Start_Timestamp" in r:
                vals[k]["_dur_ns"].append(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]))
out = {k: {c: statistics.median(v) for c, v in cs.items()} for k, cs in vals.items()}
print(json.dumps(out, indent=1))
