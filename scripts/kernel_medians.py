"""Median kernel durations (us) from a rocprofv3 --kernel-trace csv, by kernel name (short form).
usage: python scripts/kernel_medians.py run_kernel_trace.csv"""
import csv
import statistics
import sys
from collections import defaultdict

d = defaultdict(list)
with open(sys.argv[1]) as f:
    for r in csv.DictReader(f):
        d[r["Kernel_Name"]].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
out = []
for name, ts in d.items():
    if len(ts) < 20:
        continue
    short = name.replace("void ", "").replace("(anonymous namespace)::", "").split("(")[0]
    out.append(f"{short}={statistics.median(ts):.2f}")
print(" ".join(sorted(out)))
