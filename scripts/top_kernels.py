#!/usr/bin/env python3
"""Print the top kernels of a rocprofv3 --stats CSV (usage: top_kernels.py stats.csv [n])."""
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
n = int(sys.argv[2]) if len(sys.argv) > 2 else 25
tot = sum(float(r["TotalDurationNs"]) for r in rows)
print(f"total kernel time {tot / 1e6:.1f} ms over {sum(int(r['Calls']) for r in rows)} launches")
for r in rows[:n]:
    print(f'{r["Name"][:100]:100s} {r["Calls"]:>7s} {float(r["TotalDurationNs"]) / 1e6:9.1f} ms '
          f'{float(r["Percentage"]):6.2f}%')
