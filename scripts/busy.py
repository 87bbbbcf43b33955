#!/usr/bin/env python3
"""GPU busy fraction of a rocprofv3 --kernel-trace run: union of kernel intervals over the span
from the first to the last kernel, and the largest idle gaps with the kernels on either side.

  python scripts/busy.py <run_kernel_trace.csv> [n_gaps] [after_substring]

``after_substring``: start the span at the first kernel whose name contains it (skip model
construction / warm-up)."""
import csv
import sys


def main(path, n_gaps=15, after=None):
    rows = list(csv.DictReader(open(path)))
    iv = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]) for r in rows)
    if after:
        i0 = next(i for i, x in enumerate(iv) if after in x[2])
        iv = iv[i0:]
    span = iv[-1][1] - iv[0][0]
    busy, end, gaps = 0, iv[0][0], []
    prev = None
    for s, e, n in iv:
        if s > end:
            gaps.append((s - end, prev, n))
        busy += max(0, e - max(s, end))
        if e > end:
            end, prev = e, n
    tot_gap = sum(g[0] for g in gaps)
    print(f"kernels {len(iv)}  span {span / 1e6:.1f} ms  busy {busy / 1e6:.1f} ms ({busy / span:.3f})  "
          f"idle {tot_gap / 1e6:.1f} ms in {len(gaps)} gaps")
    buckets = [(1e3, "<1us"), (1e4, "1-10us"), (1e5, "10-100us"), (1e6, "0.1-1ms"), (1e12, ">1ms")]
    lo = 0
    for hi, name in buckets:
        sel = [g[0] for g in gaps if lo <= g[0] < hi]
        print(f"  gaps {name:>9s}: {len(sel):6d}  {sum(sel) / 1e6:8.1f} ms")
        lo = hi
    for g, a, b in sorted(gaps, reverse=True)[:n_gaps]:
        print(f"  {g / 1e3:9.1f} us  after {a[:60]!r}  before {b[:60]!r}")


if __name__ == "__main__":
    main(sys.argv[1], int(sys.argv[2]) if len(sys.argv) > 2 else 15, sys.argv[3] if len(sys.argv) > 3 else None)
