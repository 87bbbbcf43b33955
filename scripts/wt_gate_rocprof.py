"""Attribute the k_group_fast records of a rocprofv3 --kernel-trace csv to the libraries and legs
scripts/wt_gate_ab.py wrote to its SEQ file (launch order), and print rocprof medians:
per_weight = median launch duration; grouped = median launch duration / 100 weights; plan =
median duration of each of the 5 launches and the median per-step sum.
usage: python scripts/wt_gate_rocprof.py run_kernel_trace.csv x.seq"""
import csv
import statistics
import sys
from collections import defaultdict


def main(trace, seq_path):
    recs = []
    with open(trace) as f:
        for r in csv.DictReader(f):
            if "k_group_fast" in r["Kernel_Name"]:
                recs.append((int(r["Start_Timestamp"]), (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3))
    recs.sort()
    durs = [d for _, d in recs]
    blocks = [line.split() for line in open(seq_path) if line.strip()]
    need = sum(int(n) for *_, n in blocks)
    if need != len(durs):
        sys.exit(f"sequence wants {need} k_group_fast records, the trace holds {len(durs)}")
    pos = 0
    by = defaultdict(list)
    for lib, leg, n in blocks:
        n = int(n)
        if leg in ("per_weight", "pw_same", "pw_grp", "grouped", "plan"):
            by[(lib, leg)].append(durs[pos:pos + n])
        pos += n
    libs = sorted({lib for lib, _ in by}, key=[b[0] for b in blocks].index)
    for lib, leg in [(x, y) for y in ("per_weight", "pw_same", "pw_grp") for x in libs]:
        pw = [d for blk in by[(lib, leg)] for d in blk]
        if not pw:
            continue
        print(f"{leg:10s} {lib:18s} rocprof median {statistics.median(pw):8.2f} us/launch  n={len(pw)}  "
              f"frac {113426432 / (statistics.median(pw) * 1e-6) / 8e12:.3f}")
    for lib in libs:
        gr = [d / 100 for blk in by[(lib, "grouped")] for d in blk]
        if not gr:
            continue
        print(f"grouped    {lib:18s} rocprof median {statistics.median(gr):8.2f} us/weight  n={len(gr)}")
    for lib in libs:
        steps = [blk[i:i + 5] for blk in by[(lib, "plan")] for i in range(0, len(blk), 5)]
        if not steps:
            continue
        per = [statistics.median(s[j] for s in steps) for j in range(5)]
        print(f"plan       {lib:18s} rocprof median step {statistics.median(sum(s) for s in steps):8.2f} us  "
              f"launches " + " ".join(f"{v:.2f}" for v in per) + f"  steps={len(steps)}")


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2])
