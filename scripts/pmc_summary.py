#!/usr/bin/env python3
"""Summarise a gpurun_out/ rocprofv3 session into profiles/ (committed evidence).

  python scripts/pmc_summary.py TAG [KERNEL] [WEIGHTS_PER_PMC_LAUNCH]
(defaults: the grouped bench kernel, 30 weights per launch = pmc.sh's --steps 30) reads gpurun_out/prof_TAG/run_kernel_stats.csv and gpurun_out/pmc_TAG/*/run_counter_collection.csv,
writes profiles/TAG_bench_kernel_stats.csv, profiles/TAG_pmc_<counters>.csv (bench kernel rows
only) and profiles/pmc_traffic.json (HBM bytes per launch, MI355X_MICROARCH.md corrections:
FETCH_SIZE x2 on gfx950, WRITE_SIZE as-is, KB = 1024 B)."""
import csv
import json
import os
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
KERNEL = "k_group_fast<4, 0, false, true, true, true>"  # bench.py's grouped launch (K*90 MB > 256 MiB)
ALG = 113426432  # algorithmic bytes per [11008, 4096] int4 g128 weight
STATS_WEIGHTS = 100  # scripts/gpu_check.sh's kernel-trace run: bench.py --profile-only --steps 100


def main(tag, kernel=KERNEL, per_launch=30):
    prof = os.path.join(ROOT, "gpurun_out", f"prof_{tag}", "run_kernel_stats.csv")
    out = os.path.join(ROOT, "profiles")
    rows = list(csv.DictReader(open(prof)))
    with open(os.path.join(out, f"{tag}_bench_kernel_stats.csv"), "w", newline="") as f:
        w = csv.DictWriter(f, fieldnames=list(rows[0].keys()))
        w.writeheader()
        for r in rows:
            if "at::native" in r["Name"]:
                r = dict(r, Name=r["Name"].split("(")[0][:120] + "(...)")  # torch input generators
            w.writerow(r)
    k = next(r for r in rows if kernel in r["Name"])
    pmc_dir = os.path.join(ROOT, "gpurun_out", f"pmc_{tag}")
    med = {}
    for sub in sorted(os.listdir(pmc_dir)):
        p = os.path.join(pmc_dir, sub, "run_counter_collection.csv")
        if not os.path.exists(p):
            continue
        mine = [r for r in csv.DictReader(open(p)) if kernel in r["Kernel_Name"]]
        with open(os.path.join(out, f"{tag}_pmc_{sub.lower()}.csv"), "w", newline="") as f:
            w = csv.DictWriter(f, fieldnames=list(mine[0].keys()))
            w.writeheader()
            w.writerows(mine)
        by = {}
        for r in mine:
            by.setdefault(r["Counter_Name"], []).append(float(r["Counter_Value"]))
        for c, v in by.items():
            med[c] = statistics.median(v)
    rd = med["FETCH_SIZE"] * 1024 * 2
    wr = med["WRITE_SIZE"] * 1024
    d = {"kernel": f"{kernel} (int4 sym g128, [11008,4096] bf16, {per_launch} weights per PMC launch)",
         "weights_per_pmc_launch": per_launch,
         "rocprof_avg_ns": float(k["AverageNs"]), "rocprof_calls": int(k["Calls"]),
         "rocprof_weights_per_launch": STATS_WEIGHTS,
         "rocprof_avg_ns_per_weight": float(k["AverageNs"]) / STATS_WEIGHTS,
         "fetch_size_kb_median": med["FETCH_SIZE"], "write_size_kb_median": med["WRITE_SIZE"],
         "correction": "FETCH_SIZE x2 (gfx950 half-count for 16-B/lane streaming reads, MI355X_MICROARCH.md HBM "
                       "section); WRITE_SIZE as-is; KB = 1024 B",
         "hbm_read_bytes_per_launch": rd, "hbm_write_bytes_per_launch": wr, "hbm_bytes_per_launch": rd + wr,
         "hbm_bytes_per_weight": (rd + wr) / per_launch,
         "algorithmic_bytes_per_launch": ALG * per_launch, "traffic_over_algorithmic": (rd + wr) / (ALG * per_launch),
         "other_counters_median": {c: v for c, v in med.items() if c not in ("FETCH_SIZE", "WRITE_SIZE")},
         "source": f"profiles/{tag}_pmc_*.csv (rocprofv3 --pmc, separate passes, bench.py --profile-only); "
                   f"profiles/{tag}_bench_kernel_stats.csv (rocprofv3 --kernel-trace --stats)"}
    json.dump(d, open(os.path.join(out, "pmc_traffic.json"), "w"), indent=2)
    print(json.dumps(d, indent=2))


if __name__ == "__main__":
    main(sys.argv[1], *(sys.argv[2:3]), *([int(sys.argv[3])] if len(sys.argv) > 3 else []))
