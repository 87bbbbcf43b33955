#!/usr/bin/env python3
"""Summarise a rocprofv3 --kernel-trace --stats run of bench.py into profiles/ (committed evidence)
and cross-check the bench line's roofline against the profiler's kernel durations.

  python scripts/prof_summary.py TAG PROF_DIR BENCH_LOG

PROF_DIR holds rocprofv3's ``*_kernel_trace.csv`` / ``*_kernel_stats.csv`` of
``rocprofv3 --kernel-trace --stats -- python3 bench.py --steps K --warmup W``; BENCH_LOG is that
command's stdout (its JSON line).  Writes
  profiles/TAG_kernel_stats.csv   -- the stats table (torch generator names shortened)
  profiles/TAG_bench_line.json    -- the bench line of the same run
  profiles/TAG_headline.json      -- the headline launches picked from the trace: the grouped
      kernel's dispatches in dispatch order:
      W*L warmup, then the K*L timed launches (L = launches per step), then L per-launch probes;
      their mean duration (the headline launches are told apart from the synthetic leg's by their
      grid.y = weights per launch, e.g. 36 / 72 for Qwen3-4B; the synthetic leg uses 100), kernel time per step, and frac = alg bytes per step / kernel time per
      step / 8 TB/s next to the line's own frac.
"""
import csv
import glob
import json
import os
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PEAK = 8.0e12


def _one(pattern):
    hits = sorted(glob.glob(pattern, recursive=True))
    if not hits:
        raise SystemExit(f"no file matches {pattern}")
    return hits[0]


def _short(name):
    return name.split("(")[0][:120] + "(...)" if "at::native" in name else name


def main(tag, prof_dir, bench_log):
    out_dir = os.path.join(ROOT, "profiles")
    line = None
    for ln in open(bench_log):
        ln = ln.strip()
        if ln.startswith("{") and '"metric"' in ln:
            line = json.loads(ln)
    if line is None:
        raise SystemExit("no bench JSON line in " + bench_log)
    with open(os.path.join(out_dir, f"{tag}_bench_line.json"), "w") as f:
        json.dump(line, f, indent=1)
    stats = list(csv.DictReader(open(_one(os.path.join(prof_dir, "**", "*kernel_stats.csv")))))
    with open(os.path.join(out_dir, f"{tag}_kernel_stats.csv"), "w", newline="") as f:
        w = csv.DictWriter(f, fieldnames=list(stats[0].keys()))
        w.writeheader()
        for r in stats:
            w.writerow(dict(r, Name=_short(r["Name"])))
    trace = list(csv.DictReader(open(_one(os.path.join(prof_dir, "**", "*kernel_trace.csv")))))
    kern = line["roofline"]["kernel"]
    L = int(line["roofline"]["launches_per_step"])
    K, W = int(line["steps"]), int(line["warmup"])
    gy = {int(p["weights"]) for p in line["per_launch"]}  # grid.y of the headline launches (weights each)
    mine = [r for r in trace if kern in r["Kernel_Name"] and int(r.get("Grid_Size_Y", r.get("Grid_Size_y", 0))) in gy]
    mine.sort(key=lambda r: int(r["Start_Timestamp"]))
    timed = mine[W * L:(W + K) * L]
    if len(timed) != K * L:
        raise SystemExit(f"expected {K * L} timed launches of {kern}, found {len(timed)} after {W * L} warmup")
    durs = [int(r["End_Timestamp"]) - int(r["Start_Timestamp"]) for r in timed]
    span = int(timed[-1]["End_Timestamp"]) - int(timed[0]["Start_Timestamp"])
    alg_step = float(line["roofline"]["alg_bytes_per_step"])
    kstep = sum(durs) / K * 1e-9
    frac_prof = alg_step / kstep / PEAK
    frac_span = alg_step * K / (span * 1e-9) / PEAK
    res = {
        "kernel": kern, "launches_timed": len(timed), "launches_per_step": L, "steps": K, "warmup": W,
        "mean_launch_ns": statistics.mean(durs), "median_launch_ns": statistics.median(durs),
        "min_launch_ns": min(durs), "max_launch_ns": max(durs),
        "kernel_ms_per_step": kstep * 1e3, "span_ms_per_step": span * 1e-6 / K,
        "bench_ms_per_step": line["ms_per_step"], "bench_event_ms_per_step": line["roofline"]["event_ms_per_step"],
        "frac_from_profile_kernel_time": frac_prof, "frac_from_profile_span": frac_span,
        "frac_bench_line": line["roofline"]["frac"],
        "line_vs_profile": line["roofline"]["frac"] / frac_prof,
        "per_launch_by_shape_ns": {},
    }
    for i in range(L):
        d = durs[i::L]
        res["per_launch_by_shape_ns"][f"launch{i}"] = {"mean": statistics.mean(d), "grid_x": timed[i].get("Grid_Size_X")}
    with open(os.path.join(out_dir, f"{tag}_headline.json"), "w") as f:
        json.dump(res, f, indent=1)
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main(*sys.argv[1:4])
