#!/usr/bin/env python3
"""profiles/headline_pmc.json from scripts/pmc_headline.sh's passes (gpurun_out/pmch_TAG/):
HBM bytes of one bench step (the 5 grouped launches of the whole-model plan), FETCH_SIZE x2 +
WRITE_SIZE (MI355X_MICROARCH.md gfx950 corrections; KB = 1024 B), median per launch shape
(told apart by grid size), next to the algorithmic bytes.

  python scripts/pmc_headline_summary.py TAG"""
import csv
import json
import os
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
KERNEL = "k_group_fast<4, 0, false, true, true, true>"
sys.path.insert(0, ROOT)


def main(tag, launches_per_step=5):
    """Dispatches of the grouped kernel come in plan order, ``launches_per_step`` per step
    (q, k+v, o, gate+up, down; q and o share a grid size, so steps are cut by dispatch order):
    HBM bytes of a step = the sum over its launches; the median over the W + K profiled steps."""
    src = os.path.join(ROOT, "gpurun_out", f"pmch_{tag}")
    vals = {}
    for c in ("FETCH_SIZE", "WRITE_SIZE"):
        rows = [r for r in csv.DictReader(open(os.path.join(src, c, "run_counter_collection.csv")))
                if KERNEL in r["Kernel_Name"] and r["Counter_Name"] == c]
        rows.sort(key=lambda r: int(r["Dispatch_Id"]))
        vals[c] = [float(r["Counter_Value"]) for r in rows]
        grids = [int(r["Grid_Size"]) for r in rows]
    n = len(vals["FETCH_SIZE"])
    assert n == len(vals["WRITE_SIZE"]) and n % launches_per_step == 0, (n, len(vals["WRITE_SIZE"]))
    steps = []
    shapes = {}
    for i in range(0, n, launches_per_step):
        rd = sum(vals["FETCH_SIZE"][i:i + launches_per_step]) * 1024 * 2
        wr = sum(vals["WRITE_SIZE"][i:i + launches_per_step]) * 1024
        steps.append((rd, wr))
    for j in range(launches_per_step):
        rd = statistics.median(vals["FETCH_SIZE"][j::launches_per_step]) * 1024 * 2
        wr = statistics.median(vals["WRITE_SIZE"][j::launches_per_step]) * 1024
        shapes[f"launch{j}_grid{grids[j]}"] = {"hbm_read_bytes": rd, "hbm_write_bytes": wr}
    step = statistics.median(rd + wr for rd, wr in steps)
    shapes = dict(shapes, steps_profiled=len(steps))
    import bench  # noqa: E402  (algorithmic bytes of the same plan, no GPU needed)
    alg = 0
    for name, n, k in bench.QWEN3_4B:
        p = n * k * bench.QWEN3_LAYERS
        alg += p * 2 + p // 2 + (p // 128) * 2
    out = {"tag": tag, "kernel": KERNEL, "launches_per_step": launches_per_step, "per_launch": shapes,
           "hbm_bytes_per_step": step, "hbm_bytes_per_launch": step / launches_per_step,
           "alg_bytes_per_step": alg, "traffic_over_algorithmic": step / alg,
           "correction": "FETCH_SIZE x2 (gfx950 half-count of 16-B/lane streaming reads), WRITE_SIZE as-is, KB=1024 B",
           "source": f"scripts/pmc_headline.sh TAG={tag}: rocprofv3 --pmc FETCH_SIZE / --pmc WRITE_SIZE (separate runs) "
                     "of python3 bench.py --profile-only --steps 20 --warmup 5; median over the 25 profiled steps"}
    json.dump(out, open(os.path.join(ROOT, "profiles", "headline_pmc.json"), "w"), indent=1)
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main(sys.argv[1])
