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


def main(tag):
    src = os.path.join(ROOT, "gpurun_out", f"pmch_{tag}")
    per = {}
    for c in ("FETCH_SIZE", "WRITE_SIZE"):
        for r in csv.DictReader(open(os.path.join(src, c, "run_counter_collection.csv"))):
            if KERNEL in r["Kernel_Name"] and r["Counter_Name"] == c:
                per.setdefault(r["Grid_Size"], {}).setdefault(c, []).append(float(r["Counter_Value"]))
    shapes = {}
    step = 0.0
    for g, d in sorted(per.items(), key=lambda kv: int(kv[0])):
        rd = statistics.median(d["FETCH_SIZE"]) * 1024 * 2
        wr = statistics.median(d["WRITE_SIZE"]) * 1024
        n = len(d["FETCH_SIZE"])
        shapes[g] = {"dispatches": n, "hbm_read_bytes": rd, "hbm_write_bytes": wr}
    # launches per step: grid sizes repeat once per step except the [1024, 2560] k/v launch (one
    # grid size, one launch per step); every listed grid size is one launch per step
    step = sum(v["hbm_read_bytes"] + v["hbm_write_bytes"] for v in shapes.values())
    import bench  # noqa: E402  (algorithmic bytes of the same plan, no GPU needed)
    alg = 0
    for name, n, k in bench.QWEN3_4B:
        p = n * k * bench.QWEN3_LAYERS
        alg += p * 2 + p // 2 + (p // 128) * 2
    out = {"tag": tag, "kernel": KERNEL, "launches_per_step": len(shapes), "per_launch_shape": shapes,
           "hbm_bytes_per_step": step, "hbm_bytes_per_launch": step / len(shapes),
           "alg_bytes_per_step": alg, "traffic_over_algorithmic": step / alg,
           "correction": "FETCH_SIZE x2 (gfx950 half-count of 16-B/lane streaming reads), WRITE_SIZE as-is, KB=1024 B",
           "source": f"scripts/pmc_headline.sh TAG={tag}: rocprofv3 --pmc FETCH_SIZE / --pmc WRITE_SIZE (separate runs) "
                     "of python3 bench.py --profile-only --steps 20 --warmup 5; medians per launch shape"}
    json.dump(out, open(os.path.join(ROOT, "profiles", "headline_pmc.json"), "w"), indent=1)
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main(sys.argv[1])
