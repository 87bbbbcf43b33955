#!/usr/bin/env python3
"""Summarise a scripts/pmc_kernels.sh session (gpurun_out/pmck_TAG/) into profiles/ (committed):

  python scripts/pmc_kernels_summary.py TAG

writes profiles/TAG_kernels_stats.csv (the rocprofv3 --kernel-trace --stats summary, torch
kernel names shortened) and profiles/TAG_kernels_pmc.json: per kernel the median duration from
the kernel trace, the median of every PMC counter over its launches, HBM bytes per launch
(MI355X_MICROARCH.md corrections: FETCH_SIZE x2 on gfx950, WRITE_SIZE as-is, KB = 1024 B) next to
the algorithmic bytes, and the derived issue figures (VALU / VMEM instructions per wave, wave
lifetime, fraction of wave cycles parked on s_waitcnt vs issuing)."""
import csv
import json
import os
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
R, C = 11008, 4096
P = R * C
T = 16384  # activation tokens of the absmean leg (scripts/kernel_driver.py)
LEG_LAUNCHES = 33  # per leg: 3 warm-up launches + N = 30 timed ones (scripts/pmc_kernels.sh N)
# kernel-name substring -> (label, algorithmic bytes per launch)
KERNELS = {
    "k_group_fast<4, 0, false, true, true, false>": ("quantize int4 g128 (per-weight launch)", int(P * 2.515625)),
    "k_group_fast<4, 0, true, true, false, false>": ("AWQ fake-quant Q(W*s)/s int4 g128 (unit-wise, r02c)", P * 4 + C * 4),
    # kernel_driver runs k_fq_cols in two legs, in this order: "#0" = 12 rotating weights into 4
    # rotating outputs (an isolated op, cold), "#1" = the AWQ grid's pattern (one weight, 20 scale
    # vectors, one output)
    "k_fq_cols<4, 0, true, false>#0": ("AWQ fake-quant Q(W*s)/s int4 g128", P * 4 + C * 4),
    "k_fq_cols<4, 0, true, false>#1": ("AWQ fake-quant Q(W*s)/s int4 g128, AWQ grid pattern (one weight, 20 scales)",
                                       P * 4 + C * 4),
    "k_absmean_partial_v8": ("AWQ absmean stage 1 [16384, 4096]", T * C * 2),
    "k_colsum_final<float>": ("AWQ absmean stage 2", None),
    "k_wmean_v8": ("AWQ w_mean stage 1", P * 2),
    "k_colsum_final<double>": ("AWQ w_mean stage 2", None),
    "k_scale_v8<true>": ("AWQ smoothing W[:, c] *= s[c]", P * 4 + C * 4),
    # kernel_driver's absmean / w_mean legs in order: "#0" the [16384, 4096] / [11008, 4096]
    # operands, "#1" the AWQ pass's own Qwen3-4B pattern as issued through round 4 (one calibration
    # sample [2048, 2560]; one balance layer [9728, 2560]); the segmented launches of round 5 (16
    # samples; gate + up, then q / k / v)
    "k_absmean_1l<128>#0": ("AWQ absmean [16384, 4096], one launch (round 3)", T * C * 2),
    "k_absmean_1l<128>#1": ("AWQ absmean, one calibration sample [2048, 2560] per launch (Qwen3-4B pass through r04)",
                            2048 * 2560 * 2),
    "k_absmean_seg<128>": ("AWQ absmean, 16 samples x [2048, 2560] in one segmented launch (round 5)",
                           16 * 2048 * 2560 * 2),
    "k_wmean_1l<128, 4>#0": ("AWQ w_mean [11008, 4096] g128, one launch (round 3)", P * 2),
    "k_wmean_1l<128, 4>#1": ("AWQ w_mean, one balance layer [9728, 2560] per launch (Qwen3-4B pass through r04)",
                             9728 * 2560 * 2),
    "k_wmean_seg<128, 4>#0": ("AWQ w_mean, gate + up 2 x [9728, 2560] in one segmented launch (round 5)",
                              2 * 9728 * 2560 * 2),
    "k_wmean_seg<128, 4>#1": ("AWQ w_mean, q / k / v [4096 | 1024 | 1024, 2560] in one segmented launch (round 5)",
                              6144 * 2560 * 2),
    # MXFP4 [128, 768, 2048] (BASELINE configs[3]): read 2 B + codes 0.5 B + e8m0 scale 1/32 B per param
    "k_group_fast<2, 2, false, true, true, false>": ("MXFP4 Qwen3-30B-A3B expert half [128, 768, 2048] (one launch)",
                                                     int(128 * 768 * 2048 * (2 + 0.5 + 1 / 32))),
    # NVFP4 [128, 768, 2048]: read 2 B + codes 0.5 B + e4m3 scale 1/16 B per param + f32 per slice
    "k_nv_encode<false>": ("NVFP4 fused encode launch, Qwen3-30B-A3B expert half [128, 768, 2048] (round 4)",
                           int(128 * 768 * 2048 * (2 + 0.5 + 1 / 16)) + 128 * 4),
    "k_nv_absmax<false>": ("NVFP4 fused |w| max launch [128, 768, 2048] (round 4)", 128 * 768 * 2048 * 2),
    "k_group_fast<1, 3, false, true, true, false>": ("NVFP4 two-pass quantize pass [128, 768, 2048]",
                                                     int(128 * 768 * 2048 * (2 + 0.5 + 1 / 16)) + 128 * 4),
    "k_absmax_slices": ("NVFP4 two-pass per-slice |w| max pre-pass [128, 768, 2048]", 128 * 768 * 2048 * 2),
    # FP8_BLOCK 128x128 (round 5, qz_block.hip): read 2 B + e4m3 1 B per param + a bf16 scale per block;
    # kernel_driver runs the table-mode kernel in two legs, k+v then q
    "k_block_fp8<2, true>#0": ("FP8_BLOCK grouped launch 72 x [1024, 2560] (Qwen3-4B k+v)",
                               72 * 1024 * 2560 * 3 + 72 * 8 * 20 * 2),
    "k_block_fp8<2, true>#1": ("FP8_BLOCK grouped launch 36 x [4096, 2560] (Qwen3-4B q)",
                               36 * 4096 * 2560 * 3 + 36 * 32 * 20 * 2),
    "k_block_fp8<2, false>": ("FP8_BLOCK batch launch [36, 1024, 2560]", 36 * 1024 * 2560 * 3 + 36 * 8 * 20 * 2),
}


def _short(name):
    return name.split("(")[0][:120] + "(...)" if "at::native" in name else name


def main(tag):
    src = os.path.join(ROOT, "gpurun_out", f"pmck_{tag}")
    out = os.path.join(ROOT, "profiles")
    rows = list(csv.DictReader(open(os.path.join(src, "trace", "run_kernel_stats.csv"))))
    with open(os.path.join(out, f"{tag}_kernels_stats.csv"), "w", newline="") as f:
        w = csv.DictWriter(f, fieldnames=list(rows[0].keys()))
        w.writeheader()
        for r in rows:
            w.writerow(dict(r, Name=_short(r["Name"])))
    trace = list(csv.DictReader(open(os.path.join(src, "trace", "run_kernel_trace.csv"))))
    res = {}
    def leg(rows, part):  # "#k": the k-th block of LEG_LAUNCHES consecutive launches of the kernel
        return rows if part is None else rows[part * LEG_LAUNCHES:(part + 1) * LEG_LAUNCHES]
    for key, (label, alg) in KERNELS.items():
        sub, _, part = key.partition("#")
        part = int(part) if part else None
        mine = sorted((r for r in trace if sub in r["Kernel_Name"]), key=lambda r: int(r["Dispatch_Id"]))
        durs = [int(r["End_Timestamp"]) - int(r["Start_Timestamp"]) for r in leg(mine, part)]
        if not durs:
            continue
        d = {"label": label, "launches": len(durs), "median_ns": statistics.median(durs),
             "mean_ns": statistics.fmean(durs), "min_ns": min(durs), "counters": {}}
        for pdir in sorted(os.listdir(src)):
            p = os.path.join(src, pdir, "run_counter_collection.csv")
            if pdir == "trace" or not os.path.exists(p):
                continue
            by = {}
            rows = [r for r in csv.DictReader(open(p)) if sub in r["Kernel_Name"]]
            seen = sorted({int(r["Dispatch_Id"]) for r in rows})  # dispatches in order
            seen = [str(d) for d in seen]
            keep = set(leg(seen, part))
            for r in rows:
                if r["Dispatch_Id"] in keep:
                    by.setdefault(r["Counter_Name"], []).append(float(r["Counter_Value"]))
            for c, v in by.items():
                d["counters"][c] = statistics.median(v)
        c = d["counters"]
        if "FETCH_SIZE" in c and "WRITE_SIZE" in c:
            d["hbm_bytes"] = c["FETCH_SIZE"] * 1024 * 2 + c["WRITE_SIZE"] * 1024
        if alg:
            d["alg_bytes"] = alg
            d["alg_TBps"] = alg / d["median_ns"] / 1e3
            d["frac_of_8TBps"] = d["alg_TBps"] / 8.0
            if "hbm_bytes" in d:
                d["traffic_over_alg"] = d["hbm_bytes"] / alg
        if c.get("SQ_WAVES"):
            wv = c["SQ_WAVES"]
            d["valu_per_wave"] = c.get("SQ_INSTS_VALU", 0) / wv
            d["vmem_rd_per_wave"] = c.get("SQ_INSTS_VMEM_RD", 0) / wv
            d["vmem_wr_per_wave"] = c.get("SQ_INSTS_VMEM_WR", 0) / wv
            d["salu_per_wave"] = c.get("SQ_INSTS_SALU", 0) / wv
            d["lds_per_wave"] = c.get("SQ_INSTS_LDS", 0) / wv
            d["wave_cycles_per_wave_x4"] = c.get("SQ_WAVE_CYCLES", 0) / wv
        wc = c.get("SQ_WAIT_ANY", 0) + c.get("SQ_WAIT_INST_ANY", 0) + c.get("SQ_ACTIVE_INST_ANY", 0)
        if wc:
            d["frac_wait_any"] = c["SQ_WAIT_ANY"] / wc
            d["frac_wait_inst_any"] = c["SQ_WAIT_INST_ANY"] / wc
            d["frac_active_inst"] = c["SQ_ACTIVE_INST_ANY"] / wc
            d["frac_active_valu_of_active"] = c.get("SQ_ACTIVE_INST_VALU", 0) / max(c["SQ_ACTIVE_INST_ANY"], 1)
        res[label] = d
    with open(os.path.join(out, f"{tag}_kernels_pmc.json"), "w") as f:
        json.dump({"source": f"scripts/pmc_kernels.sh TAG={tag} (scripts/kernel_driver.py, 30 launches per kernel, "
                             "12 rotating [11008, 4096] bf16 copies)", "kernels": res}, f, indent=1)
    for k, d in res.items():
        print(f"{k:42s} med {d['median_ns'] / 1e3:7.2f} us  frac {d.get('frac_of_8TBps', 0):.3f}  "
              f"traffic/alg {d.get('traffic_over_alg', 0):.3f}  valu/wave {d.get('valu_per_wave', 0):7.1f}  "
              f"wait {d.get('frac_wait_any', 0):.2f} inst-wait {d.get('frac_wait_inst_any', 0):.2f} "
              f"active {d.get('frac_active_inst', 0):.2f}")


if __name__ == "__main__":
    main(sys.argv[1])
