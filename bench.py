#!/usr/bin/env python3
"""Benchmark of the north-star path: int4 symmetric group-128 quantize + pack of every linear
weight of a Qwen3-4B-shaped model (BASELINE.json configs[1], "Qwen3-4B AWQ int4 group_size=128 on
1xMI355X"; metric "params quantized/sec + achieved HBM GB/s, Qwen3-4B AWQ int4-g128").

One *step* = one pass of the product's compressor over the whole model: the 252 targeted
linears (36 layers x q/k/v/o/gate/up/down, 3.63 G params, public Qwen3-4B dims, random bf16
weights -- there is no checkpoint offline) quantized + packed by ``compressor.CompressionPlan``,
the exact launch plan ``save_compressed`` runs (same-shape modules of one scheme in ONE grouped
launch: 5 launches per step).  Weights (7.3 GB) and outputs (1.8 GB) stay resident in HBM, far
larger than the 256 MiB Infinity Cache, so every step streams from HBM; the device->host copy
that ``save_compressed`` adds is not in the timed region (DESIGN.md §6 gives the
PCIe-inclusive rate).

``value`` (params/s) and ``roofline.achieved`` come from the SAME timed region: wall clock
(barrier + synchronize on both sides, max over ranks) for ``value``; HIP events on the launch
stream around the same K steps for the kernel time (= the K launches back to back).  The
rocprofv3 kernel trace of the same command is summarised by scripts/prof_summary.py.

Beside it (not the headline): the north-star synthetic weight [11008, 4096] (grouped and one
launch per weight), the AWQ kernels, a 2-layer AWQ oneshot, the other BASELINE configs, and the
CPU baseline (the oracle's torch restatement on the host cores).

Multi-GPU: one process per GPU.  ``--gpus N`` under torchrun (WORLD_SIZE=N) runs as rank
RANK; ``--gpus N`` without a torchrun environment starts the N ranks itself (a
``torch.distributed.run`` child process; this process never touches the GPU), and a mismatch
between ``--gpus`` and WORLD_SIZE is an error, so ``n_gpus`` is always the ranks that ran
(``ranks_seen`` = the process group's size).  The headline is weak scaling: each rank
compresses its own Qwen3-4B-sized weight set (no collective in the timed region).  Beside it,
at every N: the row-sharded synthetic leg ([11008, 4096] split into N row
blocks, kernel-only and end-to-end including the RCCL all-gather of the packed codes and
scales) and the strong-scaling leg (ONE Qwen3-4B sharded over the ranks by the product's
plan, plus ``distributed.gather_state``'s all-gather of the compressed state dict).

Usage: python bench.py [--gpus N] [--steps K] [--warmup W]
       torchrun --nproc-per-node N bench.py --gpus N ...
"""
import argparse
import json
import os
import platform
import subprocess
import sys
import time

import torch
import torch.distributed as dist

T_START = time.perf_counter()  # after `import torch`: the phase budget starts here
ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

ROWS, COLS, GROUP, BITS = 11008, 4096, 128, 4  # north-star synthetic weight (secondary leg)
PARAMS = ROWS * COLS
# algorithmic bytes per [11008, 4096] weight: read 2 B/param + packed 0.5 B/param
# + one bf16 scale per group = 2.515625 B/param
ALG_BYTES = PARAMS * 2 + PARAMS * BITS // 8 + (PARAMS // GROUP) * 2  # 113,426,432
HBM_PEAK_GBS = 8000.0  # MI355X_MICROARCH.md: 8.0 TB/s spec
METRIC = "params quantized/sec + achieved HBM GB/s, Qwen3-4B AWQ int4-g128"
RECIPE = os.path.join(ROOT, "configs", "recipes", "awq_w4a16_g128.yaml")
# BASELINE.json configs[2]: FP8_BLOCK attention + int4 g32 MLP (reference recipe_mixed_fp8_int4.yaml, M1 corrected)
MIXED_RECIPE = os.path.join(ROOT, "configs", "recipes", "mixed_fp8_block_awq_int4.yaml")
MODEL_CFG = os.path.join(ROOT, "configs", "models", "qwen3-4b")

# Qwen3-4B linear shapes (hidden 2560, inter 9728, 32 q / 8 kv heads x 128), 36 layers
QWEN3_4B = [("q_proj", 4096, 2560), ("k_proj", 1024, 2560), ("v_proj", 1024, 2560), ("o_proj", 2560, 4096),
            ("gate_proj", 9728, 2560), ("up_proj", 9728, 2560), ("down_proj", 2560, 9728)]
QWEN3_LAYERS = 36


def kernel_name(grouped: bool, launch_weight_bytes: int, logl: int = 4, kind: int = 0, sym: bool = True) -> str:
    """The k_group_fast instantiation a quantize launch runs, from the library's build constants
    (qz_build_config): <LOGL, KIND, FQ, SYM, NT, GRP>; NT when the launch reads more than
    nt_bytes_q."""
    from quantizers_amd import _lib
    nt = launch_weight_bytes > int(_lib.build_config()["nt_bytes_q"])
    b = lambda v: str(bool(v)).lower()  # noqa: E731
    return f"k_group_fast<{logl}, {kind}, false, {b(sym)}, {b(nt)}, {b(grouped)}>"


def parse():
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=None,
                   help="ranks (one per GPU); without a torchrun environment bench.py starts them itself")
    p.add_argument("--steps", type=int, default=20)
    # 50 untimed steps (70 ms): the clocks settle about 25 steps (35 ms) into a load
    # (scripts/step_ramp.py, profiles/r05j_step_ramp.log), so the K timed steps are steady state
    p.add_argument("--warmup", type=int, default=50)
    p.add_argument("--copies", type=int, default=12)
    p.add_argument("--cpu-seconds", type=float, default=10.0)
    p.add_argument("--launch-check", action="store_true",
                   help="start the ranks, join the process group, print the rank census and exit (no GPU use)")
    p.add_argument("--no-cpu-baseline", action="store_true")
    p.add_argument("--no-extras", action="store_true", help="headline only (no secondary legs)")
    p.add_argument("--profile-only", action="store_true",
                   help="warmup + K headline steps only (rocprofv3 PMC passes); prints nothing else")
    return p.parse_args()


def cpu_baseline(seconds: float, checks=None):
    """The oracle's torch restatement of compressed-tensors (oracle/ct_torch.py), timed on the host
    cores on a bounded sample of the headline workload: repeated compress_weight calls on the
    north-star synthetic weight [11008, 4096] (seed 0, N(0, 0.02^2) bf16), one
    warm-up call, then at least 5 timed calls for about ``seconds``; best and median per call
    reported, ``value`` = the median.  The oracle is used only here (the CPU leg) and as the
    checker of ``checks`` = [(input rows, packed codes, scales)] taken from the GPU's measured
    outputs (plain-C restatement, bit for bit).

    Threads: 16 = the GPU box's CPU share for one GPU (its OMP_NUM_THREADS; gpurun sizes one
    GPU's host share at 16 of the node's os.cpu_count() cores), not os.cpu_count() as BASELINE.md
    §2 asks -- running 256 threads would take cores the box does not give one GPU's job."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import ct_torch as ct  # CPU baseline leg only
    import qref  # checker only
    ok = None
    if checks:
        ok = True
        for w_in, codes, scale in checks:
            ref_p, ref_s = qref.int_sym_group_pack(w_in, BITS, GROUP)
            ok = ok and bool(torch.equal(codes, ref_p) and torch.equal(scale.view(torch.int16), ref_s.view(torch.int16)))
    threads = min(16, os.cpu_count() or 1)
    torch.set_num_threads(threads)
    g = torch.Generator().manual_seed(0)
    w = (torch.randn(ROWS, COLS, generator=g) * 0.02).to(torch.bfloat16)
    a = ct.QArgs(num_bits=BITS, type="int", symmetric=True, strategy="group", group_size=GROUP)
    ct.compress_weight(w, a)  # warm-up
    times = []
    t_start = time.perf_counter()
    while len(times) < 5 or (time.perf_counter() - t_start < seconds and len(times) < 200):
        t0 = time.perf_counter()
        ct.compress_weight(w, a)
        times.append(time.perf_counter() - t0)
    times.sort()
    med = times[len(times) // 2]
    res = {"value": PARAMS / med, "unit": "params/s", "cores": threads, "kind": "port",
           "best_params_per_s": PARAMS / times[0], "median_s_per_call": med, "best_s_per_call": times[0],
           "calls": len(times),
           "sample": f"oracle/ct_torch.compress_weight (compressed-tensors op sequence, torch CPU) int4-g{GROUP} on "
                     f"the north-star synthetic bf16 weight [{ROWS},{COLS}] (seed 0, N(0, 0.02^2)): 1 warm-up + "
                     f"{len(times)} timed calls in {sum(times):.1f}s, value = median call, torch threads={threads} "
                     f"(the box's per-GPU CPU share), os.cpu_count()={os.cpu_count()}, cpu='{cpu_model()}'"}
    return res, ok


def cpu_model():
    try:
        out = subprocess.run(["lscpu"], capture_output=True, text=True, timeout=10).stdout
        for line in out.splitlines():
            if line.startswith("Model name"):
                return line.split(":", 1)[1].strip()
    except Exception:
        pass
    return platform.processor() or "unknown"


PASSES = 5  # event-timed passes per secondary leg; the median is reported


WARM_S = 0.08  # untimed load before a leg's passes: the clocks settle ~35 ms into a load (r05j_step_ramp)


def _event_median(fn, stream, passes=PASSES, warm=1, warm_s=WARM_S):
    """Median seconds of ``passes`` calls of ``fn`` (each enqueues one whole pass on ``stream``),
    each between its own pair of HIP events on that stream, after at least ``warm`` untimed calls
    and ``warm_s`` seconds of them (a leg that starts from an idle GPU otherwise times the clock
    ramp: 19.4 -> 17.5 us per weight over 7 grouped passes, profiles/r06e_bench_compare.txt);
    also returns every pass's seconds."""
    t0, i = time.perf_counter(), 0
    while i < warm or time.perf_counter() - t0 < warm_s:
        fn()
        i += 1
        if i >= warm:
            torch.cuda.synchronize()
    ts = []
    for _ in range(passes):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(stream)
        fn()
        e1.record(stream)
        torch.cuda.synchronize()
        ts.append(e0.elapsed_time(e1) * 1e-3)
    return sorted(ts)[len(ts) // 2], ts


def _launch_us(gq, stream, reps=10, passes=7):
    """One grouped launch's steady duration (us): ``reps`` launches back to back between one pair
    of HIP events (the gaps between them included, as in a plan step), median of ``passes``."""
    def batch():
        for _ in range(reps):
            gq.run(stream)
    return _event_median(batch, stream, passes=passes, warm=1, warm_s=0.02)[0] * 1e6 / reps


def mixed_plan_leg(ops, dev, stream, steps=20):
    """BASELINE.json configs[2] through the product: the Qwen3-4B model (public dims, random bf16)
    under the mixed recipe (configs/recipes/mixed_fp8_block_awq_int4.yaml = the reference's
    recipe_mixed_fp8_int4.yaml with quirk M1 corrected: FP8_BLOCK on q/k/v/o, int4 sym g32 on
    gate/up/down), compressed by ``compressor.CompressionPlan`` exactly as ``save_compressed`` runs
    it: 5 grouped launches per step (q, k+v, o through the FP8_BLOCK strip kernel; gate+up, down
    through the group kernel).  HIP events on the launch stream around ``steps`` whole steps;
    algorithmic bytes = every weight read once + every output written once (plan.alg_bytes());
    per-launch figures from one event pair per launch."""
    from quantizers_amd.compressor import CompressionPlan, compression_units
    torch.manual_seed(1235)
    model = build_model(dev, MIXED_RECIPE)
    units, _ = compression_units(model)
    plan = CompressionPlan(units, dev)
    def steps_pass():
        for _ in range(steps):
            plan.run(stream)
    s, _ = _event_median(steps_pass, stream, warm=1)
    s /= steps
    alg = plan.alg_bytes()
    per = []
    for gq, part, *_ in plan.grouped:
        us = _launch_us(gq, stream)
        rb = sum(w.numel() * 2 for _, w in part)
        nb = rb + sum(t.numel() * t.element_size() for o in gq.outs for t in o.values() if t is not None)
        per.append({"scheme": "FP8_BLOCK 128x128" if ops.is_fp8_block128(gq.a) else
                    f"int{gq.a.num_bits} g{gq.a.group_size}", "shape": f"{gq.rows}x{gq.cols}", "weights": gq.n,
                    "us": us, "alg_bytes": nb, "frac": nb / (us * 1e-6) / 1e9 / HBM_PEAK_GBS,
                    "read_frac": rb / (us * 1e-6) / 1e9 / HBM_PEAK_GBS})
    res = {"params": plan.params, "launches_per_step": plan.launches, "ms": s * 1e3, "params_per_s": plan.params / s,
           "alg_bytes": alg, "alg_GBps": alg / s / 1e9, "frac": alg / s / 1e9 / HBM_PEAK_GBS,
           "read_frac": plan.params * 2 / s / 1e9 / HBM_PEAK_GBS, "per_launch": per,
           "recipe": "configs/recipes/mixed_fp8_block_awq_int4.yaml",
           "timing": f"HIP events on the launch stream around {steps} CompressionPlan steps, median of {PASSES} "
                     f"such passes; per launch: bench._launch_us"}
    del plan, units, model
    torch.cuda.empty_cache()
    return res


def other_configs(ops, QuantizationArgs, dev, gen, stream):
    """BASELINE.json configs[2] (Qwen3-4B FP8_BLOCK attention + int4-g32 MLP, through the product's
    CompressionPlan) and configs[3] (Qwen3-30B-A3B experts -> MXFP4 / NVFP4): one quantize pass
    over every targeted weight."""
    res = {"qwen3_4b_mixed_fp8block_int4g32": mixed_plan_leg(ops, dev, stream)}
    # Qwen3-30B-A3B: 48 layers x 128 experts x {gate, up [768, 2048], down [2048, 768]}; 4 resident
    # layers (fused [E, 2I, H] / [E, H, I] parameters, gate/up as strided views) rotated over 48
    mx = QuantizationArgs(num_bits=4, type="float", group_size=32, scale_dtype="uint8")
    layers = []
    for _ in range(4):
        gu = (torch.randn(128, 2 * 768, 2048, device=dev, generator=gen) * 0.02).to(torch.bfloat16)
        dn = (torch.randn(128, 2048, 768, device=dev, generator=gen) * 0.02).to(torch.bfloat16)
        layers.append((gu, dn))

    # outputs preallocated, every launch's arguments marshalled once (ops.PreparedQuantize): one
    # ctypes call per launch, no allocation inside the timed passes
    views = [w for gu, dn in layers for w in (gu[:, :768], gu[:, 768:], dn)]
    preps = [ops.PreparedQuantize(w, mx, ops.alloc_outputs(tuple(w.shape), mx, None, dev)) for w in views]

    def moe_pass():
        for li in range(48):
            for j in range(3):
                k = (li % 4) * 3 + j
                preps[k].run(views[k], stream)
    npar = 48 * 128 * 3 * 768 * 2048
    t, ts = _event_median(moe_pass, stream)
    nb = npar * (2 + 0.5 + 1 / 32)
    res["qwen3_30b_a3b_experts_mxfp4"] = {"params": npar, "ms": t * 1e3, "params_per_s": npar / t,
                                          "alg_GBps": nb / t / 1e9, "frac": nb / t / 1e9 / HBM_PEAK_GBS,
                                          "ms_passes": [round(x * 1e3, 4) for x in ts],
                                          "timing": f"HIP events around each whole pass (144 launches), median of "
                                                    f"{PASSES}; outputs preallocated"}
    del preps
    res["qwen3_30b_a3b_experts_nvfp4"] = nvfp4_experts_leg(ops, QuantizationArgs, layers, dev)
    del layers
    torch.cuda.empty_cache()
    return res


NV_B_PER_PARAM = 2 + 0.5 + 1 / 16  # NVFP4: read 2 B + packed E2M1 0.5 B + one e4m3 scale per 16


def nvfp4_experts_leg(ops, QuantizationArgs, layers, dev):
    """The reference's own Qwen3-30B-A3B recipe (configs/recipes/recipe_MoE_RTN_NVFP4.yaml:16-21
    -> NVFP4: E2M1 codes, e4m3 group-16 scales, one f32 global scale per expert linear): every
    expert weight of the 48 layers (4 resident fused layers rotated, as the MXFP4 leg) through
    the fused NVFP4 path (qz_quantize_nvfp4 -> k_nv_absmax + k_nv_encode, two launches per fused
    parameter, no fills; the parameters round-robin over 2 streams as CompressionPlan issues them,
    ops.quantize_nvfp4_many; one stream reported beside it), outputs preallocated.  HIP events on the launch stream around one whole
    pass (288 launches back to back); the generic qz_quantize path (absmax pre-pass, global-scale
    launch, group kernel: five launches) timed the same way beside it.  Algorithmic bytes per
    param = 2.5625 (+ 4 B per expert linear); the path reads every weight twice (the global
    scale needs the whole slice first), so ``streamed_frac`` also prices the
    second read (4.5625 B per param)."""
    import ctypes
    from quantizers_amd import _lib
    nv = QuantizationArgs(num_bits=4, type="float", strategy="tensor_group", group_size=16,
                          scale_dtype="float8_e4m3fn")
    views = [(li, j, w) for li, (gu, dn) in enumerate(layers) for j, w in enumerate((gu[:, :768], gu[:, 768:], dn))]
    outs = {(li, j): ops.alloc_outputs(tuple(w.shape), nv, None, dev) for li, j, w in views}
    lib = _lib.load()
    ca = nv.to_c()
    ws = torch.empty(lib.qz_quantize_workspace_size(128, 2048, 768, ctypes.byref(ca)) + 256, dtype=torch.uint8,
                     device=dev)

    items = [(w, outs[(lj, j)]) for li in range(48) for lj, j, w in views[(li % 4) * 3:(li % 4) * 3 + 3]]

    def fused():  # as CompressionPlan issues NVFP4 parameters: round-robin over 2 streams
        ops.quantize_nvfp4_many(items, nv)

    def fused_one_stream():
        ops.quantize_nvfp4_many(items, nv, n_streams=1)

    def two_pass():
        for li in range(48):
            for lj, j, w in views[(li % 4) * 3:(li % 4) * 3 + 3]:
                b, r, c, ld_r, ld_b = ops._geom(w)
                o = outs[(lj, j)]
                rc = lib.qz_quantize(ops._ptr(w), b, r, c, ld_r, ld_b, ctypes.byref(ca), _lib.QZ_OUT_FP4_PACKED,
                                     ops._ptr(o["codes"]), ops._ptr(o["scale"]), ops._ptr(None),
                                     ops._ptr(o["global_scale"]), ops._ptr(ws), ws.numel(), ops._stream())
                _lib.check(rc, "qz_quantize")
    npar = 48 * 128 * 3 * 768 * 2048
    nb = npar * NV_B_PER_PARAM + 48 * 3 * 128 * 4
    res = {"params": npar, "alg_bytes": nb, "kernel": "k_nv_absmax<false> + k_nv_encode<false> (qz_quantize_nvfp4)",
           "recipe": "reference configs/recipes/recipe_MoE_RTN_NVFP4.yaml (scheme NVFP4)",
           "timing": "HIP events around each whole pass (144 fused parameters back to back), median of 7"}
    st = torch.cuda.current_stream(dev)
    for name, fn in (("fused", fused), ("fused_one_stream", fused_one_stream), ("two_pass", two_pass)):
        best, _ = _event_median(fn, st, passes=7)
        gbps = nb / best / 1e9
        leg = {"ms": best * 1e3, "params_per_s": npar / best, "alg_GBps": gbps, "frac": gbps / HBM_PEAK_GBS,
               "read_frac": npar * 2 / best / 1e9 / HBM_PEAK_GBS,
               "streamed_frac": (npar * (NV_B_PER_PARAM + 2) + 48 * 3 * 128 * 4) / best / 1e9 / HBM_PEAK_GBS}
        if name == "fused":
            res.update(leg)
        elif name == "fused_one_stream":
            res["one_stream"] = leg
        else:
            res["two_pass_qz_quantize"] = leg
    del outs
    return res


def minimax_pass(ops, QuantizationArgs, dev, gen, world, rank):
    """BASELINE.json configs[4]: MiniMax-M2.1 mixed precision (recipe_Minimax-M2.1-AWQ-MixedPrec):
    62 layers x {256 experts x (w1, w3 [1536, 3072], w2 [3072, 1536]) int4 sym g32, attention
    q [6144, 3072], k/v [1024, 3072], o [3072, 6144] FP8 g32}, layers sharded round-robin over the
    ranks (strong scaling: the model is fixed).  Two resident synthetic layers are rotated (the
    whole bf16 model, 460 GB, exceeds one GPU).  Timed between barriers, max over ranks."""
    i4 = QuantizationArgs(num_bits=4, type="int", symmetric=True, group_size=32)
    f8 = QuantizationArgs(num_bits=8, type="float", symmetric=True, group_size=32)
    n_layers, n_exp, hid, inter = 62, 256, 3072, 1536
    attn = [(6144, hid), (1024, hid), (1024, hid), (hid, 6144)]
    mine = [l for l in range(n_layers) if l % world == rank]
    res_layers = []
    for _ in range(2):
        gu = (torch.randn(n_exp, 2 * inter, hid, device=dev, generator=gen) * 0.02).to(torch.bfloat16)
        dn = (torch.randn(n_exp, hid, inter, device=dev, generator=gen) * 0.02).to(torch.bfloat16)
        at = [(torch.randn(r, c, device=dev, generator=gen) * 0.02).to(torch.bfloat16) for r, c in attn]
        res_layers.append((gu, dn, at))

    # every launch prepared once (outputs preallocated, arguments marshalled): one ctypes call each
    launches = []
    for gu, dn, at in res_layers:
        lay = [(w, i4) for w in (gu[:, :inter], gu[:, inter:], dn)] + [(w, f8) for w in at]
        launches.append([(w, ops.PreparedQuantize(w, a, ops.alloc_outputs(tuple(w.shape), a, None, dev)))
                         for w, a in lay])
    stream = torch.cuda.current_stream(dev)

    def run():
        for j, _ in enumerate(mine):
            for w, prep in launches[j % 2]:
                prep.run(w, stream)

    if world > 1:
        dist.barrier()
    t, ts = _event_median(run, stream) if mine else (0.0, [])
    if world > 1:
        dist.barrier()
    t = torch.tensor([t], device=dev, dtype=torch.float64)
    if world > 1:
        _all_reduce_max(t)
    t = t.item()
    del launches
    p_exp = n_layers * n_exp * 3 * inter * hid
    p_att = n_layers * sum(r * c for r, c in attn)
    del res_layers
    torch.cuda.empty_cache()
    return {"params": p_exp + p_att, "ms": t * 1e3, "params_per_s": (p_exp + p_att) / t, "ranks": world,
            "alg_GBps": (p_exp * (2 + 0.5 + 2 / 32) + p_att * (2 + 1 + 2 / 32)) / t / 1e9,
            "frac": (p_exp * (2 + 0.5 + 2 / 32) + p_att * (2 + 1 + 2 / 32)) / t / 1e9 / HBM_PEAK_GBS / world,
            "ms_passes_this_rank": [round(x * 1e3, 4) for x in ts],
            "timing": f"HIP events around each pass of the rank's layers (7 launches per layer, outputs "
                      f"preallocated), median of {PASSES}, max over ranks",
            "sharding": "layers round-robin over ranks (strong scaling)"}


def _all_reduce_max(t):
    if dist.get_backend() == "gloo" and t.is_cuda:
        h = t.cpu()
        dist.all_reduce(h, op=dist.ReduceOp.MAX)
        t.copy_(h)
    else:
        dist.all_reduce(t, op=dist.ReduceOp.MAX)


def _all_gather_into(out, inp):
    if dist.get_backend() == "gloo":
        parts = [torch.empty_like(inp, device="cpu") for _ in range(dist.get_world_size())]
        dist.all_gather(parts, inp.cpu())
        out.copy_(torch.cat([p.reshape(-1) for p in parts]).view_as(out))
    else:
        dist.all_gather_into_tensor(out, inp)


def awq_kernels(ops, QuantizationArgs, copies, dev, gen, stream, n=60):
    """The AWQ kernels on the headline weight shape, each with its
    algorithmic bytes and achieved HBM GB/s (rotating the HBM-resident weight copies).

    Each kernel is timed as ``n`` launches back to back between ONE pair of HIP events on the
    launch stream, the C ABI called through pre-marshalled ctypes arguments (a few us of host
    time per launch, less than a kernel), so the GPU never waits for the host: us = the steady
    time per launch, including the gap between launches.  (Bracketing each launch with its own
    event pair, as the round-2 bench did, also timed the GPU waiting for the next Python call.)"""
    import ctypes
    from quantizers_amd import _lib
    lib = _lib.load()
    P = ctypes.c_void_p
    st = P(stream.cuda_stream)
    a = QuantizationArgs(num_bits=BITS, type="int", symmetric=True, group_size=GROUP)
    ca = a.to_c()
    nc = len(copies)
    s = torch.rand(COLS, device=dev, generator=gen) + 0.5
    fq_out = torch.empty_like(copies[0])
    fq_ws = ops.workspace(lib.qz_quantize_workspace_size(1, ROWS, COLS, ctypes.byref(ca)) + 256, dev)
    x = [(torch.randn(16384, COLS, device=dev, generator=gen)).to(torch.bfloat16) for _ in range(4)]
    sums = torch.zeros(COLS, dtype=torch.float32, device=dev)
    wsum = torch.zeros(COLS, dtype=torch.float64, device=dev)
    with torch.cuda.stream(stream):
        ws_a = ops.stats_workspace(lib.qz_awq_absmean_workspace_size(16384, COLS) + 256, dev)
        ws_w = ops.stats_workspace(lib.qz_awq_weight_mean_workspace_size(ROWS, COLS, GROUP) + 256, dev)
    wp = [P(c.data_ptr()) for c in copies]
    xp = [P(t.data_ptr()) for t in x]

    def ok(rc):
        if rc:
            _lib.check(rc, "bench awq kernel")

    res = {}
    for name, fn, nbytes in [
        ("fake_quant_scaled (a5: Q(W*s)/s, int4 g128)",
         lambda i: ok(lib.qz_awq_fake_quant(wp[i % nc], 1, ROWS, COLS, COLS, PARAMS, ctypes.byref(ca), P(s.data_ptr()),
                                            P(fq_out.data_ptr()), P(fq_ws.data_ptr()), fq_ws.numel(), st)),
         PARAMS * 4 + COLS * 4),
        ("absmean_accum (a3: sum|x| over [16384, 4096] activations)",
         lambda i: ok(lib.qz_awq_absmean_accum(xp[i % 4], 16384, COLS, COLS, P(sums.data_ptr()), P(ws_a.data_ptr()),
                                               ws_a.numel(), st)), x[0].numel() * 2),
        ("weight_mean_accum (a4: |W|/group absmax, g128)",
         lambda i: ok(lib.qz_awq_weight_mean_accum(wp[i % nc], ROWS, COLS, COLS, GROUP, P(wsum.data_ptr()),
                                                   P(ws_w.data_ptr()), ws_w.numel(), st)), PARAMS * 2),
        ("scale_columns (a6: W[:, c] *= s[c])",
         lambda i: ok(lib.qz_scale_columns(wp[i % nc], ROWS, COLS, COLS, P(s.data_ptr()), i & 1, st)), PARAMS * 4),
    ]:
        def batch(fn=fn):
            for i in range(n):
                fn(i)
        t, _ = _event_median(batch, stream, passes=9)
        us = t * 1e6 / n
        res[name] = {"us": us, "alg_bytes": nbytes, "GBps": nbytes / (us * 1e-6) / 1e9,
                     "frac": nbytes / (us * 1e-6) / 1e9 / HBM_PEAK_GBS,
                     "timing": f"{n} launches back to back between one event pair, median of 9 such passes"}
    del x
    return res


def awq_oneshot_layers(dev, n_layers=3, n_seq=16, seq=2048):
    """BASELINE.json configs[1] end to end on a truncated model: Qwen3-4B (public dims, random
    bf16 weights: no checkpoint offline) with ``n_layers`` decoder layers, the AWQ int4-g128
    recipe, ``n_seq`` x ``seq`` random calibration tokens, through ``quantizers_amd.oneshot``
    (capture layer-0 inputs, per layer: activation statistics, 20-point grid search with the
    fused fake-quant kernel and the parent forwards, smoothing, propagation)."""
    from transformers import AutoConfig, AutoModelForCausalLM
    from quantizers_amd.oneshot import oneshot
    cfg = AutoConfig.from_pretrained(os.path.join(ROOT, "configs", "models", "qwen3-4b"))
    cfg.num_hidden_layers = n_layers
    torch.manual_seed(0)
    with torch.device(dev):
        model = AutoModelForCausalLM.from_config(cfg, dtype=torch.bfloat16)
    g = torch.Generator().manual_seed(42)
    data = [{"input_ids": torch.randint(0, cfg.vocab_size, (seq,), generator=g)} for _ in range(n_seq)]
    recipe = os.path.join(ROOT, "configs", "recipes", "awq_w4a16_g128.yaml")
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    oneshot(model=model, recipe=recipe, dataset=data, max_seq_length=seq, num_calibration_samples=n_seq, device=dev)
    torch.cuda.synchronize()
    t = time.perf_counter() - t0
    rep = model.awq_report
    n_map = sum(len(v) for v in rep.values())
    per_layer = list(model.awq_layer_seconds)
    del model
    torch.cuda.empty_cache()
    steady = sum(per_layer[1:]) / max(len(per_layer) - 1, 1)
    return {"model": "Qwen3-4B dims, random bf16 weights", "layers": n_layers, "calibration_tokens": n_seq * seq,
            "mappings": n_map, "s_total": t, "s_per_layer_logged": per_layer, "s_per_steady_layer": steady,
            "projected_36_layers_s": t + (36 - n_layers) * steady,
            "how": "wall clock of oneshot() on the truncated model (layer-0 input capture and first-call setup "
                   "included once); projection = that + the remaining layers at the mean of layers 1..n-1",
            "recipe": "configs/recipes/awq_w4a16_g128.yaml"}


def build_model(dev, recipe=RECIPE):
    """A Qwen3-4B-shaped causal LM (configs/models/qwen3-4b: public dims, 36 layers) with random
    bf16 weights on ``dev``, its targeted modules resolved from ``recipe`` (default: the AWQ
    int4-g128 recipe) exactly as ``oneshot`` resolves them."""
    from transformers import AutoConfig, AutoModelForCausalLM
    from quantizers_amd.oneshot import resolve_schemes
    from quantizers_amd.recipe import parse_recipe
    cfg = AutoConfig.from_pretrained(MODEL_CFG)
    with torch.device(dev):
        model = AutoModelForCausalLM.from_config(cfg, dtype=torch.bfloat16)
    schemes = resolve_schemes(model, parse_recipe(recipe))
    model.quantization_scheme_map = {n: s for n, (s, _) in schemes.items()}
    return model


def synthetic_leg(ops, QuantizationArgs, dev, gen, stream, copies_n, k):
    """North-star synthetic weight [11008, 4096] int4-g128: K weights (rotating over ``copies_n``
    HBM-resident copies, 1.08 GB) into K distinct output sets, as ONE grouped launch and as K
    per-weight launches (qz_quantize_many), each after its own warmup, HIP-event timed."""
    a = QuantizationArgs(num_bits=BITS, type="int", symmetric=True, strategy="group", group_size=GROUP)
    copies = [(torch.randn(ROWS, COLS, device=dev, generator=gen) * 0.02).to(torch.bfloat16)
              for _ in range(copies_n)]
    ws = [copies[i % copies_n] for i in range(k)]
    outs = [ops.alloc_outputs((ROWS, COLS), a, None, dev) for _ in range(k)]
    gq = ops.GroupedQuantize(ws, a, outs=outs)
    prep = ops.PreparedQuantize(copies[0], a, ops.alloc_outputs((ROWS, COLS), a, None, dev))
    many = prep.prepare_many(ws, outs=outs)
    res = {}
    for name, fn, launches in (("grouped", lambda: gq.run(stream), 1), ("per_weight", lambda: many(stream), k)):
        t, ts = _event_median(fn, stream, passes=max(PASSES, 7), warm=3)
        us_w = t * 1e6 / k
        gbps = ALG_BYTES / (us_w * 1e-6) / 1e9
        res[name] = {"kernel": kernel_name(name == "grouped", (k if name == "grouped" else 1) * PARAMS * 2),
                     "weights": k, "launches": launches, "us_per_weight": us_w, "params_per_s": PARAMS / (us_w * 1e-6),
                     "achieved_GBps": gbps, "frac": gbps / HBM_PEAK_GBS,
                     "us_per_weight_passes": [round(x * 1e6 / k, 3) for x in ts],
                     "timing": f"HIP events around each pass ({k} weights), median of {len(ts)} passes"}
    check = (copies[(k - 1) % copies_n][:256].cpu(), outs[k - 1]["codes"][:256].cpu(), outs[k - 1]["scale"][:256].cpu())
    del gq, many, prep, outs, ws
    return res, copies, check


def row_blocks(rows: int, world: int, align: int = 8):
    """BASELINE.md §2's multi-GPU split of one weight: ``world`` contiguous row blocks of equal
    height (a multiple of ``align`` rows, so an asymmetric zero point packed along dim 0 stays
    word-aligned), the last ones possibly short or empty: [(r0, r1)] per rank, and the padded
    block height every rank's all-gather slot has."""
    blk = -(-rows // world)
    blk = -(-blk // align) * align
    return [(min(r * blk, rows), min((r + 1) * blk, rows)) for r in range(world)], blk


def row_sharded_leg(ops, QuantizationArgs, dev, stream, world, rank, reps=7):
    """BASELINE.md §2 multi-GPU row: the north-star synthetic weight [11008, 4096] int4-g128 split
    into ``world`` row blocks (``row_blocks``), rank r quantizing block r (strong scaling: the
    weight is fixed).  Every rank generates the same copies (seeded), keeps only its block.

    * kernel-only: ONE grouped launch over ``n`` distinct copies of the rank's block (n x block
      bytes >= 1 GB, beyond the 256 MiB Infinity Cache), HIP events on the launch stream, median
      of ``reps``; aggregate params/s = 11008 x 4096 / (max over ranks of the time per copy);
    * end-to-end: per copy, the rank's block quantized (one launch) and the packed codes and
      scales reassembled on EVERY rank by ``all_gather_into_tensor`` into the full
      [11008, 512] int32 / [11008, 32] bf16 tensors (RCCL over xGMI); wall clock between
      barriers, max over ranks;
    * check: the gathered tensors of copy 0 equal one single-GPU quantize of the whole copy 0,
      bit for bit (rank 0)."""
    a = QuantizationArgs(num_bits=BITS, type="int", symmetric=True, strategy="group", group_size=GROUP)
    blocks, blk = row_blocks(ROWS, world)
    r0, r1 = blocks[rank]
    mine = r1 - r0
    blk_bytes = max(blk, 8) * COLS * 2
    n = max(4, min(128, -(-(1 << 30) // blk_bytes)))
    copies = []
    for i in range(n):
        g = torch.Generator(device=dev).manual_seed(5000 + i)
        full = (torch.randn(ROWS, COLS, device=dev, generator=g) * 0.02).to(torch.bfloat16)
        copies.append(full[r0:r1].clone() if mine else None)
        del full
    res = {"split": f"{world} row blocks of {blk} rows (rank {rank}: rows {r0}-{r1})", "copies": n,
           "weight": f"[{ROWS}, {COLS}] int4 sym g{GROUP}"}
    # kernel-only: one grouped launch over the n copies of this rank's block
    us_copy = 0.0
    if mine:
        outs = [ops.alloc_outputs((mine, COLS), a, None, dev) for _ in range(n)]
        gq = ops.GroupedQuantize(copies, a, outs=outs)
        us_copy = _event_median(lambda: gq.run(stream), stream, passes=reps, warm=3)[0] * 1e6 / n
        del gq, outs
    t = torch.tensor([us_copy], device=dev, dtype=torch.float64)
    if world > 1:
        _all_reduce_max(t)
    us_max = t.item()
    alg_rank = mine * COLS * 2.515625
    res["kernel_only"] = {"us_per_copy_max_rank": us_max, "us_per_copy_this_rank": us_copy,
                          "params_per_s": PARAMS / (us_max * 1e-6),
                          "per_gpu_GBps": alg_rank / (us_copy * 1e-6) / 1e9 if us_copy else None,
                          "per_gpu_frac": alg_rank / (us_copy * 1e-6) / 1e9 / HBM_PEAK_GBS if us_copy else None,
                          "per_gpu_read_frac": mine * COLS * 2 / (us_copy * 1e-6) / 1e9 / HBM_PEAK_GBS
                          if us_copy else None,
                          "how": "one grouped launch over the copies of this rank's block, HIP events, median"}
    # end to end: quantize the block, all-gather codes + scales into the full tensors
    codes_blk = torch.zeros(blk, COLS // 8, dtype=torch.int32, device=dev)
    scale_blk = torch.zeros(blk, COLS // GROUP, dtype=torch.bfloat16, device=dev)
    codes_full = torch.empty(world * blk, COLS // 8, dtype=torch.int32, device=dev)
    scale_full = torch.empty(world * blk, COLS // GROUP, dtype=torch.bfloat16, device=dev)
    prep = ops.PreparedQuantize(copies[0], a, {"codes": codes_blk[:mine], "scale": scale_blk[:mine]}) \
        if mine else None

    def one(i):
        if prep is not None:
            prep.run(copies[i % n], stream)
        if world > 1:
            _all_gather_into(codes_full, codes_blk)
            _all_gather_into(scale_full, scale_blk)

    for i in range(3):
        one(i)
    k = min(n, 32)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    t0 = time.perf_counter()
    for i in range(k):
        one(i)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    t = torch.tensor([(time.perf_counter() - t0) / k], device=dev, dtype=torch.float64)
    if world > 1:
        _all_reduce_max(t)
    e2e = t.item()
    res["end_to_end"] = {"us_per_copy": e2e * 1e6, "params_per_s": PARAMS / e2e,
                         "gathered_bytes_per_copy": world * blk * (COLS // 8 * 4 + COLS // GROUP * 2),
                         "how": "per copy: the block's quantize launch + all_gather_into_tensor of the packed codes "
                                "and the scales into the full tensors on every rank; wall clock between barriers, "
                                "max over ranks" + ("" if world > 1 else " (1 rank: nothing to gather)")}
    # bit-exact check of the reassembled copy 0 against one whole-weight quantize
    one(0)
    torch.cuda.synchronize()
    ok = None
    if rank == 0:
        g = torch.Generator(device=dev).manual_seed(5000)
        full = (torch.randn(ROWS, COLS, device=dev, generator=g) * 0.02).to(torch.bfloat16)
        ref = ops.quantize_weight(full, a)
        got_c = codes_full[:ROWS] if world > 1 else codes_blk[:ROWS]
        got_s = scale_full[:ROWS] if world > 1 else scale_blk[:ROWS]
        ok = bool(torch.equal(ref["codes"], got_c) and torch.equal(ref["scale"].view(torch.int16),
                                                                    got_s.view(torch.int16)))
        del full, ref
    res["gathered_equals_single_gpu"] = ok
    del copies, codes_full, scale_full, prep
    torch.cuda.empty_cache()
    return res


def strong_model_leg(units, dev, stream, world, rank, steps=10):
    """The product's sharded whole-model compression (strong scaling: ONE Qwen3-4B, its 252
    linears assigned to ranks by ``distributed.plan_shards`` -- LPT on bytes, as
    ``compressed_state_dict`` does -- each rank running its share as grouped launches), then the
    compressed state dict reassembled on every rank by ``distributed.gather_state`` (one RCCL
    ``all_gather_into_tensor`` into the result buffer).

    * kernel-only: HIP events around ``steps`` runs of the rank's share, max over ranks;
    * end-to-end: ``steps`` x (the share's launches + ``gather_state``), wall clock between
      barriers, max over ranks."""
    from quantizers_amd.compressor import CompressionPlan
    from quantizers_amd.distributed import gather_state, plan_shards
    shards = plan_shards([(str(i), u.nbytes) for i, u in enumerate(units)], world)
    mine = [units[int(i)] for i in shards[rank]]
    total = sum(u.nbytes // 2 for u in units)
    plan = CompressionPlan(mine, dev) if mine else None
    res = {"model_params": total, "units_total": len(units), "units_this_rank": len(mine),
           "params_this_rank": plan.params if plan else 0, "launches_this_rank": plan.launches if plan else 0}
    ms = 0.0
    if plan is not None:
        for _ in range(3):
            plan.run(stream)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(stream)
        for _ in range(steps):
            plan.run(stream)
        e1.record(stream)
        torch.cuda.synchronize()
        ms = e0.elapsed_time(e1) / steps
    t = torch.tensor([ms], device=dev, dtype=torch.float64)
    if world > 1:
        _all_reduce_max(t)
    res["kernel_only"] = {"ms_max_rank": t.item(), "ms_this_rank": ms, "params_per_s": total / (t.item() * 1e-3),
                          "how": "HIP events around the rank's share (grouped launches), max over ranks"}
    local = plan.tensors() if plan is not None else {}
    local = {k: v for k, v in local.items() if v.is_cuda}  # weight_shape stays on the host
    nbytes = sum(v.numel() * v.element_size() for v in local.values())

    def one():
        if plan is not None:
            plan.run(stream)
        return gather_state(local)  # RCCL: device buffers; gloo rehearsal: through the host

    got = one()
    n_got = len(got)
    del got
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    t0 = time.perf_counter()
    for _ in range(steps):
        got = one()
        del got
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    t = torch.tensor([(time.perf_counter() - t0) / steps], device=dev, dtype=torch.float64)
    if world > 1:
        _all_reduce_max(t)
    res["end_to_end"] = {"ms": t.item() * 1e3, "params_per_s": total / t.item(), "tensors_on_every_rank": n_got,
                         "compressed_bytes_this_rank": nbytes,
                         "how": "per step: the rank's share + distributed.gather_state (all_gather_into_tensor of "
                                "every rank's flat compressed bytes into the result buffer on every rank); wall clock "
                                "between barriers, max over ranks"}
    del plan, local
    torch.cuda.empty_cache()
    return res


def _spawn_ranks(n: int) -> int:
    """``--gpus N`` outside a torchrun environment: run N rank processes of this script under
    ``torch.distributed.run`` as a CHILD process (this process never initialises the GPU and
    never execs) and return their exit status."""
    import socket
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}",
           "--master-addr=127.0.0.1", f"--master-port={port}", os.path.abspath(__file__)] + sys.argv[1:]
    return subprocess.call(cmd)


def launch_check(world, rank, backend):
    """``--launch-check``: join the process group, census the ranks, print one JSON line on rank
    0 and exit -- the rank plumbing of ``--gpus N`` without touching a GPU (CPU-testable)."""
    dist.init_process_group("gloo")
    seen = [None] * dist.get_world_size()
    dist.all_gather_object(seen, {"rank": rank, "local_rank": int(os.environ.get("LOCAL_RANK", "0")),
                                  "pid": os.getpid()})
    if rank == 0:
        print(json.dumps({"launch_check": True, "n_gpus": world, "ranks_seen": dist.get_world_size(),
                          "ranks": seen, "backend_for_run": backend}), flush=True)
    dist.barrier()
    dist.destroy_process_group()


def main():
    args = parse()
    env_world = os.environ.get("WORLD_SIZE")
    if env_world is None and (args.gpus or 1) > 1:
        sys.exit(_spawn_ranks(args.gpus))  # the ranks print the line; nothing here touches the GPU
    world = int(env_world or "1")
    if args.gpus is not None and args.gpus != world:
        print(f"bench.py: --gpus {args.gpus} but WORLD_SIZE={world}: refusing to report an n_gpus the run "
              f"does not have", file=sys.stderr)
        sys.exit(2)
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    # QZ_BENCH_BACKEND=gloo: rehearsal of the multi-rank code path on a box with fewer GPUs than
    # ranks (ranks share devices, collectives go through host memory); the driver's N-GPU runs
    # use the default RCCL ("nccl") backend, one rank per GPU.
    backend = os.environ.get("QZ_BENCH_BACKEND", "nccl")
    if args.launch_check:
        launch_check(world, rank, backend)
        return
    n_dev = torch.cuda.device_count()  # counts devices without initialising the GPU
    if backend == "gloo":
        local = local % max(n_dev, 1)
    elif world > 1 and n_dev < world:
        print(f"bench.py: {world} ranks need {world} GPUs for RCCL, {n_dev} visible "
              f"(QZ_BENCH_BACKEND=gloo rehearses the ranks on fewer)", file=sys.stderr)
        sys.exit(2)
    if world > 1:
        torch.cuda.set_device(local)
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))
        else:
            dist.init_process_group(backend)
    dev = torch.device("cuda", local)
    torch.cuda.set_device(dev)

    from quantizers_amd import ops
    from quantizers_amd.compressor import CompressionPlan, compression_units
    from quantizers_amd.quantization import QuantizationArgs

    phases = {}  # per-rank wall seconds by phase (max over ranks goes in the line)
    t_phase = [T_START]

    def stamp(name):
        now = time.perf_counter()
        phases[name] = phases.get(name, 0.0) + now - t_phase[0]
        t_phase[0] = now

    stamp("start_to_device")
    torch.manual_seed(1234 + rank)
    model = build_model(dev)
    units, _ = compression_units(model)
    plan = CompressionPlan(units, dev)  # every pointer table / output built before timing
    stream = torch.cuda.current_stream(dev)
    params_step = plan.params
    alg_step = plan.alg_bytes()
    launches_step = plan.launches

    def region(k):
        """barrier + sync, exactly k steps, sync + barrier: (wall s max over ranks, event ms)."""
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        if world > 1:
            dist.barrier()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        e0.record(stream)
        for _ in range(k):
            plan.run(stream)
        e1.record(stream)
        torch.cuda.synchronize()
        if world > 1:
            dist.barrier()
        wall = torch.tensor([time.perf_counter() - t0], device=dev, dtype=torch.float64)
        if world > 1:
            _all_reduce_max(wall)
        return wall.item(), e0.elapsed_time(e1)

    stamp("model_and_plan")
    for _ in range(args.warmup):
        plan.run(stream)
    el, ev_ms = region(args.steps)
    stamp("headline")
    if args.profile_only:
        return

    # steady state of the same plan (informational, never `value`): 100 steps after 50 more; equal
    # to the timed region at the default W = 50 (the clocks settle about 25 steps into a load,
    # profiles/r05j_step_ramp.log); a short W's timed region reads slower than it
    for _ in range(50):
        plan.run(stream)
    s0, s1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s0.record(stream)
    for _ in range(100):
        plan.run(stream)
    s1.record(stream)
    torch.cuda.synchronize()
    steady_ms = s0.elapsed_time(s1) / 100
    steady = {"warmup_steps": 50, "steps": 100, "event_ms_per_step": steady_ms,
              "params_per_s": params_step / (steady_ms * 1e-3),
              "frac": alg_step / (steady_ms * 1e-3) / 1e9 / HBM_PEAK_GBS,
              "how": "HIP events around 100 steps after 50 more untimed ones, right after the timed region; "
                     "informational (value and roofline use the W / K given)"}

    # per-launch durations (untimed, after the regions above): each launch 10 times back to back
    # between one event pair, median of 7 such passes (_launch_us)
    per_launch = []
    for gq, part, *_ in plan.grouped:
        nb = sum(w.numel() * 2 for _, w in part) + sum(t.numel() * t.element_size() for o in gq.outs
                                                         for t in o.values() if t is not None)
        us = _launch_us(gq, stream)
        rb = sum(w.numel() * 2 for _, w in part)
        per_launch.append({"shapes": sorted({f"{r}x{c}" for r, c in gq.shapes}), "weights": gq.n,
                           "us": us, "alg_bytes": nb, "read_bytes": rb,
                           "GBps": nb / (us * 1e-6) / 1e9, "frac": nb / (us * 1e-6) / 1e9 / HBM_PEAK_GBS,
                           "read_frac": rb / (us * 1e-6) / 1e9 / HBM_PEAK_GBS})

    checks = []
    if rank == 0:  # the measured outputs of one module per shape, checked in the CPU leg
        for gq, part, *_ in plan.grouped:
            w = part[0][1]
            checks.append((w[:64].cpu(), gq.outs[0]["codes"][:64].cpu(), gq.outs[0]["scale"][:64].cpu()))

    # multi-GPU legs (BASELINE.md §2 multi-GPU row; north star: RCCL all-gather over xGMI), run at
    # every N so the driver's 1/2/4/8-GPU lines carry comparable fields
    ranks_seen = dist.get_world_size() if world > 1 else 1
    stamp("per_launch_and_checks")
    strong = strong_model_leg(units, dev, stream, world, rank, steps=10 if backend == "nccl" else 2)
    stamp("strong_scaling_leg")
    row_sharded = row_sharded_leg(ops, QuantizationArgs, dev, stream, world, rank)
    stamp("row_sharded_leg")
    # PCIe-inclusive rate (not the headline): what save_compressed pays per model on one GPU --
    # the same plan, then every output tensor copied to pinned host memory (_HostCopier: side
    # stream, one device->host copy per tensor).  One warm run first (pinned-host allocator).
    pcie = None
    if world == 1 and not args.no_extras:
        from quantizers_amd.compressor import _HostCopier

        def to_host():
            plan.run(stream)
            hc = _HostCopier(dev)
            h = hc.submit(plan.tensors())
            hc.finish()
            return h

        to_host()
        torch.cuda.synchronize()
        tp = time.perf_counter()
        host = to_host()
        torch.cuda.synchronize()
        dt = time.perf_counter() - tp
        d2h = sum(t.numel() * t.element_size() for t in host.values())
        pcie = {"ms": dt * 1e3, "params_per_s": params_step / dt, "d2h_bytes": d2h, "d2h_GBps": d2h / dt / 1e9,
                "how": "one whole-model CompressionPlan step + device->pinned-host copies of all outputs "
                       "(compressor._HostCopier), wall clock"}
        del host
    del plan, units, model
    torch.cuda.empty_cache()

    extras = {}
    cpu_check = None
    if not args.no_extras:
        gen = torch.Generator(device=dev).manual_seed(99 + rank)
        syn, copies, cpu_check = synthetic_leg(ops, QuantizationArgs, dev, gen, stream, args.copies, 100)
        extras["north_star_synthetic_11008x4096"] = syn
        extras["awq_kernels"] = awq_kernels(ops, QuantizationArgs, copies, dev, gen, stream)
        del copies
        torch.cuda.empty_cache()
        if world == 1:
            extras["awq_oneshot_qwen3_4b"] = awq_oneshot_layers(dev)
        other = other_configs(ops, QuantizationArgs, dev, gen, stream)
        other["minimax_m2_1_mixedprec_sharded"] = minimax_pass(ops, QuantizationArgs, dev, gen, world, rank)
        extras["other_configs"] = other

    stamp("extras")
    cpu, ok = None, None
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        cpu, ok = cpu_baseline(args.cpu_seconds, checks + ([cpu_check] if cpu_check else []))
    stamp("cpu_baseline")
    names = sorted(phases)
    pt = torch.tensor([phases[k] for k in names], device=dev, dtype=torch.float64)
    if world > 1:
        _all_reduce_max(pt)
    phase_max = dict(zip(names, [round(v, 3) for v in pt.tolist()]))
    print(f"bench.py rank {rank}/{world}: phase seconds {json.dumps({k: round(v, 3) for k, v in phases.items()})}",
          file=sys.stderr, flush=True)

    if rank == 0:
        value = world * params_step * args.steps / el
        ev_s = ev_ms * 1e-3
        achieved = alg_step * args.steps / ev_s / 1e9
        # HBM traffic per launch from the committed PMC passes of this same plan
        # (scripts/pmc_headline.sh -> profiles/headline_pmc.json); null when absent or stale
        traffic, traffic_src = None, None
        pmc_path = os.path.join(ROOT, "profiles", "headline_pmc.json")
        if os.path.exists(pmc_path):
            pmc = json.load(open(pmc_path))
            if pmc.get("alg_bytes_per_step") == alg_step and pmc.get("launches_per_step") == launches_step:
                traffic = pmc["hbm_bytes_per_launch"]
                traffic_src = (f"committed PMC passes, not re-read in this run: profiles/headline_pmc.json "
                               f"({pmc['tag']}), FETCH_SIZE x2 + WRITE_SIZE per launch of this same plan, "
                               f"{pmc['traffic_over_algorithmic']:.4f} x algorithmic")
        line = {
            "metric": METRIC,
            "value": value,
            "unit": "params/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": el / args.steps * 1e3,
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "bf16",
            "data": "synthetic: random-init bf16 weights of the public Qwen3-4B dims (no checkpoint offline)",
            "config": {"workload": "int4 sym group_size=128 quantize+pack (pack-quantized) of all 252 Qwen3-4B linears "
                                   "per step via compressor.CompressionPlan (the save_compressed launch plan)",
                       "model": "Qwen3-4B dims, 36 layers", "params_per_step": params_step,
                       "group_size": GROUP, "num_bits": BITS, "recipe": "configs/recipes/awq_w4a16_g128.yaml",
                       "parallelism": f"weight-shard dp{world}"},
            "hbm_GBps_step": world * alg_step * args.steps / el / 1e9,
            "roofline": {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": achieved / HBM_PEAK_GBS,
                         # the north star's "HBM-read roofline" reading: weight bytes read only
                         "read_frac": params_step * 2 * args.steps / ev_s / 1e9 / HBM_PEAK_GBS,
                         "read_achieved": params_step * 2 * args.steps / ev_s / 1e9,
                         "frac_definition": "frac = algorithmic read + write bytes (SURVEY §8d) / kernel time / "
                                            "8 TB/s; read_frac = weight bytes read / kernel time / 8 TB/s",
                         "traffic": traffic, "traffic_source": traffic_src,
                         "kernel": kernel_name(True, 36 * 9728 * 2560 * 2),
                         "kernel_ms_mean": ev_ms / (args.steps * launches_step),
                         "launches_per_step": launches_step, "alg_bytes_per_step": alg_step,
                         "alg_bytes_per_launch": alg_step / launches_step,
                         "kernel_timing": "HIP events on the launch stream around the same K steps as value "
                                          "(K x launches_per_step grouped launches back to back) / launches",
                         "event_ms_per_step": ev_ms / args.steps,
                         "traffic_unit": "HBM bytes per launch (alg_bytes_per_launch beside it)"},
            "per_launch": per_launch,
            "steady_state": steady,
            "cpu_baseline": cpu,
            "parity_check": ok,
            "ranks_seen": ranks_seen,
            "row_sharded_synthetic_11008x4096": row_sharded,
            "strong_scaling_qwen3_4b_sharded": strong,
            "pcie_inclusive": pcie,
            "phase_seconds_max_rank": phase_max,
            "wall_seconds_max_rank": round(sum(phase_max.values()), 3),
        }
        line.update(extras)
        print(json.dumps(line), flush=True)
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
