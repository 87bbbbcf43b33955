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
CPU baseline (the oracle's torch restatement on the host cores).  Multi-GPU: one process per GPU
(torchrun), each quantizes its own model-sized weight set (weak scaling, no collective in the
timed region); afterwards the ranks reassemble the compressed tensors with bucketed RCCL
all-gathers (``distributed.gather_state``), timed separately.

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
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=20)
    p.add_argument("--warmup", type=int, default=5)
    p.add_argument("--copies", type=int, default=12)
    p.add_argument("--cpu-seconds", type=float, default=10.0)
    p.add_argument("--no-cpu-baseline", action="store_true")
    p.add_argument("--no-extras", action="store_true", help="headline only (no secondary legs)")
    p.add_argument("--profile-only", action="store_true",
                   help="warmup + K headline steps only (rocprofv3 PMC passes); prints nothing else")
    return p.parse_args()


def cpu_baseline(seconds: float, checks=None):
    """The oracle's torch restatement of compressed-tensors (oracle/ct_torch.py), timed on the host
    cores on a bounded sample of the headline workload: repeated compress_weight calls on one
    Qwen3-4B gate_proj-shaped weight [9728, 2560] (the model's largest shape class).  The oracle
    is used only here (the CPU leg) and as the checker of ``checks`` = [(input rows, packed
    codes, scales)] taken from the GPU's measured outputs (plain-C restatement, bit for bit).

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
    rows, cols = 9728, 2560
    g = torch.Generator().manual_seed(0)
    w = (torch.randn(rows, cols, generator=g) * 0.02).to(torch.bfloat16)
    a = ct.QArgs(num_bits=BITS, type="int", symmetric=True, strategy="group", group_size=GROUP)
    ct.compress_weight(w, a)  # warm-up
    n, t0 = 0, time.perf_counter()
    while True:
        ct.compress_weight(w, a)
        n += 1
        el = time.perf_counter() - t0
        if (el >= seconds and n >= 3) or n >= 2000:
            break
    res = {"value": n * rows * cols / el, "unit": "params/s", "cores": threads, "kind": "port",
           "sample": f"oracle/ct_torch.compress_weight (compressed-tensors op sequence, torch CPU) int4-g{GROUP} on "
                     f"one Qwen3-4B gate_proj-shaped bf16 weight [{rows},{cols}], {n} calls in {el:.1f}s, torch "
                     f"threads={threads} (the box's per-GPU CPU share), os.cpu_count()={os.cpu_count()}, "
                     f"cpu='{cpu_model()}'"}
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


def _timed(fn, reps=3):
    fn()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(reps):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / reps


def other_configs(ops, QuantizationArgs, dev, gen):
    """BASELINE.json configs[2] (Qwen3-4B FP8_BLOCK attention + int4-g32 MLP) and configs[3]
    (Qwen3-30B-A3B experts -> MXFP4): one quantize pass over every targeted weight."""
    res = {}
    fp8b = QuantizationArgs(num_bits=8, type="float", strategy="block", block_structure=[128, 128])
    i4 = QuantizationArgs(num_bits=4, type="int", symmetric=True, group_size=32)
    ws = [(fp8b if n.endswith(("q_proj", "k_proj", "v_proj", "o_proj")) else i4,
           (torch.randn(QWEN3_LAYERS, r, c, device=dev, generator=gen) * 0.02).to(torch.bfloat16))
          for n, r, c in QWEN3_4B]
    npar = sum(w.numel() for _, w in ws)
    t = _timed(lambda: [ops.quantize_weight(w, a) for a, w in ws])
    res["qwen3_4b_mixed_fp8block_int4g32"] = {"params": npar, "ms": t * 1e3, "params_per_s": npar / t}
    del ws
    torch.cuda.empty_cache()
    # Qwen3-30B-A3B: 48 layers x 128 experts x {gate, up [768, 2048], down [2048, 768]}; 4 resident
    # layers (fused [E, 2I, H] / [E, H, I] parameters, gate/up as strided views) rotated over 48
    mx = QuantizationArgs(num_bits=4, type="float", group_size=32, scale_dtype="uint8")
    layers = []
    for _ in range(4):
        gu = (torch.randn(128, 2 * 768, 2048, device=dev, generator=gen) * 0.02).to(torch.bfloat16)
        dn = (torch.randn(128, 2048, 768, device=dev, generator=gen) * 0.02).to(torch.bfloat16)
        layers.append((gu, dn))

    def moe_pass():
        for li in range(48):
            gu, dn = layers[li % 4]
            ops.quantize_weight(gu[:, :768], mx)
            ops.quantize_weight(gu[:, 768:], mx)
            ops.quantize_weight(dn, mx)
    npar = 48 * 128 * 3 * 768 * 2048
    t = _timed(moe_pass, reps=2)
    res["qwen3_30b_a3b_experts_mxfp4"] = {"params": npar, "ms": t * 1e3, "params_per_s": npar / t,
                                          "alg_GBps": npar * (2 + 0.5 + 1 / 32) / t / 1e9}
    del layers
    torch.cuda.empty_cache()
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

    def run():
        for j, _ in enumerate(mine):
            gu, dn, at = res_layers[j % 2]
            ops.quantize_weight(gu[:, :inter], i4)
            ops.quantize_weight(gu[:, inter:], i4)
            ops.quantize_weight(dn, i4)
            for w in at:
                ops.quantize_weight(w, f8)

    run()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    t0 = time.perf_counter()
    reps = 2
    for _ in range(reps):
        run()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    t = torch.tensor([(time.perf_counter() - t0) / reps], device=dev, dtype=torch.float64)
    if world > 1:
        _all_reduce_max(t)
    t = t.item()
    p_exp = n_layers * n_exp * 3 * inter * hid
    p_att = n_layers * sum(r * c for r, c in attn)
    del res_layers
    torch.cuda.empty_cache()
    return {"params": p_exp + p_att, "ms": t * 1e3, "params_per_s": (p_exp + p_att) / t, "ranks": world,
            "alg_GBps": (p_exp * (2 + 0.5 + 2 / 32) + p_att * (2 + 1 + 2 / 32)) / t / 1e9,
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
        out.copy_(torch.stack(parts))
    else:
        dist.all_gather_into_tensor(out, inp)


def _event_us(fn, n, stream):
    """Mean per-launch duration (HIP events on the launch stream) of fn(i), i = 0..n-1."""
    for i in range(3):
        fn(i)
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(n)]
    for i in range(n):
        ev[i][0].record(stream)
        fn(i)
        ev[i][1].record(stream)
    torch.cuda.synchronize()
    return sum(a.elapsed_time(b) for a, b in ev) / n * 1e3


def awq_kernels(ops, QuantizationArgs, copies, dev, gen, stream):
    """The AWQ kernels on the headline weight shape, each with its
    algorithmic bytes and achieved HBM GB/s (rotating the HBM-resident weight copies)."""
    a = QuantizationArgs(num_bits=BITS, type="int", symmetric=True, group_size=GROUP)
    nc = len(copies)
    s = torch.rand(COLS, device=dev, generator=gen) + 0.5
    fq_out = torch.empty_like(copies[0])
    x = [(torch.randn(16384, COLS, device=dev, generator=gen)).to(torch.bfloat16) for _ in range(4)]
    sums = torch.zeros(COLS, dtype=torch.float32, device=dev)
    wsum = torch.zeros(COLS, dtype=torch.float64, device=dev)
    res = {}
    for name, fn, nbytes in [
        ("fake_quant_scaled (a5: Q(W*s)/s, int4 g128)",
         lambda i: ops.fake_quantize(copies[i % nc], a, col_scales=s, out=fq_out), PARAMS * 4 + COLS * 4),
        ("absmean_accum (a3: sum|x| over [16384, 4096] activations)",
         lambda i: ops.awq_absmean_accum(x[i % 4], sums), x[0].numel() * 2),
        ("weight_mean_accum (a4: |W|/group absmax, g128)",
         lambda i: ops.awq_weight_mean_accum(copies[i % nc], GROUP, wsum), PARAMS * 2),
        ("scale_columns (a6: W[:, c] *= s[c])",
         lambda i: ops.scale_columns_(copies[i % nc], s), PARAMS * 4),
    ]:
        us = _event_us(fn, 40, stream)
        res[name] = {"us": us, "alg_bytes": nbytes, "GBps": nbytes / (us * 1e-6) / 1e9}
    del x
    return res


def awq_oneshot_layers(dev, n_layers=2, n_seq=16, seq=2048):
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
    del model
    torch.cuda.empty_cache()
    return {"model": "Qwen3-4B dims, random bf16 weights", "layers": n_layers, "calibration_tokens": n_seq * seq,
            "mappings": n_map, "s_total": t, "s_per_layer": t / n_layers,
            "projected_36_layers_s": t / n_layers * 36, "recipe": "configs/recipes/awq_w4a16_g128.yaml"}


def build_model(dev):
    """A Qwen3-4B-shaped causal LM (configs/models/qwen3-4b: public dims, 36 layers) with random
    bf16 weights on ``dev``, its targeted modules resolved from the AWQ int4-g128 recipe exactly
    as ``oneshot`` resolves them."""
    from transformers import AutoConfig, AutoModelForCausalLM
    from quantizers_amd.oneshot import resolve_schemes
    from quantizers_amd.recipe import parse_recipe
    cfg = AutoConfig.from_pretrained(MODEL_CFG)
    with torch.device(dev):
        model = AutoModelForCausalLM.from_config(cfg, dtype=torch.bfloat16)
    schemes = resolve_schemes(model, parse_recipe(RECIPE))
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
        for _ in range(3):
            fn()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(stream)
        fn()
        e1.record(stream)
        torch.cuda.synchronize()
        us_w = e0.elapsed_time(e1) * 1e3 / k
        gbps = ALG_BYTES / (us_w * 1e-6) / 1e9
        res[name] = {"kernel": kernel_name(name == "grouped", (k if name == "grouped" else 1) * PARAMS * 2),
                     "weights": k, "launches": launches, "us_per_weight": us_w, "params_per_s": PARAMS / (us_w * 1e-6),
                     "achieved_GBps": gbps, "frac": gbps / HBM_PEAK_GBS}
    check = (copies[(k - 1) % copies_n][:256].cpu(), outs[k - 1]["codes"][:256].cpu(), outs[k - 1]["scale"][:256].cpu())
    del gq, many, prep, outs, ws
    return res, copies, check


def main():
    args = parse()
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    # QZ_BENCH_BACKEND=gloo: rehearsal of the multi-rank code path on a box with fewer GPUs than
    # ranks (ranks share devices, collectives go through host memory); the driver's N-GPU runs
    # use the default RCCL ("nccl") backend, one rank per GPU.
    backend = os.environ.get("QZ_BENCH_BACKEND", "nccl")
    if backend == "gloo":
        local = local % max(torch.cuda.device_count(), 1)
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

    for _ in range(args.warmup):
        plan.run(stream)
    el, ev_ms = region(args.steps)
    if args.profile_only:
        return

    # per-launch durations of one extra (untimed) step, one event pair per launch
    per_launch = []
    for gq, part, *_ in plan.grouped:
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(stream)
        gq.run(stream)
        e1.record(stream)
        torch.cuda.synchronize()
        nb = sum(w.numel() * 2 for _, w in part) + sum(t.numel() * t.element_size() for o in gq.outs
                                                         for t in o.values() if t is not None)
        us = e0.elapsed_time(e1) * 1e3
        per_launch.append({"shapes": sorted({f"{r}x{c}" for r, c in gq.shapes}), "weights": gq.n,
                           "us": us, "alg_bytes": nb,
                           "GBps": nb / (us * 1e-6) / 1e9})

    checks = []
    if rank == 0:  # the measured outputs of one module per shape, checked in the CPU leg
        for gq, part, *_ in plan.grouped:
            w = part[0][1]
            checks.append((w[:64].cpu(), gq.outs[0]["codes"][:64].cpu(), gq.outs[0]["scale"][:64].cpu()))

    # reassembly across ranks (north star: RCCL all-gather over xGMI), outside the timing
    allgather = None
    if world > 1:
        from quantizers_amd.distributed import gather_state
        local_t = plan.tensors()
        nbytes = sum(t.numel() * t.element_size() for t in local_t.values())
        gather_state({f"r{rank}.{k}": v for k, v in local_t.items()})  # warm (communicator, buffers)
        torch.cuda.synchronize()
        dist.barrier()
        ta = time.perf_counter()
        got = gather_state({f"r{rank}.{k}": v for k, v in local_t.items()})
        torch.cuda.synchronize()
        dist.barrier()
        allgather = {"ms": (time.perf_counter() - ta) * 1e3, "bytes_per_rank": nbytes,
                     "tensors_gathered": len(got), "how": "distributed.gather_state: bucketed all_gather_into_tensor"}
        del got, local_t
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
        other = other_configs(ops, QuantizationArgs, dev, gen)
        other["minimax_m2_1_mixedprec_sharded"] = minimax_pass(ops, QuantizationArgs, dev, gen, world, rank)
        extras["other_configs"] = other

    cpu, ok = None, None
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        cpu, ok = cpu_baseline(args.cpu_seconds, checks + ([cpu_check] if cpu_check else []))

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
                traffic_src = (f"profiles/headline_pmc.json ({pmc['tag']}): FETCH_SIZE x2 + WRITE_SIZE per launch, "
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
                         "frac": achieved / HBM_PEAK_GBS, "traffic": traffic, "traffic_source": traffic_src,
                         "kernel": kernel_name(True, 36 * 9728 * 2560 * 2),
                         "kernel_ms_mean": ev_ms / (args.steps * launches_step),
                         "launches_per_step": launches_step, "alg_bytes_per_step": alg_step,
                         "alg_bytes_per_launch": alg_step / launches_step,
                         "kernel_timing": "HIP events on the launch stream around the same K steps as value "
                                          "(K x launches_per_step grouped launches back to back) / launches",
                         "event_ms_per_step": ev_ms / args.steps,
                         "traffic_unit": "HBM bytes per launch (alg_bytes_per_launch beside it)"},
            "per_launch": per_launch,
            "cpu_baseline": cpu,
            "parity_check": ok,
            "allgather": allgather,
            "pcie_inclusive": pcie,
        }
        line.update(extras)
        print(json.dumps(line), flush=True)
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
