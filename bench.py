#!/usr/bin/env python3
"""Benchmark of the north-star kernel: int4 symmetric group-128 quantize + pack of a synthetic
bf16 weight [11008, 4096] (BASELINE.json configs[1]: "Qwen3-4B AWQ int4 group_size=128 on
1xMI355X"; metric "params quantized/sec + achieved HBM GB/s").

One *step* = one fused quantize+pack pass over one [11008, 4096] bf16 weight already resident
in HBM, into that step's own output tensors.  The step rotates over COPIES distinct input buffers
(> the 256 MiB Infinity Cache) so every step streams its weight from HBM, not L3 (BASELINE.md
timing protocol).  The K timed steps are ONE grouped launch (qz_quantize_grouped: grid.y = step,
a device table of per-step weight/output pointers), the way the library quantizes many
same-shape weights; the one-launch-per-weight rate (qz_quantize_many) is reported beside it
(``per_weight_launch``), and ``--per-weight-launch`` makes it the timed path.  Multi-GPU: one process per GPU, each quantizes its own weight
shard set (weak scaling, no collective in the timed region); after timing, ranks reassemble
the packed tensors with one RCCL all-gather (reported separately, as the north star asks).

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

ROWS, COLS, GROUP, BITS = 11008, 4096, 128, 4
PARAMS = ROWS * COLS
# algorithmic bytes per launch: read 2 B/param + packed 0.5 B/param + bf16 scale/group
ALG_BYTES = PARAMS * 2 + PARAMS * BITS // 8 + (PARAMS // GROUP) * 2  # 113,426,432
HBM_PEAK_GBS = 8000.0  # MI355X_MICROARCH.md: 8.0 TB/s spec
METRIC = "params quantized/sec + achieved HBM GB/s, Qwen3-4B AWQ int4-g128"
KERNEL_NAME_SINGLE = "k_group_fast<4, 0, false, true, false>"  # one launch per weight (90 MB < 256 MiB)
NT_BYTES = 256 << 20  # QZ_NT_BYTES: launches reading more use nt loads + 4 KiB tiles


def grouped_kernel_name(k):
    nt = k * PARAMS * 2 > NT_BYTES
    return f"k_group_fast<4, 0, false, true, {str(nt).lower()}, true>"

# Qwen3-4B linear shapes (hidden 2560, inter 9728, 32 q / 8 kv heads x 128), 36 layers
QWEN3_4B = [("q_proj", 4096, 2560), ("k_proj", 1024, 2560), ("v_proj", 1024, 2560), ("o_proj", 2560, 4096),
            ("gate_proj", 9728, 2560), ("up_proj", 9728, 2560), ("down_proj", 2560, 9728)]
QWEN3_LAYERS = 36


def parse():
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=200)
    p.add_argument("--warmup", type=int, default=20)
    p.add_argument("--copies", type=int, default=12)
    p.add_argument("--cpu-seconds", type=float, default=10.0)
    p.add_argument("--no-cpu-baseline", action="store_true")
    p.add_argument("--no-model-pass", action="store_true")
    p.add_argument("--per-weight-launch", action="store_true",
                   help="time one qz_quantize launch per step (qz_quantize_many) instead of one grouped launch")
    p.add_argument("--python-loop", action="store_true",
                   help="one Python qz_quantize call per step instead of one qz_quantize_many call")
    p.add_argument("--graph", action="store_true",
                   help="replay the K steps as one captured hipGraph (measured slower, see DESIGN.md §6)")
    p.add_argument("--profile-only", action="store_true",
                   help="just warmup + K launches (for rocprofv3 runs); prints nothing else")
    return p.parse_args()


def cpu_model():
    try:
        out = subprocess.run(["lscpu"], capture_output=True, text=True, timeout=10).stdout
        for line in out.splitlines():
            if line.startswith("Model name"):
                return line.split(":", 1)[1].strip()
    except Exception:
        pass
    return platform.processor() or "unknown"


def cpu_baseline(seconds: float, measured=None):
    """The oracle's torch-op restatement of compressed-tensors (oracle/ct_torch.py), timed on the
    host cores on the same synthetic weight.  The oracle is used only here (the
    CPU leg): besides the timing it checks the GPU's measured output slices ``measured`` =
    (input rows, packed codes, scales[, codes, scales of the per-weight launch]) bit for bit
    against the plain-C restatement."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import ct_torch as ct  # CPU baseline leg only
    import qref  # checker only
    ok = None
    if measured is not None:
        w_in, outs = measured[0], measured[1:]
        ref_p, ref_s = qref.int_sym_group_pack(w_in, BITS, GROUP)
        ok = all(bool(torch.equal(codes, ref_p) and torch.equal(scale.view(torch.int16), ref_s.view(torch.int16)))
                 for codes, scale in zip(outs[0::2], outs[1::2]))

    threads = min(16, os.cpu_count() or 1)  # the GPU box's CPU share is 16
    torch.set_num_threads(threads)
    g = torch.Generator().manual_seed(0)
    w = (torch.randn(ROWS, COLS, generator=g) * 0.02).to(torch.bfloat16)
    a = ct.QArgs(num_bits=BITS, type="int", symmetric=True, strategy="group", group_size=GROUP)
    ct.compress_weight(w, a)  # warm-up
    n, t0 = 0, time.perf_counter()
    while True:
        ct.compress_weight(w, a)
        n += 1
        el = time.perf_counter() - t0
        if (el >= seconds and n >= 3) or n >= 1000:
            break
    res = {"value": n * PARAMS / el, "unit": "params/s", "cores": threads, "kind": "port",
            "sample": f"oracle/ct_torch.compress_weight (compressed-tensors op sequence, torch CPU) on the same "
                      f"bf16 [{ROWS},{COLS}] int4-g{GROUP} weight, {n} calls in {el:.1f}s, "
                      f"torch threads={threads}, os.cpu_count()={os.cpu_count()}, cpu='{cpu_model()}'"}
    return res, ok


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


def read_pmc_traffic(kernel, weights_per_launch):
    """HBM bytes per launch of ``kernel`` from the committed rocprofv3 PMC passes
    (profiles/pmc_traffic.json: bytes per weight x the weights one launch processes), or None."""
    path = os.path.join(ROOT, "profiles", "pmc_traffic.json")
    try:
        with open(path) as f:
            d = json.load(f)
        if not d.get("kernel", "").startswith(kernel):
            return None, None
        return d["hbm_bytes_per_weight"] * weights_per_launch, d.get("source")
    except Exception:
        return None, None


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
    from quantizers_amd.quantization import QuantizationArgs

    a = QuantizationArgs(num_bits=BITS, type="int", symmetric=True, strategy="group", group_size=GROUP)
    gen = torch.Generator(device=dev).manual_seed(1234 + rank)
    copies = [(torch.randn(ROWS, COLS, device=dev, generator=gen) * 0.02).to(torch.bfloat16)
              for _ in range(args.copies)]
    out = ops.quantize_weight(copies[0], a)  # allocates outputs + workspace
    bufs = {"codes": out["codes"], "scale": out["scale"], "zero_point": out["zero_point"]}
    stream = torch.cuda.current_stream(dev)
    prep = ops.PreparedQuantize(copies[0], a, bufs)

    def step(i, st=stream):
        prep.run(copies[i % args.copies], st)

    # Default: the K steps are ONE grouped launch (qz_quantize_grouped) over K (weight, outputs)
    # pairs: step i reads copy i % COPIES and writes its own codes/scales (K distinct output
    # sets, so no two steps of the launch write the same bytes).
    grouped = not (args.per_weight_launch or args.python_loop or args.graph)
    # everything is marshalled BEFORE the warmup, so each timed region directly follows its own
    # W warmup steps (the card's clocks depend on the preceding ~ms of load: scripts/idle_gap.py)
    outs_k = [{"codes": torch.empty_like(bufs["codes"]), "scale": torch.empty_like(bufs["scale"]),
               "zero_point": None} for _ in range(args.steps)]
    if grouped:
        # (--profile-only: the warmup launch has the timed launch's size, so every launch of the
        # grouped kernel in a rocprofv3 pass covers K weights)
        nw = args.steps if args.profile_only else max(args.warmup, 1)
        warm = ops.GroupedQuantize([copies[i % args.copies] for i in range(nw)], a,
                                   outs=[{"codes": torch.empty_like(bufs["codes"]),
                                          "scale": torch.empty_like(bufs["scale"]), "zero_point": None}
                                         for _ in range(nw)])
        gq = ops.GroupedQuantize([copies[i % args.copies] for i in range(args.steps)], a, outs=outs_k)

    # --graph: the K timed steps captured once into a hipGraph and replayed with one host call.
    # Measured on MI355X: kernels inside the replay run 25.4 us vs 21.0 us launched on the stream
    # (per-node release fences), and the stream launches already run back to back (median gap 0).
    graph = None
    if args.graph:
        graph = torch.cuda.CUDAGraph()
        cap = torch.cuda.Stream(dev)
        cap.wait_stream(stream)
        with torch.cuda.graph(graph, stream=cap):
            for i in range(args.steps):
                step(i, torch.cuda.current_stream(dev))
        stream.wait_stream(cap)
        graph.replay()  # untimed: first replay uploads the graph
        torch.cuda.synchronize()

    # One launch per weight: qz_quantize_many -- one host call that enqueues the K qz_quantize
    # launches (each over its own resident copy, into the K distinct output sets) -- so the ~20 us
    # Python/ctypes cost per call cannot leave the GPU idle between the ~21 us kernels.
    many = None if (graph is not None or args.python_loop) else \
        prep.prepare_many([copies[i % args.copies] for i in range(args.steps)], outs=outs_k)

    def run_steps(grouped_launch=grouped):
        if grouped_launch:
            gq.run(stream)
        elif graph is not None:
            graph.replay()
        elif many is not None:
            many(stream)
        else:
            for i in range(args.steps):
                step(i)

    def warmup(grouped_launch):
        if grouped_launch:
            warm.run(stream)  # W warmup steps (one grouped launch)
        else:
            for i in range(args.warmup):
                step(i)

    if args.profile_only:
        warmup(grouped)
        run_steps()
        torch.cuda.synchronize()
        return

    def timed_region(grouped_launch):
        """barrier + sync, exactly K steps, sync + barrier; wall seconds (max over ranks) and the
        HIP-event time of the region on the launch stream (ms)."""
        ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        if world > 1:
            dist.barrier()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        ev0.record(stream)
        run_steps(grouped_launch)
        ev1.record(stream)
        torch.cuda.synchronize()
        if world > 1:
            dist.barrier()
        wall = time.perf_counter() - t0
        t = torch.tensor([wall], device=dev, dtype=torch.float64)
        if world > 1:
            _all_reduce_max(t)
        return t.item(), ev0.elapsed_time(ev1)

    # ---- contract timing.  HIP events on the launch stream bracket the same region: for the
    # grouped launch their elapsed time IS the kernel's launch duration; for per-weight launches
    # elapsed / K is the average launch duration (back-to-back, no host gaps).
    warmup(grouped)
    el, region_ms = timed_region(grouped)
    n_launches = 1 if grouped else args.steps
    k_ms_mean = region_ms / n_launches

    # ---- secondary: one launch per weight (qz_quantize_many), same K steps into the same K
    # distinct output sets, after its own W warmup steps; then one event pair around each launch
    # (adds the event packets' ~1-2 us per launch)
    per_weight = None
    if grouped:
        warmup(False)
        pw_el, pw_region_ms = timed_region(False)
        pw_us = pw_region_ms / args.steps * 1e3
        per_weight = {"kernel": KERNEL_NAME_SINGLE, "us_per_launch": pw_us,
                      "params_per_s": world * PARAMS * args.steps / pw_el,
                      "achieved_GBps": ALG_BYTES / (pw_us * 1e-6) / 1e9,
                      "frac": ALG_BYTES / (pw_us * 1e-6) / 1e9 / HBM_PEAK_GBS,
                      "timing": "HIP events around K back-to-back qz_quantize launches (one qz_quantize_many call, "
                                "the K distinct output sets of the grouped launch) / K, after W warmup launches"}
    starts = [torch.cuda.Event(enable_timing=True) for _ in range(args.steps)]
    ends = [torch.cuda.Event(enable_timing=True) for _ in range(args.steps)]
    for i in range(args.steps):
        starts[i].record(stream)
        step(i)
        ends[i].record(stream)
    torch.cuda.synchronize()
    durs = sorted(s.elapsed_time(e) for s, e in zip(starts, ends))
    if per_weight is not None:
        per_weight["us_per_launch_events_mean"] = sum(durs) / len(durs) * 1e3
        per_weight["us_per_launch_events_median"] = durs[len(durs) // 2] * 1e3
    k_ms_each_mean = sum(durs) / len(durs)
    k_ms_each_med = durs[len(durs) // 2]

    # ---- the measured buffers' first 256 rows, checked against the oracle in the CPU leg below
    measured = None
    if rank == 0:
        last = (args.steps - 1) % args.copies
        o_last = outs_k[args.steps - 1] if (grouped or many is not None) else bufs
        measured = (copies[last][:256].cpu(), o_last["codes"][:256].cpu(), o_last["scale"][:256].cpu())
        if grouped:  # the per-step event-pair launches wrote bufs from the same copy: must agree too
            measured = measured + (bufs["codes"][:256].cpu(), bufs["scale"][:256].cpu())
    many_used = many is not None
    if grouped:
        del gq, warm
    del outs_k, many
    torch.cuda.empty_cache()

    # ---- reassembly across ranks (north star: RCCL all-gather over xGMI), outside the timing
    allgather = None
    if world > 1:
        gathered_codes = torch.empty((world,) + tuple(bufs["codes"].shape), dtype=bufs["codes"].dtype, device=dev)
        gathered_scale = torch.empty((world,) + tuple(bufs["scale"].shape), dtype=bufs["scale"].dtype, device=dev)
        for _ in range(3):
            _all_gather_into(gathered_codes, bufs["codes"])
            _all_gather_into(gathered_scale, bufs["scale"])
        torch.cuda.synchronize()
        dist.barrier()
        ta = time.perf_counter()
        reps = 10
        for _ in range(reps):
            _all_gather_into(gathered_codes, bufs["codes"])
            _all_gather_into(gathered_scale, bufs["scale"])
        torch.cuda.synchronize()
        allgather = (time.perf_counter() - ta) / reps * 1e3

    # ---- the AWQ kernels (a3-a6) on the same resident weights
    awq = None
    if not args.no_model_pass:
        awq = awq_kernels(ops, QuantizationArgs, copies, dev, gen, stream)

    # ---- whole-model pass: every Qwen3-4B linear (36 layers, batched per shape)
    model_pass = None
    if not args.no_model_pass:
        del copies
        torch.cuda.empty_cache()
        ws = []
        for name, n, k in QWEN3_4B:
            ws.append((name, (torch.randn(QWEN3_LAYERS, n, k, device=dev, generator=gen) * 0.02).to(torch.bfloat16)))
        outs = [ops.quantize_weight(w, a) for _, w in ws]  # warm + allocate
        torch.cuda.synchronize()
        reps = 5
        tm = time.perf_counter()
        for _ in range(reps):
            for (_, w), o in zip(ws, outs):
                ops.quantize_weight(w, a, out={"codes": o["codes"], "scale": o["scale"], "zero_point": o["zero_point"]})
        torch.cuda.synchronize()
        mp = (time.perf_counter() - tm) / reps
        nparams = sum(w.numel() for _, w in ws)
        model_pass = {"params": nparams, "ms": mp * 1e3, "params_per_s": nparams / mp,
                      "alg_GBps": nparams * (2 + BITS / 8 + 2 / GROUP) / mp / 1e9, "launches": len(ws)}

    # ---- AWQ oneshot (scale search + smoothing) on a 2-layer Qwen3-4B, BASELINE configs[1]
    awq_e2e = None
    if not args.no_model_pass and world == 1:
        awq_e2e = awq_oneshot_layers(dev)

    # ---- the other BASELINE configs, one whole-model pass each (reported beside the headline)
    other = None
    if not args.no_model_pass:
        other = other_configs(ops, QuantizationArgs, dev, gen)
        other["minimax_m2_1_mixedprec_sharded"] = minimax_pass(ops, QuantizationArgs, dev, gen, world, rank)

    cpu, ok = None, None
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        cpu, ok = cpu_baseline(args.cpu_seconds, measured)

    if rank == 0:
        ms_step = el / args.steps * 1e3
        value = world * PARAMS * args.steps / el
        per_launch = args.steps if grouped else 1  # weights one launch processes
        kernel = grouped_kernel_name(args.steps) if grouped else KERNEL_NAME_SINGLE
        achieved = ALG_BYTES * per_launch / (k_ms_mean * 1e-3) / 1e9
        traffic, tsrc = read_pmc_traffic(kernel, per_launch)
        line = {
            "metric": METRIC,
            "value": value,
            "unit": "params/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": ms_step,
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "bf16",
            "data": "synthetic: torch.randn*0.02 bf16 weights (no checkpoint); same shape as Qwen3-4B's 11008x4096",
            "config": {"workload": f"int4 sym group_size={GROUP} quantize+pack (pack-quantized) of bf16 W[{ROWS},{COLS}]"
                                   f", {args.copies} rotating HBM-resident copies",
                       "rows": ROWS, "cols": COLS, "group_size": GROUP, "num_bits": BITS,
                       "parallelism": f"weight-shard dp{world}"},
            "hbm_GBps_step": world * ALG_BYTES * args.steps / el / 1e9,
            "roofline": {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": achieved / HBM_PEAK_GBS, "traffic": traffic,
                         "kernel": kernel, "kernel_ms_mean": k_ms_mean, "weights_per_launch": per_launch,
                         "kernel_timing": ("HIP events around the timed region = the one grouped launch "
                                           "(qz_quantize_grouped) of the K steps" if grouped else
                                           "HIP events around the K back-to-back launches of the timed region / K"
                                           + (" (one hipGraph replay)" if graph is not None else
                                              " (one qz_quantize_many call)" if many_used else
                                              " (Python loop of qz_quantize calls)")),
                         "alg_bytes_per_launch": ALG_BYTES * per_launch,
                         "alg_bytes_per_weight": ALG_BYTES, "traffic_source": tsrc},
            "per_weight_launch": per_weight if grouped else {
                "kernel": KERNEL_NAME_SINGLE, "us_per_launch_events_mean": k_ms_each_mean * 1e3,
                "us_per_launch_events_median": k_ms_each_med * 1e3},
            "cpu_baseline": cpu,
            "parity_check": ok,
            "allgather_ms": allgather,
            "qwen3_4b_all_linears": model_pass,
            "awq_kernels": awq,
            "awq_oneshot_qwen3_4b": awq_e2e,
            "other_configs": other,
        }
        print(json.dumps(line), flush=True)
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
