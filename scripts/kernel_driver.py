#!/usr/bin/env python3
"""Run each north-star kernel a fixed number of times on the [11008, 4096] bf16 headline weight
(12 rotating HBM-resident copies, > the 256 MiB Infinity Cache) -- the program the rocprofv3
PMC passes of scripts/pmc_kernels.sh profile.  Prints per-kernel HIP-event times.

  python scripts/kernel_driver.py [N]      (N launches per kernel, default 30)
"""
import os
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from quantizers_amd import ops  # noqa: E402
from quantizers_amd.quantization import QuantizationArgs  # noqa: E402

R, C, G = 11008, 4096, 128


def main(n=30):
    dev = torch.device("cuda:0")
    gen = torch.Generator(device=dev).manual_seed(0)
    copies = [(torch.randn(R, C, device=dev, generator=gen) * 0.02).to(torch.bfloat16) for _ in range(12)]
    a = QuantizationArgs(num_bits=4, type="int", symmetric=True, group_size=G)
    s = torch.rand(C, device=dev, generator=gen) + 0.5
    grid_s = [torch.rand(C, device=dev, generator=gen) + 0.5 for _ in range(20)]
    fq_out = [torch.empty_like(copies[0]) for _ in range(4)]
    x = [torch.randn(16384, C, device=dev, generator=gen).to(torch.bfloat16) for _ in range(4)]
    sums = torch.zeros(C, dtype=torch.float32, device=dev)
    wsum = torch.zeros(C, dtype=torch.float64, device=dev)
    outs = [ops.alloc_outputs((R, C), a, None, dev) for _ in range(n)]
    prep = ops.PreparedQuantize(copies[0], a, outs[0])
    many = prep.prepare_many([copies[i % 12] for i in range(n)], outs=outs)
    gq = ops.GroupedQuantize([copies[i % 12] for i in range(n)], a, outs=outs)
    kernels = [
        ("quantize_per_weight", lambda i: prep.run(copies[i % 12]), 1),
        ("fake_quant_cols", lambda i: ops.fake_quantize(copies[i % 12], a, col_scales=s, out=fq_out[i % 4]), 1),
        # the AWQ dense grid's pattern (awq._grid_fixed): ONE weight fake-quantized under 20 scale
        # vectors into the same output (the balance layer's own weight)
        ("fake_quant_grid", lambda i: ops.fake_quantize(copies[0], a, col_scales=grid_s[i % 20], out=fq_out[0]), 1),
        ("absmean", lambda i: ops.awq_absmean_accum(x[i % 4], sums), 1),
        ("weight_mean", lambda i: ops.awq_weight_mean_accum(copies[i % 12], G, wsum), 1),
        ("scale_columns", lambda i: ops.scale_columns_(copies[i % 12], s), 1),
    ]
    # NVFP4 (the reference's Qwen3-30B-A3B recipe): one fused expert half [128, 768, 2048] per
    # launch (strided slices of [128, 1536, 2048]), 4 resident parameters rotated (1.6 GB)
    nv = QuantizationArgs(num_bits=4, type="float", strategy="tensor_group", group_size=16,
                          scale_dtype="float8_e4m3fn")
    gus = [(torch.randn(128, 1536, 2048, device=dev, generator=gen) * 0.02).to(torch.bfloat16) for _ in range(4)]
    nv_out = ops.alloc_outputs((128, 768, 2048), nv, None, dev)
    import ctypes
    from quantizers_amd import _lib
    lib, ca = _lib.load(), nv.to_c()
    nv_ws = torch.empty(lib.qz_quantize_workspace_size(128, 768, 2048, ctypes.byref(ca)) + 256, dtype=torch.uint8,
                        device=dev)

    def nv_two_pass(i):
        w = gus[i % 4][:, :768]
        rc = lib.qz_quantize(ops._ptr(w), 128, 768, 2048, 2048, 1536 * 2048, ctypes.byref(ca), _lib.QZ_OUT_FP4_PACKED,
                             ops._ptr(nv_out["codes"]), ops._ptr(nv_out["scale"]), ops._ptr(None),
                             ops._ptr(nv_out["global_scale"]), ops._ptr(nv_ws), nv_ws.numel(), ops._stream())
        _lib.check(rc, "qz_quantize")
    # MXFP4 (BASELINE.json configs[3]): the same fused expert halves, E2M1 codes + E8M0 scales, g32
    mx = QuantizationArgs(num_bits=4, type="float", group_size=32, scale_dtype="uint8")
    mx_out = ops.alloc_outputs((128, 768, 2048), mx, None, dev)
    kernels += [
        ("mxfp4_experts", lambda i: ops.quantize_weight(gus[i % 4][:, 768:], mx, out=mx_out), 1),
        ("nvfp4_fused", lambda i: ops.quantize_weight(gus[i % 4][:, :768], nv, out=nv_out), 1),
        ("nvfp4_two_pass", nv_two_pass, 1),
    ]
    # FP8_BLOCK 128x128 (BASELINE configs[2], the mixed recipe's attention half): the strip kernel
    # as CompressionPlan issues it -- grouped launches over the Qwen3-4B k+v (72 x [1024, 2560]) and
    # q (36 x [4096, 2560]) weights -- and one batch launch over a [36, 1024, 2560] stack
    fb = QuantizationArgs(num_bits=8, type="float", strategy="block", block_structure=[128, 128])
    kv = [(torch.randn(1024, 2560, device=dev, generator=gen) * 0.02).to(torch.bfloat16) for _ in range(72)]
    qw = [(torch.randn(4096, 2560, device=dev, generator=gen) * 0.02).to(torch.bfloat16) for _ in range(36)]
    g_kv, g_q = ops.GroupedQuantize(kv, fb), ops.GroupedQuantize(qw, fb)
    stk = (torch.randn(36, 1024, 2560, device=dev, generator=gen) * 0.02).to(torch.bfloat16)
    stk_out = ops.alloc_outputs(tuple(stk.shape), fb, None, dev)
    kernels += [
        ("fp8_block_grouped_kv", lambda i: g_kv.run(), 1),
        ("fp8_block_grouped_q", lambda i: g_q.run(), 1),
        ("fp8_block_stack_kv", lambda i: ops.quantize_weight(stk, fb, out=stk_out), 1),
    ]
    # the AWQ statistics in the pass's own pattern (Qwen3-4B: hidden 2560, 16 calibration samples of
    # 2048 tokens per batched forward): absmean per sample as the hook issued it through round 4 and
    # all 16 samples as one segmented launch (round 5); w_mean per balance layer ([9728, 2560]) and
    # per mapping as one segmented launch (gate + up; q / k / v)
    xl = [torch.randn(16 * 2048, 2560, device=dev, generator=gen).to(torch.bfloat16) for _ in range(2)]
    smp = [[x[j * 2048:(j + 1) * 2048] for j in range(16)] for x in xl]
    sums_l = [torch.zeros(2560, dtype=torch.float32, device=dev) for _ in range(16)]
    gu_map = [[(torch.randn(9728, 2560, device=dev, generator=gen) * 0.02).to(torch.bfloat16) for _ in range(2)]
              for _ in range(3)]
    qkv = [(torch.randn(r, 2560, device=dev, generator=gen) * 0.02).to(torch.bfloat16) for r in (4096, 1024, 1024)]
    wsum_l = [torch.zeros(2560, dtype=torch.float64, device=dev) for _ in range(3)]
    kernels += [
        ("absmean_sample_2048x2560", lambda i: ops.awq_absmean_accum(smp[i % 2][i % 16], sums_l[0]), 1),
        ("absmean_seg_16x2048x2560", lambda i: ops.awq_absmean_segments(smp[i % 2], sums_l), 1),
        ("wmean_balance_9728x2560", lambda i: ops.awq_weight_mean_accum(gu_map[i % 3][i % 2], G, wsum_l[0]), 1),
        ("wmean_seg_gate_up", lambda i: ops.awq_weight_mean_segments(gu_map[i % 3], G, wsum_l[:2]), 1),
        ("wmean_seg_q_k_v", lambda i: ops.awq_weight_mean_segments(qkv, G, wsum_l), 1),
    ]
    st = torch.cuda.current_stream()
    for name, fn, _ in kernels:
        for i in range(3):
            fn(i)
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(st)
        for i in range(n):
            fn(i)
        e1.record(st)
        torch.cuda.synchronize()
        print(f"{name:22s} {e0.elapsed_time(e1) * 1e3 / n:8.2f} us/launch (events over {n} launches)", flush=True)
    many()
    gq.run()
    torch.cuda.synchronize()
    time.sleep(0.01)


if __name__ == "__main__":
    main(int(sys.argv[1]) if len(sys.argv) > 1 else 30)
