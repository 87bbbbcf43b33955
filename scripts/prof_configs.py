#!/usr/bin/env python3
"""Per-kernel profile of the model-level passes (run under rocprofv3 --kernel-trace --stats):
Qwen3-4B FP8_BLOCK attention + int4-g32 MLP, int4-g128 all linears, Qwen3-30B-A3B experts MXFP4,
one resident layer each (kernel durations, not wall time)."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from quantizers_amd import ops  # noqa: E402
from quantizers_amd.quantization import QuantizationArgs  # noqa: E402

dev = torch.device("cuda:0")
g = torch.Generator(device=dev).manual_seed(0)
L = 36
shapes = [("q", 4096, 2560), ("k", 1024, 2560), ("v", 1024, 2560), ("o", 2560, 4096),
          ("gate", 9728, 2560), ("up", 9728, 2560), ("down", 2560, 9728)]
fp8b = QuantizationArgs(num_bits=8, type="float", strategy="block", block_structure=[128, 128])
i4g32 = QuantizationArgs(num_bits=4, type="int", symmetric=True, group_size=32)
i4g128 = QuantizationArgs(num_bits=4, type="int", symmetric=True, group_size=128)
mx = QuantizationArgs(num_bits=4, type="float", group_size=32, scale_dtype="uint8")
nv = QuantizationArgs(num_bits=4, type="float", strategy="tensor_group", group_size=16, scale_dtype="float8_e4m3fn")
f8g = QuantizationArgs(num_bits=8, type="float", group_size=32)
ws = {n: (torch.randn(L, r, c, device=dev, generator=g) * 0.02).to(torch.bfloat16) for n, r, c in shapes}
for _ in range(5):
    for n, w in ws.items():
        ops.quantize_weight(w, fp8b if n in "qkvo" else i4g32)
    for n, w in ws.items():
        ops.quantize_weight(w, i4g128)
    for n, w in ws.items():
        ops.quantize_weight(w, f8g)
    ops.quantize_weight(ws["gate"], nv)
torch.cuda.synchronize()
del ws
gu = (torch.randn(128, 1536, 2048, device=dev, generator=g) * 0.02).to(torch.bfloat16)
dn = (torch.randn(128, 2048, 768, device=dev, generator=g) * 0.02).to(torch.bfloat16)
for _ in range(5):
    ops.quantize_weight(gu[:, :768], mx)
    ops.quantize_weight(gu[:, 768:], mx)
    ops.quantize_weight(dn, mx)
torch.cuda.synchronize()
print("done")
