#!/usr/bin/env python3
"""Diagnose NVFP4 mismatches on the extreme-magnitude slices of tests/test_nvfp4_gpu.py:
per slice, differing code bytes / scales vs the C oracle, with the group's inputs."""
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (ROOT, os.path.join(ROOT, "tests"), os.path.join(ROOT, "oracle")):
    sys.path.insert(0, p)
import qref  # noqa: E402
from quantizers_amd import ops  # noqa: E402
from quantizers_amd.quantization import QuantizationArgs  # noqa: E402
from test_nvfp4_gpu import NV, _OA, _rand  # noqa: E402

a = QuantizationArgs(**NV)
base = _rand((6, 64, 256), seed=77, scale=1.0)
mult = torch.tensor([2.0 ** -120, 2.0 ** -60, 1.0, 2.0 ** 40, 2.0 ** 100, 1.0]).view(6, 1, 1)
w = (base.float() * mult).to(torch.bfloat16)
w[5] = (base[5].float() * (2.0 ** torch.arange(-30, 34, dtype=torch.float32).view(64, 1))).to(torch.bfloat16)
got = ops.quantize_weight(w.to("cuda:0"), a)
for i in range(6):
    ref = qref.compress_weight(w[i], _OA)
    gc, rc = got["codes"][i].cpu(), ref["weight_packed"].view(torch.uint8)
    gs, rs = got["scale"][i].cpu().view(torch.uint8), ref["weight_scale"].view(torch.uint8)
    dc, ds = (gc != rc).nonzero().tolist(), (gs != rs).nonzero().tolist()
    print(f"slice {i}: gscale got {got['global_scale'][i].item()!r} ref {ref['weight_global_scale'].item()!r}; "
          f"codes differ {len(dc)}, scales differ {len(ds)}")
    for r, c in dc[:4]:
        g = c // 8
        x = w[i, r, g * 16:(g + 1) * 16].float()
        print(f"  code [{r},{c}] got {int(gc[r, c]):#04x} ref {int(rc[r, c]):#04x}; scale got {int(gs[r, g]):#04x} "
              f"ref {int(rs[r, g]):#04x}; elems {x[(c % 8) * 2].item()!r}, {x[(c % 8) * 2 + 1].item()!r}; "
              f"group absmax {x.abs().max().item()!r}")
    for r, g in ds[:4]:
        x = w[i, r, g * 16:(g + 1) * 16].float()
        print(f"  scale [{r},{g}] got {int(gs[r, g]):#04x} ref {int(rs[r, g]):#04x}; group absmax {x.abs().max().item()!r}")
