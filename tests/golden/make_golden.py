"""Generate the committed golden fixtures (tests/golden/*.safetensors) from the CPU oracle.

Inputs are seeded (SURVEY.md §8c suggested set): W bf16 [256, 512] N(0, 0.02^2) plus edge
cases (0.1% x20 outliers, an all-zero group, exact +-7.5*s / 0.5*s ties), every scheme the
reference's recipes use.  Outputs are the on-disk tensors of oracle/ct_torch.compress_weight
(which oracle/quant_ref.c reproduces bit for bit).  Parity with compressed-tensors itself is
unpinned (the package is absent); these fixtures pin the oracle across rounds and the GPU
library against committed data.

Run: python tests/golden/make_golden.py   (rewrites the fixtures; commit them)
"""
import os
import sys

import torch
from safetensors.torch import save_file

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, "..", "..", "oracle"))
import ct_torch as ct  # noqa: E402

CASES = {
    "int4_sym_g128": ct.QArgs(num_bits=4, group_size=128),
    "int4_sym_g32": ct.QArgs(num_bits=4, group_size=32),
    "int4_asym_g128": ct.QArgs(num_bits=4, group_size=128, symmetric=False),
    "int4_asym_g32": ct.QArgs(num_bits=4, group_size=32, symmetric=False),
    "int8_sym_channel": ct.QArgs(num_bits=8, strategy="channel"),
    "fp8_g32": ct.QArgs(num_bits=8, type="float", group_size=32),
    "fp8_block128": ct.QArgs(num_bits=8, type="float", strategy="block", block_structure=(128, 128)),
    "fp8_channel": ct.QArgs(num_bits=8, type="float", strategy="channel"),
    "mxfp4_g32": ct.QArgs(num_bits=4, type="float", group_size=32, scale_dtype="e8m0"),
    "nvfp4_g16": ct.QArgs(num_bits=4, type="float", strategy="tensor_group", group_size=16, scale_dtype="fp8"),
}


def inputs():
    g = torch.Generator().manual_seed(0)
    w = torch.randn(256, 512, generator=g) * 0.02
    e = w.clone()
    m = torch.rand(256, 512, generator=g) < 0.001
    e[m] *= 20
    e[0, :128] = 0.0
    e[2, :128] = 0.0
    e[2, :5] = torch.tensor([0.75, -0.75, 0.05, -0.05, 0.15])
    return {"w_gauss": w.to(torch.bfloat16), "w_edge": e.to(torch.bfloat16)}


def main():
    ins = inputs()
    save_file(ins, os.path.join(HERE, "inputs.safetensors"))
    for case, a in CASES.items():
        out = {}
        for k, w in ins.items():
            for name, t in ct.compress_weight(w, a).items():
                if t.dtype == torch.float8_e4m3fn:
                    t = t.view(torch.uint8)
                out[f"{k}.{name}"] = t.contiguous()
        save_file(out, os.path.join(HERE, f"{case}.safetensors"),
                  metadata={k: str(v) for k, v in vars(a).items()})
    print("wrote", len(CASES), "fixtures")


if __name__ == "__main__":
    main()
