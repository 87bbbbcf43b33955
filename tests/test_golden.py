"""Committed golden fixtures (tests/golden, made by make_golden.py): the CPU oracle (both
restatements) reproduces them on CPU; the HIP library reproduces them on the GPU."""
import os

import pytest
import torch
from safetensors import safe_open
from safetensors.torch import load_file

import ct_torch as ct
import qref

HERE = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
CASES = sorted(f[:-12] for f in os.listdir(HERE)
               if f.endswith(".safetensors") and f != "inputs.safetensors" and not f.startswith("awq_"))


def _args(case):
    with safe_open(os.path.join(HERE, f"{case}.safetensors"), "pt") as f:
        md = f.metadata()
    kw = {}
    for k, v in md.items():
        if v == "None":
            v = None
        elif v in ("True", "False"):
            v = v == "True"
        elif v.lstrip("-").isdigit():
            v = int(v)
        elif v.startswith("("):
            v = tuple(int(x) for x in v.strip("()").split(",") if x.strip())
        kw[k] = v
    return ct.QArgs(**kw)


def _eq(a, b, key):
    if a.dtype == torch.float8_e4m3fn:
        a = a.view(torch.uint8)
    if a.dtype == torch.bfloat16:
        a, b = a.view(torch.int16), b.view(torch.int16)
    assert a.shape == b.shape and torch.equal(a.cpu(), b.cpu()), key


def test_cases_present():
    assert len(CASES) == 10


@pytest.mark.parametrize("case", CASES)
def test_oracle_reproduces_golden(case):
    a = _args(case)
    ins = load_file(os.path.join(HERE, "inputs.safetensors"))
    gold = load_file(os.path.join(HERE, f"{case}.safetensors"))
    for k, w in ins.items():
        for impl in (ct.compress_weight, qref.compress_weight):
            out = impl(w, a)
            for name in [n for n in gold if n.startswith(k + ".")]:
                _eq(out[name[len(k) + 1:]], gold[name], f"{case}/{name}")


@pytest.mark.gpu
@pytest.mark.parametrize("case", CASES)
def test_gpu_reproduces_golden(cuda, case):
    from quantizers_amd import ops
    from quantizers_amd.quantization import QuantizationArgs
    a = _args(case)
    qa = QuantizationArgs(num_bits=a.num_bits, type=a.type, symmetric=a.symmetric, strategy=a.strategy,
                          group_size=a.group_size, block_structure=list(a.block_structure) if a.block_structure else None,
                          scale_dtype={None: None, "fp8": "float8_e4m3fn", "e8m0": "uint8"}[a.scale_dtype])
    ins = load_file(os.path.join(HERE, "inputs.safetensors"))
    gold = load_file(os.path.join(HERE, f"{case}.safetensors"))
    for k, w in ins.items():
        out = ops.compress_weight(w.to(cuda), qa)
        names = [n for n in gold if n.startswith(k + ".")]
        assert {n[len(k) + 1:] for n in names} == set(out)
        for name in names:
            _eq(out[name[len(k) + 1:]], gold[name], f"{case}/{name}")
