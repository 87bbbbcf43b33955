"""ctypes binding of oracle/quant_ref.c (TEST INFRASTRUCTURE ONLY — see ct_torch.py header).

Returns results in the same tensor layout as ``ct_torch.compress_weight`` so tests can compare
the two restatements, and the GPU library against either, bit for bit.
"""
from __future__ import annotations

import ctypes
import os
import subprocess

import numpy as np
import torch

_HERE = os.path.dirname(os.path.abspath(__file__))
_SO = os.path.join(_HERE, "build", "libquant_ref.so")
_lib = None

ST = {"tensor": 0, "channel": 1, "group": 2, "block": 3, "tensor_group": 4}


class _Args(ctypes.Structure):
    _fields_ = [(n, ctypes.c_int) for n in
                ("num_bits", "type", "symmetric", "strategy", "group_size", "block_h", "block_w", "scale_fmt")]


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(_SO):
            subprocess.check_call(["make", "-s", "-C", _HERE])
        _lib = ctypes.CDLL(_SO)
        P = ctypes.c_void_p
        I64 = ctypes.c_int64
        _lib.qref_quantize.argtypes = [P, I64, I64, ctypes.POINTER(_Args), P, P, P, P]
        _lib.qref_pack_int32.argtypes = [P, I64, I64, ctypes.c_int, P]
        _lib.qref_pack_int32_dim0.argtypes = [P, I64, I64, ctypes.c_int, P]
        _lib.qref_pack_fp4.argtypes = [P, I64, P]
        _lib.qref_int_sym_group_pack.argtypes = [P, I64, I64, ctypes.c_int, ctypes.c_int, P, P]
    return _lib


def _ptr(t: torch.Tensor):
    return ctypes.c_void_p(t.data_ptr())


def _n_groups(a, R, C):
    if a.strategy == "tensor":
        return (1,)
    if a.strategy == "channel":
        return (R, 1)
    if a.strategy in ("group", "tensor_group"):
        return (R, C // a.group_size)
    bh, bw = a.block_structure
    return (R // bh, C // bw)


def compress_weight(w: torch.Tensor, a) -> dict:
    """Same contract as ct_torch.compress_weight, computed by the C restatement."""
    assert w.dtype == torch.bfloat16 and w.dim() == 2
    w = w.contiguous()
    R, C = w.shape
    args = _Args(a.num_bits, 0 if a.type == "int" else 1, int(a.symmetric), ST[a.strategy],
                 a.group_size or 0, *(a.block_structure or (0, 0)),
                 {None: 0, "fp8": 2, "e8m0": 3}[a.scale_dtype])
    gshape = _n_groups(a, R, C)
    ng = int(np.prod(gshape))
    q = torch.empty(R, C, dtype=torch.uint8)
    sb = torch.empty(ng, dtype=torch.int16)
    zp = torch.empty(ng, dtype=torch.int8)
    gsc = torch.zeros(1, dtype=torch.float32)
    rc = lib().qref_quantize(_ptr(w), R, C, ctypes.byref(args), _ptr(q), _ptr(sb), _ptr(zp), _ptr(gsc))
    if rc != 0:
        raise ValueError("qref_quantize failed")
    out = {}
    if a.type == "int":
        pf = 32 // a.num_bits
        packed = torch.empty(R, (C + pf - 1) // pf, dtype=torch.int32)
        lib().qref_pack_int32(_ptr(q), R, C, a.num_bits, _ptr(packed))
        out["weight_packed"] = packed
        out["weight_scale"] = sb.view(torch.bfloat16).reshape(gshape)
        out["weight_shape"] = torch.tensor([R, C])
        if not a.symmetric and a.strategy in ("group", "channel"):
            z = zp.reshape(gshape).contiguous()
            H = (z.shape[0] + pf - 1) // pf
            zpk = torch.empty(H, z.shape[1], dtype=torch.int32)
            lib().qref_pack_int32_dim0(_ptr(z), z.shape[0], z.shape[1], a.num_bits, _ptr(zpk))
            out["weight_zero_point"] = zpk
        out["_q_int8"] = q.view(torch.int8)
        out["_zp_int8"] = zp.reshape(gshape)
    elif a.num_bits == 8:
        out["weight"] = q.view(torch.float8_e4m3fn)
        out["weight_scale"] = sb.view(torch.bfloat16).reshape(gshape)
    else:
        packed = torch.empty(R, C // 2, dtype=torch.uint8)
        lib().qref_pack_fp4(_ptr(q), R * C, _ptr(packed))
        out["weight_packed"] = packed
        if a.strategy == "tensor_group":
            out["weight_global_scale"] = gsc
            out["weight_scale"] = sb.to(torch.uint8).view(torch.float8_e4m3fn).reshape(gshape)
        else:
            out["weight_scale"] = sb.to(torch.uint8).reshape(gshape)
    return out


def int_sym_group_pack(w: torch.Tensor, bits: int, g: int):
    """Fused single-pass C leg timed by bench.py's cpu_baseline (1 thread)."""
    R, C = w.shape
    packed = torch.empty(R, C * bits // 32, dtype=torch.int32)
    scale = torch.empty(R, C // g, dtype=torch.bfloat16)
    rc = lib().qref_int_sym_group_pack(_ptr(w), R, C, bits, g, _ptr(packed), _ptr(scale))
    if rc != 0:
        raise ValueError("bad shape")
    return packed, scale
