"""The models' rotary position embedding of 128-wide heads in one HIP pass during the AWQ pass.

transformers' ``apply_rotary_pos_emb`` (with ``rotate_half``; the reference pins 4.57) runs a
cat, a negation and three elementwise kernels per tensor, twice per attention forward (q and k)
-- 21 attention forwards per layer in the AWQ grid.  ``fused_rotary`` swaps the function in every
model module whose ``apply_rotary_pos_emb`` / ``rotate_half`` are that exact code
(bytecode-equal to the restatements below) for one that runs ``qz_rotary128`` per tensor (the
same three roundings: bf16(x * cos), bf16(rotate_half(x) * sin), their bf16 sum) on bf16 GPU
heads of width 128 -- compared bit for bit with the original on its first call per device and
not used again if they differ.  The originals are restored when the context exits."""
from __future__ import annotations

import contextlib
import logging
import os
import sys
from typing import Dict

import torch
from torch import nn

from . import ops
from .moe_eager import _bits_equal
from .patching import same_code

log = logging.getLogger(__name__)

FUSED_ROTARY = os.environ.get("QZ_FUSED_ROTARY", "1") == "1"  # A/B knob: qz_rotary128 for apply_rotary_pos_emb
_OK: Dict[torch.device, bool] = {}  # qz_rotary128 verified against apply_rotary_pos_emb (per device)


def rotate_half(x):
    x1 = x[..., : x.shape[-1] // 2]
    x2 = x[..., x.shape[-1] // 2 :]
    return torch.cat((-x2, x1), dim=-1)


def apply_rotary_pos_emb(q, k, cos, sin, unsqueeze_dim=1):
    cos = cos.unsqueeze(unsqueeze_dim)
    sin = sin.unsqueeze(unsqueeze_dim)
    q_embed = (q * cos) + (rotate_half(q) * sin)
    k_embed = (k * cos) + (rotate_half(k) * sin)
    return q_embed, k_embed


def _eligible(t: torch.Tensor, cos: torch.Tensor, sin: torch.Tensor) -> bool:
    return (t.is_cuda and t.dtype == torch.bfloat16 and t.dim() == 4 and t.shape[-1] == 128 and t.stride(-1) == 1
            and t.numel() > 0 and t.data_ptr() % 8 == 0 and all(s % 4 == 0 for s in t.stride()[:-1])
            and cos.dtype == torch.bfloat16 and sin.dtype == torch.bfloat16 and cos.dim() == 3
            and cos.shape == sin.shape and cos.stride() == sin.stride() and cos.shape[0] in (1, t.shape[0])
            and cos.shape[1] == t.shape[2] and cos.shape[2] == 128 and cos.stride(-1) == 1
            and all(s % 4 == 0 for s in cos.stride()[:-1]) and cos.data_ptr() % 8 == 0 and sin.data_ptr() % 8 == 0)


def _fused(orig):
    def apply(q, k, cos, sin, unsqueeze_dim=1):
        if unsqueeze_dim != 1 or not (_eligible(q, cos, sin) and _eligible(k, cos, sin)):
            return orig(q, k, cos, sin, unsqueeze_dim)
        ok = _OK.get(q.device)
        if ok is None:
            want = orig(q, k, cos, sin, unsqueeze_dim)
            try:
                ok = _bits_equal(ops.rotary128(q, cos, sin), want[0]) and _bits_equal(ops.rotary128(k, cos, sin), want[1])
            except (RuntimeError, ValueError) as e:
                log.info("rotary: qz_rotary128 unavailable (%s)", e)
                ok = False
            _OK[q.device] = ok
            if not ok:
                log.info("rotary: qz_rotary128 differs from apply_rotary_pos_emb on %s; the original kept", q.device)
            return want
        if not ok:
            return orig(q, k, cos, sin, unsqueeze_dim)
        return ops.rotary128(q, cos, sin), ops.rotary128(k, cos, sin)
    apply.__qz_fused__ = True
    return apply


@contextlib.contextmanager
def fused_rotary(model: nn.Module):
    """Inside the context, every module that defines one of ``model``'s classes and holds the
    reference ``apply_rotary_pos_emb`` / ``rotate_half`` uses the fused version."""
    patched = []
    try:
        if FUSED_ROTARY:
            seen = set()
            for m in model.modules():
                name = type(m).__module__
                if name in seen:
                    continue
                seen.add(name)
                mod = sys.modules.get(name)
                fn = getattr(mod, "apply_rotary_pos_emb", None)
                if (fn is not None and not getattr(fn, "__qz_fused__", False) and same_code(fn, apply_rotary_pos_emb)
                        and same_code(getattr(mod, "rotate_half", None), rotate_half)):
                    mod.apply_rotary_pos_emb = _fused(fn)
                    patched.append((mod, fn))
        yield len(patched)
    finally:
        for mod, fn in patched:
            mod.apply_rotary_pos_emb = fn
