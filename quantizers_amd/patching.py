"""Helpers for the AWQ pass's in-place forward swaps (dense_mlp, dense_norm, rotary, moe_eager):
a swap applies only to code that is exactly the transformers code it restates; and the guard
that keeps the pass off the pinned hipBLASLt fault (``bmm_guard``)."""
from __future__ import annotations

import contextlib
import dis
import logging
import os
from typing import Callable, List, Tuple

import torch

log = logging.getLogger(__name__)


def _instructions(fn: Callable) -> List[Tuple[str, object]]:
    code = fn.__code__
    out = []
    for ins in dis.get_instructions(code):
        val = ins.argval
        if hasattr(val, "co_code"):  # nested code objects: compare by their own instructions
            val = tuple(_instructions(type("F", (), {"__code__": val})))
        out.append((ins.opname, val))
    return out


def same_code(fn, ref: Callable) -> bool:
    """``fn`` (or the function it wraps) has the same instructions and operand values as ``ref``
    -- docstrings, names of the file / line numbers aside."""
    fn = getattr(fn, "__wrapped__", fn)
    if getattr(fn, "__code__", None) is None:
        return False
    try:
        return _instructions(fn) == _instructions(ref)
    except TypeError:
        return False


# --------------------------------------------------------------------------------------------
# Guard against the pinned library fault: torch 2.10's bundled hipBLASLt raised
# hipErrorIllegalAddress on MI355X for a bf16 strided-batched GEMM in the "NT" layout of
# F.linear -- torch.bmm(x [16, 2048, 768], out [16, 2048, 768].transpose(1, 2)), K = 768
# (profiles/r03b_bmm_probe.log, reproduced with no repository code loaded).  Nothing in this
# repository issues such a product, but a model's own forward could during the AWQ pass; inside
# ``bmm_guard()`` every bf16 batched product of that layout and inner size runs as one 2-D GEMM
# per batch entry instead of the strided-batched kernel (logged once per shape).
PINNED_BMM_K = 768
_ROUTE_DEVICES = ("cuda",)  # tests add "cpu" to exercise the routing without a GPU
_routed_shapes: set = set()


def pinned_bmm_defect(a, b) -> bool:
    """True for a bf16 batched product a [..., M, K] @ b [..., K, N] whose b is a transposed view
    (stride(-2) == 1: the NT layout) with K == 768 and equal batch dims -- the pinned fault's class."""
    return (isinstance(a, torch.Tensor) and isinstance(b, torch.Tensor) and a.dtype == torch.bfloat16
            and b.dtype == torch.bfloat16 and a.dim() >= 3 and a.dim() == b.dim()
            and a.shape[:-2] == b.shape[:-2] and a.shape[-1] == PINNED_BMM_K and b.shape[-2] == PINNED_BMM_K
            and b.stride(-2) == 1 and b.stride(-1) != 1 and a.device.type in _ROUTE_DEVICES)


def _per_batch_mm(a, b):
    key = (tuple(a.shape), tuple(b.shape))
    if key not in _routed_shapes:
        _routed_shapes.add(key)
        log.warning("bmm_guard: bf16 NT batched GEMM %s @ %s (K=%d, the pinned hipBLASLt fault's class) runs "
                    "as per-batch 2-D GEMMs", key[0], key[1], PINNED_BMM_K)
    lead = a.shape[:-2]
    a3, b3 = a.reshape(-1, *a.shape[-2:]), b.reshape(-1, *b.shape[-2:])
    # torch.stack of plain mm results (no out=): stays autograd-safe if a forward inside the
    # guard runs with grad enabled
    out = torch.stack([torch.mm(a3[i], b3[i]) for i in range(a3.shape[0])])
    return out.reshape(*lead, a.shape[-2], b.shape[-1])


BMM_GUARD = True


@contextlib.contextmanager
def bmm_guard():
    """torch.bmm / torch.matmul / Tensor.matmul / Tensor.__matmul__ with the pinned defect's
    operands go through ``_per_batch_mm`` inside the context; everything else is untouched.
    ``BMM_GUARD = False`` leaves torch as it is."""
    if not BMM_GUARD:
        yield
        return
    saved = (torch.bmm, torch.matmul, torch.Tensor.matmul, torch.Tensor.__matmul__)

    def wrap(orig):
        # anything but the defect's operands goes to the original, whose result is returned as is:
        # Tensor.__matmul__'s NotImplemented for a non-tensor operand (so __rmatmul__ runs) included
        def f(a, b, *args, **kw):
            if not args and not kw and pinned_bmm_defect(a, b):
                return _per_batch_mm(a, b)
            return orig(a, b, *args, **kw)
        f.__wrapped_orig__ = orig
        return f
    torch.bmm, torch.matmul = wrap(saved[0]), wrap(saved[1])
    torch.Tensor.matmul, torch.Tensor.__matmul__ = wrap(saved[2]), wrap(saved[3])
    try:
        yield
    finally:
        torch.bmm, torch.matmul, torch.Tensor.matmul, torch.Tensor.__matmul__ = saved
