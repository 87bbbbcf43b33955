"""Helpers for the AWQ pass's in-place forward swaps (dense_mlp, dense_norm, rotary, moe_eager):
a swap applies only to code that is exactly the transformers code it restates."""
from __future__ import annotations

import dis
from typing import Callable, List, Tuple


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
