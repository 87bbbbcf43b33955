"""Dense gated MLPs in the model's own arithmetic with the SiLU·up step as one HIP pass.

transformers' dense MLPs (Qwen3MLP, LlamaMLP, ... -- the reference pins 4.57) compute
``down_proj(act_fn(gate_proj(x)) * up_proj(x))``: between the projections a SiLU pass and a
multiply pass over [tokens, intermediate] bf16.  During the AWQ pass (calibration, the 20-point
grid of the gate/up mapping whose parent is the MLP, propagation) ``fused_mlps`` gives every such
module a forward that calls the same three Linear modules in the same order (their hooks fire as
before) and replaces the two elementwise passes by ``qz_silu_mul`` -- compared bit for bit with
``act_fn(gate) * up`` on its first call per device and not used again if they differ.

A module qualifies when its class's forward is that exact expression (bytecode-equal to
``_reference_forward``), its projections are ``nn.Linear`` and its activation is a SiLU."""
from __future__ import annotations

import contextlib
import logging
import os
from typing import Dict

import torch
from torch import nn

from . import ops
from .moe_eager import _bits_equal
from .patching import same_code

log = logging.getLogger(__name__)

FUSED_MLP = os.environ.get("QZ_FUSED_MLP", "1") == "1"  # A/B knob: qz_silu_mul in dense MLP forwards
_OK: Dict[torch.device, bool] = {}  # qz_silu_mul verified against act_fn(gate) * up (per device)


def _reference_forward(self, x):
    down_proj = self.down_proj(self.act_fn(self.gate_proj(x)) * self.up_proj(x))
    return down_proj


def qualifies(m: nn.Module) -> bool:
    return (same_code(type(m).forward, _reference_forward)
            and all(isinstance(getattr(m, n, None), nn.Linear) for n in ("gate_proj", "up_proj", "down_proj"))
            and type(getattr(m, "act_fn", None)).__name__ in ("SiLUActivation", "SiLU")
            and not getattr(m.act_fn, "inplace", False))


class FusedMLP:
    """Instance-level forward for one qualifying MLP (see the module docstring)."""

    def __init__(self, module: nn.Module):
        self.m = module

    def forward(self, x):
        m = self.m
        gate, up = m.gate_proj(x), m.up_proj(x)
        if not (gate.is_cuda and gate.dtype == torch.bfloat16 and up.dtype == torch.bfloat16 and gate.numel()):
            return m.down_proj(m.act_fn(gate) * up)
        ok = _OK.get(gate.device)
        if ok is None:
            want = m.act_fn(gate) * up
            ok = _OK[gate.device] = _bits_equal(ops.silu_mul(gate, up), want)
            if not ok:
                log.info("MLP: qz_silu_mul differs from act_fn(gate) * up on %s; composed ops kept", gate.device)
            return m.down_proj(want)
        return m.down_proj(ops.silu_mul(gate, up) if ok else m.act_fn(gate) * up)


@contextlib.contextmanager
def fused_mlps(model: nn.Module):
    """Every qualifying dense MLP of ``model`` forwards through ``FusedMLP`` inside the context
    (GPU bf16 only; CPU tensors take the composed ops); the class forwards are restored after."""
    patched = []
    try:
        if FUSED_MLP:
            for mod in model.modules():
                if "forward" not in mod.__dict__ and qualifies(mod):
                    mod.forward = FusedMLP(mod).forward  # instance attribute: Module.__call__ uses it
                    patched.append(mod)
        yield len(patched)
    finally:
        for mod in patched:
            if "forward" in mod.__dict__:
                del mod.forward
