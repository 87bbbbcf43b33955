"""Model introspection: which weights the recipe targets, under the reference's names.

The reference pins transformers 4.57, where MoE experts are per-expert ``nn.Linear`` modules
(``...mlp.experts.<e>.gate_proj``); this image has transformers 5.x, which fuses them into 3-D
parameters (``experts.gate_up_proj [E, 2I, H]``, ``experts.down_proj [E, H, I]``; SURVEY.md
finding 5).  ``iter_linears`` presents both layouts under the 4.57 per-expert names, so the
reference's recipe regexes (e.g. recipe_MoE_RTN_NVFP4.yaml:21) match either way, and groups
same-shaped expert slices so the GPU kernel quantizes all experts of a layer in one launch
(the C ABI's batch dimension).
"""
from __future__ import annotations

import re

from dataclasses import dataclass
from typing import Dict, List, Optional, Tuple

import torch
from torch import nn


@dataclass
class LinearRef:
    """One quantization target: a 2-D weight [out, in] (possibly a view into a fused param)."""

    name: str
    module: nn.Module
    param_name: str  # attribute on ``module`` holding the storage
    index: Optional[Tuple[int, slice]] = None  # (expert, row slice) for fused experts
    type_name: str = "Linear"

    @property
    def weight(self) -> torch.Tensor:
        p = getattr(self.module, self.param_name)
        if self.index is None:
            return p.data
        e, rows = self.index
        return p.data[e, rows]

    @property
    def bias(self) -> Optional[torch.Tensor]:
        if self.index is None:
            b = getattr(self.module, "bias", None)
            return b.data if b is not None else None
        return None


def _fused_expert_specs(mod: nn.Module):
    """Known fused-expert parameter layouts -> [(param, [(proj_name, row_slice_fn)])]."""
    specs = []
    if hasattr(mod, "gate_up_proj") and isinstance(getattr(mod, "gate_up_proj"), nn.Parameter) \
            and getattr(mod, "gate_up_proj").dim() == 3:
        two_i = mod.gate_up_proj.shape[1]
        half = two_i // 2
        specs.append(("gate_up_proj", [("gate_proj", slice(0, half)), ("up_proj", slice(half, two_i))]))
    if hasattr(mod, "down_proj") and isinstance(getattr(mod, "down_proj"), nn.Parameter) \
            and getattr(mod, "down_proj").dim() == 3:
        specs.append(("down_proj", [("down_proj", slice(None))]))
    # MiniMax-style w1/w3 (gate/up) and w2 (down) fused variants
    for pn, proj in (("w1", "w1"), ("w2", "w2"), ("w3", "w3")):
        p = getattr(mod, pn, None)
        if isinstance(p, nn.Parameter) and p.dim() == 3:
            specs.append((pn, [(proj, slice(None))]))
    return specs


# transformers-5 runtime names -> the checkpoint names of the transformers version the reference
# pins (4.57).  Mixtral-family MoE blocks are ``block_sparse_moe`` with experts ``w1`` (gate),
# ``w3`` (up), ``w2`` (down) on disk (transformers/conversion_mapping.py "mixtral"/"minimax_m2");
# Qwen-style MoE keeps ``mlp.experts.<e>.{gate,up,down}_proj``.
MIXTRAL_FAMILY = ("mixtral", "minimax", "minimax_m2")


def model_type(model: nn.Module) -> str:
    return getattr(getattr(model, "config", None), "model_type", "") or ""


def checkpoint_name(name: str, mtype: str) -> str:
    if mtype in MIXTRAL_FAMILY:
        return re.sub(r"\.mlp(?=\.|$)", ".block_sparse_moe", name)
    return name


def _expert_proj_names(mtype: str):
    if mtype in MIXTRAL_FAMILY:
        return {"gate_proj": "w1", "up_proj": "w3", "down_proj": "w2"}
    return {"gate_proj": "gate_proj", "up_proj": "up_proj", "down_proj": "down_proj"}


def iter_linears(model: nn.Module, prefix: str = "", mtype: Optional[str] = None) -> List[LinearRef]:
    """Every quantization target under ``model`` with its checkpoint name (``prefix`` is
    prepended for a sub-module such as one decoder layer)."""
    mtype = model_type(model) if mtype is None else mtype
    pn = _expert_proj_names(mtype)
    out: List[LinearRef] = []
    for name, mod in model.named_modules():
        if prefix:
            name = f"{prefix}.{name}" if name else prefix
        if isinstance(mod, nn.Linear):
            out.append(LinearRef(name=checkpoint_name(name, mtype), module=mod, param_name="weight", type_name="Linear"))
            continue
        for pname, projs in _fused_expert_specs(mod):
            n_exp = getattr(mod, pname).shape[0]
            for e in range(n_exp):
                for proj, rows in projs:
                    out.append(LinearRef(name=checkpoint_name(f"{name}.{e}.{pn.get(proj, proj)}", mtype), module=mod,
                                         param_name=pname, index=(e, rows), type_name="Linear"))
    return out


def is_fused_experts(mod: nn.Module) -> bool:
    return bool(_fused_expert_specs(mod))


def batch_groups(refs: List[LinearRef]) -> List[List[LinearRef]]:
    """Group refs that are same-shaped slices of one fused parameter (one kernel launch)."""
    groups: Dict[Tuple[int, str, str], List[LinearRef]] = {}
    order: List[Tuple[int, str, str]] = []
    for r in refs:
        if r.index is None:
            key = (id(r), "", "")
        else:
            key = (id(r.module), r.param_name, str(r.index[1]))
        if key not in groups:
            groups[key] = []
            order.append(key)
        groups[key].append(r)
    return [groups[k] for k in order]


def stacked_view(group: List[LinearRef]) -> torch.Tensor:
    """[E, rows, cols] strided view over a fused-expert group (or [1, r, c] for a Linear)."""
    if len(group) == 1 and group[0].index is None:
        return group[0].weight.unsqueeze(0)
    r0 = group[0]
    p = getattr(r0.module, r0.param_name).data
    experts = [g.index[0] for g in group]
    if experts != list(range(experts[0], experts[0] + len(experts))):
        return torch.stack([g.weight for g in group])
    return p[experts[0]:experts[0] + len(experts), r0.index[1]]


def decoder_layers(model: nn.Module) -> nn.ModuleList:
    """The transformer block list (model.model.layers for HF causal LMs)."""
    n = getattr(getattr(model, "config", None), "num_hidden_layers", None)
    for name, mod in model.named_modules():
        if isinstance(mod, nn.ModuleList) and len(mod) > 0 and (n is None or len(mod) == n):
            if name.endswith("layers") or name.endswith(".h") or name.endswith("blocks"):
                return mod
    raise ValueError("could not find the decoder layer list")
