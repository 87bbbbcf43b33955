"""AWQ (activation-aware weight quantization) on the MI355X kernels.

Restates the algorithm of [3P] llmcompressor ``AWQModifier`` (llmcompressor>=0.9, called from
scripts/do_oneshot.py:179-187 through the recipes' ``AWQModifier`` blocks, e.g.
configs/recipes/recipe_awq_w4a16.yaml:11-31):

1. per smooth->balance mapping, the running mean |x| of the balance layers' input channels
   (``qz_awq_absmean_accum``; fp32 sums, decision D8);
2. ``w_mean`` = mean over rows of |W| / (group absmax + 1e-6) over the balance layers
   (``qz_awq_weight_mean_accum``; bf16 elementwise, fp64 sums);
3. a grid of ``n_grid`` ratios r: s = clamp(x_mean^r / (w_mean^(1-r) + 1e-4), 1e-4),
   normalised by sqrt(max*min) (``qz_awq_grid_scales``); each balance layer's weight is
   replaced by Q(W*s)/s in one fused pass (``qz_awq_fake_quant``) with that layer's own
   scheme, the parent module re-runs on the cached inputs, and the MSE against the
   unquantized outputs picks the first best ratio (strict <);
4. ``_apply_smoothing``: balance W[:, c] *= s[c]; smooth norm w /= s, or a smooth Linear's
   last len(s) output rows (and bias) /= s (``qz_scale_columns`` / ``qz_scale_rows``).

Mappings whose balance in_features differ from the smooth layer's output width are skipped
(GQA v_proj->o_proj, decision D9).  The parent forwards are PyTorch GEMMs.
"""
from __future__ import annotations

import logging
import re
from dataclasses import dataclass
from typing import Any, Dict, List, Optional, Tuple

import torch
from torch import nn

from . import ops
from .quantization import QuantizationArgs
from .recipe import AWQMapping

log = logging.getLogger(__name__)

# llmcompressor's default mappings for Llama/Qwen-style decoder blocks
DEFAULT_MAPPINGS = [
    AWQMapping("re:.*input_layernorm$", ["re:.*q_proj$", "re:.*k_proj$", "re:.*v_proj$"]),
    AWQMapping("re:.*v_proj$", ["re:.*o_proj$"]),
    AWQMapping("re:.*post_attention_layernorm$", ["re:.*gate_proj$", "re:.*up_proj$"]),
    AWQMapping("re:.*up_proj$", ["re:.*down_proj$"]),
]


def _rx(t: str) -> str:
    return t[3:] if t.startswith("re:") else re.escape(t) + "$"


@dataclass
class ResolvedMapping:
    smooth_name: str
    smooth: nn.Module
    balance_names: List[str]
    balance: List[nn.Linear]
    parent_name: str
    parent: nn.Module


def _common_parent(names: List[str]) -> str:
    parts = [n.split(".") for n in names]
    common = []
    for xs in zip(*parts):
        if all(x == xs[0] for x in xs):
            common.append(xs[0])
        else:
            break
    return ".".join(common)


def resolve_mappings(layer: nn.Module, prefix: str, mappings: List[AWQMapping],
                     quantized: Dict[str, QuantizationArgs]) -> List[ResolvedMapping]:
    """Resolve regex mappings inside one decoder layer (names are relative to the model)."""
    mods = {f"{prefix}.{n}" if n else prefix: m for n, m in layer.named_modules()}
    out: List[ResolvedMapping] = []
    for mp in mappings:
        srx = _rx(mp.smooth_layer)
        smooth_names = [n for n in mods if re.match(srx, n)]
        for sname in smooth_names:
            # balance layers: in the same sub-block as the smooth layer (closest matches)
            balance = []
            for brx in mp.balance_layers:
                cands = [n for n, m in mods.items() if re.match(_rx(brx), n) and isinstance(m, nn.Linear)]
                if not cands:
                    continue
                # pick the candidate sharing the longest prefix with the smooth layer
                best = max(cands, key=lambda n: len(_common_parent([n, sname])))
                balance.append(best)
            if not balance:
                continue
            smod = mods[sname]
            width = smod.weight.shape[0]
            lin = [mods[b] for b in balance]
            if any(l.in_features != width for l in lin):
                log.info("AWQ: skipping mapping %s -> %s (shape mismatch, D9)", sname, balance)
                continue
            if not all(b in quantized for b in balance):
                log.info("AWQ: skipping mapping %s -> %s (balance layers not quantized)", sname, balance)
                continue
            pname = balance[0] if len(balance) == 1 else _common_parent(balance)
            out.append(ResolvedMapping(sname, smod, balance, lin, pname, mods[pname]))
    return out


class _ParentCache:
    """Forward pre-hook on a parent module: cache its (args, kwargs) per calibration batch."""

    def __init__(self, module: nn.Module):
        self.calls: List[Tuple[tuple, dict]] = []
        self.h = module.register_forward_pre_hook(self._hook, with_kwargs=True)

    def _hook(self, mod, args, kwargs):
        self.calls.append((tuple(a.detach() if torch.is_tensor(a) else a for a in args), dict(kwargs)))

    def remove(self):
        self.h.remove()


class _AbsMean:
    """Forward pre-hook on a balance layer: sum |x| per input channel (GPU kernel)."""

    def __init__(self, module: nn.Linear):
        self.sum = None
        self.count = 0
        self.h = module.register_forward_pre_hook(self._hook)

    def _hook(self, mod, args):
        x = args[0]
        if self.sum is None:
            self.sum = torch.zeros(x.shape[-1], dtype=torch.float32, device=x.device)
        self.count += ops.awq_absmean_accum(x.detach(), self.sum)

    def mean(self) -> torch.Tensor:
        return self.sum / max(self.count, 1)

    def remove(self):
        self.h.remove()


def _run_parent(parent: nn.Module, calls) -> List[torch.Tensor]:
    outs = []
    for args, kwargs in calls:
        o = parent(*args, **kwargs)
        if isinstance(o, tuple):
            o = o[0]
        outs.append(o)
    return outs


def _loss(ref: List[torch.Tensor], got: List[torch.Tensor]) -> float:
    tot = torch.zeros((), dtype=torch.float64, device=ref[0].device)
    n = 0
    for a, b in zip(ref, got):
        tot += (a - b).reshape(-1).float().pow(2).sum().double()
        n += a.numel()
    return (tot / n).item()


def _group_size_for_mean(a: QuantizationArgs, cols: int) -> int:
    if a.strategy in ("group", "tensor_group"):
        return a.group_size
    if a.strategy in ("channel", "block"):
        return cols  # D9b: block / channel balance layers normalised per row
    return cols


@torch.no_grad()
def awq_layer(layer: nn.Module, prefix: str, layer_inputs: List[Tuple[tuple, dict]], mappings: List[AWQMapping],
              quantized: Dict[str, QuantizationArgs], duo_scaling: bool = True, n_grid: int = 20) -> Dict[str, Any]:
    """Run AWQ on one decoder layer in place.  ``layer_inputs`` are the cached (args, kwargs)
    of the layer for every calibration batch.  Returns per-mapping diagnostics."""
    resolved = resolve_mappings(layer, prefix, mappings, quantized)
    if not resolved:
        return {}
    # 1. one calibration pass: activation statistics + parent inputs
    stats = {r.smooth_name: _AbsMean(r.balance[0]) for r in resolved}
    caches = {r.smooth_name: _ParentCache(r.parent) for r in resolved}
    try:
        for args, kwargs in layer_inputs:
            layer(*args, **kwargs)
    finally:
        for h in list(stats.values()) + list(caches.values()):
            h.remove()
    report = {}
    for r in resolved:
        x_mean = stats[r.smooth_name].mean()
        # 2. w_mean over the balance layers (each with its own group size)
        cols = r.balance[0].in_features
        wsum = torch.zeros(cols, dtype=torch.float64, device=x_mean.device)
        rows = 0
        for name, lin in zip(r.balance_names, r.balance):
            rows += ops.awq_weight_mean_accum(lin.weight.data, _group_size_for_mean(quantized[name], cols), wsum)
        w_mean = (wsum / rows).float()
        calls = caches[r.smooth_name].calls
        ref_out = _run_parent(r.parent, calls)
        # 3. grid search
        orig = [lin.weight.data.clone() for lin in r.balance]
        best, best_ratio, best_scales, history = float("inf"), -1.0, None, []
        scales = torch.empty_like(x_mean)
        for i in range(n_grid):
            ratio = i / n_grid
            ops.awq_grid_scales(x_mean, w_mean, ratio, duo_scaling, out=scales)
            for name, lin, w0 in zip(r.balance_names, r.balance, orig):
                ops.fake_quantize(w0, quantized[name], col_scales=scales, out=lin.weight.data)
            loss = _loss(ref_out, _run_parent(r.parent, calls))
            history.append(loss)
            if loss < best:
                best, best_ratio, best_scales = loss, ratio, scales.clone()
        for lin, w0 in zip(r.balance, orig):
            lin.weight.data.copy_(w0)
        if best_scales is None:
            raise RuntimeError(f"AWQ: no finite loss for {r.smooth_name} (history {history})")
        # 4. apply smoothing
        for lin in r.balance:
            ops.scale_columns_(lin.weight.data, best_scales, divide=False)
        sw = r.smooth.weight.data
        if sw.dim() == 1:
            ops.scale_rows_(sw, best_scales, divide=True)
        else:
            ops.scale_rows_(sw[-best_scales.numel():], best_scales, divide=True)
        b = getattr(r.smooth, "bias", None)
        if b is not None:
            ops.scale_rows_(b.data[-best_scales.numel():], best_scales, divide=True)
        report[r.smooth_name] = {"balance": r.balance_names, "best_ratio": best_ratio, "best_loss": best,
                                 "history": history}
        del ref_out
    return report
