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

Mapping resolution follows llmcompressor ``_set_resolved_mappings``: every module matching
``smooth_layer``; its balance layers are all targets under the smooth layer's parent matching
a ``balance_layers`` regex; a Linear balance whose in_features differ from a Linear smooth
layer's out_features is dropped (GQA v_proj->o_proj, decision D9); the loss parent is the
single balance layer, else the lowest common ancestor that is not a ModuleList.

MoE experts (transformers-5 fused ``gate_up_proj`` / ``down_proj`` parameters) are resolved
under the per-expert names of the reference's transformers 4.57 layout (model.py), so the
MiniMax recipes' ``post_attention_layernorm -> w1, w3`` (all experts, parent = the MoE block)
and ``w3 -> w2`` (one expert, parent = that expert's w2) mappings work unchanged
(recipe_Minimax-M2.1-AWQ-MixedPrec.yaml:49-56).  ``moe_calibrate_all_experts=True`` semantics:
an expert's linears see every calibration token (the experts module's input), not only the
tokens routed to it; with False, only the routed tokens (from the router's top-k indices).
Inputs of a per-expert ``w2`` are recomputed from the cached experts input and a snapshot of
the pre-smoothing gate/up weights, so nothing of size tokens x experts is kept resident.
The parent forwards are PyTorch GEMMs; the grid's losses stay on the device (one host sync
per mapping).
"""
from __future__ import annotations

import contextlib
import logging
import os
import re
import threading
from dataclasses import dataclass
from typing import Any, Callable, Dict, List, Optional, Tuple

import numpy as np
import torch
from torch import nn

from . import _lib, moe_eager, ops
from .model import LinearRef, batch_groups, checkpoint_name, is_fused_experts, iter_linears, stacked_view
from .quantization import QuantizationArgs
from .recipe import AWQMapping

log = logging.getLogger(__name__)

PHASE_TIMING = False  # diagnostics (set True): synchronised per-phase wall times, logged per layer

# D8: the dtype of the AWQ statistics and grid scales.  "bf16" (default since round 5): SURVEY
# A.6's reading of llmcompressor -- the running mean |x| kept in the activation dtype
# ((prev_mean * prev_n + batch_sum) / n, every op rounded to bf16; the batch sum accumulated in
# f32 and rounded once), w_mean a bf16 column sum per balance layer summed in bf16, the grid scale
# formula evaluated in bf16, so W * s, Q(W*s)/s and the smoothing multiply by bf16 scales.  "fp32":
# rounds 1-4 (x_mean f32 sums, w_mean f64 sums, scales f32).  On a 2-layer Qwen3-4B the two
# readings differ in 3 of 6 argmins and 17.9 % of the packed int4 words (profiles/r05_d8_probe.txt),
# so the choice is exposed (oneshot(awq_dtype=...), --awq-dtype).  The grid loss is an f64 sum of
# f32(bf16(a - b))^2 in both (llmcompressor's f32 per-batch sum differs only in summation order).
AWQ_DTYPES = ("bf16", "fp32")
AWQ_DTYPE = "bf16"


def _div_count_bf16(t: torch.Tensor, n: int) -> torch.Tensor:
    """bf16 tensor / a token or row count as torch's GPU kernel computes it (the product with the
    f32 reciprocal of the count; DESIGN.md §4 D8 "device semantics"), written out so the bits do not
    depend on the tensor's device (torch's CPU kernel divides)."""
    return (t.float() * float(np.float32(1.0) / np.float32(n))).to(torch.bfloat16)


def _running_mean_bf16(parts) -> Optional[torch.Tensor]:
    """llmcompressor's _accumulate_mean in bf16 over per-batch f32 sums [(sum [C], n), ...] in
    batch order: m = s_0 / n_0, then m = (m * count + s_j) / (count + n_j), each division by a
    count in torch's GPU form (``_div_count_bf16``; oracle: ct_torch.awq_running_mean_from_sums_literal
    with device_division=True)."""
    m, c = None, 0
    for part, n in parts:
        if n == 0:
            continue
        sb = part.to(torch.bfloat16)
        m = _div_count_bf16(sb if m is None else m * c + sb, c + n)
        c += n
    return m


def _layer_means_bf16(parts) -> torch.Tensor:
    """_compute_layer_means' bf16 combination of per-balance-layer column sums [(sum, rows), ...]
    in balance order: each sum rounded once to bf16, added in bf16, / the total rows in torch's GPU
    form (oracle: ct_torch.awq_layer_means_from_sums_literal, device_division=True)."""
    acc, rows = None, 0
    for part, n in parts:
        sb = part.to(torch.bfloat16)
        acc = sb if acc is None else acc + sb
        rows += n
    return _div_count_bf16(acc, rows)


def _running_means_bf16(parts: torch.Tensor, counts: List[List[int]]) -> torch.Tensor:
    """``_running_mean_bf16`` for E operands at once: parts [E, P, C] f32 per-batch sums, counts
    [E][P] tokens.  Each step is the op the per-operand form issues with Python-int scalars on the
    device -- bf16(f32(m) * c), bf16 + bf16, and the division by a scalar as a product with its f32
    reciprocal (PyTorch's GPU kernel for a tensor / CPU-scalar division) -- taken with per-operand
    f32 factors, so every row is bit-identical to the per-operand loop.  The factors of all steps
    go to the device in one pinned, non-blocking copy (a pageable copy per step would make the
    host wait for the stream).  Operands without tokens give 0."""
    import numpy as np
    E, P, C = parts.shape
    dev = parts.device
    n = np.asarray(counts, dtype=np.int64).reshape(E, P)
    fac = np.zeros((P, 4, E), dtype=np.float32)  # [step][c, 1/(c+n), first, apply][operand]
    seen = np.zeros(E, dtype=np.int64)
    steps = []
    for j in range(P):
        live = n[:, j] > 0
        if not live.any():
            continue
        fac[j, 0] = seen.astype(np.float32)
        fac[j, 1] = 1.0
        fac[j, 1, live] = np.float32(1.0) / (seen[live] + n[live, j]).astype(np.float32)
        fac[j, 2] = live & (seen == 0)
        fac[j, 3] = live
        seen = seen + np.where(live, n[:, j], 0)
        steps.append(j)
    f = torch.from_numpy(fac)
    if dev.type == "cuda":
        f = f.pin_memory().to(dev, non_blocking=True)
    m = torch.zeros(E, C, dtype=torch.bfloat16, device=dev)
    for j in steps:
        cf, inv, first, apply = (f[j, k][:, None] for k in range(4))
        sb = parts[:, j].to(torch.bfloat16)
        t = torch.where(first > 0, sb, (m.float() * cf).to(torch.bfloat16) + sb)
        m = torch.where(apply > 0, (t.float() * inv).to(torch.bfloat16), m)
    return m


def _grid_scales_bf16(x_mean: torch.Tensor, w_mean: Optional[torch.Tensor], ratio: float, duo: bool,
                      out: Optional[torch.Tensor] = None) -> torch.Tensor:
    """One grid point's scale vector(s) evaluated in bf16 as torch evaluates llmcompressor's
    formula on bf16 statistics ([C] or a [B, C] stack of independent mappings): clamp(x^r /
    (w^(1-r) + 1e-4), 1e-4) / sqrt(max * min), inf / nan -> 1.  Returned as f32 (exact bf16
    values) for the kernels' column-scale arguments."""
    xb = x_mean.to(torch.bfloat16)
    if duo:
        s = (xb.pow(ratio) / (w_mean.to(torch.bfloat16).pow(1 - ratio) + 1e-4)).clamp(min=1e-4)
    else:
        s = xb.pow(ratio).clamp(min=1e-4)
    s = s / (s.amax(-1, keepdim=True) * s.amin(-1, keepdim=True)).sqrt()
    s = torch.where(torch.isinf(s) | torch.isnan(s), torch.ones_like(s), s)
    if out is None:
        return s.float()
    out.copy_(s)
    return out


PHASES: Dict[str, float] = {}  # phase name -> seconds, accumulated while PHASE_TIMING


@contextlib.contextmanager
def phase(name: str):
    """Accumulate the synchronised wall time of a block under ``name`` (only with the module
    constant ``awq.PHASE_TIMING = True``: the synchronisations perturb the overlap they measure, so
    it is a diagnostic mode)."""
    if not PHASE_TIMING:
        yield
        return
    import time
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    try:
        yield
    finally:
        torch.cuda.synchronize()
        PHASES[name] = PHASES.get(name, 0.0) + time.perf_counter() - t0
_D9_LOGGED: set = set()  # (layer class, balance suffix) pairs already reported at INFO

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
    smooth: Any                      # norm / Linear module, or a LinearRef (virtual expert linear)
    balance_names: List[str]
    balance: List[LinearRef]
    parent_name: str
    parent: Optional[nn.Module]      # real module re-run for the loss; None = virtual
    parent_kind: str = "module"      # "module" | "linear" (one virtual linear) | "expert" (one expert MLP)
    parent_expert: int = -1
    origin: int = -1                 # index of the AWQMapping it came from


def _common_parent(names: List[str]) -> str:
    parts = [n.split(".") for n in names]
    common = []
    for xs in zip(*parts):
        if all(x == xs[0] for x in xs):
            common.append(xs[0])
        else:
            break
    return ".".join(common)


def _out_features(m) -> int:
    return m.weight.shape[0]


def resolve_mappings(layer: nn.Module, prefix: str, mappings: List[AWQMapping],
                     quantized: Dict[str, QuantizationArgs], mtype: str = "") -> List[ResolvedMapping]:
    """Resolve regex mappings inside one decoder layer (names are checkpoint names)."""
    mods = {checkpoint_name(f"{prefix}.{n}" if n else prefix, mtype): m for n, m in layer.named_modules()}
    lins = {r.name: r for r in iter_linears(layer, prefix, mtype)}
    virtual = {n: r for n, r in lins.items() if r.index is not None}
    out: List[ResolvedMapping] = []
    for mi, mp in enumerate(mappings):
        srx = _rx(mp.smooth_layer)
        snames = [n for n in mods if re.match(srx, n)] + [n for n in virtual if re.match(srx, n)]
        for sname in snames:
            smooth = virtual.get(sname) or mods[sname]
            sparent = sname.rpartition(".")[0]
            smooth_is_linear = isinstance(smooth, (nn.Linear, LinearRef))
            width = smooth.weight.shape[0]
            balance: List[str] = []
            for brx in mp.balance_layers:
                for n in lins:
                    if not n.startswith(sparent + ".") or n in balance:
                        continue
                    if not re.match(_rx(brx), n[len(sparent) + 1:]):
                        continue
                    if smooth_is_linear and lins[n].weight.shape[1] != width:
                        # at INFO once per (layer class, balance suffix): every GQA layer repeats it
                        key = (type(layer).__name__, n[len(prefix):])
                        log.log(logging.DEBUG if key in _D9_LOGGED else logging.INFO,
                                "AWQ: dropping balance %s of %s (shape mismatch, D9)", n, sname)
                        _D9_LOGGED.add(key)
                        continue
                    balance.append(n)
            if not balance:
                continue
            if not all(b in quantized for b in balance):
                log.info("AWQ: skipping mapping %s -> %s (balance layers not quantized)", sname, balance)
                continue
            refs = [lins[b] for b in balance]
            if len(balance) == 1:
                pname = balance[0]
                if refs[0].index is None:
                    out.append(ResolvedMapping(sname, smooth, balance, refs, pname, refs[0].module, origin=mi))
                else:
                    out.append(ResolvedMapping(sname, smooth, balance, refs, pname, None, "linear", refs[0].index[0],
                                               origin=mi))
                continue
            pname = _common_parent(balance)
            kind, expert = "module", -1
            while True:
                m = mods.get(pname)
                if m is not None and not isinstance(m, nn.ModuleList) and not is_fused_experts(m):
                    break
                if m is None and all(r.index is not None for r in refs) and \
                        len({(id(r.module), r.index[0]) for r in refs}) == 1 and pname.rpartition(".")[2].isdigit():
                    kind, expert = "expert", refs[0].index[0]  # one expert's MLP (4.57: experts.<e>)
                    break
                pname = pname.rpartition(".")[0]
            out.append(ResolvedMapping(sname, smooth, balance, refs, pname, mods.get(pname) if kind == "module" else None,
                                       kind, expert, origin=mi))
    return out


_SAMPLES: List[int] = [0]  # > 0 while a batched layer call stands for that many calibration samples


def _split_samples(x: torch.Tensor) -> List[torch.Tensor]:
    """Inside a batched calibration call (``_SAMPLES[0]`` = n samples stacked sample-major): the
    per-sample pieces of a hooked input -- [n, S, ...] split along dim 0, a flattened [n * S, ...]
    into n equal row blocks -- i.e. exactly what the per-sample calls handed the hook."""
    n = _SAMPLES[0]
    if n <= 1:
        return [x]
    if x.dim() >= 3 and x.shape[0] == n:
        return [x[i:i + 1] for i in range(n)]
    if x.shape[0] % n == 0:
        return list(x.chunk(n, dim=0))
    raise RuntimeError(f"AWQ: cannot split a hooked input of shape {tuple(x.shape)} into {n} samples")


def stack_layer_calls(layer_inputs: List[Tuple[tuple, dict]]) -> Optional[Tuple[tuple, dict]]:
    """The per-sample decoder-layer calls as ONE call with the hidden states stacked along the
    batch dimension, when every other argument is the same for all samples and broadcasts over
    the batch (same sequence length, same positions / rotary tables / mask); else None."""
    if len(layer_inputs) < 2:
        return None
    a0, k0 = layer_inputs[0]
    if not a0 or not torch.is_tensor(a0[0]) or a0[0].dim() != 3 or a0[0].shape[0] != 1:
        return None
    for a, k in layer_inputs[1:]:
        if len(a) != len(a0) or not torch.is_tensor(a[0]) or a[0].shape != a0[0].shape \
                or not _same(tuple(a[1:]), tuple(a0[1:])) or not _same(k, k0):
            return None
    for v in list(a0[1:]) + list(k0.values()):
        for t in (v if isinstance(v, (tuple, list)) else (v,)):
            if torch.is_tensor(t) and t.dim() >= 3 and t.shape[0] != 1:
                return None
    return (torch.cat([a[0] for a, _ in layer_inputs], dim=0),) + tuple(a0[1:]), dict(k0)


# ------------------------------------------------------------------ concurrent sample calls
CALIB_THREADS = int(os.environ.get("QZ_CALIB_THREADS", "4"))  # per-sample layer calls on N host threads / streams (r03c: MoE layers 0.74-0.81 -> 0.68-0.70 s)
_SLOT = threading.local()  # .j = the calibration sample the current thread's layer call belongs to
_calib_streams: Dict[Tuple[str, int], List] = {}


def _slot() -> Optional[int]:
    return getattr(_SLOT, "j", None)


def run_samples(fn: Callable[[int], Any], n: int, threads: int = 0) -> List[Any]:
    """``[fn(j) for j in range(n)]`` -- with ``threads`` > 1 (default ``QZ_CALIB_THREADS``) the
    calls run on that many host threads, each enqueueing on its own stream (sample j on thread
    j % threads), so one sample's host work and syncs (the MoE blocks' routing reads) overlap
    the others' kernels.  Every call computes exactly what it would alone; the hooks below file
    what they see under the sample index (``_SLOT``) and ``finish()`` combines it in sample
    order, so the results are bit-identical to the sequential calls."""
    threads = threads or CALIB_THREADS
    if threads <= 1 or n < 2 or not torch.cuda.is_available():
        return [fn(j) for j in range(n)]
    main = torch.cuda.current_stream()
    dev = main.device
    key = (str(dev), threads)
    if key not in _calib_streams:
        _calib_streams[key] = [torch.cuda.Stream(dev) for _ in range(threads)]
    streams = _calib_streams[key]
    for st in streams:
        st.wait_stream(main)
    out: List[Any] = [None] * n
    errs: List[BaseException] = []

    def worker(t: int):
        try:
            with torch.cuda.device(dev), torch.cuda.stream(streams[t]), torch.no_grad():
                for j in range(t, n, threads):
                    if errs:
                        return
                    _SLOT.j = j
                    out[j] = fn(j)
        except BaseException as e:  # noqa: BLE001 -- re-raised in the caller
            errs.append(e)
        finally:
            _SLOT.j = None

    ths = [threading.Thread(target=worker, args=(t,), name=f"qz-calib-{t}") for t in range(threads)]
    for th in ths:
        th.start()
    for th in ths:
        th.join()
    for st in streams:
        main.wait_stream(st)
    if errs:
        raise errs[0]
    return out


class _ParentCache:
    """Forward pre-hook on a parent module: cache its (args, kwargs) per calibration batch."""

    def __init__(self, module: nn.Module):
        self.calls: List[Tuple[tuple, dict]] = []
        self.slots: Dict[int, List[Tuple[tuple, dict]]] = {}
        self.h = module.register_forward_pre_hook(self._hook, with_kwargs=True)

    def _hook(self, mod, args, kwargs):
        call = (tuple(a.detach() if torch.is_tensor(a) else a for a in args), dict(kwargs))
        j = _slot()
        if j is None:
            self.calls.append(call)
        else:
            self.slots.setdefault(j, []).append(call)

    def finish(self):
        for j in sorted(self.slots):
            self.calls.extend(self.slots[j])
        self.slots = {}

    def remove(self):
        self.h.remove()


class _AbsMean:
    """Forward pre-hook on a balance layer: sum |x| per input channel (GPU kernel).  ``bf16``
    (D8): every calibration batch's sum is kept apart and ``mean()`` is the bf16 running mean."""

    def __init__(self, module: Optional[nn.Module] = None, bf16: bool = False):
        self.sum = None
        self.count = 0
        self.bf16 = bf16
        self.parts: List[Tuple[torch.Tensor, int]] = []
        self.slots: Dict[int, List[Tuple[torch.Tensor, int]]] = {}
        self.h = module.register_forward_pre_hook(self._hook) if module is not None else None

    def _hook(self, mod, args):
        j = _slot()
        xs = _split_samples(args[0])
        if j is None and len(xs) > 1:  # a batched calibration forward: every sample in one launch
            self.add_samples(xs)
            return
        for x in xs:  # one add per calibration sample, as per-sample calls did
            if j is None:
                self.add(x)
            elif x.numel():  # concurrent samples: this sample's total alone, added in order by finish()
                part = torch.zeros(x.shape[-1], dtype=torch.float32, device=x.device)
                self.slots.setdefault(j, []).append((part, ops.awq_absmean_accum(x.detach(), part)))

    def add_samples(self, xs: List[torch.Tensor]):
        """``add(x)`` for every sample in order, as ONE segmented launch (ops.awq_absmean_segments):
        each sample's total from zero, bit-identical to its own call, then combined as the
        sequential adds combine them (f32 sum += total in sample order; bf16: one part each)."""
        xs = [x.detach() if x.dtype == torch.bfloat16 else x.detach().to(torch.bfloat16) for x in xs]
        live = [i for i, x in enumerate(xs) if x.numel()]
        if not live:
            for x in xs:
                self.add(x)
            return
        buf = torch.zeros(len(live), xs[live[0]].shape[-1], dtype=torch.float32, device=xs[live[0]].device)
        counts = ops.awq_absmean_segments([xs[i] for i in live], list(buf))
        slot = {i: k for k, i in enumerate(live)}
        for i, x in enumerate(xs):
            if not x.numel():
                self.add(x)
                continue
            part, n = buf[slot[i]], counts[slot[i]]
            if self.bf16:
                self.parts.append((part, n))
            else:
                if self.sum is None:
                    self.sum = torch.zeros_like(part)
                self.sum += part
            self.count += n

    def finish(self):
        """sum = ((0 + t_0) + t_1) + ... over the samples in order: the kernel adds each call's
        total to sum[c] with one f32 add, so adding the per-sample totals (each 0 + t_j = t_j)
        in sample order gives the sequential calls' bits."""
        for j in sorted(self.slots):
            for part, n in self.slots[j]:
                if self.bf16:
                    self.parts.append((part, n))
                    self.count += n
                    continue
                if self.sum is None:
                    self.sum = torch.zeros_like(part)
                self.sum += part
                self.count += n
        self.slots = {}

    def add(self, x: torch.Tensor):
        if self.bf16:  # one sum per calibration batch, combined by mean()
            part = torch.zeros(x.shape[-1], dtype=torch.float32, device=x.device)
            n = ops.awq_absmean_accum(x.detach(), part) if x.numel() else 0
            self.parts.append((part, n))
            self.count += n
            return
        if self.sum is None:
            self.sum = torch.zeros(x.shape[-1], dtype=torch.float32, device=x.device)
        if x.numel():
            self.count += ops.awq_absmean_accum(x.detach(), self.sum)

    def mean(self) -> torch.Tensor:
        if self.bf16:
            return _running_mean_bf16(self.parts)
        return self.sum / max(self.count, 1)

    def remove(self):
        if self.h is not None:
            self.h.remove()


class _ExpertInputs:
    """Inputs of the fused experts module (all tokens + the router's top-k choice) per
    calibration batch, and per-expert activations recomputed from them on demand."""

    def __init__(self, module: nn.Module, calibrate_all: bool):
        self.module = module
        self.calibrate_all = calibrate_all
        self.x: List[torch.Tensor] = []
        self.topk: List[Optional[torch.Tensor]] = []
        self.gate_up0: Optional[torch.Tensor] = None  # pre-smoothing snapshot
        self._xcat: Optional[torch.Tensor] = None  # every batch's tokens, concatenated (lazily)
        self.slots: Dict[int, Tuple[list, list]] = {}
        self.h = module.register_forward_pre_hook(self._hook)

    def _hook(self, mod, args):
        xs = _split_samples(args[0].detach())
        tk = _split_samples(args[1].detach()) if len(args) > 1 and torch.is_tensor(args[1]) else [None] * len(xs)
        j = _slot()
        if j is None:
            self.x.extend(xs)
            self.topk.extend(tk)
        else:
            sx, st = self.slots.setdefault(j, ([], []))
            sx.extend(xs)
            st.extend(tk)

    def finish(self):
        for j in sorted(self.slots):
            self.x.extend(self.slots[j][0])
            self.topk.extend(self.slots[j][1])
        self.slots = {}

    def remove(self):
        self.h.remove()

    def snapshot(self):
        if self.gate_up0 is None and hasattr(self.module, "gate_up_proj"):
            self.gate_up0 = self.module.gate_up_proj.data.clone()

    def tokens(self, i: int, e: int) -> torch.Tensor:
        x = self.x[i]
        if self.calibrate_all or self.topk[i] is None:
            return x
        return x[(self.topk[i] == e).any(dim=-1)]

    def hidden(self, i: int, e: int) -> torch.Tensor:
        """act(x W_gate^T) * (x W_up^T) for expert e: the input of its down projection."""
        return moe_eager._act_mul(self.module, nn.functional.linear(self.tokens(i, e), self.gate_up0[e]))

    def hidden_cat(self, e: int) -> torch.Tensor:
        """``cat([hidden(i, e) for every batch i])`` as ONE GEMM over the concatenated tokens:
        hipBLASLt gives every row the same bits either way at these shapes
        (``profiles/r02ao_concat_probe.log``), and a 128-expert layer issues 128 GEMMs instead of 2,048."""
        if self.calibrate_all or any(t is None for t in self.topk):
            if self._xcat is None:
                self._xcat = torch.cat(self.x) if len(self.x) > 1 else self.x[0]
            x = self._xcat
        else:
            x = torch.cat([self.tokens(i, e) for i in range(len(self.x))])
        return moe_eager._act_mul(self.module, nn.functional.linear(x, self.gate_up0[e]))


CONCAT_EXPERT_INPUTS = os.environ.get("QZ_CONCAT_EXPERT_INPUTS", "1") == "1"
EXPERT_MAJOR = os.environ.get("QZ_EXPERT_MAJOR", "1") == "1"  # expert searches: experts outer, grid inner
BATCHED_LOSS = os.environ.get("QZ_BATCHED_LOSS", "1") == "1"  # expert searches: one ordered reduce per search
MULTI_LOSS = int(os.environ.get("QZ_MULTI_LOSS", "8"))  # expert searches: grid outputs per loss launch (<= 8)
OVERLAP_LOSS = os.environ.get("QZ_OVERLAP_LOSS", "0") == "1"  # expert searches: loss kernels on a side stream (measured slower: off)
GRID_GRAPHS = os.environ.get("QZ_GRID_GRAPHS", "0") == "1"  # MoE-block grids: forwards replayed from one HIP graph (r03i: replays ~10% faster, capture costs more: off)


class _GraphedForward:
    """The parent forward of a fixed-routing MoE-block grid, replayed from one HIP graph.

    Every grid point re-runs the same MoE block on the same cached inputs, with the same
    routing (``moe_eager.fixed_routing``) and the balance weights rewritten in place: the same
    kernels on the same addresses each time.  Issued from Python that is ~260 launches per
    forward (two GEMMs per routed expert on 4 streams), which the host cannot issue as fast as
    the GPU runs them.  The first grid forward runs eagerly, is captured once (capture runs
    nothing), replayed, and the replay's outputs are compared bit for bit with the eager ones;
    on a match the remaining grid points replay the graph, otherwise (or when capture fails,
    e.g. a host sync inside the forward) they run eagerly.  The outputs of a replay live in the
    graph's buffers until the next replay, which is enqueued on the same stream after the loss
    kernels that read them."""

    def __init__(self, run: Callable[[], List[torch.Tensor]], name: str):
        self.run, self.name = run, name
        self.graph: Optional[Any] = None
        self.outs: Optional[List[torch.Tensor]] = None
        self.state: Optional[bool] = None  # None: not tried yet; True: replaying; False: eager

    def __call__(self) -> List[torch.Tensor]:
        if self.state:
            self.graph.replay()
            return self.outs
        if self.state is False:
            return self.run()
        with phase("MoE-block grid: first forward, capture, check"):
            return self._first()

    def _first(self) -> List[torch.Tensor]:
        want = self.run()
        self.state = False
        try:
            g = torch.cuda.CUDAGraph()
            with torch.cuda.graph(g, capture_error_mode="thread_local"):
                outs = self.run()
            g.replay()
            ok = len(outs) == len(want) and all(moe_eager._bits_equal(a, b) for a, b in zip(want, outs))
        except RuntimeError as e:
            log.info("AWQ: %s grid forward not capturable (%s); eager forwards", self.name, e)
            return want
        if ok:
            self.graph, self.outs, self.state = g, outs, True
        else:
            log.info("AWQ: %s graph replay differs from the eager forward; eager forwards", self.name)
        return want

    def close(self) -> None:
        """Release the graph once its last replay has finished: the executable graph owns the
        runtime's side streams and argument buffers for its multi-stream replay, and its outputs
        live in the graph's private memory pool."""
        if self.graph is not None:
            torch.cuda.synchronize()
        self.graph = self.outs = None


def _batched_losses(hs, ref_out, wq_all, losses) -> None:
    """Expert-major grid losses with stage 1 only per (expert, grid point) -- the partial sums go
    to their own row of one [experts, grid, nb] f64 buffer -- and ONE ordered reduce launch for
    the whole search (qz_awq_sq_err_reduce): a launch and ~5 us of latency-bound stage 2 fewer per
    loss, the same fixed-order sums, so the same bits as awq_sq_err_accum per loss."""
    n_grid, n_exp = wq_all.shape[0], len(hs)
    nb = ops.awq_sq_err_partials_count(ref_out[0].shape)
    part = torch.empty(n_exp, n_grid, nb, dtype=torch.float64, device=wq_all.device)
    multi = MULTI_LOSS if all(ro.is_contiguous() for ro in ref_out) else 1
    outs = [torch.empty_like(ref_out[0]) for _ in range(multi)] if multi > 1 else []
    for k, (h, ro) in enumerate(zip(hs, ref_out)):
        if multi > 1:  # up to `multi` grid points' outputs, then one loss launch reading ro once
            h2 = h.reshape(-1, h.shape[-1])
            for g0 in range(0, n_grid, multi):
                gs = range(g0, min(n_grid, g0 + multi))
                for j, g in enumerate(gs):
                    torch.mm(h2, wq_all[g, k].t(), out=outs[j].view(-1, outs[j].shape[-1]))
                ops.awq_sq_err_partials_multi(ro, outs[:len(gs)], part[k, g0:g0 + len(gs)])
            continue
        for g in range(n_grid):
            ops.awq_sq_err_partials(ro, nn.functional.linear(h, wq_all[g, k]), part[k, g])
    tot = torch.zeros(n_exp, n_grid, dtype=torch.float64, device=wq_all.device)
    ops.awq_sq_err_reduce(part.view(n_exp * n_grid, nb), nb, tot)
    losses += tot.t()


def _overlapped_losses(hs, ref_out, wq_all, losses) -> None:
    """Expert-major grid losses with each loss kernel (memory-bound) on a side stream, so it runs
    beside the next GEMM (MFMA-bound) instead of after it.  The GEMM outputs alternate between two
    buffers (a GEMM waits for the loss that last read its buffer); the GEMM is ``mm(h, W^T)``, the
    same call ``F.linear`` makes, and every loss accumulates into its own slot: the same bits."""
    dev = hs[0].device
    main = torch.cuda.current_stream(dev)
    side = torch.cuda.Stream(dev)
    side.wait_stream(main)
    n_grid = wq_all.shape[0]
    bufs = [torch.empty(ref_out[0].shape, dtype=ref_out[0].dtype, device=dev) for _ in range(2)]
    done: List[Optional[torch.cuda.Event]] = [None, None]
    step = 0
    for k, (h, ro) in enumerate(zip(hs, ref_out)):
        if ro.shape != bufs[0].shape:
            bufs = [torch.empty(ro.shape, dtype=ro.dtype, device=dev) for _ in range(2)]
            done = [None, None]
            side.wait_stream(main)
            main.wait_stream(side)
        for g in range(n_grid):
            i = step % 2
            if done[i] is not None:
                main.wait_event(done[i])
            torch.mm(h.reshape(-1, h.shape[-1]), wq_all[g, k].t(), out=bufs[i].view(-1, bufs[i].shape[-1]))
            ready = torch.cuda.Event()
            ready.record(main)
            side.wait_event(ready)
            with torch.cuda.stream(side):
                ops.awq_sq_err_accum(ro, bufs[i], losses[g, k:k + 1])
                done[i] = torch.cuda.Event()
                done[i].record(side)
            step += 1
    main.wait_stream(side)
    for b in bufs:
        b.record_stream(side)


def _virtual_input(ei: _ExpertInputs, ref: LinearRef, i: int) -> torch.Tensor:
    if ref.param_name == "down_proj" or ref.param_name == "w2":
        return ei.hidden(i, ref.index[0])
    return ei.tokens(i, ref.index[0])


def _is_tokenwise(m: nn.Module) -> bool:
    """Parents that act on every token independently: a Linear, a gated MLP, a MoE block
    (router + fused experts).  Attention and whole decoder layers are not."""
    if isinstance(m, nn.Linear):
        return True
    name = type(m).__name__
    if name.endswith("MLP") or "SparseMoe" in name or any(is_fused_experts(c) for c in m.children()):
        return not any("Attention" in type(c).__name__ for c in m.modules())
    return False


def _tokenwise_concat(parent: nn.Module, calls):
    """A token-wise parent (MLP, MoE block, Linear) can run its calibration calls as ONE call
    over all tokens: same per-token math and the same loss sum, larger GEMMs and one expert
    loop per grid point instead of one per calibration batch.  Other parents (attention:
    positions, masks) keep their per-batch calls."""
    if len(calls) < 2 or not _is_tokenwise(parent):
        return calls
    xs = []
    for args, kwargs in calls:
        if kwargs or len(args) != 1 or not torch.is_tensor(args[0]) or args[0].dim() != 3 or args[0].shape[0] != 1:
            return calls
        xs.append(args[0])
    if any(x.shape[2] != xs[0].shape[2] for x in xs):
        return calls
    return [((torch.cat(xs, dim=1),), {})]


def _same(a, b) -> bool:
    """Structural equality of two cached call arguments (tensors by value)."""
    if torch.is_tensor(a) or torch.is_tensor(b):
        return torch.is_tensor(a) and torch.is_tensor(b) and a.shape == b.shape and a.dtype == b.dtype and \
            a.device == b.device and (a is b or torch.equal(a, b))
    if isinstance(a, (tuple, list)) or isinstance(b, (tuple, list)):
        return type(a) is type(b) and len(a) == len(b) and all(_same(x, y) for x, y in zip(a, b))
    if isinstance(a, dict) or isinstance(b, dict):
        return isinstance(a, dict) and isinstance(b, dict) and a.keys() == b.keys() and \
            all(_same(a[k], b[k]) for k in a)
    return a is b or (type(a) is type(b) and a == b)


def _batchwise_concat(calls, max_tokens: int = 1 << 17):
    """A non-token-wise parent (self-attention) whose calibration calls differ only in their
    ``hidden_states`` (every sample the same length, the same positions / rotary embeddings /
    mask, all with batch 1) runs them as calls over up to ``max_tokens`` tokens stacked along
    the batch dimension: the per-sequence attention is unchanged (the mask and the position
    embeddings broadcast over the batch), the loss sums the same elements, and there are ~16x
    fewer launches and larger GEMM / attention kernels per grid point."""
    if len(calls) < 2:
        return calls

    def hidden(call):
        args, kwargs = call
        if args:
            return args[0] if len(args) == 1 and "hidden_states" not in kwargs else None
        return kwargs.get("hidden_states")

    hs = [hidden(c) for c in calls]
    if any(h is None or not torch.is_tensor(h) or h.dim() != 3 or h.shape[0] != 1 or h.shape != hs[0].shape
           for h in hs):
        return calls
    args0, kw0 = calls[0]
    rest0 = {k: v for k, v in kw0.items() if k != "hidden_states"}
    for args, kwargs in calls[1:]:
        if bool(args) != bool(args0) or not _same(rest0, {k: v for k, v in kwargs.items() if k != "hidden_states"}):
            return calls
    for v in rest0.values():  # batch-1 tensors must broadcast: only leading dims of size 1
        for t in (v if isinstance(v, (tuple, list)) else (v,)):
            if torch.is_tensor(t) and t.dim() >= 3 and t.shape[0] != 1:
                return calls
    per = max(1, max_tokens // hs[0].shape[1])
    out = []
    for i in range(0, len(hs), per):
        h = torch.cat(hs[i:i + per], dim=0)
        out.append(((h,), dict(rest0)) if args0 else ((), dict(rest0, hidden_states=h)))
    return out


def _run_parent(parent: nn.Module, calls) -> List[torch.Tensor]:
    outs = []
    for args, kwargs in calls:
        o = parent(*args, **kwargs)
        if isinstance(o, tuple):
            o = o[0]
        outs.append(o)
    return outs


def _sq_err(ref: List[torch.Tensor], got: List[torch.Tensor]) -> torch.Tensor:
    """mean squared error over all calibration outputs, fp64 on the device (no host sync):
    one fused kernel per output (qz_awq_sq_err_accum) instead of sub / cast / pow / sum."""
    tot = torch.zeros(1, dtype=torch.float64, device=ref[0].device)
    n = 0
    for a, b in zip(ref, got):
        if a.dtype == torch.bfloat16 and b.dtype == torch.bfloat16:
            ops.awq_sq_err_accum(a, b, tot)
        else:
            tot += (a - b).reshape(-1).float().pow(2).sum().double()
        n += a.numel()
    return tot[0] / max(n, 1)


def _group_size_for_mean(a: QuantizationArgs, cols: int) -> int:
    if a.strategy in ("group", "tensor_group"):
        return a.group_size
    if a.strategy in ("channel", "block"):
        return cols  # D9b: block / channel balance layers normalised per row
    return cols


def _w_mean(groups: List[List[LinearRef]], quantized: Dict[str, QuantizationArgs], cols: int, bf16: bool,
            device, refs: Optional[List[LinearRef]] = None) -> torch.Tensor:
    """w_mean over the balance layers.  fp32 (D8 rounds 1-4): one f64 column sum over every row
    of every balance layer, / rows, as f32.  bf16: llmcompressor's _compute_layer_means -- each
    balance linear's column sum (f64 on the device, rounded to bf16), summed over the layers in
    bf16 in the mapping's balance order (``refs``; the module order llmcompressor iterates),
    divided by the row count in bf16."""
    if not bf16:
        wsum = torch.zeros(cols, dtype=torch.float64, device=device)
        rows = 0
        for part, n in _w_mean_parts([(_view(g), _group_size_for_mean(quantized[g[0].name], cols)) for g in groups],
                                     cols, device):
            wsum += part  # ((0 + v_0) + v_1) + ...: the sequential calls' f64 adds
            rows += n
        return (wsum / rows).float()
    # every balance linear is a layer of its own (each expert slice too)
    return _layer_means_bf16(_w_mean_parts([(ref.weight, _group_size_for_mean(quantized[ref.name], cols)) for ref in
                                            (refs if refs is not None else [x for g in groups for x in g])],
                                           cols, device))


def _w_mean_parts(items: List[Tuple[torch.Tensor, int]], cols: int, device) -> List[Tuple[torch.Tensor, int]]:
    """[(weight, group size)] -> [(its f64 column sums from zero, its rows)] in order: the weights
    of one group size in segmented launches (ops.awq_weight_mean_segments: one launch per mapping
    instead of one per balance layer, each sum bit-identical to its own call)."""
    parts = [torch.zeros(cols, dtype=torch.float64, device=device) for _ in items]
    rows = [0] * len(items)
    by_g: Dict[int, List[int]] = {}
    for i, (_, g) in enumerate(items):
        by_g.setdefault(g, []).append(i)
    for g, idx in by_g.items():
        for i, n in zip(idx, ops.awq_weight_mean_segments([items[i][0] for i in idx], g, [parts[i] for i in idx])):
            rows[i] = n
    return list(zip(parts, rows))


def _launch_groups(r: ResolvedMapping, quantized: Dict[str, QuantizationArgs]):
    """Balance refs grouped into single batched launches (same fused parameter, same scheme)."""
    out = []
    for g in batch_groups(r.balance):
        if len(g) > 1 and len({id(quantized[x.name]) for x in g}) > 1:
            out.extend([[x] for x in g])
        else:
            out.append(g)
    return out


def _view(g: List[LinearRef]) -> torch.Tensor:
    return g[0].weight if len(g) == 1 else stacked_view(g)


def _independent_batches(resolved: List[ResolvedMapping]) -> List[List[ResolvedMapping]]:
    """Split the mapping sequence into runs whose grid searches do not depend on each other's
    smoothing: consecutive mappings from one AWQMapping entry whose loss parent is their single
    balance layer and whose smooth/balance layers are all distinct (per-expert w3 -> w2,
    up -> down of every expert).  Everything else stays a run of one, in order."""
    out: List[List[ResolvedMapping]] = []
    for r in resolved:
        single = len(r.balance) == 1 and r.parent_kind in ("linear", "module") and \
            r.parent_name == r.balance_names[0]
        if out and single and len(out[-1]) >= 1:
            prev = out[-1]
            p = prev[0]
            p_single = len(p.balance) == 1 and p.parent_name == p.balance_names[0]
            touched = {x.smooth_name for x in prev} | {x.balance_names[0] for x in prev}
            if p_single and p.origin == r.origin and r.smooth_name not in touched and \
                    r.balance_names[0] not in touched:
                prev.append(r)
                continue
        out.append([r])
    return out


def _grid_ranks(enabled: bool) -> Tuple[int, int]:
    """(world, rank) for splitting a mapping's grid ratios, (1, 0) when not distributed."""
    import torch.distributed as dist
    if not enabled or not (dist.is_available() and dist.is_initialized()) or dist.get_world_size() == 1:
        return 1, 0
    return dist.get_world_size(), dist.get_rank()


def _all_reduce_sum(t: torch.Tensor) -> None:
    import torch.distributed as dist
    if dist.get_backend() == "gloo" and t.is_cuda:  # gloo: host staging
        h = t.cpu()
        dist.all_reduce(h)
        t.copy_(h)
    else:
        dist.all_reduce(t)


def _sharded_search(batch: List[ResolvedMapping], search_chunk, chunk: int = 1, n_grid: int = 20) -> List[Any]:
    """Run ``search_chunk`` (a list of mappings -> a list of results) over consecutive chunks of
    a batch of independent mappings; under torch.distributed rank r takes chunks r, r + world,
    ... and the results are exchanged as ONE device tensor collective: every mapping's (found
    flag, best ratio, best loss, loss history [n_grid], scale vector) is a row of an f64 matrix
    [mappings, 3 + n_grid + max cols] that is non-zero on exactly one rank, all-reduced (sum, RCCL
    on nccl) -- exact, so every rank applies identical smoothing.  Chunk boundaries do not depend
    on the world size, so the result is bit-identical to one process."""
    import torch.distributed as dist
    chunks = [batch[i:i + chunk] for i in range(0, len(batch), chunk)]
    if not (dist.is_available() and dist.is_initialized()) or dist.get_world_size() == 1:
        return [f for c in chunks for f in search_chunk(c)]
    world, rank = dist.get_world_size(), dist.get_rank()
    dev = batch[0].balance[0].weight.device
    cols = [r.balance[0].weight.shape[-1] for r in batch]
    width = 3 + n_grid + max(cols)
    table = torch.zeros(len(batch), width, dtype=torch.float64, device=dev)
    for j in range(rank, len(chunks), world):
        for k, f in enumerate(search_chunk(chunks[j])):
            if f is None:
                continue
            m = j * chunk + k
            ratio, best, history, scales = f
            row = table[m]
            row[0] = 1.0
            row[1] = ratio
            row[2] = best
            row[3:3 + n_grid] = torch.tensor(history, dtype=torch.float64, device=dev)
            row[3 + n_grid:3 + n_grid + scales.numel()] = scales.to(torch.float64)
    _all_reduce_sum(table)
    out: List[Any] = []
    for m, r in enumerate(batch):
        row = table[m]
        if row[0].item() == 0.0:
            out.append(None)
            continue
        head = row[:3 + n_grid].cpu().tolist()
        out.append((head[1], head[2], head[3:3 + n_grid],
                    row[3 + n_grid:3 + n_grid + cols[m]].to(torch.float32).contiguous()))
    return out


def _expert_batchable(batch: List[ResolvedMapping], quantized: Dict[str, QuantizationArgs], calibrate_all: bool) -> bool:
    """Every expert's w3 -> w2 of one fused module, one scheme: searchable as batched launches."""
    if not calibrate_all or len(batch) < 2:
        return False
    r0 = batch[0]
    b0 = r0.balance[0]
    if r0.parent_kind != "linear" or b0.param_name not in ("down_proj", "w2"):
        return False
    return all(r.parent_kind == "linear" and r.balance[0].module is b0.module and
               r.balance[0].param_name == b0.param_name and
               quantized[r.balance_names[0]] is quantized[r0.balance_names[0]] for r in batch)


STATEFUL_OBSERVERS = ("minmax", "static_minmax")


class _ObserverState:
    """Per-balance-layer weight observer memory across the AWQ grid (D7, stateful reading):
    ``minmax`` = moving average of the group min/max (``averaging_constant``, default 0.01),
    ``static_minmax`` = running extremes; the first grid point initialises the state.  Updates
    run in the weight dtype with torch's op order (past + c * (cur - past)), as
    oracle/ct_torch.moving_average_minmax restates."""

    def __init__(self, a: QuantizationArgs):
        self.a = a
        self.c = float((a.observer_kwargs or {}).get("averaging_constant", 0.01))
        self.mn = self.mx = None

    def update(self, mn: torch.Tensor, mx: torch.Tensor):
        if self.mn is None:
            self.mn, self.mx = mn, mx
        elif self.a.observer == "static_minmax":
            self.mn, self.mx = torch.minimum(self.mn, mn), torch.maximum(self.mx, mx)
        else:
            self.mn = self.mn + self.c * (mn - self.mn)
            self.mx = self.mx + self.c * (mx - self.mx)
        return self.mn, self.mx


def _fake_quant_stateful(w0: torch.Tensor, a: QuantizationArgs, scales: torch.Tensor, out: torch.Tensor,
                         st: _ObserverState) -> None:
    """Q(W*s)/s with qparams from the layer's observer memory: W*s (bf16) -> group min/max
    (qz_observe_minmax) -> state update -> calculate_qparams -> fake-quantize with those qparams
    (qz_quantize_qparams, bf16 output, sign of zero kept) -> / s (qz_scale_columns)."""
    ws = w0.clone()
    ops.scale_columns_(ws, scales, divide=False)
    mn, mx = st.update(*ops.observe_minmax(ws, a))
    scale, zp = ops.calculate_qparams(mn, mx, a)
    fq = ops.quantize(ws, scale, zp if not a.symmetric else None, a, out_fmt=_lib.QZ_OUT_FAKEQUANT)
    ops.scale_columns_(fq, scales, divide=True)
    out.copy_(fq)


def _expert_chunk(n_tokens: int, inter: int, hidden: int, budget: int = 4 << 30) -> int:
    """Experts per batched search chunk: their w2 inputs and reference outputs stay resident."""
    per_expert = n_tokens * (inter + hidden) * 2
    return int(max(1, min(16, budget // max(per_expert, 1))))


@torch.no_grad()
def awq_layer(layer: nn.Module, prefix: str, layer_inputs: List[Tuple[tuple, dict]], mappings: List[AWQMapping],
              quantized: Dict[str, QuantizationArgs], duo_scaling: bool = True, n_grid: int = 20,
              mtype: str = "", calibrate_all_experts: bool = True,
              stateful_observers: bool = False, batched_calls: bool = False,
              awq_dtype: Optional[str] = None) -> Dict[str, Any]:
    """Run AWQ on one decoder layer in place.  ``layer_inputs`` are the cached (args, kwargs)
    of the layer for every calibration batch.  Returns per-mapping diagnostics.

    ``stateful_observers``: balance layers whose scheme names the ``minmax`` / ``static_minmax``
    observer keep that observer's memory across the 20 grid points of their search (D7's
    stateful reading); default: every observation is memoryless (D7).
    ``batched_calls``: run the calibration pass as one call over the stacked samples
    (``stack_layer_calls``; the hooks see the same per-sample inputs) -- the caller has checked
    that the batched layer forward is bit-identical to the per-sample one.
    ``awq_dtype``: "bf16" / "fp32" statistics and grid scales (D8, ``AWQ_DTYPE`` when None)."""
    awq_dtype = AWQ_DTYPE if awq_dtype is None else awq_dtype
    if awq_dtype not in AWQ_DTYPES:
        raise ValueError(f"awq_dtype must be one of {AWQ_DTYPES}, got {awq_dtype!r}")
    bf16 = awq_dtype == "bf16"

    def grid_scales(xm, wm, ratio, out=None):
        if bf16:
            return _grid_scales_bf16(xm, wm, ratio, duo_scaling, out=out)
        if xm.dim() == 2:
            return ops.awq_grid_scales_batched(xm, wm, ratio, duo_scaling, out=out)
        return ops.awq_grid_scales(xm, wm, ratio, duo_scaling, out=out)
    resolved = resolve_mappings(layer, prefix, mappings, quantized, mtype)
    if not resolved:
        return {}
    # 1. one calibration pass: activation statistics + parent inputs (before any smoothing)
    hooks = []
    stats: Dict[str, _AbsMean] = {}
    caches: Dict[str, _ParentCache] = {}
    experts: Dict[int, _ExpertInputs] = {}
    for r in resolved:
        b0 = r.balance[0]
        if b0.index is None:
            stats[r.smooth_name] = _AbsMean(b0.module, bf16)
            hooks.append(stats[r.smooth_name])
        elif id(b0.module) not in experts:
            experts[id(b0.module)] = _ExpertInputs(b0.module, calibrate_all_experts)
            hooks.append(experts[id(b0.module)])
        if r.parent_kind == "module":
            caches[r.smooth_name] = _ParentCache(r.parent)
            hooks.append(caches[r.smooth_name])
        elif id(r.balance[0].module) not in experts:
            experts[id(r.balance[0].module)] = _ExpertInputs(r.balance[0].module, calibrate_all_experts)
            hooks.append(experts[id(r.balance[0].module)])
    stacked = stack_layer_calls(layer_inputs) if batched_calls else None
    calib = phase("calibration pass")
    calib.__enter__()
    try:
        if stacked is not None:  # one batched call; the hooks split it back into the samples
            _SAMPLES[0] = len(layer_inputs)
            try:
                layer(*stacked[0], **stacked[1])
            finally:
                _SAMPLES[0] = 0
        else:
            run_samples(lambda j: (layer(*layer_inputs[j][0], **layer_inputs[j][1]), None)[1], len(layer_inputs))
    finally:
        for h in hooks:
            h.remove()
        calib.__exit__(None, None, None)
    for h in hooks:
        h.finish()
    for ei in experts.values():
        ei.snapshot()
    n_batches = len(layer_inputs)

    def search(r: ResolvedMapping, grid_shard: bool = False):
        """Grid search of one mapping; returns (best_ratio, best_loss, history, best_scales) or None.
        ``grid_shard``: split the grid ratios over the ranks (all ranks run this mapping)."""
        b0 = r.balance[0]
        if b0.index is None:
            x_mean = stats[r.smooth_name].mean()
        else:
            ei = experts[id(b0.module)]
            am = _AbsMean(bf16=bf16)
            # in chunks of one segmented launch: each batch's expert input is a fresh GEMM output,
            # so only STATS_SEGS of them are alive at once (same sums, same order: ADVICE r05)
            for i0 in range(0, n_batches, ops.STATS_SEGS):
                am.add_samples([_virtual_input(ei, b0, i) for i in range(i0, min(i0 + ops.STATS_SEGS, n_batches))])
            if am.count == 0:  # expert never routed to (moe_calibrate_all_experts=False)
                log.info("AWQ: skipping mapping %s (no calibration tokens)", r.smooth_name)
                return None
            x_mean = am.mean()
        groups = _launch_groups(r, quantized)
        # 2. w_mean over the balance layers (each with its own group size)
        w_mean = _w_mean(groups, quantized, b0.weight.shape[1], bf16, x_mean.device, r.balance)
        # parent: forward closure over the calibration batches
        if r.parent_kind == "module":
            calls = caches[r.smooth_name].calls
            calls = _tokenwise_concat(r.parent, calls) if _is_tokenwise(r.parent) else _batchwise_concat(calls)
            run: Callable[[], List[torch.Tensor]] = lambda p=r.parent, c=calls: _run_parent(p, c)
        else:
            ei = experts[id(b0.module)]
            e = r.parent_expert
            if r.parent_kind == "linear":
                xin = [_virtual_input(ei, b0, i) for i in range(n_batches)]
                run = lambda x=xin, ref=b0: [nn.functional.linear(t, ref.weight) for t in x]
            else:
                xin = [ei.tokens(i, e) for i in range(n_batches)]
                mod = b0.module

                def run(x=xin, mod=mod, e=e):
                    outs = []
                    for t in x:
                        h = moe_eager._act_mul(mod, nn.functional.linear(t, mod.gate_up_proj[e]))
                        outs.append(nn.functional.linear(h, mod.down_proj[e]))
                    return outs
        return _grid(r, groups, run, x_mean, w_mean, grid_shard)

    def _grid(r, groups, run, x_mean, w_mean, grid_shard):
        """Steps 3-4 of ``search``: the 20-point grid and its argmin.  Balance layers all inside
        fused experts: the router and the cached inputs are unchanged by the grid, so the
        experts' routing is fixed across its forwards (moe_eager.fixed_routing) -- the reference
        forward included, which takes the planned form too."""
        fixed = r.parent_kind == "module" and all(b.index is not None for b in r.balance)
        with moe_eager.fixed_routing() if fixed else contextlib.nullcontext():
            return _grid_fixed(r, groups, run, x_mean, w_mean, grid_shard, fixed)

    def _grid_fixed(r, groups, run, x_mean, w_mean, grid_shard, fixed):
        ref_out = run()
        # 3. grid search: losses stay on the device.  Under torch.distributed (and outside a
        # sharded batch of mappings) the ratios are split over the ranks: rank r
        # evaluates ratios r, r + world, ...; the loss vector is summed over ranks (every other
        # entry is an exact 0), so every rank sees the bit-identical history of one process
        orig = [_view(g).clone() for g in groups]
        tmp = [torch.empty_like(o) for o in orig]
        scales = torch.empty(x_mean.shape, dtype=torch.float32, device=x_mean.device)
        world, rank = _grid_ranks(grid_shard)
        obs = [(_ObserverState(quantized[g[0].name])
                if stateful_observers and quantized[g[0].name].observer in STATEFUL_OBSERVERS else None)
               for g in groups]
        if any(o is not None for o in obs):
            world, rank = 1, 0  # the observer memory runs through the grid in order: no ratio split
        losses = torch.zeros(n_grid, dtype=torch.float64, device=x_mean.device)
        graphed = None
        if fixed and GRID_GRAPHS and x_mean.is_cuda:
            run = graphed = _GraphedForward(run, r.smooth_name)
        for i in range(rank, n_grid, world):
            ratio = i / n_grid
            grid_scales(x_mean, w_mean, ratio, out=scales)
            for g, w0, t, o in zip(groups, orig, tmp, obs):
                if o is not None:
                    _fake_quant_stateful(w0, quantized[g[0].name], scales, t, o)
                    _view(g).copy_(t)
                elif len(g) == 1:
                    ops.fake_quantize(w0, quantized[g[0].name], col_scales=scales, out=g[0].weight)
                else:
                    ops.fake_quantize(w0, quantized[g[0].name], col_scales=scales, out=t)
                    _view(g).copy_(t)
            losses[i] = _sq_err(ref_out, run())
        if graphed is not None:
            graphed.close()
        for g, w0 in zip(groups, orig):
            _view(g).copy_(w0)
        if world > 1:
            _all_reduce_sum(losses)
        history = losses.cpu().tolist()
        finite = [(l, i) for i, l in enumerate(history) if l == l]
        if not finite:
            raise RuntimeError(f"AWQ: no finite loss for {r.smooth_name} (history {history})")
        best, best_i = min(finite)  # first best ratio (strict <): min over (loss, index)
        best_ratio = best_i / n_grid
        return best_ratio, best, history, grid_scales(x_mean, w_mean, best_ratio)

    def apply(r: ResolvedMapping, found):
        """4. _apply_smoothing: balance columns *= s, smooth rows (and bias) /= s."""
        if found is None:
            report[r.smooth_name] = {"balance": r.balance_names, "parent": r.parent_name, "skipped": "no tokens"}
            return
        best_ratio, best, history, best_scales = found
        for g in _launch_groups(r, quantized):
            ops.scale_columns_(_view(g), best_scales, divide=False)
        sw = r.smooth.weight if isinstance(r.smooth, LinearRef) else r.smooth.weight.data
        if sw.dim() == 1:
            ops.scale_rows_(sw, best_scales, divide=True)
        else:
            ops.scale_rows_(sw[-best_scales.numel():], best_scales, divide=True)
        b = None if isinstance(r.smooth, LinearRef) else getattr(r.smooth, "bias", None)
        if b is not None:
            ops.scale_rows_(b.data[-best_scales.numel():], best_scales, divide=True)
        report[r.smooth_name] = {"balance": r.balance_names, "parent": r.parent_name, "best_ratio": best_ratio,
                                 "best_loss": best, "history": history}

    def search_experts(chunk: List[ResolvedMapping]):
        """Grid search of several experts' w3 -> w2 mappings at once: w2 inputs recomputed per
        expert (as in ``search``), then per grid point ONE batched scale launch, ONE batched
        fake-quant launch (one scale vector per expert) and one GEMM per expert over all its
        calibration tokens; per-expert losses stay on the device."""
        refs = [r.balance[0] for r in chunk]
        mod, pname = refs[0].module, refs[0].param_name
        ei = experts[id(mod)]
        a = quantized[chunk[0].balance_names[0]]
        es = [ref.index[0] for ref in refs]
        w2 = getattr(mod, pname).data  # [E, H, I]
        if CONCAT_EXPERT_INPUTS and all(r.param_name in ("down_proj", "w2") for r in refs):
            hid = [[ei.hidden_cat(ref.index[0])] for ref in refs]  # [e] -> [[T, I]]
        else:
            hid = [[_virtual_input(ei, ref, i) for i in range(n_batches)] for ref in refs]  # [e][i] -> [T_i, I]
        cols = w2.shape[2]
        xm = torch.empty(len(refs), cols, dtype=torch.float32, device=w2.device)
        wm = torch.empty_like(xm)
        hs = [torch.cat(h) if len(h) > 1 else h[0] for h in hid]  # all tokens of an expert: [T, I]
        del hid
        if bf16:
            # one sum per calibration batch (the batches' token runs of each expert), all experts'
            # runs in segmented launches; the running means of all experts at once
            counts = [[ei.tokens(i, ref.index[0]).shape[0] for i in range(n_batches)] for ref in refs]
            parts = torch.zeros(len(refs), n_batches, cols, dtype=torch.float32, device=w2.device)
            pieces, outs = [], []
            for k in range(len(refs)):
                for i, piece in enumerate(torch.split(hs[k], counts[k])):
                    if piece.numel():  # the segmented kernel reads bf16 (fp16 / fp32 models: ADVICE r05)
                        pieces.append(piece if piece.dtype == torch.bfloat16 else piece.to(torch.bfloat16))
                        outs.append(parts[k, i])
            ops.awq_absmean_segments(pieces, outs)
            xm.copy_(_running_means_bf16(parts, counts))
            # each expert's w2 is a balance layer of its own: bf16(column sum) / rows
            wsums = torch.zeros(len(refs), cols, dtype=torch.float64, device=w2.device)
            gs = _group_size_for_mean(a, cols)
            rows = ops.awq_weight_mean_segments([ref.weight for ref in refs], gs, list(wsums))
            assert len(set(rows)) == 1
            wm.copy_(_div_count_bf16(wsums.to(torch.bfloat16), rows[0]))
        else:
            for k, ref in enumerate(refs):
                am = _AbsMean(bf16=bf16)
                am.add(hs[k])
                xm[k] = am.mean()
                wm[k] = _w_mean([[ref]], quantized, cols, bf16, w2.device)
        # one GEMM per expert and grid point over all its tokens (2-D GEMMs: the path every
        # other mapping uses)
        w0 = torch.stack([w2[e] for e in es])  # [k, H, I] (pre-search weights)
        ref_out = [nn.functional.linear(h, w0[k]) for k, h in enumerate(hs)]
        n_el = ref_out[0].numel()
        wq = torch.empty_like(w0)
        scales = torch.empty(n_grid, len(refs), cols, dtype=torch.float32, device=w2.device)
        losses = torch.zeros(n_grid, len(refs), dtype=torch.float64, device=w2.device)
        if EXPERT_MAJOR:
            # every grid point's fake-quantized weights first, then expert by expert over the grid:
            # an expert's inputs and reference output are re-read 20 times back to back (from the
            # 256 MB Infinity Cache where they fit) instead of once per pass over all experts.
            # Same GEMM and loss per (grid point, expert): bit-identical losses.
            wq_all = torch.empty((n_grid,) + tuple(w0.shape), dtype=w0.dtype, device=w0.device)
            for g in range(n_grid):
                grid_scales(xm, wm, g / n_grid, out=scales[g])
                ops.fake_quantize_batched(w0, a, scales[g], out=wq_all[g])
            if OVERLAP_LOSS and w0.is_cuda:
                _overlapped_losses(hs, ref_out, wq_all, losses)
            elif BATCHED_LOSS and w0.is_cuda and all(ro.shape == ref_out[0].shape for ro in ref_out):
                _batched_losses(hs, ref_out, wq_all, losses)
            else:
                for k, (h, ro) in enumerate(zip(hs, ref_out)):
                    for g in range(n_grid):
                        ops.awq_sq_err_accum(ro, nn.functional.linear(h, wq_all[g, k]), losses[g, k:k + 1])
            del wq_all
        else:
            for g in range(n_grid):
                grid_scales(xm, wm, g / n_grid, out=scales[g])
                ops.fake_quantize_batched(w0, a, scales[g], out=wq)
                for k, (h, ro) in enumerate(zip(hs, ref_out)):
                    ops.awq_sq_err_accum(ro, nn.functional.linear(h, wq[k]), losses[g, k:k + 1])
        hist = (losses / max(n_el, 1)).cpu()
        out = []
        for k in range(len(refs)):
            history = hist[:, k].tolist()
            finite = [(l, i) for i, l in enumerate(history) if l == l]
            if not finite:
                raise RuntimeError(f"AWQ: no finite loss for {chunk[k].smooth_name} (history {history})")
            best, bi = min(finite)
            out.append((bi / n_grid, best, history, scales[bi, k].clone()))
        return out

    report: Dict[str, Any] = {}
    for batch in _independent_batches(resolved):
        if len(batch) == 1:
            r0 = batch[0]
            kind = ("grid, MoE-block parent" if r0.parent_kind == "module" and all(b.index is not None for b in r0.balance)
                    else f"grid, {r0.parent_kind} parent")
            with phase(kind):
                apply(r0, search(r0, grid_shard=True))
            continue
        # mutually independent single-layer-parent mappings (e.g. every expert's w3 -> w2):
        # search all (sharded over ranks under torch.distributed), then smooth in order
        stateful = stateful_observers and any(quantized[r.balance_names[0]].observer in STATEFUL_OBSERVERS
                                              for r in batch)
        with phase("expert searches"):
            if not stateful and _expert_batchable(batch, quantized, calibrate_all_experts):
                b0 = batch[0].balance[0]
                ei = experts[id(b0.module)]
                n_tok = sum(x.shape[0] for x in ei.x)
                w2 = getattr(b0.module, b0.param_name)
                found = _sharded_search(batch, search_experts, _expert_chunk(n_tok, w2.shape[2], w2.shape[1]), n_grid)
            else:
                found = _sharded_search(batch, lambda c: [search(c[0])], 1, n_grid)
            for r, f in zip(batch, found):
                apply(r, f)
    return report
