"""compressed-tensors checkpoint writer / reader.

Replaces ``model.save_pretrained(output_dir, save_compressed=True)`` (scripts/do_oneshot.py:197):
every targeted weight is quantized + packed on the GPU by the fused kernel (``CompressionPlan``:
same-shape dense modules of one scheme in ONE grouped launch, fused-expert slices of one
parameter in a single batched launch; results copied to pinned host memory asynchronously) and
written under the
compressed-tensors names the reference itself pins in
scripts/recombine_weights_MiniMax-M2.1.py:54-65 (``weight_packed``, ``weight_scale``,
``weight_shape``, ``weight_zero_point``; ``weight`` for float-quantized; plus
``weight_global_scale`` for NVFP4), with ``config.json.quantization_config`` laid out as in
scripts/recombine_weights_MiniMax-M2.1.py:82-134.  MoE experts are written per expert
(``...experts.<e>.<proj>``), the layout of the transformers version the reference pins.
"""
from __future__ import annotations

import json
import logging
import os
import time
from dataclasses import dataclass
from typing import Dict, List, Optional, Sequence, Tuple

import torch
import torch.distributed as dist
from safetensors.torch import load_file, save_file
from torch import nn

from . import ops

log = logging.getLogger(__name__)
from .model import LinearRef, batch_groups, checkpoint_name, iter_linears, model_type, stacked_view
from .quantization import QuantizationArgs, QuantizationScheme, compression_format

CT_VERSION = "0.13.1.dev0+quantizers_amd"  # format revision written (reference run: recombine...py:133)
SHARD_BYTES = 5 * 1024 ** 3


def _args_dict(a: Optional[QuantizationArgs]):
    if a is None:
        return None
    return {"actorder": a.actorder, "block_structure": a.block_structure, "dynamic": a.dynamic,
            "group_size": a.group_size, "num_bits": a.num_bits, "observer": a.observer,
            "observer_kwargs": dict(a.observer_kwargs or {}), "scale_dtype": a.scale_dtype,
            "strategy": a.strategy, "symmetric": a.symmetric, "type": a.type, "zp_dtype": a.zp_dtype}


def quantization_config(model: nn.Module) -> dict:
    return quantization_config_for(model.quantization_scheme_map,
                                   [r.name for r in iter_linears(model)])


def quantization_config_for(scheme_map: Dict[str, QuantizationScheme], linear_names: List[str]) -> dict:
    """``config.json.quantization_config`` for the given per-module schemes (unquantized
    linears are listed under ``ignore``)."""
    groups = {}
    seen = {}
    for name, sch in scheme_map.items():
        if id(sch) in seen:
            continue
        gname = f"group_{len(groups)}"
        seen[id(sch)] = gname
        fmt = compression_format(sch.weights, sch.input_activations)
        groups[gname] = {"targets": list(sch.targets), "weights": _args_dict(sch.weights),
                         "input_activations": _args_dict(sch.input_activations),
                         "output_activations": _args_dict(sch.output_activations), "format": fmt}
    fmts = {g["format"] for g in groups.values()}
    ignore = sorted(n for n in linear_names if n not in scheme_map)
    return {"config_groups": groups, "format": fmts.pop() if len(fmts) == 1 else "mixed-precision",
            "global_compression_ratio": None, "ignore": ignore, "kv_cache_scheme": None,
            "quant_method": "compressed-tensors", "quantization_status": "compressed",
            "sparsity_config": {}, "transform_config": {}, "version": CT_VERSION}


# ------------------------------------------------------------------ compression units / plan
@dataclass
class CompressUnit:
    """One compressor work item: a dense Linear weight, or the same-shaped slices of one fused
    expert parameter (``stacked``: one batched launch over ``[E, rows, cols]``)."""

    refs: List[LinearRef]
    scheme: QuantizationScheme
    stacked: bool

    def view(self) -> torch.Tensor:
        w = stacked_view(self.refs)
        return w if self.stacked else w[0]

    def base(self) -> Optional[torch.Tensor]:
        """The fused parameter a stacked / expert unit is a view of (None for a dense Linear)."""
        r0 = self.refs[0]
        return getattr(r0.module, r0.param_name).data if r0.index is not None else None

    @property
    def nbytes(self) -> int:
        return sum(r.weight.numel() for r in self.refs) * 2


def compression_units(model: nn.Module) -> Tuple[List[CompressUnit], Dict[str, torch.Tensor]]:
    """The targeted weights as compression units, and every tensor written unchanged (unquantized
    fused-expert slices, biases of quantized Linears, all other parameters and buffers), keyed by
    checkpoint name."""
    scheme_map: Dict[str, QuantizationScheme] = getattr(model, "quantization_scheme_map", {})
    refs = iter_linears(model)
    units: List[CompressUnit] = []
    raw: Dict[str, torch.Tensor] = {}
    replaced_params = set()  # id() of fused parameters whose content is written per expert
    for group in batch_groups(refs):
        r0 = group[0]
        if r0.index is not None:
            replaced_params.add(id(getattr(r0.module, r0.param_name)))
        if r0.index is not None and all(g.name in scheme_map for g in group) \
                and len({id(scheme_map[g.name]) for g in group}) == 1:
            units.append(CompressUnit(list(group), scheme_map[r0.name], stacked=True))
            continue
        for g in group:  # dense Linear, or fused slices with mixed targets: one unit each
            if g.name in scheme_map:
                units.append(CompressUnit([g], scheme_map[g.name], stacked=False))
                if g.index is None and g.bias is not None:
                    raw[f"{g.name}.bias"] = g.bias.detach()
            elif g.index is not None:
                raw[f"{g.name}.weight"] = g.weight.detach()
    mtype = model_type(model)
    quant_linears = {g.name for g in refs if g.name in scheme_map and g.index is None}
    for name, prm in model.named_parameters():
        if id(prm) in replaced_params:
            continue
        cname = checkpoint_name(name, mtype)
        mod_name, _, leaf = cname.rpartition(".")
        if mod_name in quant_linears and leaf in ("weight", "bias"):
            continue
        raw.setdefault(cname, prm.detach())
    for name, buf in model.named_buffers():
        cname = checkpoint_name(name, mtype)
        if cname not in raw and not name.endswith("inv_freq"):
            raw[cname] = buf.detach()
    return units, raw


class CompressionPlan:
    """Prepared kernel launches for a set of compression units whose weights are on ``device``
    (staged there when the model is host-resident).  Dense units of one scheme and shape are ONE
    grouped launch (``ops.GroupedQuantize``: the launch ramp paid once per shape, 5 launches for
    all 252 Qwen3-4B linears; one mixed-shape launch per scheme measured 3 % slower);
    NVFP4 dense units of one shape are one ``qz_quantize_grouped_nvfp4`` call (two launches);
    FP8_BLOCK dense units of one shape are one launch of the strip kernel (``qz_quantize_grouped``,
    qz_block.hip); stacked fused experts and other schemes are one call each.  ``run()`` only enqueues
    the launches (graph/bench friendly, outputs preallocated); ``tensors()`` returns the on-disk tensors by name."""

    def __init__(self, units: Sequence[CompressUnit], device, stager=None):
        self.device = torch.device(device)
        self.grouped = []  # (GroupedQuantize, [(unit, weight)], args, int_q, fmt)
        self.singles = []  # (unit, weight, preallocated outputs, args, int_q, fmt)
        buckets: Dict[tuple, list] = {}
        self.params = 0
        staged = False
        bases: Dict[int, torch.Tensor] = {}  # host fused parameter -> its staged device copy
        for u in units:
            a = u.scheme.weights
            w = u.view()
            if w.device != self.device:  # host-resident weight: pinned, double-buffered staging
                if stager is None:
                    from .staging import H2DStager
                    stager = H2DStager(self.device)
                base = u.base()
                if base is not None and not w.is_contiguous() and base.is_contiguous() \
                        and w.untyped_storage().data_ptr() == base.untyped_storage().data_ptr():
                    # a strided slice of a fused expert parameter (gate / up halves): stage the
                    # parameter once, contiguously, and take the same view on the device -- no
                    # host-side gather copy (58 GB of them cost 7 s on Qwen3-30B-A3B)
                    key = base.data_ptr()
                    if key not in bases:
                        bases[key] = stager.copy(base)
                    w = bases[key].as_strided(w.size(), w.stride(), w.storage_offset() - base.storage_offset())
                else:
                    w = stager.copy(w)
                staged = True
            self.params += w.numel()
            int_q, fmt = ops._compress_plan(a, u.scheme.input_activations is not None)
            if not u.stacked and ops.grouped_ok(a, w):
                # one launch per (scheme, shape); one mixed-shape launch per scheme
                # (qz_quantize_grouped_var) measured 3 % slower on Qwen3-4B (r02q A/B)
                key = (id(u.scheme), tuple(w.shape))
                buckets.setdefault(key, []).append((u, w))
            else:
                self.singles.append((u, w, ops.alloc_outputs(tuple(w.shape), a, fmt, self.device), a, int_q, fmt))
        for items in buckets.values():
            a = items[0][0].scheme.weights
            int_q, fmt = ops._compress_plan(a, items[0][0].scheme.input_activations is not None)
            if len({tuple(w.shape) for _, w in items}) > 8:  # at most 8 shapes per launch
                items.sort(key=lambda uw: tuple(uw[1].shape))
            parts: List[list] = [[]]
            seen: set = set()
            for uw in items:  # <= 65535 weights and <= 8 shapes per launch
                shp = tuple(uw[1].shape)
                if len(parts[-1]) == 65535 or (shp not in seen and len(seen) == 8):
                    parts.append([])
                    seen = set()
                parts[-1].append(uw)
                seen.add(shp)
            for part in parts:
                gq = ops.GroupedQuantize([w for _, w in part], a, fmt)
                self.grouped.append((gq, part, a, int_q, fmt))
        self._ready = None  # completion of the staging copies: every run() waits for it
        if staged:
            self._ready = torch.cuda.Event()
            self._ready.record(stager.stream)

    @property
    def launches(self) -> int:
        return len(self.grouped) + len(self.singles)

    def alg_bytes(self) -> int:
        """Algorithmic HBM bytes of one run(): every weight read once + every output written once."""
        n = self.params * 2
        outs = [o for gq, *_ in self.grouped for o in gq.outs] + [o for _, _, o, *_ in self.singles]
        for o in outs:
            for t in o.values():
                if t is not None:
                    n += t.numel() * t.element_size()
        return n

    def run(self, stream=None) -> None:
        main = stream if stream is not None else torch.cuda.current_stream(self.device)
        if self._ready is not None:
            main.wait_event(self._ready)
        for gq, *_ in self.grouped:  # one stream: spreading the launches over 2-3 streams measured
            if not gq.nvfp4:         # slower (r02r A/B) -- except NVFP4's two-launch calls:
                gq.run(main)
        nvg = [gq for gq, *_ in self.grouped if gq.nvfp4]
        if nvg:  # Qwen3-4B NVFP4, 7 calls: 3.14-3.18 -> 2.95-2.96 ms on 2 streams (r04y_nv_streams_dense.log)
            sts = ops.nvfp4_streams(self.device, main)
            for i, gq in enumerate(nvg):
                gq.run(sts[i % len(sts)])
            ops.join_streams(sts)
        if self.singles:
            # float schemes carry fmt None (the kernel's default output, ops._compress_plan)
            two_stream = lambda a, fmt: a.is_nvfp4 and fmt in (None, ops.default_out_fmt(a))  # noqa: E731
            nv = [(w, o, a) for u, w, o, a, int_q, fmt in self.singles if two_stream(a, fmt)]
            with torch.cuda.stream(main):
                for u, w, o, a, int_q, fmt in self.singles:
                    if not two_stream(a, fmt):
                        ops.quantize_weight(w, a, out_fmt=fmt, out=o)
            # NVFP4 parameters (stacked fused experts): two streams, one's |w| max launch beside
            # the other's encode (ops.quantize_nvfp4_many); grouped by scheme
            by_args: Dict[int, list] = {}
            for w, o, a in nv:
                by_args.setdefault(id(a), [a, []])[1].append((w, o))
            for a, items in by_args.values():
                ops.quantize_nvfp4_many(items, a, stream=main)

    def tensors(self) -> Dict[str, torch.Tensor]:
        """The on-disk tensors of every unit (device tensors; ``weight_shape`` on the host)."""
        out: Dict[str, torch.Tensor] = {}
        for gq, part, a, int_q, fmt in self.grouped:
            for (u, w), q in zip(part, gq.outs):
                for k, v in ops._compressed_tensors(q, tuple(w.shape), a, int_q, fmt).items():
                    out[f"{u.refs[0].name}.{k}"] = v
        for u, w, q, a, int_q, fmt in self.singles:
            comp = ops._compressed_tensors(q, tuple(w.shape), a, int_q, fmt)
            for i, g in enumerate(u.refs):
                for k, v in comp.items():
                    if k == "weight_shape":
                        out[f"{g.name}.{k}"] = v.clone()  # one tensor per module (no shared storage)
                    elif not u.stacked:
                        out[f"{g.name}.{k}"] = v
                    else:
                        out[f"{g.name}.{k}"] = v[i].reshape(v.shape[1:] if v.dim() > 1 else (1,))
        return out


def _chunks(units: Sequence[CompressUnit], budget: int, device) -> List[List[CompressUnit]]:
    """Split units so the weights staged on ``device`` per plan stay under ``budget`` bytes
    (device-resident weights need no staging and form one plan)."""
    out: List[List[CompressUnit]] = [[]]
    size = 0
    for u in units:
        staged = u.refs[0].weight.device != torch.device(device)
        nb = u.nbytes if staged else 0
        if out[-1] and size + nb > budget:
            out.append([])
            size = 0
        out[-1].append(u)
        size += nb
    return [c for c in out if c]


class _HostCopier:
    """Asynchronous device -> pinned-host copies on a side stream: the copies of one plan overlap
    the next plan's kernels; at most ``budget`` bytes of device results are kept alive waiting
    for their copies."""

    def __init__(self, device, budget: int = 8 << 30):
        self.device = torch.device(device)
        self.stream = torch.cuda.Stream(self.device)
        self.pending = []  # (done event, device tensors, bytes)
        self.inflight = 0
        self.budget = budget

    def submit(self, items: Dict[str, torch.Tensor]) -> Dict[str, torch.Tensor]:
        """Enqueue the device -> host copies of ``items``; returns host tensors (valid once
        ``last_event`` completes).  Tensors that are views of one device storage (the per-expert
        slices of a stacked output) travel as ONE copy of that storage, and their host views are
        cut from its pinned copy: a few large DMAs instead of one per tensor."""
        dev_items = {k: t for k, t in items.items() if t.is_cuda}
        host = {k: t for k, t in items.items() if not t.is_cuda}
        if not dev_items:
            return host
        ready = torch.cuda.Event()
        ready.record(torch.cuda.current_stream(self.device))
        self.stream.wait_event(ready)
        stores: Dict[int, Tuple[torch.UntypedStorage, int]] = {}  # storage ptr -> (storage, buffer offset)
        total = 0
        for t in dev_items.values():
            st = t.untyped_storage()
            if st.data_ptr() not in stores:
                stores[st.data_ptr()] = (st, total)
                total += (st.nbytes() + 63) // 64 * 64
        buf = torch.empty(max(total, 1), dtype=torch.uint8, pin_memory=True)
        with torch.cuda.stream(self.stream):
            for st, off in stores.values():
                src = torch.empty(0, dtype=torch.uint8, device=self.device).set_(st, 0, (st.nbytes(),), (1,))
                buf[off:off + st.nbytes()].copy_(src, non_blocking=True)
        for k, t in dev_items.items():
            st, off = stores[t.untyped_storage().data_ptr()]
            flat = buf[off:off + st.nbytes()].view(t.dtype)
            host[k] = flat.as_strided(t.size(), t.stride(), flat.storage_offset() + t.storage_offset())
        done = torch.cuda.Event()
        done.record(self.stream)
        self.pending.append((done, list(dev_items.values()), total))
        self.inflight += total
        while self.inflight > self.budget and len(self.pending) > 1:
            self._retire()
        return host

    @property
    def last_event(self):
        """Completion event of the latest submit (None before the first device copy)."""
        return self.pending[-1][0] if self.pending else None

    def _retire(self):
        done, _, nb = self.pending.pop(0)
        done.synchronize()
        self.inflight -= nb

    def finish(self):
        while self.pending:
            self._retire()


def _dist_info() -> Tuple[int, int]:
    if dist.is_available() and dist.is_initialized():
        return dist.get_world_size(), dist.get_rank()
    return 1, 0


STAGE_BYTES = 4 << 30  # host-resident weights staged on the device per plan
WRITE_THREADS = 4  # concurrent shard-file writers


def _compress_chunks(units: Sequence[CompressUnit], device, copier: Optional["_HostCopier"], timings: Dict[str, float]):
    """Compress ``units`` plan by plan (at most STAGE_BYTES of host weights staged per plan);
    yields each plan's on-disk tensors -- pinned-host views when ``copier`` is given (valid once
    ``copier.last_event`` completes), device tensors otherwise."""
    stager = None
    if device.type == "cuda" and any(u.refs[0].weight.device != device for u in units):
        from .staging import H2DStager
        stager = H2DStager(device)  # one pair of pinned buffers for every chunk
    for k in ("plan", "run", "tensors", "submit"):
        timings.setdefault(k, 0.0)
    for chunk in _chunks(units, STAGE_BYTES, device):
        t0 = time.perf_counter()
        plan = CompressionPlan(chunk, device, stager)
        t1 = time.perf_counter()
        plan.run()
        t2 = time.perf_counter()
        t = plan.tensors()
        t3 = time.perf_counter()
        out = copier.submit(t) if copier is not None else t
        timings["plan"] += t1 - t0
        timings["run"] += t2 - t1
        timings["tensors"] += t3 - t2
        timings["submit"] += time.perf_counter() - t3
        del plan
        yield out
    if stager is not None:
        timings["staging"] = dict(stager.stats)


def _raw_to_host(raw: Dict[str, torch.Tensor], device,
                 copier: Optional["_HostCopier"] = None) -> Tuple[Dict[str, torch.Tensor], Optional["_HostCopier"]]:
    """The unchanged tensors on the host: device ones through a pinned copier (``copier``, or a
    new one; returned, to be finished by the caller), host ones as they are -- except those
    sharing storage with another output (tied embeddings), cloned because safetensors refuses
    shared storage."""
    out: Dict[str, torch.Tensor] = {}
    dev_raw = {k: v for k, v in raw.items() if v.is_cuda}
    if dev_raw:
        copier = copier if copier is not None else _HostCopier(device)
        out.update(copier.submit(dev_raw))
    host_raw = {k: v for k, v in raw.items() if not v.is_cuda}
    users: Dict[int, int] = {}
    for v in host_raw.values():
        users[v.untyped_storage().data_ptr()] = users.get(v.untyped_storage().data_ptr(), 0) + 1
    for k, v in host_raw.items():
        out[k] = v.clone() if users[v.untyped_storage().data_ptr()] > 1 else v
    return out, copier


@torch.no_grad()
def compressed_state_dict(model: nn.Module, device=None, to_host: bool = True,
                          dst: Optional[int] = None) -> Dict[str, torch.Tensor]:
    """All tensors to write: compressed targeted weights + untouched parameters/buffers.

    One process: every unit is compressed by ``CompressionPlan`` (grouped launches) and copied
    to pinned host memory asynchronously.  Under ``torch.distributed`` (one process per GPU, every
    rank holding the same model): the units are assigned to ranks by bytes (LPT,
    ``distributed.plan_shards``), each rank compresses its share with no collective on the data
    path, and ``distributed.gather_state`` reassembles the compressed tensors with bucketed RCCL
    all-gathers -- on every rank (``dst=None``) or only on rank ``dst`` (others get ``{}``)."""
    device = torch.device(device) if device is not None else torch.device("cuda", torch.cuda.current_device())
    units, raw = compression_units(model)
    world, rank = _dist_info()
    mine = units
    res = getattr(model, "quantization_residency", None)
    owned_raw: Dict[str, torch.Tensor] = {}
    if world > 1 and res is not None:
        # owner-keeps residency (oneshot over a meta skeleton): compress what this rank holds --
        # a unit kept by two ranks (it straddles their shards) is taken by the lower one
        sp = save_plan(units, raw, world, res.max_shard_bytes)
        taken = set().union(*[set(sp.units_of[r]) for r in range(rank)]) if rank else set()
        mine = [units[i] for i in sp.units_of[rank] if i not in taken]
        if dst is None or dst != 0:  # receivers other than rank 0 get each unchanged tensor from its owner
            owned_raw = {k: raw[k] for k in sp.raw_of[rank] if not raw[k].is_meta}
    elif world > 1:
        from .distributed import plan_shards
        plan = plan_shards([(str(i), u.nbytes) for i, u in enumerate(units)], world)
        keep = {int(k) for k in plan[rank]}
        mine = [u for i, u in enumerate(units) if i in keep]
    copier = _HostCopier(device) if (to_host and world == 1 and device.type == "cuda") else None
    local: Dict[str, torch.Tensor] = {}
    tm: Dict[str, float] = {}
    for t in _compress_chunks(mine, device, copier, tm):
        local.update(t)
    if copier is not None:
        copier.finish()
    log.info("compressed_state_dict phases (s): %s", tm)
    receiver = world == 1 or dst is None or rank == dst
    if world > 1:
        from .distributed import gather_state
        local.update({f"\0raw.{k}": v for k, v in owned_raw.items()})
        local = gather_state(local, dst=dst, to_host=to_host)
        # unchanged tensors a skeleton rank holds only as meta come from their owners
        for k in [k for k in local if k.startswith("\0raw.")]:
            v = local.pop(k)
            if raw.get(k[5:]) is not None and raw[k[5:]].is_meta:
                raw[k[5:]] = v
    if not receiver:
        return {}
    raw = {k: v for k, v in raw.items() if not v.is_meta}
    out = dict(local)
    if to_host:
        host_raw, rc = _raw_to_host(raw, device)
        out.update(host_raw)
        if rc is not None:
            rc.finish()
    else:
        out.update(raw)
    return out


def _unit_layout(u: CompressUnit) -> List[Tuple[str, int]]:
    """Names and byte sizes of a unit's on-disk tensors, known before anything runs (the
    shapes ``ops._compressed_tensors`` gives each module, per expert for a stacked unit)."""
    a = u.scheme.weights
    int_q, _ = ops._compress_plan(a, u.scheme.input_activations is not None)
    rows, cols = (int(x) for x in u.refs[0].weight.shape[-2:])
    gshape = ops.n_groups(a, rows, cols)
    ng = 1
    for d in gshape:
        ng *= d
    scale_b = ng * torch.empty((), dtype=ops._scale_dtype(a)).element_size()
    sizes: Dict[str, int] = {}
    if a.type == "int":
        pf = 32 // a.num_bits
        if int_q:
            sizes["weight"] = rows * cols
        else:
            sizes["weight_packed"] = rows * ((cols + pf - 1) // pf) * 4
            sizes["weight_shape"] = 2 * 8
        sizes["weight_scale"] = scale_b
        if not a.symmetric and a.strategy in ("group", "channel"):
            sizes["weight_zero_point"] = ng if int_q else (gshape[0] + pf - 1) // pf * gshape[1] * 4
    elif a.num_bits == 8:
        sizes["weight"] = rows * cols
        sizes["weight_scale"] = scale_b
    else:
        sizes["weight_packed"] = rows * cols // 2
        sizes["weight_scale"] = scale_b
        if a.is_nvfp4:
            sizes["weight_global_scale"] = 4
    return [(f"{r.name}.{k}", nb) for r in u.refs for k, nb in sizes.items()]


def _split_shards(items: Sequence[Tuple[str, int]], max_shard_bytes: int) -> List[List[str]]:
    """The shard split of ``items`` (checkpoint order): a shard closes when the next tensor would
    take it past ``max_shard_bytes`` (a tensor larger than that is a shard of its own)."""
    shards: List[List[str]] = [[]]
    size = 0
    for n, nb in items:
        if shards[-1] and size + nb > max_shard_bytes:
            shards.append([])
            size = 0
        shards[-1].append(n)
        size += nb
    return shards


@dataclass
class SavePlan:
    """Who writes what, computed identically on every rank before anything is compressed.

    ``order``: every checkpoint tensor (name, bytes) in checkpoint order -- compression units in
    model order, names sorted within a unit, then the unchanged tensors by name; ``shards``: the
    split of that order into files (``files``); ``owner[s]``: the rank that writes shard ``s``
    (contiguous runs of shards, balanced by bytes); ``units_of[r]`` / ``raw_of[r]``: the units
    rank ``r`` compresses and the unchanged tensors it writes -- exactly those with a tensor in
    one of its shards (a unit straddling two ranks' shards is compressed by both)."""

    order: List[Tuple[str, int]]
    shards: List[List[str]]
    files: List[str]
    owner: List[int]
    units_of: List[List[int]]
    raw_of: List[List[str]]

    @property
    def total_bytes(self) -> int:
        return sum(nb for _, nb in self.order)

    def weight_map(self) -> Dict[str, str]:
        return {n: f for names, f in zip(self.shards, self.files) for n in names}


def save_plan(units: Sequence[CompressUnit], raw: Dict[str, torch.Tensor], world: int,
              max_shard_bytes: int = SHARD_BYTES) -> SavePlan:
    order: List[Tuple[str, int]] = []
    unit_of: Dict[str, int] = {}
    for i, u in enumerate(units):
        lay = sorted(_unit_layout(u))
        order.extend(lay)
        for n, _ in lay:
            unit_of[n] = i
    order.extend(sorted((k, v.numel() * v.element_size()) for k, v in raw.items()))
    shards = _split_shards(order, max_shard_bytes)
    n = len(shards)
    files = ["model.safetensors"] if n == 1 else [f"model-{i + 1:05d}-of-{n:05d}.safetensors" for i in range(n)]
    size = dict(order)
    total = max(1, sum(size.values()))
    owner, before = [], 0
    for names in shards:  # rank of a shard = where its byte midpoint falls: contiguous, balanced
        nb = sum(size[x] for x in names)
        owner.append(min(world - 1, int(world * (before + nb / 2) / total)))
        before += nb
    units_of: List[set] = [set() for _ in range(world)]
    raw_of: List[List[str]] = [[] for _ in range(world)]
    for names, r in zip(shards, owner):
        for x in names:
            if x in unit_of:
                units_of[r].add(unit_of[x])
            else:
                raw_of[r].append(x)
    return SavePlan(order, shards, files, owner, [sorted(s) for s in units_of], raw_of)


def save_compressed(model: nn.Module, output_dir: str, max_shard_bytes: int = SHARD_BYTES, device=None) -> str:
    """Write safetensors shards + index + config.json(quantization_config).

    The shard split is fixed up front from the tensors' names and sizes (``save_plan``: the same
    files, byte for byte, whatever the number of ranks).  One process writes every shard; under
    ``torch.distributed`` (one process per GPU) each rank compresses only the units whose
    tensors fall in ITS shards, copies them device -> host over its own PCIe link and writes
    those files itself -- no compressed byte crosses xGMI or funnels through rank 0; rank 0 adds
    the index and config.  The ranks must therefore share ``output_dir`` (one node, or a shared
    filesystem): checked before anything is written (``_check_shared_dir``).  Either way a shard is handed to a writer thread as soon as its bytes
    are on the host, while later plans compress.  Every rank returns after all files exist."""
    world, rank = _dist_info()
    device = torch.device(device) if device is not None else torch.device("cuda", torch.cuda.current_device())
    qcfg = quantization_config(model)
    if hasattr(model, "config"):
        # so a later model.config.save_pretrained(output_dir) keeps the compressed-tensors config
        model.config.quantization_config = qcfg
    t0 = time.perf_counter()
    res = getattr(model, "quantization_residency", None)
    if res is not None and (res.max_shard_bytes != max_shard_bytes or res.world != world):
        raise ValueError(f"this model's ranks keep the tensors of a {res.world}-rank save plan with "
                         f"max_shard_bytes={res.max_shard_bytes} (oneshot(max_shard_bytes=...)); "
                         f"save_compressed was called with {world} rank(s) and {max_shard_bytes}")
    if world > 1:
        _check_shared_dir(output_dir, rank)
    units, raw = compression_units(model)
    plan = save_plan(units, raw, world, max_shard_bytes)
    mine = [units[i] for i in plan.units_of[rank]]
    my_raw = {k: raw[k] for k in plan.raw_of[rank]}
    writer = _PlannedShardWriter(output_dir, plan, rank)
    copier = _HostCopier(device) if device.type == "cuda" else None
    tm: Dict[str, float] = {}
    for t in _compress_chunks(mine, device, copier, tm):
        writer.add(t, copier.last_event if copier is not None else None)
    host_raw, rc = _raw_to_host(my_raw, device, copier)  # same copier stream: its last event covers all
    writer.add(host_raw, copier.last_event if copier is not None else (rc.last_event if rc is not None else None))
    n_tensors, n_bytes = writer.close()
    if copier is not None:
        copier.finish()
    if rc is not None and rc is not copier:
        rc.finish()
    log.info("save_compressed rank %d/%d: %d shard(s), %d tensors, %.2f GB; phases (s): %s", rank, world,
             plan.owner.count(rank), n_tensors, n_bytes / 1e9, tm)
    if rank == 0:
        if len(plan.files) > 1:
            with open(os.path.join(output_dir, "model.safetensors.index.json"), "w") as f:
                json.dump({"metadata": {"total_size": plan.total_bytes},
                           "weight_map": dict(sorted(plan.weight_map().items()))}, f, indent=2)
        _write_config(model, qcfg, output_dir)
        log.info("save_compressed: %d files, %.2f GB in %.2fs", len(plan.files), plan.total_bytes / 1e9,
                 time.perf_counter() - t0)
    if world > 1:
        dist.barrier()
    return output_dir


def _check_shared_dir(output_dir: str, rank: int) -> None:
    """Every rank writes its own shards into ``output_dir``, so the directory must be the SAME
    directory on every rank (one node, or a filesystem shared by all nodes): rank 0 drops a probe
    file there and every rank must read it back, else the save stops before writing anything."""
    import uuid
    os.makedirs(output_dir, exist_ok=True)
    box = [uuid.uuid4().hex if rank == 0 else None]
    dist.broadcast_object_list(box, 0)
    probe = os.path.join(output_dir, f".qz_rank_probe_{box[0]}")
    if rank == 0:
        with open(probe, "w") as f:
            f.write(box[0])
    dist.barrier()
    try:
        ok = open(probe).read() == box[0]
    except OSError:
        ok = False
    seen: List = [None] * dist.get_world_size()
    dist.all_gather_object(seen, ok)
    if rank == 0:
        os.remove(probe)
    if not all(seen):
        raise RuntimeError(f"save_compressed: {output_dir} is not one shared directory for all ranks (ranks "
                           f"{[r for r, v in enumerate(seen) if not v]} cannot see rank 0's files); every rank "
                           f"writes its own shards, so run the ranks on one node or on a shared filesystem")


class _PlannedShardWriter:
    """Writes this rank's shards of a ``SavePlan``: tensors arrive in any grouping (plan by plan,
    then the unchanged ones); a shard is handed to a pool thread (WRITE_THREADS) once all its
    tensors are here, under its final file name.  Tensors of other ranks' shards are dropped
    (the halves of a straddling unit); a tensor whose size differs from the plan is an error."""

    def __init__(self, output_dir: str, plan: SavePlan, rank: int):
        from concurrent.futures import ThreadPoolExecutor
        os.makedirs(output_dir, exist_ok=True)
        self.dir, self.plan = output_dir, plan
        self.size = dict(plan.order)
        self.mine = [s for s, r in enumerate(plan.owner) if r == rank]
        self.shard_of = {n: s for s in self.mine for n in plan.shards[s]}
        self.missing = {s: len(plan.shards[s]) for s in self.mine}
        self.held: Dict[int, Dict[str, torch.Tensor]] = {s: {} for s in self.mine}
        self.ready = None
        self.pool = ThreadPoolExecutor(max_workers=max(1, WRITE_THREADS))
        self.futures = []
        self.count = self.bytes = 0

    def add(self, items: Dict[str, torch.Tensor], ready=None) -> None:
        if ready is not None:
            self.ready = ready  # one copy stream: the latest event covers every earlier copy
        for n, t in items.items():
            if n not in self.size:  # a tensor the plan never saw would silently be lost
                raise ValueError(f"save plan: {n} is not in the checkpoint plan")
            s = self.shard_of.get(n)
            if s is None or n in self.held[s]:  # another rank's shard (a straddling unit's other half)
                continue
            nb = t.numel() * t.element_size()
            if nb != self.size[n]:
                raise ValueError(f"save plan: {n} has {nb} bytes, the plan expected {self.size[n]}")
            self.held[s][n] = t
            self.missing[s] -= 1
            if self.missing[s] == 0:
                shard = {x: self.held[s][x] for x in self.plan.shards[s]}  # checkpoint order
                self.held[s] = {}
                self.count += len(shard)
                self.bytes += sum(self.size[x] for x in shard)
                path = os.path.join(self.dir, self.plan.files[s])
                self.futures.append(self.pool.submit(_write_shard_file, shard, path, self.ready))

    def close(self) -> Tuple[int, int]:
        try:
            for f in self.futures:
                f.result()
        finally:
            self.pool.shutdown()
        left = {self.plan.files[s]: n for s, n in self.missing.items() if n}
        if left:
            raise RuntimeError(f"save plan: shards never completed (tensors missing): {left}")
        return self.count, self.bytes


def _write_shard_file(shard: Dict[str, torch.Tensor], path: str, ready) -> None:
    if ready is not None:
        ready.synchronize()  # the shard's device -> host copies have landed
    tmp = os.path.join(os.path.dirname(path), "." + os.path.basename(path) + ".tmp")
    save_file({k: (v.cpu() if v.is_cuda else v).contiguous() for k, v in shard.items()}, tmp,
              metadata={"format": "pt"})
    os.replace(tmp, path)


def _write_config(model: nn.Module, qcfg: dict, output_dir: str) -> None:
    cfg = model.config.to_dict() if hasattr(model, "config") else {}
    cfg["quantization_config"] = qcfg
    with open(os.path.join(output_dir, "config.json"), "w") as f:
        json.dump(cfg, f, indent=2, default=str)
    _write_recipe(getattr(model, "quantization_recipe", None), output_dir)


def _write_recipe(recipe, output_dir: str) -> None:
    """recipe.yaml beside the checkpoint (llmcompressor's save_pretrained wrapper stores the
    applied recipe the same way): the recipe file's text, or the dict/YAML text it was given."""
    import yaml
    if recipe is None:
        return
    path = os.path.join(output_dir, "recipe.yaml")
    if isinstance(recipe, str):
        text = open(recipe).read() if os.path.exists(recipe) else recipe
    elif isinstance(recipe, (dict, list)):
        try:
            text = yaml.safe_dump(recipe, sort_keys=False)
        except yaml.YAMLError:
            return
    else:
        return
    with open(path, "w") as f:
        f.write(text)


def _load_all(path: str) -> Dict[str, torch.Tensor]:
    idx = os.path.join(path, "model.safetensors.index.json")
    if os.path.exists(idx):
        files = sorted(set(json.load(open(idx))["weight_map"].values()))
    else:
        files = ["model.safetensors"]
    sd = {}
    for fn in files:
        sd.update(load_file(os.path.join(path, fn)))
    return sd


@torch.no_grad()
def load_decompressed(path: str, device=None) -> Dict[str, torch.Tensor]:
    """Read a compressed checkpoint back to bf16 weights (decompressors on the GPU)."""
    device = torch.device(device) if device is not None else torch.device("cuda", torch.cuda.current_device())
    cfg = json.load(open(os.path.join(path, "config.json")))["quantization_config"]
    sd = _load_all(path)
    group_args = {g: QuantizationArgs(**{k: v for k, v in c["weights"].items()}) for g, c in cfg["config_groups"].items()}
    out = {}
    bases = {}
    for k in sd:
        for suf in (".weight_packed", ".weight_scale", ".weight"):
            if k.endswith(suf):
                bases.setdefault(k[: -len(suf)], set()).add(suf)
    for base, sufs in bases.items():
        if ".weight_scale" not in sufs:
            continue
        args = _args_for(base, cfg, group_args)
        scale = sd[f"{base}.weight_scale"].to(device)
        zp = sd.get(f"{base}.weight_zero_point")
        gs = sd.get(f"{base}.weight_global_scale")
        if args.type == "int":
            codes = sd[f"{base}.weight_packed"].to(device) if f"{base}.weight_packed" in sd else sd[f"{base}.weight"].to(device)
            shape = tuple(int(x) for x in sd[f"{base}.weight_shape"].tolist()) if f"{base}.weight_shape" in sd else tuple(codes.shape)
            if zp is not None and not args.symmetric:
                zp = ops.unpack_zero_points(zp.to(device), args.num_bits, scale.shape) if zp.dtype == torch.int32 else zp.to(device)
            fmt = None if codes.dtype == torch.int32 else 1
            out[f"{base}.weight"] = ops.dequantize(codes, shape, args, scale, zp, in_fmt=fmt).cpu()
        elif args.num_bits == 8:
            codes = sd[f"{base}.weight"].to(device)
            out[f"{base}.weight"] = ops.dequantize(codes, tuple(codes.shape), args, scale).cpu()
        else:
            codes = sd[f"{base}.weight_packed"].to(device)
            shape = (codes.shape[0], codes.shape[1] * 2)
            out[f"{base}.weight"] = ops.dequantize(codes, shape, args, scale, None,
                                                   gs.to(device) if gs is not None else None).cpu()
    for k, v in sd.items():
        if any(k.endswith(s) for s in (".weight_packed", ".weight_scale", ".weight_shape", ".weight_zero_point",
                                       ".weight_global_scale")):
            continue
        if k not in out:
            out[k] = v
    return out


def _args_for(base: str, cfg: dict, group_args: Dict[str, QuantizationArgs]) -> QuantizationArgs:
    from .recipe import match_any
    for g, c in cfg["config_groups"].items():
        if match_any(base, "Linear", [t for t in c["targets"] if t.startswith("re:") or t == base]):
            return group_args[g]
    if len(group_args) == 1:
        return next(iter(group_args.values()))
    for g, c in cfg["config_groups"].items():
        if "Linear" in c["targets"]:
            return group_args[g]
    raise ValueError(f"no config group for {base}")
