"""Multi-GPU weight quantization: one process per GPU, weights sharded across ranks, results
reassembled with one RCCL all-gather over xGMI (BASELINE.json configs[4]).

The reference is single-process (its only parallelism is model_free_ptq's file thread pool,
scripts/quant_GLM-4.7-Flash-FP8.py:22).  Quantize+pack has no cross-weight dependency, so:

* ``plan_shards`` assigns whole weights (or whole fused-expert groups) to ranks by bytes,
  longest-processing-time first (deterministic: every rank computes the same plan);
* each rank compresses its share with the fused HIP kernel -- no collective on the data path;
* ``gather_state`` flattens each rank's compressed tensors into one byte buffer and runs ONE
  ``all_gather_into_tensor`` (padded to the largest shard; xGMI is point-to-point, so a single
  large collective beats many small ones) straight into the result buffer, whose per-rank
  slices every rank unflattens as views -- or ``gather`` to one rank only (``dst``).
* ``save_compressed`` does not gather at all: each rank writes its own shard files
  (``compressor.save_compressed``).

Works with backend "nccl" (RCCL, GPU tensors) and "gloo" (CPU tensors, used by the CPU tests).
"""
from __future__ import annotations

import heapq
from typing import Callable, Dict, List, Optional, Sequence, Tuple

import torch
import torch.distributed as dist

Item = Tuple[str, int]  # (key, cost in bytes)


def plan_shards(items: Sequence[Item], world: int) -> List[List[str]]:
    """LPT assignment of weights to ranks (ties broken by key so every rank agrees)."""
    heap = [(0, r) for r in range(world)]
    heapq.heapify(heap)
    out: List[List[str]] = [[] for _ in range(world)]
    for key, cost in sorted(items, key=lambda kv: (-kv[1], kv[0])):
        load, r = heapq.heappop(heap)
        out[r].append(key)
        heapq.heappush(heap, (load + cost, r))
    return out


def _layout(tensors: Dict[str, torch.Tensor]) -> Tuple[int, List[Tuple[str, str, Tuple[int, ...], int]]]:
    """Byte layout of ``tensors`` (sorted by name) in one flat buffer, every tensor 16-B aligned:
    (total bytes, [(name, dtype, shape, byte offset)])."""
    meta = []
    off = 0
    for k in sorted(tensors):
        t = tensors[k]
        nb = t.numel() * t.element_size()
        meta.append((k, str(t.dtype).replace("torch.", ""), tuple(t.shape), off))
        off += (nb + 15) // 16 * 16
    return off, meta


def _flatten(tensors: Dict[str, torch.Tensor], device, meta=None, capacity: Optional[int] = None) -> torch.Tensor:
    """Copy ``tensors`` into one uint8 buffer of ``capacity`` bytes (default: the layout's size)
    on ``device`` at the offsets of ``meta`` (``_layout``); the padding is zeroed."""
    size, lay = _layout(tensors) if meta is None else (None, meta)
    if size is None:
        last = lay[-1] if lay else None
        size = 0 if last is None else last[3] + (_nbytes(last) + 15) // 16 * 16
    cap = size if capacity is None else capacity
    flat = torch.empty(cap, dtype=torch.uint8, device=device)
    end = 0
    for k, _, _, o in lay:
        t = tensors[k].contiguous()
        nb = t.numel() * t.element_size()
        if o > end:
            flat[end:o].zero_()
        if nb:
            flat[o:o + nb].copy_(t.reshape(-1).view(torch.uint8), non_blocking=True)
        end = o + nb
    if cap > end:
        flat[end:].zero_()
    return flat


def _nbytes(entry) -> int:
    _, dt, shape, _ = entry
    n = 1
    for d in shape:
        n *= d
    return n * torch.empty((), dtype=getattr(torch, dt)).element_size()


def _unflatten(flat: torch.Tensor, meta, copy: bool = True) -> Dict[str, torch.Tensor]:
    out = {}
    for ent in meta:
        k, dt, shape, off = ent
        t = flat[off:off + _nbytes(ent)].view(getattr(torch, dt)).reshape(shape)
        out[k] = t.clone() if copy else t
    return out


GATHER_BUCKET_BYTES = 1 << 30  # bytes per rank per all-gather round


def gather_state(local: Dict[str, torch.Tensor], device=None, dst: Optional[int] = None, to_host: bool = False,
                 bucket_bytes: int = GATHER_BUCKET_BYTES) -> Dict[str, torch.Tensor]:
    """Reassemble every rank's tensors: the union of all ranks' ``local`` dicts on every rank
    (``dst=None``) or on rank ``dst`` only (the other ranks return ``{}``).

    Each rank's tensors are packed into one flat byte buffer (padded to the largest rank's size).
    ``dst=None``: the buffers travel by ``all_gather_into_tensor`` -- ONE collective straight into
    the result buffer when every rank's share fits ``bucket_bytes``, otherwise rounds of
    ``bucket_bytes`` per rank (a bounded staging footprint); a few large RCCL collectives over the
    point-to-point xGMI links rather than one per tensor.  ``dst=r``: the same rounds by
    ``gather`` to rank ``r`` alone (no bytes delivered to ranks that drop them).  ``to_host``:
    the receivers' results land in pinned host memory (the writer's input), otherwise on
    ``device``."""
    world = dist.get_world_size() if dist.is_initialized() else 1
    if world == 1:
        if not to_host:
            return dict(local)
        return {k: (v.cpu() if v.is_cuda else v) for k, v in local.items()}
    return _gather_packed(local, device, dst, to_host, bucket_bytes)


def _gather_packed(local: Dict[str, torch.Tensor], device, dst: Optional[int], to_host: bool,
                   bucket_bytes: int) -> Dict[str, torch.Tensor]:
    """gather_state's collective path (any world size, so a 1-rank RCCL group exercises it)."""
    world = dist.get_world_size()
    rank = dist.get_rank()
    nccl = dist.get_backend() == "nccl"
    if device is None:
        device = torch.device("cuda", torch.cuda.current_device()) if nccl else torch.device("cpu")
    size, meta = _layout(local)
    metas: List = [None] * world
    dist.all_gather_object(metas, (size, meta))
    maxn = max(m[0] for m in metas)
    receiver = dst is None or rank == dst
    out: Dict[str, torch.Tensor] = {}
    if maxn == 0:
        return out if receiver else {}
    if maxn <= bucket_bytes and not to_host:
        # one round, received in place: rank r's tensors are views of recv[r * maxn:]
        send = _flatten(local, device, meta, capacity=maxn)
        if dst is None:
            recv = torch.empty(world * maxn, dtype=torch.uint8, device=device)
            dist.all_gather_into_tensor(recv, send)
        else:
            recv = torch.empty(world * maxn, dtype=torch.uint8, device=device) if receiver else None
            dist.gather(send, [recv[r * maxn:(r + 1) * maxn] for r in range(world)] if receiver else None, dst=dst)
        if not receiver:
            return {}
        for r in range(world):
            out.update(_unflatten(recv[r * maxn:(r + 1) * maxn], metas[r][1], copy=False))
        return out
    flat = _flatten(local, device, meta)
    host_dev = torch.device("cpu") if to_host else torch.device(device)
    pin = to_host and flat.is_cuda
    dest = [torch.empty(metas[r][0], dtype=torch.uint8, device=host_dev, pin_memory=pin) for r in range(world)] \
        if receiver else None
    step = max(16, min(bucket_bytes, maxn) // 16 * 16)
    send = torch.zeros(step, dtype=torch.uint8, device=device)
    recv = torch.empty(world * step, dtype=torch.uint8, device=device) if receiver else None
    for off in range(0, maxn, step):
        n = min(step, maxn - off)
        valid = max(0, min(n, flat.numel() - off))
        if valid:
            send[:valid].copy_(flat[off:off + valid])
        if dst is None:
            dist.all_gather_into_tensor(recv[: world * n], send[:n])
        else:
            dist.gather(send[:n], [recv[r * n:(r + 1) * n] for r in range(world)] if receiver else None, dst=dst)
        if receiver:
            for r in range(world):
                take = max(0, min(n, metas[r][0] - off))
                if take:
                    dest[r][off:off + take].copy_(recv[r * n: r * n + take], non_blocking=pin)
    if not receiver:
        return {}
    if pin:
        torch.cuda.current_stream(device).synchronize()
    for r in range(world):
        out.update(_unflatten(dest[r], metas[r][1], copy=False))
    return out


def sharded_compress(weights: Dict[str, torch.Tensor], compress: Callable[[str, torch.Tensor], Dict[str, torch.Tensor]],
                     device=None) -> Dict[str, torch.Tensor]:
    """Compress ``weights`` (name -> tensor; every rank passes the same dict, tensors may live on
    the host) with ranks splitting the work, then all-gather: returns ``{f"{name}.{k}": t}`` for
    all weights on every rank."""
    world = dist.get_world_size() if dist.is_initialized() else 1
    rank = dist.get_rank() if dist.is_initialized() else 0
    plan = plan_shards([(k, v.numel() * v.element_size()) for k, v in weights.items()], world)
    local: Dict[str, torch.Tensor] = {}
    for name in plan[rank]:
        for k, t in compress(name, weights[name]).items():
            local[f"{name}.{k}"] = t
    return gather_state(local, device)
