"""Multi-GPU weight quantization: one process per GPU, weights sharded across ranks, results
reassembled with one RCCL all-gather over xGMI (BASELINE.json configs[4]).

The reference is single-process (its only parallelism is model_free_ptq's file thread pool,
scripts/quant_GLM-4.7-Flash-FP8.py:22).  Quantize+pack has no cross-weight dependency, so:

* ``plan_shards`` assigns whole weights (or whole fused-expert groups) to ranks by bytes,
  longest-processing-time first (deterministic: every rank computes the same plan);
* each rank compresses its share with the fused HIP kernel -- no collective on the data path;
* ``gather_state`` flattens each rank's compressed tensors into one byte buffer and runs ONE
  ``all_gather_into_tensor`` (padded to the largest shard; xGMI is point-to-point, so a single
  large collective beats many small ones), then every rank unflattens the full state dict.

Works with backend "nccl" (RCCL, GPU tensors) and "gloo" (CPU tensors, used by the CPU tests).
"""
from __future__ import annotations

import heapq
from typing import Callable, Dict, List, Sequence, Tuple

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


def _flatten(tensors: Dict[str, torch.Tensor], device) -> Tuple[torch.Tensor, List[Tuple[str, str, Tuple[int, ...], int]]]:
    meta = []
    parts = []
    off = 0
    for k in sorted(tensors):
        t = tensors[k].contiguous()
        b = t.view(torch.uint8).reshape(-1) if t.numel() else torch.empty(0, dtype=torch.uint8, device=t.device)
        meta.append((k, str(t.dtype).replace("torch.", ""), tuple(t.shape), off))
        parts.append(b.to(device))
        off += b.numel()
        pad = (-off) % 16  # keep every tensor 16-B aligned inside the buffer (view(dtype))
        if pad:
            parts.append(torch.zeros(pad, dtype=torch.uint8, device=device))
            off += pad
    flat = torch.cat(parts) if parts else torch.empty(0, dtype=torch.uint8, device=device)
    return flat, meta


def _unflatten(flat: torch.Tensor, meta) -> Dict[str, torch.Tensor]:
    out = {}
    for k, dt, shape, off in meta:
        dtype = getattr(torch, dt)
        n = int(torch.tensor(shape).prod().item()) if shape else 1
        nb = n * torch.empty((), dtype=dtype).element_size()
        out[k] = flat[off:off + nb].view(dtype).reshape(shape).clone()
    return out


def gather_state(local: Dict[str, torch.Tensor], device=None) -> Dict[str, torch.Tensor]:
    """All ranks get the union of every rank's tensors (one all_gather_into_tensor)."""
    if not dist.is_initialized() or dist.get_world_size() == 1:
        return dict(local)
    world = dist.get_world_size()
    if device is None:
        device = torch.device("cuda", torch.cuda.current_device()) if dist.get_backend() == "nccl" else torch.device("cpu")
    flat, meta = _flatten(local, device)
    metas: List = [None] * world
    dist.all_gather_object(metas, (flat.numel(), meta))
    maxn = max(m[0] for m in metas)
    buf = torch.zeros(maxn, dtype=torch.uint8, device=device)
    buf[: flat.numel()] = flat
    allbuf = torch.empty(world * maxn, dtype=torch.uint8, device=device)
    dist.all_gather_into_tensor(allbuf, buf)
    out: Dict[str, torch.Tensor] = {}
    for r in range(world):
        n, m = metas[r]
        out.update(_unflatten(allbuf[r * maxn: r * maxn + n], m))
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
