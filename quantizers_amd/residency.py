"""Multi-rank residency: ONE host copy of the model, layers broadcast over RCCL (BASELINE.json
configs[4], MiniMax-M2.1: ~460 GB of bf16 weights, which eight per-rank host copies could not
hold; the reference loads exactly one, scripts/do_oneshot.py:86-94).

Under torch.distributed, rank 0 holds the loaded model and every other rank a meta-device
skeleton of the same architecture (``cli.load_model``).  ``Residency`` then:

* materialises the non-layer tensors (embeddings, final norm, lm_head, rotary buffers) on every
  rank's device by one broadcast from rank 0;
* as the layer-sequential pass reaches decoder layer i, broadcasts that layer's tensors from
  rank 0 (one flat byte buffer per layer: a single large collective over xGMI) -- every rank then
  runs the layer's AWQ search with the grid split over the ranks, as before;
* after the layer, each rank keeps on its device only the tensors of the checkpoint shards it
  will write (``compressor.save_plan``: the same plan ``save_compressed`` follows) and turns the
  rest back into meta tensors.  Rank 0 keeps the whole model (returned to its host when it does
  not fit the device), so the returned model stays complete there.

Host memory: one model (rank 0).  Device memory per rank: its 1/N share of the checkpoint plus
one layer, and during the pass the non-layer tensors (embeddings, lm_head -- one copy when tied --,
final norm), which ``release_outside`` returns to meta on the ranks that do not write them.  Nothing of the compressed result crosses xGMI afterwards: each rank compresses and
writes its own shards."""
from __future__ import annotations

from typing import Dict, Iterable, List, Optional, Set, Tuple

import torch
import torch.distributed as dist
from torch import nn

Slot = Tuple[nn.Module, bool, str]  # (module, is a buffer, attribute name)


def _world() -> Tuple[int, int]:
    if dist.is_available() and dist.is_initialized():
        return dist.get_world_size(), dist.get_rank()
    return 1, 0


def slots(module: nn.Module, exclude: Optional[nn.Module] = None) -> List[Slot]:
    """Every parameter / buffer slot under ``module`` in a deterministic order (the same on every
    rank for the same architecture), skipping the sub-tree ``exclude``."""
    skip = {id(m) for m in exclude.modules()} if exclude is not None else set()
    out: List[Slot] = []
    for _, m in module.named_modules():
        if id(m) in skip:
            continue
        for name, p in m._parameters.items():
            if p is not None:
                out.append((m, False, name))
        for name, b in m._buffers.items():
            if b is not None:
                out.append((m, True, name))
    return out


def _get(s: Slot) -> torch.Tensor:
    m, is_buf, name = s
    return (m._buffers if is_buf else m._parameters)[name]


def _set(s: Slot, t: torch.Tensor) -> None:
    m, is_buf, name = s
    if is_buf:
        m._buffers[name] = t
    else:
        p = m._parameters[name]
        if p.is_meta or t.is_meta or p.device != t.device:
            m._parameters[name] = nn.Parameter(t, requires_grad=p.requires_grad)
        else:
            p.data = t


def skeleton_mode(model: nn.Module) -> bool:
    """Collective (under torch.distributed): True when some rank holds a meta skeleton of the
    model.  Rank 0 must then hold the weights; a mix of complete models on several ranks is the
    replicated mode (every rank loaded the model) and stays as it was."""
    world, rank = _world()
    if world == 1:
        return False
    has_meta = any(t.is_meta for t in list(model.parameters()) + list(model.buffers()))
    flags: List = [None] * world
    dist.all_gather_object(flags, has_meta)
    if not any(flags):
        return False
    if flags[0]:
        raise ValueError("rank 0 must hold the model's weights (the other ranks may hold a meta skeleton)")
    return True


def _broadcast(flat: torch.Tensor, src: int) -> None:
    if dist.get_backend() == "gloo" and flat.is_cuda:  # gloo rehearsal: through the host
        h = flat.cpu()
        dist.broadcast(h, src)
        flat.copy_(h)
    else:
        dist.broadcast(flat, src)


def _alias_groups(ss: List[Slot]) -> List[int]:
    """For each slot, the index of the first slot holding the SAME tensor object (tied weights,
    e.g. lm_head.weight is embed_tokens.weight under tie_word_embeddings)."""
    first: Dict[int, int] = {}
    return [first.setdefault(id(_get(s)), i) for i, s in enumerate(ss)]


def broadcast_slots(ss: List[Slot], device, src: int = 0) -> None:
    """Make the tensors of ``ss`` valid on every rank's ``device``: rank ``src`` provides them
    (already on ``device``), the others receive ONE flat byte buffer and take views of it.  A
    tensor held by several slots (tied weights) travels once, and every slot that holds it on
    ``src`` holds one shared tensor on the other ranks too (``src``'s alias structure is sent
    along), so ties survive on every rank and no rank's checkpoint gains an untied copy."""
    world, rank = _world()
    if world == 1:  # no other rank to send to: src's tensors are already in place
        return
    alias = _alias_groups(ss) if rank == src else None
    if world > 1:
        box = [alias]
        dist.broadcast_object_list(box, src)
        alias = box[0]
    if len(alias) != len(ss):
        raise ValueError(f"broadcast_slots: rank {rank} has {len(ss)} slots, rank {src} {len(alias)}")
    lay, off = {}, 0
    for i, s in enumerate(ss):
        if alias[i] != i:
            continue
        t = _get(s)
        nb = t.numel() * t.element_size()
        lay[i] = (off, nb, t.shape, t.dtype)
        off += (nb + 255) // 256 * 256
    if off == 0:
        return
    flat = torch.empty(off, dtype=torch.uint8, device=device)
    if rank == src:
        for i, (o, nb, _, _) in lay.items():
            if nb:
                flat[o:o + nb].copy_(_get(ss[i]).detach().contiguous().reshape(-1).view(torch.uint8))
    _broadcast(flat, src)
    if rank != src:
        for i, s in enumerate(ss):
            if alias[i] == i:
                o, nb, shape, dtype = lay[i]
                _set(s, flat[o:o + nb].view(dtype).view(shape))
            else:  # tied: the very object the first holder now has
                m, is_buf, name = s
                (m._buffers if is_buf else m._parameters)[name] = _get(ss[alias[i]])


class Residency:
    """Owner-keeps bookkeeping for one oneshot pass (see the module docstring)."""

    def __init__(self, model: nn.Module, device, max_shard_bytes: int):
        from .compressor import compression_units, save_plan
        from .model import checkpoint_name, model_type
        self.world, self.rank = _world()
        self.device = torch.device(device)
        units, raw = compression_units(model)
        plan = save_plan(units, raw, self.world, max_shard_bytes)
        mtype = model_type(model)
        by_name: Dict[str, Slot] = {}
        for name, _ in model.named_parameters():
            mod, _, leaf = name.rpartition(".")
            by_name[checkpoint_name(name, mtype)] = (model.get_submodule(mod) if mod else model, False, leaf)
        for name, _ in model.named_buffers():
            mod, _, leaf = name.rpartition(".")
            by_name.setdefault(checkpoint_name(name, mtype), (model.get_submodule(mod) if mod else model, True, leaf))
        keep: Set[Tuple[int, bool, str]] = set()
        for i in plan.units_of[self.rank]:
            for r in units[i].refs:
                keep.add((id(r.module), False, r.param_name))
        for n in plan.raw_of[self.rank]:
            s = by_name.get(n)
            if s is None:  # an unquantized slice of a fused expert parameter: "<expert>.<proj>.weight"
                s = self._fused_slot(model, n)
            if s is not None:
                keep.add((id(s[0]), s[1], s[2]))
        self.keep = keep
        self.max_shard_bytes = max_shard_bytes

    @staticmethod
    def _fused_slot(model: nn.Module, name: str) -> Optional[Slot]:
        from .model import iter_linears
        for r in iter_linears(model):
            if r.index is not None and f"{r.name}.weight" == name:
                return (r.module, False, r.param_name)
        return None

    def owns(self, s: Slot) -> bool:
        return self.rank == 0 or (id(s[0]), s[1], s[2]) in self.keep

    def materialise_outside(self, model: nn.Module, layers: nn.ModuleList) -> None:
        """Non-layer tensors on every rank's device (rank 0 moves its own there first)."""
        ss = slots(model, exclude=layers)
        if self.rank == 0:
            # id(host tensor) -> (that tensor, kept alive so its id stays unique; its device copy)
            moved: Dict[int, Tuple[torch.Tensor, torch.Tensor]] = {}
            for s in ss:
                t = _get(s)
                if id(t) in moved:  # a tied slot (lm_head under tie_word_embeddings): the SAME new object
                    m, is_buf, name = s
                    (m._buffers if is_buf else m._parameters)[name] = moved[id(t)][1]
                elif t.device != self.device:
                    _set(s, t.detach().to(self.device))
                    moved[id(t)] = (t, _get(s))
        broadcast_slots(ss, self.device)

    def release_outside(self, model: nn.Module, layers: nn.ModuleList) -> None:
        """After the pass: ranks other than 0 return the non-layer tensors they will not write to
        meta (a tensor held by several slots stays when any of its slots is owned), so a helper
        rank ends holding only its 1/N share of the checkpoint."""
        if self.rank == 0:
            return
        ss = slots(model, exclude=layers)
        alias = _alias_groups(ss)
        owned = {alias[i] for i, s in enumerate(ss) if self.owns(s)}
        for i, s in enumerate(ss):
            if alias[i] in owned:
                continue
            t = _get(s)
            if alias[i] == i:
                _set(s, torch.empty(t.shape, dtype=t.dtype, device="meta"))
            else:
                m, is_buf, name = s
                (m._buffers if is_buf else m._parameters)[name] = _get(ss[alias[i]])

    def fetch(self, layer: nn.Module, onload) -> Optional[Dict]:
        """Layer i on every rank's device: rank 0 onloads it (``onload(layer)`` -> the host tensors
        to return it to, or None when it is device-resident), then one broadcast."""
        host = None
        if self.rank == 0 and any(_get(s).device != self.device for s in slots(layer)):
            host = onload(layer)
        broadcast_slots(slots(layer), self.device)
        return host

    def release(self, layer: nn.Module) -> None:
        """After layer i: ranks other than 0 keep (as their own device tensors) only what they
        will write, the rest becomes meta again."""
        if self.rank == 0:
            return
        for s in slots(layer):
            t = _get(s)
            if self.owns(s):
                _set(s, t.detach().clone())
            else:
                _set(s, torch.empty(t.shape, dtype=t.dtype, device="meta"))

    def distribute(self, model: nn.Module, layers: Iterable[nn.Module], onload, offload) -> None:
        """No calibration pass (RTN recipes): every layer still travels once, so each rank ends
        with the tensors it will write."""
        for layer in layers:
            host = self.fetch(layer, onload)
            self.release(layer)
            if host is not None:
                offload(layer, host)
