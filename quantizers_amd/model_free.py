"""Data-free checkpoint quantization: safetensors in -> compressed-tensors safetensors out,
without instantiating the model (drop-in for ``llmcompressor.model_free_ptq`` as called at
scripts/quant_GLM-4.7-Flash-FP8.py:11-24: ``model_free_ptq(model_stub, save_directory,
scheme="FP8_BLOCK", ignore=[...], max_workers=16, device="cuda:0")``).

Every floating 2-D ``<module>.weight`` tensor whose module name is not matched by ``ignore``
is a quantization target (a checkpoint has no module types; the reference's ignore list names
the non-Linear 2-D tensors such as ``model.embed_tokens``).  Per shard file:

  disk --(max_workers reader threads: pread of each target's bytes into pinned slots, DMA per slot;
       staging.DiskStager)--> device --fused HIP quantize+pack (ops.compress_weights: the file's
       same-shape weights in one grouped launch)--> --async D2H, pinned--> host
       --(WRITE_THREADS writer threads, after the copy event)--> disk

The targets are chosen from each file's safetensors header alone; the other tensors (norms,
embeddings, ignored weights) are memory-mapped and read when the output shard is written.  The
reads of files i+1 .. i+LOOKAHEAD and the writes of earlier files overlap the GPU work on file i.  Output shards keep
the input file names; ``model.safetensors.index.json`` and ``config.json`` (with
``quantization_config``) are rewritten and every other file (tokenizer, generation config) is
copied.  Multi-GPU: under ``torch.distributed`` (one process per GPU), files are assigned to
ranks by size (LPT, ``distributed.plan_shards``); each rank writes its own files -- there is no
data-path collective -- and rank 0 writes the index and config from the gathered weight maps.

Decision D13: a target whose shape does not divide the group / block size is left unquantized
and listed under ``ignore`` (compressed-tensors would raise for a strict block layout).
Weights must be bf16 (the kernels' input type); other floating dtypes raise ``ValueError``.
"""
from __future__ import annotations

import argparse
import json
import logging
import os
import shutil
import time
from concurrent.futures import ThreadPoolExecutor
from typing import Dict, List, Optional, Union

import torch
import torch.distributed as dist
from safetensors import safe_open
from safetensors.torch import save_file

from . import ops
from .compressor import _HostCopier, quantization_config_for
from .distributed import plan_shards
from .quantization import QuantizationArgs, QuantizationScheme, preset_scheme
from .recipe import match_any
from .staging import DiskStager, safetensors_header

log = logging.getLogger(__name__)

_FLOATS = (torch.bfloat16, torch.float16, torch.float32)
LOOKAHEAD = 2  # files whose reads are queued ahead of the one being quantized
WRITE_THREADS = 4  # output shards written concurrently


def _scheme(scheme: Union[str, QuantizationScheme, dict]) -> QuantizationScheme:
    if isinstance(scheme, QuantizationScheme):
        return scheme
    if isinstance(scheme, str):
        return preset_scheme(scheme, ["Linear"])
    if isinstance(scheme, dict):  # {"weights": {...}, "targets": [...]} as in a recipe config group
        w = scheme.get("weights", scheme)
        return QuantizationScheme(targets=list(scheme.get("targets", ["Linear"])), weights=QuantizationArgs(**w))
    raise TypeError(f"scheme must be a preset name, QuantizationScheme or dict, got {type(scheme)}")


def _shard_files(model_dir: str) -> List[str]:
    idx = os.path.join(model_dir, "model.safetensors.index.json")
    if os.path.exists(idx):
        with open(idx) as f:
            return sorted(set(json.load(f)["weight_map"].values()))
    files = sorted(f for f in os.listdir(model_dir) if f.endswith(".safetensors"))
    if not files:
        raise ValueError(f"no safetensors files in {model_dir}")
    return files


def _divisible(shape, a: QuantizationArgs) -> bool:
    rows, cols = shape
    if a.strategy in ("group", "tensor_group"):
        return cols % a.group_size == 0
    if a.strategy == "block":
        bh, bw = a.block_structure
        return rows % bh == 0 and cols % bw == 0
    return True


def is_target(name: str, t_shape, t_dtype, ignore: List[str]) -> bool:
    if not name.endswith(".weight") or len(t_shape) != 2 or t_dtype not in _FLOATS:
        return False
    return not match_any(name[: -len(".weight")], "Linear", ignore)


# Phase record of the latest model_free_ptq call on this process (scripts/model_free_bench.py):
# host spans (read_wait / write: perf_counter start, end, bytes) and device spans (kernel / d2h:
# pairs of timing events, resolved to seconds when the call ends).
LAST_RUN: Dict[str, object] = {}


def _span(kind: str, t0: float, nbytes: int) -> None:
    spans = LAST_RUN.setdefault("host", [])
    spans.append((kind, t0, time.perf_counter(), nbytes))  # list.append is atomic under the GIL


def _read(path: str) -> Dict[str, torch.Tensor]:
    t0 = time.perf_counter()
    out = {}
    with safe_open(path, framework="pt", device="cpu") as f:
        for k in f.keys():
            out[k] = f.get_tensor(k)
    _span("read", t0, sum(t.numel() * t.element_size() for t in out.values()))
    return out


_DT_TAGS = {"BF16": torch.bfloat16, "F16": torch.float16, "F32": torch.float32}


def _select(meta, sch: QuantizationScheme, ignore: List[str]):
    """A file's tensors split by the header alone: (target names to quantize, their modules, D13
    skips).  A floating 2-D target that is not bf16 raises (the kernels read bf16)."""
    a = sch.weights
    targets, mods, skipped = [], [], []
    for name in sorted(meta):
        tag, shape, _ = meta[name]
        dt = _DT_TAGS.get(tag)
        if dt is None or not is_target(name, shape, dt, ignore):
            continue
        mod = name[: -len(".weight")]
        if dt != torch.bfloat16:
            raise ValueError(f"{name}: weights must be bfloat16 for the GPU quantizer (got {dt})")
        if not _divisible(shape, a):
            log.warning("model_free_ptq: %s %s not divisible by the scheme's groups/blocks; left unquantized (D13)",
                        name, tuple(shape))
            skipped.append(mod)
            continue
        targets.append(name)
        mods.append(mod)
    return targets, mods, skipped


def _rest(path: str, meta, targets: List[str]) -> Dict[str, torch.Tensor]:
    """The file's other tensors (norms, embeddings, ignored or skipped weights), unchanged: memory-
    mapped host tensors, read when the output shard is written."""
    keep = set(targets)
    out = {}
    with safe_open(path, framework="pt", device="cpu") as f:
        for k in meta:
            if k not in keep:
                out[k] = f.get_tensor(k)
    return out


def _quantize_file(ws: List[torch.Tensor], mods: List[str], sch: QuantizationScheme, device, copier=None
                   ) -> Dict[str, torch.Tensor]:
    """One shard's compressed tensors: ONE ``ops.compress_weights`` call over the file's device-
    resident targets (same-shape weights in one grouped launch); with ``copier`` they come back
    through pinned memory asynchronously (valid once the copier's last event completes)."""
    if not ws:
        return {}
    in_bytes = sum(w.numel() * 2 for w in ws)
    kern = _dev_pair(torch.cuda.current_stream(device))
    comps = ops.compress_weights(ws, sch.weights, has_activation_quant=sch.input_activations is not None)
    kern[1].record(torch.cuda.current_stream(device))
    dev_out = {f"{mod}.{k}": v for mod, comp in zip(mods, comps) for k, v in comp.items()}
    out_bytes = sum(v.numel() * v.element_size() for v in dev_out.values() if v.is_cuda)
    LAST_RUN.setdefault("dev", []).append(("kernel", kern, in_bytes + out_bytes))
    if copier is None:
        return {k: (v.to("cpu") if v.is_cuda else v) for k, v in dev_out.items()}
    d2h = _dev_pair(copier.stream, after=torch.cuda.current_stream(device))
    out = copier.submit(dev_out)
    d2h[1].record(copier.stream)
    LAST_RUN.setdefault("dev", []).append(("d2h", d2h, out_bytes))
    return out


def _dev_pair(stream, after=None):
    """A (start, end) pair of timing events; start recorded now on ``stream`` (behind ``after``'s
    work so far when given), end recorded by the caller."""
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    if after is not None:
        stream.wait_stream(after)
    e0.record(stream)
    return e0, e1


def _write_shard(out: Dict[str, torch.Tensor], path: str, ready) -> None:
    if ready is not None:
        ready.synchronize()  # the shard's device->host copies have landed
    t0 = time.perf_counter()
    save_file({k: v.contiguous() for k, v in out.items()}, path, {"format": "pt"})
    _span("write", t0, os.path.getsize(path))


def run_summary() -> Dict[str, Dict[str, float]]:
    """Per phase of the latest call: busy seconds (the sum of its spans), bytes, GB/s while busy;
    ``wall`` = the call's wall seconds.  Device phases are resolved from their events (the call
    has synchronised)."""
    res: Dict[str, Dict[str, float]] = {}
    for kind, t0, t1, nb in LAST_RUN.get("host", []):
        r = res.setdefault(kind, {"s": 0.0, "bytes": 0})
        r["s"] += t1 - t0
        r["bytes"] += nb
    for kind, (e0, e1), nb in LAST_RUN.get("dev", []):
        r = res.setdefault(kind, {"s": 0.0, "bytes": 0})
        r["s"] += e0.elapsed_time(e1) * 1e-3
        r["bytes"] += nb
    for r in res.values():
        r["GBps"] = r["bytes"] / r["s"] / 1e9 if r["s"] else 0.0
    res["wall"] = {"s": LAST_RUN.get("wall", 0.0)}
    return res


def model_free_ptq(model_stub: str, save_directory: str, scheme: Union[str, QuantizationScheme, dict] = "FP8_BLOCK",
                   ignore: Optional[List[str]] = None, max_workers: int = 4,
                   device: Union[str, torch.device, None] = None) -> str:
    """Quantize every targeted weight of the checkpoint at ``model_stub`` (a local directory:
    this build has no hub access) into ``save_directory``.  Returns ``save_directory``."""
    ignore = list(ignore or [])
    sch = _scheme(scheme)
    if sch.weights is None:
        raise ValueError("scheme has no weight quantization")
    world = dist.get_world_size() if dist.is_initialized() else 1
    rank = dist.get_rank() if dist.is_initialized() else 0
    LAST_RUN.clear()
    t_call = time.perf_counter()
    if device is None:
        device = torch.device("cuda", torch.cuda.current_device())
    device = torch.device(device)
    if device.type != "cuda":
        raise ValueError("model_free_ptq runs on a ROCm device (no CPU fallback)")
    if not os.path.isdir(model_stub):
        raise ValueError(f"model_stub must be a local checkpoint directory (no hub access): {model_stub}")
    os.makedirs(save_directory, exist_ok=True)
    files = _shard_files(model_stub)
    sizes = [(f, os.path.getsize(os.path.join(model_stub, f))) for f in files]
    mine = plan_shards(sizes, world)[rank]
    mine = [f for f in files if f in set(mine)]  # keep file order for the pipeline
    quantized: List[str] = []
    skipped: List[str] = []
    weight_map: Dict[str, str] = {}
    total = 0
    with ThreadPoolExecutor(max_workers=max(2, max_workers)) as pool, \
            ThreadPoolExecutor(max_workers=WRITE_THREADS) as wpool:
        stager = DiskStager(device, pool)
        copier = _HostCopier(device)

        def enqueue(fn):  # header, target selection, and the file's reads + DMAs queued on the pool
            path = os.path.join(model_stub, fn)
            hdr = safetensors_header(path)
            targets, mods, sk = _select(hdr[1], sch, ignore)
            return path, hdr, targets, mods, sk, stager.load(path, targets, hdr)

        pending = []
        writes = []
        try:
            for f in mine[:LOOKAHEAD]:
                pending.append(enqueue(f))
            for i, fn in enumerate(mine):
                path, hdr, targets, mods, sk, fl = pending[i]
                pending[i] = None
                if i + LOOKAHEAD < len(mine):
                    pending.append(enqueue(mine[i + LOOKAHEAD]))
                t_wait = time.perf_counter()
                dev = stager.wait(fl)  # the quantize launches (current stream) see the loaded weights
                _span("read_wait", t_wait, fl.nbytes)  # the main thread blocked on this file's reads + DMAs
                out = _rest(path, hdr[1], targets)
                out.update(_quantize_file([dev[n] for n in targets], mods, sch, device, copier))
                del dev, fl
                quantized.extend(mods)
                skipped.extend(sk)
                ready = copier.last_event
                for k, t in out.items():
                    weight_map[k] = fn
                    total += t.numel() * t.element_size()
                writes.append(wpool.submit(_write_shard, out, os.path.join(save_directory, fn), ready))
            for w in writes:
                w.result()
        finally:  # on an error: the files queued ahead are closed once their reads can no longer run
            for p in pending:
                if p is not None:
                    stager.release(p[5])
        copier.finish()
    torch.cuda.synchronize(device)
    LAST_RUN["wall"] = time.perf_counter() - t_call
    state = (weight_map, total, quantized, skipped)
    if world > 1:
        allst = [None] * world
        dist.all_gather_object(allst, state)
    else:
        allst = [state]
    if rank == 0:
        wm, tot, q, sk = {}, 0, [], []
        for s in allst:
            wm.update(s[0])
            tot += s[1]
            q += s[2]
            sk += s[3]
        _write_metadata(model_stub, save_directory, sch, wm, tot, sorted(q), sorted(set(ignore) | set(sk)), files)
    if world > 1:
        dist.barrier()
    return save_directory


def _write_metadata(src: str, dst: str, sch: QuantizationScheme, weight_map, total, quantized, ignore, files):
    for f in os.listdir(src):
        p = os.path.join(src, f)
        if f in files or f in ("config.json", "model.safetensors.index.json") or not os.path.isfile(p):
            continue
        shutil.copy2(p, os.path.join(dst, f))
    if len(files) > 1 or os.path.exists(os.path.join(src, "model.safetensors.index.json")):
        with open(os.path.join(dst, "model.safetensors.index.json"), "w") as f:
            json.dump({"metadata": {"total_size": total}, "weight_map": dict(sorted(weight_map.items()))}, f, indent=2)
    cfg_path = os.path.join(src, "config.json")
    cfg = json.load(open(cfg_path)) if os.path.exists(cfg_path) else {}
    smap = {n: sch for n in quantized}
    qc = quantization_config_for(smap, [])
    qc["ignore"] = list(ignore)  # the caller's ignore entries + D13 skips (no module types here)
    cfg["quantization_config"] = qc
    with open(os.path.join(dst, "config.json"), "w") as f:
        json.dump(cfg, f, indent=2)


def main(argv=None):
    p = argparse.ArgumentParser(description="data-free quantization of a safetensors checkpoint on MI355X")
    p.add_argument("model", help="local checkpoint directory")
    p.add_argument("output", help="output directory")
    p.add_argument("--scheme", default="FP8_BLOCK")
    p.add_argument("--ignore", nargs="*", default=["lm_head"])
    p.add_argument("--max-workers", type=int, default=4)
    p.add_argument("--device", default=None)
    a = p.parse_args(argv)
    logging.basicConfig(level=logging.INFO)
    if "WORLD_SIZE" in os.environ and int(os.environ["WORLD_SIZE"]) > 1 and not dist.is_initialized():
        local = int(os.environ.get("LOCAL_RANK", "0"))
        torch.cuda.set_device(local)
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    model_free_ptq(a.model, a.output, a.scheme, a.ignore, a.max_workers, a.device)
    if dist.is_initialized():
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
