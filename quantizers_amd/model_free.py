"""Data-free checkpoint quantization: safetensors in -> compressed-tensors safetensors out,
without instantiating the model (drop-in for ``llmcompressor.model_free_ptq`` as called at
scripts/quant_GLM-4.7-Flash-FP8.py:11-24: ``model_free_ptq(model_stub, save_directory,
scheme="FP8_BLOCK", ignore=[...], max_workers=16, device="cuda:0")``).

Every floating 2-D ``<module>.weight`` tensor whose module name is not matched by ``ignore``
is a quantization target (a checkpoint has no module types; the reference's ignore list names
the non-Linear 2-D tensors such as ``model.embed_tokens``).  Per shard file:

  disk --(reader threads, mmap)--> host --H2D (pinned staging)--> fused HIP quantize+pack (ops.compress_weights:
       the file's same-shape weights in one grouped launch) --async D2H, pinned--> host
       --(writer threads, after the copy event)--> disk

Reads of file i+1 and writes of file i-1 overlap the GPU work on file i.  Output shards keep
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
from .staging import H2DStager

log = logging.getLogger(__name__)

_FLOATS = (torch.bfloat16, torch.float16, torch.float32)


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


def _read(path: str) -> Dict[str, torch.Tensor]:
    out = {}
    with safe_open(path, framework="pt", device="cpu") as f:
        for k in f.keys():
            out[k] = f.get_tensor(k)
    return out


def _quantize_file(tensors: Dict[str, torch.Tensor], sch: QuantizationScheme, ignore: List[str], device,
                   quantized: List[str], skipped: List[str], copier=None, stager=None) -> Dict[str, torch.Tensor]:
    """One shard's output tensors.  Every target of the file goes to the device (through the
    pinned staging buffers of ``stager`` when given), then ONE
    ``ops.compress_weights`` call quantizes them (same-shape weights in one grouped launch);
    with ``copier`` the compressed tensors come back through pinned memory asynchronously (valid
    once the copier's last event completes)."""
    a = sch.weights
    out: Dict[str, torch.Tensor] = {}
    mods: List[str] = []
    ws: List[torch.Tensor] = []
    for name in sorted(tensors):
        t = tensors[name]
        if not is_target(name, tuple(t.shape), t.dtype, ignore):
            out[name] = t
            continue
        mod = name[: -len(".weight")]
        if t.dtype != torch.bfloat16:
            raise ValueError(f"{name}: weights must be bfloat16 for the GPU quantizer (got {t.dtype})")
        if not _divisible(t.shape, a):
            log.warning("model_free_ptq: %s %s not divisible by the scheme's groups/blocks; left unquantized (D13)",
                        name, tuple(t.shape))
            skipped.append(mod)
            out[name] = t
            continue
        mods.append(mod)
        ws.append(stager.copy(t) if stager is not None else t.to(device))
    if not ws:
        return out
    if stager is not None:
        stager.wait()  # the quantize launches (current stream) see the staged weights
    comps = ops.compress_weights(ws, a, has_activation_quant=sch.input_activations is not None)
    dev_out = {f"{mod}.{k}": v for mod, comp in zip(mods, comps) for k, v in comp.items()}
    if copier is not None:
        out.update(copier.submit(dev_out))
    else:
        out.update({k: (v.to("cpu") if v.is_cuda else v) for k, v in dev_out.items()})
    quantized.extend(mods)
    return out


def _write_shard(out: Dict[str, torch.Tensor], path: str, ready) -> None:
    if ready is not None:
        ready.synchronize()  # the shard's device->host copies have landed
    save_file({k: v.contiguous() for k, v in out.items()}, path, {"format": "pt"})


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
    with ThreadPoolExecutor(max_workers=max(2, max_workers)) as pool:
        reads = [pool.submit(_read, os.path.join(model_stub, f)) for f in mine[:2]]
        writes = []
        copier = _HostCopier(device)
        stager = H2DStager(device)
        for i, fn in enumerate(mine):
            tensors = reads[i].result()
            if i + 2 < len(mine):
                reads.append(pool.submit(_read, os.path.join(model_stub, mine[i + 2])))
            out = _quantize_file(tensors, sch, ignore, device, quantized, skipped, copier, stager)
            ready = copier.last_event
            for k, t in out.items():
                weight_map[k] = fn
                total += t.numel() * t.element_size()
            writes.append(pool.submit(_write_shard, out, os.path.join(save_directory, fn), ready))
            reads[i] = None
        for w in writes:
            w.result()
        copier.finish()
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
