"""compressed-tensors checkpoint writer / reader.

Replaces ``model.save_pretrained(output_dir, save_compressed=True)`` (scripts/do_oneshot.py:197):
every targeted weight is quantized + packed on the GPU by the fused kernel (ops.compress_weight;
fused-expert slices of one parameter in a single batched launch) and written under the
compressed-tensors names the reference itself pins in
scripts/recombine_weights_MiniMax-M2.1.py:54-65 (``weight_packed``, ``weight_scale``,
``weight_shape``, ``weight_zero_point``; ``weight`` for float-quantized; plus
``weight_global_scale`` for NVFP4), with ``config.json.quantization_config`` laid out as in
scripts/recombine_weights_MiniMax-M2.1.py:82-134.  MoE experts are written per expert
(``...experts.<e>.<proj>``), the layout of the transformers version the reference pins.
"""
from __future__ import annotations

import json
import os
from typing import Dict, List, Optional

import torch
from safetensors.torch import load_file, save_file
from torch import nn

from . import ops
from .model import batch_groups, checkpoint_name, iter_linears, model_type, stacked_view
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


@torch.no_grad()
def compressed_state_dict(model: nn.Module, device=None) -> Dict[str, torch.Tensor]:
    """All tensors to write: compressed targeted weights + untouched parameters/buffers."""
    scheme_map: Dict[str, QuantizationScheme] = getattr(model, "quantization_scheme_map", {})
    device = torch.device(device) if device is not None else torch.device("cuda", torch.cuda.current_device())
    refs = iter_linears(model)
    out: Dict[str, torch.Tensor] = {}
    replaced_params = set()  # id() of parameters whose content is written per module
    for group in batch_groups(refs):
        r0 = group[0]
        p = getattr(r0.module, r0.param_name)
        if r0.index is not None:
            replaced_params.add(id(p))
        q = [g for g in group if g.name in scheme_map]
        if not q:
            if r0.index is not None:  # unquantized fused expert slices: per-expert `.weight`
                for g in group:
                    out[f"{g.name}.weight"] = g.weight.detach().to("cpu").clone()
            continue
        if len(q) != len(group):  # mixed targets inside one fused group: compress one by one
            subgroups = [[g] for g in group]
        else:
            subgroups = [group]
        for sg in subgroups:
            if sg[0].name not in scheme_map:
                for g in sg:
                    out[f"{g.name}.weight"] = g.weight.detach().to("cpu").clone()
                continue
            sch = scheme_map[sg[0].name]
            w = stacked_view(sg).to(device)
            if r0.index is None:
                w = w[0]
            comp = ops.compress_weight(w, sch.weights, has_activation_quant=sch.input_activations is not None)
            for i, g in enumerate(sg):
                for k, v in comp.items():
                    if k == "weight_shape":
                        out[f"{g.name}.{k}"] = v.clone()
                    elif w.dim() == 3:
                        out[f"{g.name}.{k}"] = v[i].detach().to("cpu").clone().reshape(
                            v.shape[1:] if v.dim() > 1 else (1,))
                    else:
                        out[f"{g.name}.{k}"] = v.detach().to("cpu").clone()
                if r0.index is None and g.bias is not None:
                    out[f"{g.name}.bias"] = g.bias.detach().to("cpu").clone()
    mtype = model_type(model)
    quant_linears = {g.name for g in refs if g.name in scheme_map and g.index is None}
    for name, prm in model.named_parameters():
        if id(prm) in replaced_params:
            continue
        cname = checkpoint_name(name, mtype)
        mod_name, _, leaf = cname.rpartition(".")
        if mod_name in quant_linears and leaf in ("weight", "bias"):
            continue
        if cname not in out:
            out[cname] = prm.detach().to("cpu").clone()
    for name, buf in model.named_buffers():
        cname = checkpoint_name(name, mtype)
        if cname not in out and not name.endswith("inv_freq"):
            out[cname] = buf.detach().to("cpu").clone()
    return out


def save_compressed(model: nn.Module, output_dir: str, max_shard_bytes: int = SHARD_BYTES, device=None) -> str:
    """Write safetensors shards + index + config.json(quantization_config)."""
    os.makedirs(output_dir, exist_ok=True)
    sd = compressed_state_dict(model, device)
    names = sorted(sd)
    shards: List[Dict[str, torch.Tensor]] = [{}]
    size = 0
    for n in names:
        nb = sd[n].numel() * sd[n].element_size()
        if shards[-1] and size + nb > max_shard_bytes:
            shards.append({})
            size = 0
        shards[-1][n] = sd[n].contiguous()
        size += nb
    meta = {"format": "pt"}
    if len(shards) == 1:
        save_file(shards[0], os.path.join(output_dir, "model.safetensors"), metadata=meta)
    else:
        wmap = {}
        total = 0
        for i, sh in enumerate(shards):
            fn = f"model-{i + 1:05d}-of-{len(shards):05d}.safetensors"
            save_file(sh, os.path.join(output_dir, fn), metadata=meta)
            for n, t in sh.items():
                wmap[n] = fn
                total += t.numel() * t.element_size()
        with open(os.path.join(output_dir, "model.safetensors.index.json"), "w") as f:
            json.dump({"metadata": {"total_size": total}, "weight_map": wmap}, f, indent=2)
    cfg = model.config.to_dict() if hasattr(model, "config") else {}
    cfg["quantization_config"] = quantization_config(model)
    with open(os.path.join(output_dir, "config.json"), "w") as f:
        json.dump(cfg, f, indent=2, default=str)
    _write_recipe(getattr(model, "quantization_recipe", None), output_dir)
    return output_dir


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
