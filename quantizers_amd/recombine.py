"""Recombine an FP8 (block-scaled) source checkpoint with a compressed-tensors checkpoint of its
MoE experts into one mixed-precision checkpoint (the reference does this
for MiniMax-M2.1 in scripts/recombine_weights_MiniMax-M2.1.py).

Why it exists: the quantizer works from bf16 weights, so an FP8 release is upcast, its experts
are AWQ-smoothed + int4-quantized, and the result is merged back into the original FP8 file set:

* FP8 tensors stay as they are; a projection's ``*_proj.weight_scale_inv`` (the FP8 block scale
  of DeepSeek-style checkpoints) is renamed ``*_proj.weight_scale`` (compressed-tensors name), and
  every other ``*_scale_inv`` is dropped (recombine...py:270-277);
* every expert weight matching ``expert_pattern`` is replaced by ALL the compressed tensors of that
  module present in the compressed checkpoint (``weight_packed``, ``weight_scale``,
  ``weight_shape``, ``weight_zero_point``, ``weight_g_idx``; recombine...py:56-67, 278-283);
* the smoothing layers (``post_attention_layernorm.weight``; the norms AWQ rescaled in front of the
  experts) come from the compressed checkpoint when present (recombine...py:284-291);
* ``config.json`` = the FP8 source config with a ``mixed-precision`` ``quantization_config``:
  group_0 = FP8 block 128x128 weights (+ dynamic per-token FP8 activations) for ``Linear``,
  group_1 = the compressed checkpoint's expert scheme (recombine...py:71-137); ``ignore`` is the
  compressed checkpoint's.

This is pure tensor surgery (no arithmetic); it runs on the CPU through safetensors, streaming one
source file at a time with the compressed files opened lazily (memory-mapped).
"""
from __future__ import annotations

import argparse
import json
import os
import re
import shutil
from dataclasses import dataclass, field
from typing import Dict, List, Optional

import torch
from safetensors import safe_open
from safetensors.torch import save_file

EXPERT_PATTERN = r".*block_sparse_moe\.experts\.\d+\.(w1|w2|w3)\.weight$"
SMOOTHING_PATTERN = r".*post_attention_layernorm\.weight$"
COMPRESSED_SUFFIXES = ("weight_packed", "weight_scale", "weight_shape", "weight_zero_point", "weight_g_idx")


@dataclass
class RecombineStats:
    experts_replaced: int = 0
    smoothing_replaced: int = 0
    scale_inv_renamed: int = 0
    scale_inv_dropped: int = 0
    tensors: int = 0
    bytes: int = 0
    missing_experts: List[str] = field(default_factory=list)


def _natural(s: str):
    return [int(t) if i & 1 else t.casefold() for i, t in enumerate(re.split(r"(\d+)", s))]


class _Lazy:
    """name -> tensor over a compressed checkpoint, files opened on first use."""

    def __init__(self, path: str):
        self.path = path
        idx = os.path.join(path, "model.safetensors.index.json")
        if os.path.exists(idx):
            self.where = json.load(open(idx))["weight_map"]
        else:
            self.where = {}
            for fn in sorted(f for f in os.listdir(path) if f.endswith(".safetensors")):
                with safe_open(os.path.join(path, fn), framework="pt") as f:
                    for k in f.keys():
                        self.where[k] = fn
        self.handles: Dict[str, object] = {}

    def get(self, name: str) -> Optional[torch.Tensor]:
        fn = self.where.get(name)
        if fn is None:
            return None
        h = self.handles.get(fn)
        if h is None:
            h = safe_open(os.path.join(self.path, fn), framework="pt")
            self.handles[fn] = h
        return h.get_tensor(name)


def mixed_precision_config(fp8_cfg: dict, compressed_cfg: dict) -> dict:
    cq = compressed_cfg.get("quantization_config", {})
    groups = {"group_0": {
        "targets": ["Linear"],
        "weights": {"type": "float", "num_bits": 8, "strategy": "block", "block_structure": [128, 128],
                    "symmetric": True, "dynamic": False},
        "input_activations": {"type": "float", "num_bits": 8, "strategy": "token", "symmetric": True,
                              "dynamic": True},
        "format": "float-quantized"}}
    for i, g in enumerate(cq.get("config_groups", {}).values()):
        g = dict(g)
        g["targets"] = ["Linear"] + [t for t in g.get("targets", []) if t != "Linear"]
        groups[f"group_{i + 1}"] = g
    out = dict(fp8_cfg)
    out["quantization_config"] = {
        "quant_method": "compressed-tensors", "format": "mixed-precision", "quantization_status": "compressed",
        "config_groups": groups, "ignore": cq.get("ignore", []), "kv_cache_scheme": None,
        "global_compression_ratio": None, "sparsity_config": {}, "transform_config": {},
        "version": cq.get("version", "0.13.1.dev0+quantizers_amd")}
    return out


def output_file_name(fp8_file: str) -> str:
    """Output shard name of a source shard, as the reference names them
    (recombine_weights_MiniMax-M2.1.py:68-72, specialised for MiniMax-M2.1: ``...-of-00130``
    becomes ``...-of-00125``); other names are kept."""
    return fp8_file.replace("00130", "00125")


def recombine(fp8_path: str, compressed_path: str, output_path: str, expert_pattern: str = EXPERT_PATTERN,
              smoothing_pattern: str = SMOOTHING_PATTERN, dry_run: bool = False) -> RecombineStats:
    st = RecombineStats()
    with open(os.path.join(fp8_path, "model.safetensors.index.json")) as f:
        src_map = json.load(f)["weight_map"]
    comp = _Lazy(compressed_path)
    files = sorted(set(src_map.values()), key=_natural)
    ex_rx, sm_rx = re.compile(expert_pattern), re.compile(smoothing_pattern)
    if not dry_run:
        os.makedirs(output_path, exist_ok=True)
    weight_map: Dict[str, str] = {}
    for fn in files:
        merged: Dict[str, torch.Tensor] = {}
        with safe_open(os.path.join(fp8_path, fn), framework="pt") as f:
            for name in f.keys():
                if name.endswith("_proj.weight_scale_inv"):
                    merged[name.replace("weight_scale_inv", "weight_scale")] = f.get_tensor(name)
                    st.scale_inv_renamed += 1
                elif name.endswith("_scale_inv"):
                    st.scale_inv_dropped += 1
                elif ex_rx.match(name):
                    base = name[: -len(".weight")]
                    got = {f"{base}.{s}": comp.get(f"{base}.{s}") for s in COMPRESSED_SUFFIXES}
                    got = {k: v for k, v in got.items() if v is not None}
                    if got:
                        merged.update(got)
                        st.experts_replaced += 1
                    else:  # reference drops the tensor silently; we record it
                        st.missing_experts.append(base)
                elif sm_rx.match(name):
                    t = comp.get(name)
                    merged[name] = t if t is not None else f.get_tensor(name)
                    st.smoothing_replaced += t is not None
                else:
                    merged[name] = f.get_tensor(name)
        st.tensors += len(merged)
        st.bytes += sum(t.numel() * t.element_size() for t in merged.values())
        out_fn = output_file_name(fn)
        for k in merged:
            weight_map[k] = out_fn
        if not dry_run:
            save_file({k: v.contiguous() for k, v in merged.items()}, os.path.join(output_path, out_fn),
                      metadata={"format": "pt"})
    if not dry_run:
        with open(os.path.join(output_path, "model.safetensors.index.json"), "w") as f:
            json.dump({"metadata": {"total_size": st.bytes, "format": "pt"}, "weight_map": weight_map}, f, indent=2)
        cfg = mixed_precision_config(json.load(open(os.path.join(fp8_path, "config.json"))),
                                     json.load(open(os.path.join(compressed_path, "config.json"))))
        with open(os.path.join(output_path, "config.json"), "w") as f:
            json.dump(cfg, f, indent=2)
        for extra in os.listdir(fp8_path):  # tokenizer, generation config, remote code
            p = os.path.join(fp8_path, extra)
            if os.path.isfile(p) and not extra.endswith(".safetensors") and extra not in (
                    "config.json", "model.safetensors.index.json"):
                shutil.copy2(p, os.path.join(output_path, extra))
    return st


def main(argv=None):
    p = argparse.ArgumentParser(description="merge an FP8 checkpoint with compressed-tensors experts")
    p.add_argument("--fp8-path", required=True)
    p.add_argument("--compressed-path", required=True)
    p.add_argument("--output-path", required=True)
    p.add_argument("--dry-run", action="store_true")
    a = p.parse_args(argv)
    st = recombine(a.fp8_path, a.compressed_path, a.output_path, dry_run=a.dry_run)
    print(json.dumps({k: (v if not isinstance(v, list) else len(v)) for k, v in st.__dict__.items()}))


if __name__ == "__main__":
    main()
