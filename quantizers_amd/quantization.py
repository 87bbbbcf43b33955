"""Host-side mirror of compressed-tensors' quantization configuration objects.

The reference's recipes (configs/recipes/*.yaml) are parsed by [3P] llmcompressor into
compressed-tensors ``QuantizationArgs`` / ``QuantizationScheme`` objects; this module provides
the same names, fields, defaults and validation errors so a recipe written for the reference
configures this framework identically.  Only the weight side drives
the GPU path; activation args are carried through to the saved ``quantization_config``.
"""
from __future__ import annotations

import copy
from dataclasses import dataclass, field, asdict
from typing import Any, Dict, List, Optional

from . import _lib

STRATEGIES = ("tensor", "channel", "group", "block", "token", "tensor_group")


@dataclass
class QuantizationArgs:
    """compressed-tensors ``QuantizationArgs`` (fields used in recipe_awq_w4a16.yaml:16-24 etc.)."""

    num_bits: int = 8
    type: str = "int"
    symmetric: bool = True
    group_size: Optional[int] = None
    strategy: Optional[str] = None
    block_structure: Optional[List[int]] = None
    dynamic: Any = False
    actorder: Optional[str] = None
    observer: Optional[str] = None
    observer_kwargs: Dict[str, Any] = field(default_factory=dict)
    scale_dtype: Optional[str] = None  # None | "float8_e4m3fn" (NVFP4) | "uint8" (MX E8M0)
    zp_dtype: Optional[str] = None

    def __post_init__(self):
        self.type = str(self.type).lower()
        if self.type not in ("int", "float"):
            raise ValueError(f"invalid quantization type {self.type}")
        if self.strategy is not None:
            self.strategy = str(self.strategy).lower()
            if self.strategy not in STRATEGIES:
                raise ValueError(f"invalid strategy {self.strategy}")
        if isinstance(self.block_structure, str):  # "128x128"
            self.block_structure = [int(x) for x in self.block_structure.lower().split("x")]
        # strategy inference (compressed-tensors validate_model_after)
        if self.strategy is None:
            if self.block_structure is not None:
                self.strategy = "block"
            elif self.group_size is not None:
                self.strategy = "channel" if self.group_size == -1 else "group"
            else:
                self.strategy = "tensor"
        if self.strategy in ("group", "tensor_group"):
            if self.group_size is None or self.group_size <= 0:
                raise ValueError(f"strategy {self.strategy} requires group_size > 0")
        if self.strategy == "block":
            if not self.block_structure or len(self.block_structure) != 2:
                raise ValueError("block strategy requires block_structure [h, w]")
        if self.type == "float":
            if self.num_bits not in (4, 8):
                raise ValueError("float quantization supports num_bits 4 (e2m1) or 8 (e4m3)")
            if not self.symmetric:
                raise ValueError("Asymmetric Quantization is not supported for float types")
        elif not (1 <= self.num_bits <= 8):
            raise ValueError("int quantization supports num_bits <= 8")
        if self.observer is None and not self.dynamic:
            self.observer = "minmax"

    # ------------------------------------------------------------------ predicates
    @property
    def is_mx(self) -> bool:
        return self.type == "float" and self.num_bits == 4 and self.scale_dtype in ("uint8", "e8m0")

    @property
    def is_nvfp4(self) -> bool:
        return self.type == "float" and self.num_bits == 4 and self.strategy == "tensor_group"

    def to_c(self) -> "_lib.QzArgs":
        st = {"tensor": _lib.QZ_TENSOR, "channel": _lib.QZ_CHANNEL, "group": _lib.QZ_GROUP,
              "block": _lib.QZ_BLOCK, "tensor_group": _lib.QZ_TENSOR_GROUP}[self.strategy]
        if self.is_mx:
            sf = _lib.QZ_SCALE_E8M0
        elif self.is_nvfp4:
            sf = _lib.QZ_SCALE_E4M3
        else:
            sf = _lib.QZ_SCALE_NATIVE
        bh, bw = (self.block_structure or (0, 0))
        return _lib.QzArgs(self.num_bits, _lib.QZ_INT if self.type == "int" else _lib.QZ_FLOAT,
                           int(bool(self.symmetric)), st, int(self.group_size or 0), int(bh), int(bw), sf)

    def to_dict(self) -> Dict[str, Any]:
        d = asdict(self)
        return d


@dataclass
class QuantizationScheme:
    """compressed-tensors ``QuantizationScheme``: targets + weight/activation args + format."""

    targets: List[str]
    weights: Optional[QuantizationArgs] = None
    input_activations: Optional[QuantizationArgs] = None
    output_activations: Optional[QuantizationArgs] = None
    format: Optional[str] = None


def _w(**kw) -> QuantizationArgs:
    return QuantizationArgs(**kw)


# compressed-tensors PRESET_SCHEMES (weight halves; activation args kept for the config)
def preset_scheme(name: str, targets: List[str]) -> QuantizationScheme:
    n = name.upper()
    acts = None
    if n in ("W8A16",):
        w = _w(num_bits=8, type="int", symmetric=True, strategy="channel")
    elif n in ("W4A16",):
        w = _w(num_bits=4, type="int", symmetric=True, strategy="group", group_size=128)
    elif n in ("W4A16_ASYM",):
        w = _w(num_bits=4, type="int", symmetric=False, strategy="group", group_size=128)
    elif n in ("W8A8", "INT8"):
        w = _w(num_bits=8, type="int", symmetric=True, strategy="channel")
        acts = _w(num_bits=8, type="int", symmetric=True, strategy="token", dynamic=True)
    elif n in ("W4A8",):
        w = _w(num_bits=4, type="int", symmetric=True, strategy="group", group_size=128)
        acts = _w(num_bits=8, type="int", symmetric=True, strategy="token", dynamic=True)
    elif n in ("FP8",):
        w = _w(num_bits=8, type="float", symmetric=True, strategy="tensor")
        acts = _w(num_bits=8, type="float", symmetric=True, strategy="tensor")
    elif n in ("FP8_DYNAMIC",):
        w = _w(num_bits=8, type="float", symmetric=True, strategy="channel")
        acts = _w(num_bits=8, type="float", symmetric=True, strategy="token", dynamic=True)
    elif n in ("FP8_BLOCK",):
        w = _w(num_bits=8, type="float", symmetric=True, strategy="block", block_structure=[128, 128])
        acts = _w(num_bits=8, type="float", symmetric=True, strategy="group", group_size=128, dynamic=True)
    elif n in ("NVFP4A16",):
        w = _w(num_bits=4, type="float", symmetric=True, strategy="tensor_group", group_size=16,
               scale_dtype="float8_e4m3fn")
    elif n in ("NVFP4",):
        w = _w(num_bits=4, type="float", symmetric=True, strategy="tensor_group", group_size=16,
               scale_dtype="float8_e4m3fn")
        acts = _w(num_bits=4, type="float", symmetric=True, strategy="tensor_group", group_size=16,
                  dynamic="local", scale_dtype="float8_e4m3fn")
    elif n in ("MXFP4A16",):
        w = _w(num_bits=4, type="float", symmetric=True, strategy="group", group_size=32, scale_dtype="uint8")
    elif n in ("MXFP4",):
        w = _w(num_bits=4, type="float", symmetric=True, strategy="group", group_size=32, scale_dtype="uint8")
        acts = _w(num_bits=4, type="float", symmetric=True, strategy="group", group_size=32, dynamic=True,
                  scale_dtype="uint8")
    else:
        raise ValueError(f"unknown preset scheme {name!r}")
    w.observer = w.observer or "minmax"
    return QuantizationScheme(targets=list(targets), weights=w, input_activations=acts)


def compression_format(w: QuantizationArgs, acts: Optional[QuantizationArgs] = None) -> str:
    """compressed-tensors format inference for the on-disk tensors."""
    if w.type == "int":
        if acts is not None and w.num_bits == 8:
            return "int-quantized"
        return "pack-quantized"
    if w.num_bits == 8:
        return "float-quantized"
    if w.is_mx:
        return "mxfp4-pack-quantized"
    return "nvfp4-pack-quantized"


def copy_args(a: QuantizationArgs, **kw) -> QuantizationArgs:
    b = copy.deepcopy(a)
    for k, v in kw.items():
        setattr(b, k, v)
    return b
