"""quantizers_amd — MI355X-native (gfx950) weight-quantization path for mratsim/quantizers.

The host side mirrors the reference's drop-in surface (scripts/do_oneshot.py + YAML recipes,
llmcompressor ``oneshot`` / compressed-tensors quantization API); the per-linear quantize step
(AWQ statistics and scale-search fake-quant, per-group min/max -> scale/zero-point,
round-clamp-pack to int4 / int8 / FP8-E4M3 / MXFP4 / NVFP4) runs in hand-written HIP kernels
behind the C ABI declared in include/quantizers_amd.h.
"""
from .quantization import QuantizationArgs, QuantizationScheme, preset_scheme  # noqa: F401

__version__ = "0.1.0"
