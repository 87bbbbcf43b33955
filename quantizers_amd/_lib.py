"""ctypes binding of the C ABI in include/quantizers_amd.h (libquantizers_amd.so, gfx950).

The library is built in-tree by ``__graft_entry__.build()`` (``make -C quantizers_amd/csrc``).
There is no CPU fallback: if the shared object is missing or fails to load, every op raises.
"""
from __future__ import annotations

import ctypes
import os

_HERE = os.path.dirname(os.path.abspath(__file__))
# QUANTIZERS_AMD_LIB overrides the path (tuning builds under scripts/tune_fast.sh only)
LIB_PATH = os.environ.get("QUANTIZERS_AMD_LIB") or os.path.join(_HERE, "libquantizers_amd.so")

# enums (include/quantizers_amd.h)
QZ_INT, QZ_FLOAT = 0, 1
QZ_TENSOR, QZ_CHANNEL, QZ_GROUP, QZ_BLOCK, QZ_TENSOR_GROUP = 0, 1, 2, 3, 4
QZ_SCALE_NATIVE, QZ_SCALE_E4M3, QZ_SCALE_E8M0 = 0, 2, 3
QZ_OUT_PACKED_INT32, QZ_OUT_INT8, QZ_OUT_FP8, QZ_OUT_FP4_PACKED, QZ_OUT_FAKEQUANT = 0, 1, 2, 3, 4

QZ_ERR_NULL, QZ_ERR_SHAPE, QZ_ERR_GROUP, QZ_ERR_BLOCK = -1, -2, -3, -4
QZ_ERR_BITS, QZ_ERR_ASYM_FLOAT, QZ_ERR_FORMAT, QZ_ERR_WORKSPACE, QZ_ERR_ALIGN = -5, -6, -7, -8, -9
QZ_ERR_UNAVAILABLE = -10

# every symbol the header declares (tests check the library exports all of them)
EXPORTS = (
    "qz_strerror", "qz_version", "qz_build_config", "qz_quantize_workspace_size", "qz_quantize", "qz_quantize_qparams",
    "qz_observe_minmax", "qz_calculate_qparams", "qz_dequantize", "qz_pack_int32",
    "qz_awq_absmean_workspace_size", "qz_awq_absmean_accum", "qz_awq_weight_mean_workspace_size",
    "qz_awq_weight_mean_accum", "qz_awq_absmean_segments_workspace_size", "qz_awq_absmean_accum_segments",
    "qz_awq_weight_mean_segments_workspace_size", "qz_awq_weight_mean_accum_segments",
    "qz_awq_grid_scales", "qz_awq_fake_quant", "qz_scale_columns", "qz_scale_rows",
    "qz_awq_grid_scales_batched", "qz_awq_fake_quant_batched", "qz_awq_sq_err_workspace_size",
    "qz_awq_sq_err_accum", "qz_quantize_many", "qz_quantize_grouped", "qz_quantize_grouped_var",
    "qz_grouped_blocks", "qz_awq_sq_err_partials_count", "qz_awq_sq_err_partials", "qz_awq_sq_err_reduce",
    "qz_awq_sq_err_partials_multi", "qz_awq_stats_layout", "qz_moe_combine",
    "qz_moe_silu_mul", "qz_expert_gemms", "qz_silu_mul", "qz_rmsnorm128",
    "qz_rotary128", "qz_nvfp4_sync_size", "qz_quantize_nvfp4",
    "qz_quantize_grouped_nvfp4", "qz_expert_gemms_library", "qz_expert_gemms_status",
)


class QzArgs(ctypes.Structure):
    """``qz_args`` (mirrors compressed-tensors QuantizationArgs fields)."""

    _fields_ = [(n, ctypes.c_int32) for n in
                ("num_bits", "type", "symmetric", "strategy", "group_size", "block_h", "block_w", "scale_fmt")]


class QzError(RuntimeError):
    pass


_lib = None


def load() -> ctypes.CDLL:
    """Load the HIP library; raise loudly if it is missing (no fallback)."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise QzError(f"{LIB_PATH} not built; run __graft_entry__.build() or make -C quantizers_amd/csrc")
    lib = ctypes.CDLL(LIB_PATH)
    P, I64, I32, SZ = ctypes.c_void_p, ctypes.c_int64, ctypes.c_int32, ctypes.c_size_t
    A = ctypes.POINTER(QzArgs)
    sig = {
        "qz_strerror": ([ctypes.c_int], ctypes.c_char_p),
        "qz_version": ([], ctypes.c_int),
        "qz_build_config": ([], ctypes.c_char_p),
        "qz_quantize_workspace_size": ([I64, I64, I64, A], SZ),
        "qz_quantize": ([P, I64, I64, I64, I64, I64, A, I32, P, P, P, P, P, SZ, P], ctypes.c_int),
        "qz_quantize_many": ([I64, P, P, P, P, P, I64, I64, I64, I64, I64, A, I32, P, SZ, P], ctypes.c_int),
        "qz_quantize_grouped": ([I64, P, I64, I64, A, I32, P], ctypes.c_int),
        "qz_quantize_grouped_var": ([I64, P, P, P, A, I32, P], ctypes.c_int),
        "qz_grouped_blocks": ([I64, I64], ctypes.c_int64),
        "qz_quantize_qparams": ([P, I64, I64, I64, I64, I64, A, I32, P, P, P, P, P], ctypes.c_int),
        "qz_observe_minmax": ([P, I64, I64, I64, I64, I64, A, P, P, P, SZ, P], ctypes.c_int),
        "qz_calculate_qparams": ([P, P, I64, A, P, P, P, P], ctypes.c_int),
        "qz_dequantize": ([P, I64, I64, I64, A, I32, P, P, P, P, P], ctypes.c_int),
        "qz_pack_int32": ([P, I64, I64, I32, I32, P, P], ctypes.c_int),
        "qz_awq_absmean_workspace_size": ([I64, I64], SZ),
        "qz_awq_absmean_accum": ([P, I64, I64, I64, P, P, SZ, P], ctypes.c_int),
        "qz_awq_weight_mean_workspace_size": ([I64, I64, I32], SZ),
        "qz_awq_weight_mean_accum": ([P, I64, I64, I64, I32, P, P, SZ, P], ctypes.c_int),
        "qz_awq_absmean_segments_workspace_size": ([I32, P, I64], SZ),
        "qz_awq_absmean_accum_segments": ([I32, P, P, I64, P, P, P, SZ, P], ctypes.c_int),
        "qz_awq_weight_mean_segments_workspace_size": ([I32, P, I64, I32], SZ),
        "qz_awq_weight_mean_accum_segments": ([I32, P, P, I64, P, I32, P, P, SZ, P], ctypes.c_int),
        "qz_awq_stats_layout": ([I32, I64, I64, I32, P], ctypes.c_int),
        "qz_awq_grid_scales": ([P, P, I64, ctypes.c_float, I32, P, P], ctypes.c_int),
        "qz_awq_fake_quant": ([P, I64, I64, I64, I64, I64, A, P, P, P, SZ, P], ctypes.c_int),
        "qz_awq_grid_scales_batched": ([P, P, I64, I64, ctypes.c_float, I32, P, P], ctypes.c_int),
        "qz_awq_sq_err_workspace_size": ([I64, I64], SZ),
        "qz_awq_sq_err_accum": ([P, P, I64, I64, I64, I64, P, P, SZ, P], ctypes.c_int),
        "qz_awq_sq_err_partials_count": ([I64, I64], I64),
        "qz_awq_sq_err_partials": ([P, P, I64, I64, I64, I64, P, P], ctypes.c_int),
        "qz_awq_sq_err_reduce": ([P, I64, I64, I64, P, P], ctypes.c_int),
        "qz_awq_sq_err_partials_multi": ([P, P, I32, I64, I64, P, I64, P], ctypes.c_int),
        "qz_awq_fake_quant_batched": ([P, I64, I64, I64, I64, I64, A, P, I64, P, P, SZ, P], ctypes.c_int),
        "qz_scale_columns": ([P, I64, I64, I64, P, I32, P], ctypes.c_int),
        "qz_scale_rows": ([P, I64, I64, I64, P, I32, P], ctypes.c_int),
        "qz_moe_combine": ([P, I64, I64, P, I32, P, P, I64, I32, P, P], ctypes.c_int),
        "qz_moe_silu_mul": ([P, I64, I64, I64, P, P], ctypes.c_int),
        "qz_silu_mul": ([P, I64, P, I64, I64, I64, P, P], ctypes.c_int),
        "qz_rmsnorm128": ([P, I64, I64, P, ctypes.c_float, P, P], ctypes.c_int),
        "qz_rotary128": ([P, I64, I64, I64, I64, I64, I64, P, P, I64, I64, P, I64, I64, I64, P], ctypes.c_int),
        "qz_nvfp4_sync_size": ([I64], SZ),
        "qz_quantize_nvfp4": ([P, I64, I64, I64, I64, A, P, P, P, P, SZ, P], ctypes.c_int),
        "qz_quantize_grouped_nvfp4": ([I64, P, I64, I64, A, P, SZ, P], ctypes.c_int),
        "qz_expert_gemms_library": ([ctypes.c_char_p], ctypes.c_int),
        "qz_expert_gemms_status": ([], ctypes.c_char_p),
        "qz_expert_gemms": ([P, I64, P, I64, I64, I64, I64, P, I64, P, P, P, I32, P, SZ, P], ctypes.c_int),
    }
    for name, (argtypes, restype) in sig.items():
        fn = getattr(lib, name)
        fn.argtypes = argtypes
        fn.restype = restype
    _lib = lib
    return lib


def build_config() -> dict:
    """The library's compile-time tuning constants (qz_build_config) as a dict."""
    out = {}
    for kv in load().qz_build_config().decode().split(";"):
        k, _, v = kv.partition("=")
        out[k] = int(v) if v.lstrip("-").isdigit() else v
    return out


_VALUE_ERRORS = {QZ_ERR_SHAPE, QZ_ERR_GROUP, QZ_ERR_BLOCK, QZ_ERR_BITS, QZ_ERR_ASYM_FLOAT, QZ_ERR_FORMAT,
                 QZ_ERR_ALIGN}


def check(rc: int, what: str = "") -> None:
    """Map C-ABI return codes to the reference's exception types (ValueError for bad args)."""
    if rc == 0:
        return
    msg = load().qz_strerror(rc).decode()
    if rc in _VALUE_ERRORS:
        raise ValueError(f"{what}: {msg}")
    raise QzError(f"{what}: {msg} (code {rc})")
