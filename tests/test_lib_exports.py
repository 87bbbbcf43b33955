"""The C-ABI library loads and exports every function include/quantizers_amd.h declares
(no compute calls: this runs without a GPU)."""
import ctypes
import os
import re

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _declared():
    src = open(os.path.join(ROOT, "include", "quantizers_amd.h")).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(qz_[a-z0-9_]+)\s*\(", src)))


def test_library_exports_header_symbols():
    from quantizers_amd import _lib
    lib = ctypes.CDLL(_lib.LIB_PATH)
    decl = _declared()
    assert len(decl) >= 16
    missing = [n for n in decl if not hasattr(lib, n)]
    assert not missing, missing
    assert set(decl) == set(_lib.EXPORTS)


def test_host_only_entry_points():
    from quantizers_amd import _lib
    lib = _lib.load()
    assert lib.qz_version() == 200
    cfg = _lib.build_config()
    assert cfg["arch"] == "gfx950" and isinstance(cfg["nt_bytes_q"], int)
    assert lib.qz_strerror(-3).decode().startswith("tensor column shape")
    a = _lib.QzArgs(4, 0, 1, 2, 128, 0, 0, 0)
    assert lib.qz_quantize_workspace_size(1, 11008, 4096, ctypes.byref(a)) > 0
    bad = _lib.QzArgs(4, 0, 1, 2, 100, 0, 0, 0)
    assert lib.qz_quantize_workspace_size(1, 16, 128, ctypes.byref(bad)) == 0


def test_expert_gemms_binding_host_only():
    """qz_expert_gemms binds the hipBLASLt PyTorch already loaded, by its path, never loading a
    copy itself; a library that is not loaded is refused with a reason (no GPU needed)."""
    import torch
    from quantizers_amd import _lib
    lib = _lib.load()
    bad = os.path.join(ROOT, "no_such_dir", "libhipblaslt.so")
    assert lib.qz_expert_gemms_library(bad.encode()) in (_lib.QZ_ERR_UNAVAILABLE, _lib.QZ_ERR_FORMAT)
    assert b"libhipblaslt.so" in lib.qz_expert_gemms_status()
    torch_lt = os.path.join(os.path.dirname(torch.__file__), "lib", "libhipblaslt.so")
    assert lib.qz_expert_gemms_library(torch_lt.encode()) == 0
    assert lib.qz_expert_gemms_status().startswith(b"bound: ")
    assert lib.qz_expert_gemms_library(torch_lt.encode()) == 0  # idempotent


def test_nvfp4_host_queries():
    from quantizers_amd import _lib
    lib = _lib.load()
    assert lib.qz_nvfp4_sync_size(128) == 64 * 128  # one 64-B line {key, tile count} per slice
    assert lib.qz_nvfp4_sync_size(-1) == 0
