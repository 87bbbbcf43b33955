"""PyTorch-facing wrappers of the HIP quantization kernels (device memory + stream plumbing).

Names and argument meaning follow compressed-tensors / llmcompressor (the reference's
quantization dependencies, called from scripts/do_oneshot.py:179-197):

=========================  ==========================================================
this module                 replaces ([3P] = third-party)
=========================  ==========================================================
``observe_minmax``          llmcompressor observer ``memoryless_minmax`` (a7)
``calculate_qparams``       compressed_tensors ``calculate_qparams`` (a8)
``quantize``                compressed_tensors ``quantize`` with given qparams (a9)
``fake_quantize``           compressed_tensors ``fake_quantize`` (AWQ grid, a5)
``dequantize``              compressed_tensors ``dequantize`` / decompressors
``pack_to_int32``           compressed_tensors ``pack_to_int32`` (a10)
``compress_weight``         observer -> qparams -> quantize -> pack, one fused pass
                            (ModelCompressor.compress_model per module, a9-a12)
``awq_*``                   llmcompressor AWQModifier statistics / smoothing (a3-a6)
=========================  ==========================================================

All tensors must live on a ROCm device; weights are bf16 2-D ``[N, K]`` or a 3-D batch of
slices ``[E, N, K]`` (fused MoE experts).  There is no CPU fallback.
"""
from __future__ import annotations

import ctypes
import os
from typing import Callable, Dict, List, Optional, Sequence, Tuple

import torch

from . import _lib
from .quantization import QuantizationArgs

_P = ctypes.c_void_p


def _ptr(t: Optional[torch.Tensor]):
    return _P(t.data_ptr()) if t is not None else _P(0)


def _stream():
    return _P(torch.cuda.current_stream().cuda_stream)


def _check_dev(t: torch.Tensor, name: str):
    if not t.is_cuda:
        raise ValueError(f"{name} must be a ROCm device tensor (no CPU fallback)")


_ws_cache: Dict[Tuple[int, int], torch.Tensor] = {}
_stats_ws_cache: Dict[Tuple[int, int], torch.Tensor] = {}
_sync_cache: Dict[Tuple[int, int], torch.Tensor] = {}


def workspace(nbytes: int, device) -> torch.Tensor:
    """Per-(device, stream) grow-only scratch buffer (the library never allocates)."""
    dev = torch.device(device)
    key = (dev.index or 0, torch.cuda.current_stream(dev).cuda_stream)
    buf = _ws_cache.get(key)
    if buf is None or buf.numel() < nbytes:
        buf = torch.empty(max(nbytes, 1 << 16), dtype=torch.uint8, device=dev)
        _ws_cache[key] = buf
    return buf


def stats_workspace(nbytes: int, device) -> torch.Tensor:
    """Per-(device, stream) grow-only scratch of the AWQ statistics calls, zeroed when allocated:
    its head holds the one-launch reduction's arrival counters, which every call leaves zero
    (quantizers_amd.h, statistics workspace contract) -- so it is never shared with other calls."""
    dev = torch.device(device)
    key = (dev.index or 0, torch.cuda.current_stream(dev).cuda_stream)
    buf = _stats_ws_cache.get(key)
    if buf is None or buf.numel() < nbytes:
        buf = torch.zeros(max(nbytes, 1 << 16), dtype=torch.uint8, device=dev)
        _stats_ws_cache[key] = buf
    return buf


def sync_workspace(n_slices: int, device, stream=None) -> torch.Tensor:
    """Per-(device, stream) grow-only sync region of the NVFP4 path (qz_quantize_nvfp4 /
    qz_quantize_grouped_nvfp4: each slice's |w| maximum and tile count), zeroed when allocated: every call leaves it
    zero (quantizers_amd.h), and calls on one stream never overlap, so it is shared by them."""
    dev = torch.device(device)
    st = stream if stream is not None else torch.cuda.current_stream(dev)
    key = (dev.index or 0, st.cuda_stream)
    nbytes = int(_lib.load().qz_nvfp4_sync_size(int(n_slices)))
    buf = _sync_cache.get(key)
    if buf is None or buf.numel() < nbytes:
        with torch.cuda.stream(st):
            buf = torch.zeros(max(nbytes, 1 << 16), dtype=torch.uint8, device=dev)
        _sync_cache[key] = buf
    return buf


def _drop_sync(device, stream=None) -> None:
    """Forget the stream's NVFP4 sync region after a failed call (the library clears it on the
    stream too; a fresh zeroed region is allocated by the next call either way)."""
    dev = torch.device(device)
    st = stream if stream is not None else torch.cuda.current_stream(dev)
    _sync_cache.pop((dev.index or 0, st.cuda_stream), None)


def _nvfp4_fused_ok(a: QuantizationArgs, out_fmt: int, geom, w: torch.Tensor) -> bool:
    b, r, c, ld_r, ld_b = geom
    return (a.is_nvfp4 and a.group_size == 16 and out_fmt == _lib.QZ_OUT_FP4_PACKED and ld_r == c
            and (b == 1 or ld_b % 8 == 0) and w.data_ptr() % 16 == 0)


def awq_stats_layout(which: str, rows: int, cols: int, group_size: int = 0) -> Dict[str, int]:
    """The fixed summation plan of awq_absmean_accum (``which="absmean"``, rows = tokens) or
    awq_weight_mean_accum (``"wmean"``) for a [rows, cols] input (qz_awq_stats_layout)."""
    out = (ctypes.c_int64 * 8)()
    rc = _lib.load().qz_awq_stats_layout(0 if which == "absmean" else 1, rows, cols, int(group_size), out)
    _lib.check(rc, "qz_awq_stats_layout")
    return dict(zip(("one_launch", "window", "rows_per_chunk", "chunks", "slots", "final_groups", "head_bytes", "chunks_per_group"),
                    list(out)))


def _geom(w: torch.Tensor):
    """(batch, rows, cols, ld_row, ld_batch) for a 2-D or 3-D bf16 weight view."""
    if w.dtype != torch.bfloat16:
        raise ValueError(f"weights must be bfloat16 (got {w.dtype})")
    if w.dim() == 2:
        w3 = w.unsqueeze(0)
    elif w.dim() == 3:
        w3 = w
    else:
        raise ValueError("weight must be 2-D [N, K] or 3-D [E, N, K]")
    if w3.stride(2) != 1:
        raise ValueError("weight rows must be contiguous (stride(-1) == 1)")
    b, r, c = w3.shape
    ld_b = w3.stride(0) if b > 1 else r * w3.stride(1)
    return b, r, c, w3.stride(1), ld_b


def n_groups(a: QuantizationArgs, rows: int, cols: int) -> Tuple[int, ...]:
    """Per-slice scale shape (compressed-tensors layout)."""
    if a.strategy == "tensor":
        return (1,)
    if a.strategy == "channel":
        return (rows, 1)
    if a.strategy in ("group", "tensor_group"):
        if cols % a.group_size:
            raise ValueError(f"tensor column shape must be divisible by the given group_size {a.group_size}")
        return (rows, cols // a.group_size)
    if a.strategy == "block":
        bh, bw = a.block_structure
        if rows % bh or cols % bw:
            raise ValueError("Block quantization requires exact division")
        return (rows // bh, cols // bw)
    raise ValueError(f"strategy {a.strategy} not supported for weights")


def _scale_dtype(a: QuantizationArgs):
    if a.is_mx:
        return torch.uint8
    if a.is_nvfp4:
        return torch.float8_e4m3fn
    return torch.bfloat16


def default_out_fmt(a: QuantizationArgs) -> int:
    if a.type == "int":
        return _lib.QZ_OUT_PACKED_INT32
    if a.num_bits == 8:
        return _lib.QZ_OUT_FP8
    return _lib.QZ_OUT_FP4_PACKED


def _alloc_codes(out_fmt: int, a: QuantizationArgs, lead, rows, cols, device):
    if out_fmt == _lib.QZ_OUT_PACKED_INT32:
        pf = 32 // a.num_bits
        return torch.empty(*lead, rows, (cols + pf - 1) // pf, dtype=torch.int32, device=device)
    if out_fmt == _lib.QZ_OUT_INT8:
        return torch.empty(*lead, rows, cols, dtype=torch.int8, device=device)
    if out_fmt == _lib.QZ_OUT_FP8:
        return torch.empty(*lead, rows, cols, dtype=torch.float8_e4m3fn, device=device)
    if out_fmt == _lib.QZ_OUT_FP4_PACKED:
        return torch.empty(*lead, rows, cols // 2, dtype=torch.uint8, device=device)
    return torch.empty(*lead, rows, cols, dtype=torch.bfloat16, device=device)


def quantize_weight(w: torch.Tensor, a: QuantizationArgs, out_fmt: Optional[int] = None,
                    out: Optional[Dict[str, torch.Tensor]] = None) -> Dict[str, torch.Tensor]:
    """Fused memoryless observe + calculate_qparams + quantize (+ pack).

    Returns ``codes`` (packed int32 / int8 / e4m3 / packed fp4), ``scale``, ``zero_point``
    (int8 per group) and, for NVFP4, ``global_scale`` (f32 per slice).  ``out`` may supply
    preallocated tensors (bench / graph capture).
    """
    _check_dev(w, "weight")
    b, r, c, ld_r, ld_b = _geom(w)
    lead = tuple(w.shape[:-2])
    out_fmt = default_out_fmt(a) if out_fmt is None else out_fmt
    ca = a.to_c()
    gshape = n_groups(a, r, c)
    dev = w.device
    o = dict(out or {})
    if "codes" not in o:
        o["codes"] = _alloc_codes(out_fmt, a, lead, r, c, dev)
    if "scale" not in o:
        o["scale"] = torch.empty(*lead, *gshape, dtype=_scale_dtype(a), device=dev)
    if "zero_point" not in o:  # symmetric: no zero-point tensor (compressed-tensors stores none)
        o["zero_point"] = None if a.symmetric else torch.empty(*lead, *gshape, dtype=torch.int8, device=dev)
    if a.is_nvfp4 and "global_scale" not in o:
        o["global_scale"] = torch.empty(max(b, 1), dtype=torch.float32, device=dev)
    lib = _lib.load()
    if _nvfp4_fused_ok(a, out_fmt, (b, r, c, ld_r, ld_b), w):
        sync = sync_workspace(b, dev)
        rc = lib.qz_quantize_nvfp4(_ptr(w), b, r, c, ld_b, ctypes.byref(ca), _ptr(o["codes"]), _ptr(o["scale"]),
                                   _ptr(o["global_scale"]), _ptr(sync), sync.numel(), _stream())
        if rc:
            _drop_sync(dev)
        _lib.check(rc, "qz_quantize_nvfp4")
        o.pop("workspace", None)
        return o
    ws_n = lib.qz_quantize_workspace_size(b, r, c, ctypes.byref(ca))
    ws = o.get("workspace")
    if ws is None or ws.numel() < ws_n:
        ws = workspace(ws_n, dev)
    rc = lib.qz_quantize(_ptr(w), b, r, c, ld_r, ld_b, ctypes.byref(ca), out_fmt, _ptr(o["codes"]),
                         _ptr(o["scale"]), _ptr(o["zero_point"]), _ptr(o.get("global_scale")),
                         _ptr(ws), ws.numel(), _stream())
    _lib.check(rc, "qz_quantize")
    o.pop("workspace", None)
    return o


def is_fp8_block128(a: QuantizationArgs) -> bool:
    """compressed-tensors' FP8_BLOCK preset: e4m3 codes, one bf16 scale per 128 x 128 block."""
    return (a.strategy == "block" and a.type == "float" and a.num_bits == 8
            and list(a.block_structure or ()) == [128, 128])


def grouped_ok(a: QuantizationArgs, w: torch.Tensor) -> bool:
    """True when one grouped launch covers this scheme and weight: qz_quantize_grouped (the
    single-pass group path, or FP8_BLOCK's strip kernel) or, for NVFP4,
    qz_quantize_grouped_nvfp4 (two launches per group)."""
    dense = w.dim() == 2 and w.is_contiguous() and w.dtype == torch.bfloat16 and w.data_ptr() % 16 == 0
    if is_fp8_block128(a):
        return dense and w.shape[0] % 128 == 0 and w.shape[1] % 128 == 0
    g = a.group_size or 0
    if a.is_nvfp4 and g != 16:
        return False
    return (a.strategy in ("group", "tensor_group") and 8 <= g <= 512 and (g & (g - 1)) == 0
            and dense and w.shape[1] % g == 0)


def _check_no_alias(ws: Sequence[torch.Tensor], outs: Sequence[Dict[str, torch.Tensor]]) -> None:
    """Raise if any output tensor overlaps any input weight (sorted sweep, O(n log n))."""
    import bisect
    ins = sorted((w.data_ptr(), w.data_ptr() + w.numel() * w.element_size()) for w in ws)
    starts = [lo for lo, _ in ins]
    run_hi = []  # running max of the end addresses, so one bisect answers "any input overlaps"
    m = 0
    for _, hi in ins:
        m = max(m, hi)
        run_hi.append(m)
    for o in outs:
        for k in ("codes", "scale", "zero_point"):
            t = o.get(k)
            if t is None or t.numel() == 0:
                continue
            lo, hi = t.data_ptr(), t.data_ptr() + t.numel() * t.element_size()
            j = bisect.bisect_left(starts, hi) - 1  # inputs starting before this output's end
            if j >= 0 and run_hi[j] > lo:
                raise ValueError("GroupedQuantize: an output aliases a weight")


def alloc_outputs(shape, a: QuantizationArgs, out_fmt: Optional[int], device) -> Dict[str, torch.Tensor]:
    """quantize_weight's output tensors for a [rows, cols] or [E, rows, cols] weight."""
    out_fmt = default_out_fmt(a) if out_fmt is None else out_fmt
    lead, (r, c) = tuple(shape[:-2]), tuple(shape[-2:])
    gshape = n_groups(a, r, c)
    o = {"codes": _alloc_codes(out_fmt, a, lead, r, c, device),
         "scale": torch.empty(*lead, *gshape, dtype=_scale_dtype(a), device=device),
         "zero_point": None if a.symmetric else torch.empty(*lead, *gshape, dtype=torch.int8, device=device)}
    if a.is_nvfp4:
        o["global_scale"] = torch.empty(max(int(torch.Size(lead).numel()), 1), dtype=torch.float32, device=device)
    return o


class GroupedQuantize:
    """``qz_quantize_grouped``: n dense weights of one scheme quantized in ONE launch, the
    per-launch ramp paid once.  Same-shape weights: grid.y = weight.  Mixed shapes (up to 8,
    ``qz_quantize_grouped_var``): one flat grid whose workgroups find their weight from
    per-shape segments passed as kernel arguments -- a whole model's same-scheme linears in one
    launch.  The device tables are built once here;
    ``run(stream=None)`` is one ctypes call + one kernel launch.  Outputs are exactly
    ``quantize_weight``'s, one dict per weight (``outs``; allocated when not given)."""

    def __init__(self, ws: Sequence[torch.Tensor], a: QuantizationArgs, out_fmt: Optional[int] = None,
                 outs: Optional[Sequence[Dict[str, torch.Tensor]]] = None):
        if not ws:
            raise ValueError("GroupedQuantize needs at least one weight")
        if len(ws) > 65535:
            raise ValueError("GroupedQuantize: at most 65535 weights per launch")
        for w in ws:
            _check_dev(w, "weight")
            if w.dim() != 2 or not grouped_ok(a, w) or w.device != ws[0].device:
                raise ValueError("GroupedQuantize: every weight must be a dense, 16-B aligned bf16 [rows, cols] "
                                 "tensor on one device, under a single-pass group scheme")
        shapes = [tuple(w.shape) for w in ws]
        self.mixed = len(set(shapes)) > 1
        self.nvfp4 = a.is_nvfp4
        if (self.nvfp4 or is_fp8_block128(a)) and self.mixed:
            raise ValueError("GroupedQuantize: NVFP4 / FP8_BLOCK weights of one launch must share one shape")
        self.a = a
        dev = ws[0].device
        self.out_fmt = default_out_fmt(a) if out_fmt is None else out_fmt
        if self.nvfp4 and self.out_fmt != _lib.QZ_OUT_FP4_PACKED:
            # qz_quantize_grouped_nvfp4 writes packed E2M1 codes only
            raise ValueError("GroupedQuantize: NVFP4 grouped launches write packed FP4 codes only "
                             "(use quantize_weight for other output formats)")
        self.ca = a.to_c()
        if outs is None:
            outs = [alloc_outputs(shp, a, self.out_fmt, dev) for shp in shapes]
        if len(outs) != len(ws):
            raise ValueError("GroupedQuantize: one output dict per weight")
        _check_no_alias(ws, outs)
        if any(o["codes"].data_ptr() % 16 for o in outs):  # the table contract (quantizers_amd.h)
            raise ValueError("GroupedQuantize: every codes output must be 16-B aligned")
        if not a.symmetric and any(o.get("zero_point") is None for o in outs):
            raise ValueError("GroupedQuantize: asymmetric schemes need a zero_point output per weight")
        n = len(ws)
        self.lib = _lib.load()
        # mixed shapes: the table lists equal shapes consecutively (the launch's segments)
        first: Dict[tuple, int] = {}
        for i, shp in enumerate(shapes):
            first.setdefault(shp, i)
        order = sorted(range(n), key=lambda i: first[shapes[i]]) if self.mixed else list(range(n))
        last = ("global_scale" if self.nvfp4 else "zero_point")  # NVFP4: row 3 = the f32 global scale
        rows = [[ws[i].data_ptr() for i in order], [outs[i]["codes"].data_ptr() for i in order],
                [outs[i]["scale"].data_ptr() for i in order],
                [0 if outs[i].get(last) is None else outs[i][last].data_ptr() for i in order]]
        if self.mixed:
            if len(set(shapes)) > 8:
                raise ValueError("GroupedQuantize: at most 8 distinct shapes per launch")
            self._rows = (ctypes.c_int64 * n)(*[shapes[i][0] for i in order])
            self._cols = (ctypes.c_int64 * n)(*[shapes[i][1] for i in order])
        self.table = torch.tensor(rows, dtype=torch.int64).reshape(-1).to(dev)
        self.n = n
        self.rows, self.cols = shapes[0]
        self.shapes = shapes
        self.weights, self.outs = list(ws), list(outs)  # keep every pointer alive

    def run(self, stream=None) -> List[Dict[str, torch.Tensor]]:
        st = _P(stream.cuda_stream) if stream is not None else _stream()
        if self.nvfp4:
            sync = sync_workspace(self.n, self.weights[0].device, stream)
            rc = self.lib.qz_quantize_grouped_nvfp4(self.n, _ptr(self.table), self.rows, self.cols, ctypes.byref(self.ca),
                                                    _ptr(sync), sync.numel(), st)
            if rc:
                _drop_sync(self.weights[0].device, stream)
            _lib.check(rc, "qz_quantize_grouped_nvfp4")
            return self.outs
        if self.mixed:
            rc = self.lib.qz_quantize_grouped_var(self.n, _ptr(self.table), ctypes.cast(self._rows, _P),
                                                  ctypes.cast(self._cols, _P), ctypes.byref(self.ca), self.out_fmt,
                                                  st)
            _lib.check(rc, "qz_quantize_grouped_var")
        else:
            rc = self.lib.qz_quantize_grouped(self.n, _ptr(self.table), self.rows, self.cols, ctypes.byref(self.ca),
                                              self.out_fmt, st)
            _lib.check(rc, "qz_quantize_grouped")
        return self.outs


def quantize_weights(ws: Sequence[torch.Tensor], a: QuantizationArgs,
                     out_fmt: Optional[int] = None) -> List[Dict[str, torch.Tensor]]:
    """Quantize many weights of one scheme: same-shape dense weights under a single-pass group
    scheme go through ONE grouped launch per shape (qz_quantize_grouped); anything else is one
    ``quantize_weight`` launch per weight.  Results are identical either way."""
    res: List[Optional[Dict[str, torch.Tensor]]] = [None] * len(ws)
    by_shape: Dict[tuple, List[int]] = {}
    nv_other_fmt = a.is_nvfp4 and out_fmt not in (None, _lib.QZ_OUT_FP4_PACKED)
    for i, w in enumerate(ws):
        if grouped_ok(a, w) and not nv_other_fmt:
            by_shape.setdefault((tuple(w.shape), w.device), []).append(i)
        else:
            res[i] = quantize_weight(w, a, out_fmt)
    for idx in by_shape.values():
        for s in range(0, len(idx), 65535):
            part = idx[s:s + 65535]
            outs = GroupedQuantize([ws[i] for i in part], a, out_fmt).run()
            for i, o in zip(part, outs):
                res[i] = o
    return res  # type: ignore[return-value]


NVFP4_STREAMS = 2  # 1 / 2 / 3 streams: 21.2 / 20.2 / 21.0 ms per Qwen3-30B-A3B experts pass (r04w)
_side_streams: Dict[Tuple[int, int, int], torch.cuda.Stream] = {}


def nvfp4_streams(device, stream=None, n_streams: Optional[int] = None) -> List[torch.cuda.Stream]:
    """The streams NVFP4 work is spread over: the caller's stream first, then ``n_streams - 1``
    side streams (cached per caller stream) that wait for it; ``join_streams`` makes the caller's
    stream wait for them.  Two streams let one NVFP4 call's |w| max launch (read-bound) run beside
    the previous call's encode launch (VALU-heavy)."""
    dev = torch.device(device)
    main = stream if stream is not None else torch.cuda.current_stream(dev)
    sts = [main]
    for k in range(1, max(1, NVFP4_STREAMS if n_streams is None else n_streams)):
        key = (dev.index or 0, main.cuda_stream, k)
        if key not in _side_streams:
            _side_streams[key] = torch.cuda.Stream(dev)
        sts.append(_side_streams[key])
    for s in sts[1:]:
        s.wait_stream(main)
    return sts


def join_streams(sts: List[torch.cuda.Stream]) -> None:
    """The first stream waits for the others: later work on it -- and any reuse of the memory the
    side streams touched through it -- is ordered after theirs."""
    for s in sts[1:]:
        sts[0].wait_stream(s)


def quantize_nvfp4_many(items: Sequence[Tuple[torch.Tensor, Dict[str, torch.Tensor]]], a: QuantizationArgs,
                        stream=None, n_streams: Optional[int] = None) -> None:
    """``quantize_weight(w, a, out=o)`` for every (w, o) of NVFP4 items, round-robin over
    ``nvfp4_streams`` (each stream with its own sync region).  Qwen3-30B-A3B experts pass
    21.2-21.3 -> 20.2-20.3 ms on 2 streams, 3 streams 21.0 ms, outputs identical
    (profiles/r04w_nv_streams_probe.log)."""
    if not items:
        return
    sts = nvfp4_streams(items[0][0].device, stream, n_streams)
    for i, (w, o) in enumerate(items):
        with torch.cuda.stream(sts[i % len(sts)]):
            quantize_weight(w, a, out=o)
    join_streams(sts)


def fake_quantize(w: torch.Tensor, a: QuantizationArgs, col_scales: Optional[torch.Tensor] = None,
                  out: Optional[torch.Tensor] = None) -> torch.Tensor:
    """``fake_quantize(w)`` with memoryless qparams; with ``col_scales`` s it is AWQ's
    ``Q(W * s) / s`` (llmcompressor _compute_best_scale inner step), one fused pass."""
    _check_dev(w, "weight")
    b, r, c, ld_r, ld_b = _geom(w)
    if out is None:
        out = torch.empty(w.shape, dtype=torch.bfloat16, device=w.device)
    if col_scales is not None:
        col_scales = col_scales.to(device=w.device, dtype=torch.float32).contiguous()
        if col_scales.numel() != c:
            raise ValueError("col_scales must have one entry per input column")
    ca = a.to_c()
    lib = _lib.load()
    ws_n = lib.qz_quantize_workspace_size(b, r, c, ctypes.byref(ca)) + 4 * b + 256
    ws = workspace(ws_n, w.device)
    rc = lib.qz_awq_fake_quant(_ptr(w), b, r, c, ld_r, ld_b, ctypes.byref(ca), _ptr(col_scales), _ptr(out),
                               _ptr(ws), ws.numel(), _stream())
    _lib.check(rc, "qz_awq_fake_quant")
    return out


def fake_quantize_batched(w: torch.Tensor, a: QuantizationArgs, col_scales: torch.Tensor,
                          out: Optional[torch.Tensor] = None) -> torch.Tensor:
    """Q(W_b * s_b) / s_b for a [B, N, K] batch with one scale vector per slice (``col_scales``
    [B, K]): the batched grid step of per-expert AWQ mappings (qz_awq_fake_quant_batched)."""
    _check_dev(w, "weight")
    b, r, c, ld_r, ld_b = _geom(w)
    cs = col_scales.to(device=w.device, dtype=torch.float32).contiguous()
    if w.dim() != 3 or cs.shape != (b, c):
        raise ValueError("fake_quantize_batched: w [B, N, K] and col_scales [B, K]")
    if out is None:
        out = torch.empty(w.shape, dtype=torch.bfloat16, device=w.device)
    ca = a.to_c()
    lib = _lib.load()
    ws_n = lib.qz_quantize_workspace_size(b, r, c, ctypes.byref(ca)) + 4 * b + 256
    ws = workspace(ws_n, w.device)
    rc = lib.qz_awq_fake_quant_batched(_ptr(w), b, r, c, ld_r, ld_b, ctypes.byref(ca), _ptr(cs), c, _ptr(out),
                                       _ptr(ws), ws.numel(), _stream())
    _lib.check(rc, "qz_awq_fake_quant_batched")
    return out


def observe_minmax(w: torch.Tensor, a: QuantizationArgs) -> Tuple[torch.Tensor, torch.Tensor]:
    _check_dev(w, "weight")
    b, r, c, ld_r, ld_b = _geom(w)
    lead = tuple(w.shape[:-2])
    a2 = a if a.strategy != "tensor_group" else QuantizationArgs(
        num_bits=a.num_bits, type=a.type, symmetric=a.symmetric, strategy="group", group_size=a.group_size)
    gshape = n_groups(a2, r, c)
    mn = torch.empty(*lead, *gshape, dtype=torch.bfloat16, device=w.device)
    mx = torch.empty_like(mn)
    ng = mn.numel()
    ws = workspace(8 * ng + 256, w.device)
    ca = a.to_c()
    rc = _lib.load().qz_observe_minmax(_ptr(w), b, r, c, ld_r, ld_b, ctypes.byref(ca), _ptr(mn), _ptr(mx),
                                       _ptr(ws), ws.numel(), _stream())
    _lib.check(rc, "qz_observe_minmax")
    return mn, mx


def calculate_qparams(min_vals: torch.Tensor, max_vals: torch.Tensor, a: QuantizationArgs,
                      global_scale: Optional[torch.Tensor] = None):
    """compressed-tensors ``calculate_qparams`` on device (bf16 min/max in, scale/zp out)."""
    _check_dev(min_vals, "min_vals")
    mn = min_vals.to(torch.bfloat16).contiguous()
    mx = max_vals.to(torch.bfloat16).contiguous()
    scale = torch.empty(mn.shape, dtype=_scale_dtype(a), device=mn.device)
    zp = torch.empty(mn.shape, dtype=torch.int8, device=mn.device)
    gs = None
    if a.is_nvfp4:
        if global_scale is None:
            raise ValueError("NVFP4 qparams need a global_scale")
        gs = global_scale.to(torch.float32).contiguous()
    ca = a.to_c()
    rc = _lib.load().qz_calculate_qparams(_ptr(mn), _ptr(mx), mn.numel(), ctypes.byref(ca), _ptr(gs),
                                          _ptr(scale), _ptr(zp), _stream())
    _lib.check(rc, "qz_calculate_qparams")
    return scale, zp


def quantize(w: torch.Tensor, scale: torch.Tensor, zero_point: Optional[torch.Tensor], a: QuantizationArgs,
             out_fmt: Optional[int] = None, global_scale: Optional[torch.Tensor] = None) -> torch.Tensor:
    """compressed-tensors ``quantize`` with caller-supplied qparams -> codes in ``out_fmt``."""
    _check_dev(w, "weight")
    b, r, c, ld_r, ld_b = _geom(w)
    lead = tuple(w.shape[:-2])
    out_fmt = default_out_fmt(a) if out_fmt is None else out_fmt
    codes = _alloc_codes(out_fmt, a, lead, r, c, w.device)
    ca = a.to_c()
    zp = zero_point.to(torch.int8).contiguous() if zero_point is not None else None
    gs = global_scale.to(torch.float32).contiguous() if global_scale is not None else None
    rc = _lib.load().qz_quantize_qparams(_ptr(w), b, r, c, ld_r, ld_b, ctypes.byref(ca), out_fmt,
                                         _ptr(scale.contiguous()), _ptr(zp), _ptr(gs), _ptr(codes), _stream())
    _lib.check(rc, "qz_quantize_qparams")
    return codes


def dequantize(codes: torch.Tensor, shape, a: QuantizationArgs, scale: torch.Tensor,
               zero_point: Optional[torch.Tensor] = None, global_scale: Optional[torch.Tensor] = None,
               in_fmt: Optional[int] = None) -> torch.Tensor:
    """Decompress codes back to bf16 ``shape`` ([N, K] or [E, N, K])."""
    _check_dev(codes, "codes")
    in_fmt = default_out_fmt(a) if in_fmt is None else in_fmt
    shape = tuple(int(s) for s in shape)
    if len(shape) == 2:
        b, (r, c) = 1, shape
    else:
        b, r, c = shape
    out = torch.empty(shape, dtype=torch.bfloat16, device=codes.device)
    zp = zero_point.to(torch.int8).contiguous() if zero_point is not None else None
    gs = global_scale.to(torch.float32).contiguous() if global_scale is not None else None
    ca = a.to_c()
    rc = _lib.load().qz_dequantize(_ptr(codes.contiguous()), b, r, c, ctypes.byref(ca), in_fmt,
                                   _ptr(scale.contiguous()), _ptr(zp), _ptr(gs), _ptr(out), _stream())
    _lib.check(rc, "qz_dequantize")
    return out


def pack_to_int32(value: torch.Tensor, num_bits: int, packed_dim: int = 1) -> torch.Tensor:
    """compressed-tensors ``pack_to_int32`` (int8 [R, C] -> int32)."""
    _check_dev(value, "value")
    if value.dtype != torch.int8:
        raise ValueError("Tensor must be quantized to torch.int8 before packing")
    if num_bits > 8:
        raise ValueError("Packing is only supported for less than 8 bits")
    v = value.contiguous()
    r, c = v.shape
    pf = 32 // num_bits
    shape = (r, (c + pf - 1) // pf) if packed_dim == 1 else ((r + pf - 1) // pf, c)
    out = torch.empty(shape, dtype=torch.int32, device=v.device)
    rc = _lib.load().qz_pack_int32(_ptr(v), r, c, num_bits, packed_dim, _ptr(out), _stream())
    _lib.check(rc, "qz_pack_int32")
    return out


def _compress_plan(a: QuantizationArgs, has_activation_quant: bool) -> Tuple[bool, Optional[int]]:
    """(int_q, out_fmt) of a module's compressed-tensors format: int8 weights of a W8A8 scheme stay
    unpacked (``weight``), other int schemes are ``pack-quantized`` (4/8-bit packed by the kernel,
    other widths quantized to int8 and packed by ``pack_to_int32``); float schemes use the
    kernel's default output (FP8 bytes / packed FP4)."""
    if a.type != "int":
        return False, None
    int_q = has_activation_quant and a.num_bits == 8
    fmt = _lib.QZ_OUT_INT8 if (int_q or a.num_bits not in (4, 8)) else _lib.QZ_OUT_PACKED_INT32
    return int_q, fmt


def _compressed_tensors(q: Dict[str, torch.Tensor], w_shape, a: QuantizationArgs, int_q: bool,
                        fmt: Optional[int]) -> Dict[str, torch.Tensor]:
    """A quantize_weight result -> the module's on-disk tensors (names pinned by
    scripts/recombine_weights_MiniMax-M2.1.py:54-65)."""
    out: Dict[str, torch.Tensor] = {}
    if a.type == "int":
        codes = q["codes"]
        if fmt == _lib.QZ_OUT_INT8 and not int_q:
            codes = pack_to_int32(codes.reshape(-1, codes.shape[-1]), a.num_bits).reshape(
                *codes.shape[:-1], -1)
        if int_q:
            out["weight"] = codes
        else:
            out["weight_packed"] = codes
            out["weight_shape"] = torch.tensor(list(w_shape[-2:]))
        out["weight_scale"] = q["scale"]
        if not a.symmetric and a.strategy in ("group", "channel"):
            zp = q["zero_point"]
            if int_q:
                out["weight_zero_point"] = zp
            elif zp.dim() == 2:
                out["weight_zero_point"] = pack_to_int32(zp, a.num_bits, packed_dim=0)
            else:
                out["weight_zero_point"] = torch.stack([pack_to_int32(z, a.num_bits, packed_dim=0) for z in zp])
        return out
    if a.num_bits == 8:
        out["weight"] = q["codes"]
        out["weight_scale"] = q["scale"]
    else:
        out["weight_packed"] = q["codes"]
        out["weight_scale"] = q["scale"]
        if a.is_nvfp4:
            gs = q["global_scale"]
            out["weight_global_scale"] = gs if len(w_shape) == 3 else gs.reshape(1)
    return out


def compress_weight(w: torch.Tensor, a: QuantizationArgs, has_activation_quant: bool = False) -> Dict[str, torch.Tensor]:
    """One module's on-disk tensors (names pinned by scripts/recombine_weights_MiniMax-M2.1.py:54-65):
    pack-quantized -> weight_packed/weight_scale/weight_shape[/weight_zero_point];
    float-quantized -> weight/weight_scale; nvfp4/mxfp4-pack-quantized -> weight_packed/weight_scale
    [/weight_global_scale]."""
    int_q, fmt = _compress_plan(a, has_activation_quant)
    return _compressed_tensors(quantize_weight(w, a, out_fmt=fmt), tuple(w.shape), a, int_q, fmt)


def compress_weights(ws: Sequence[torch.Tensor], a: QuantizationArgs,
                     has_activation_quant: bool = False) -> List[Dict[str, torch.Tensor]]:
    """``compress_weight`` over many modules of one scheme -- the compressor's per-module loop
    (ModelCompressor.compress_model, reached from scripts/do_oneshot.py:197).  Same-shape dense
    weights under a single-pass group scheme are quantized in ONE grouped launch per shape
    (qz_quantize_grouped: the ~3 us launch ramp paid once per shape, not once per module); any
    other weight is one launch.  Results are bit-identical to ``compress_weight`` per module."""
    int_q, fmt = _compress_plan(a, has_activation_quant)
    qs = quantize_weights(ws, a, out_fmt=fmt)
    return [_compressed_tensors(q, tuple(w.shape), a, int_q, fmt) for q, w in zip(qs, ws)]


# ------------------------------------------------------------------------------- AWQ
def awq_absmean_accum(x: torch.Tensor, sums: torch.Tensor) -> int:
    """sums[c] += sum_t |x[t, c]| (fp32, deterministic).  Returns the token count added."""
    _check_dev(x, "activations")
    if x.dtype != torch.bfloat16:
        x = x.to(torch.bfloat16)
    x2 = x.reshape(-1, x.shape[-1])
    if x2.stride(-1) != 1:
        x2 = x2.contiguous()
    t, c = x2.shape
    lib = _lib.load()
    ws = stats_workspace(lib.qz_awq_absmean_workspace_size(t, c) + 256, x.device)
    rc = lib.qz_awq_absmean_accum(_ptr(x2), t, c, x2.stride(0), _ptr(sums), _ptr(ws), ws.numel(), _stream())
    _lib.check(rc, "qz_awq_absmean_accum")
    return t


def awq_weight_mean_accum(w: torch.Tensor, group_size: int, wsum: torch.Tensor) -> int:
    """wsum[c] += sum_r |W[r,c]| / (group absmax + 1e-6) (fp64, deterministic: fixed-order
    reduction, ``awq_stats_layout``).  Returns rows added."""
    _check_dev(w, "weight")
    if w.dtype != torch.bfloat16:  # the kernel reads bf16 weights (as every quantize kernel)
        raise ValueError(f"awq_weight_mean_accum: weights must be bfloat16 (got {w.dtype})")
    w2 = w.reshape(-1, w.shape[-1])
    if w2.stride(-1) != 1:
        w2 = w2.contiguous()
    r, c = w2.shape
    lib = _lib.load()
    ws = stats_workspace(lib.qz_awq_weight_mean_workspace_size(r, c, int(group_size)) + 256, w.device)
    rc = lib.qz_awq_weight_mean_accum(_ptr(w2), r, c, w2.stride(0), int(group_size), _ptr(wsum), _ptr(ws), ws.numel(),
                                      _stream())
    _lib.check(rc, "qz_awq_weight_mean_accum")
    return r


STATS_SEGS = 16  # segments per segmented statistics launch (QZ_STATS_SEGS)


def _rows2d(t: torch.Tensor) -> torch.Tensor:
    t2 = t.reshape(-1, t.shape[-1])
    return t2 if t2.stride(-1) == 1 else t2.contiguous()


def _segments(fn_ws, fn_run, single, ts: List[torch.Tensor], outs: List[torch.Tensor], *extra) -> List[int]:
    """Issue ts[i] -> outs[i] as segmented launches of <= STATS_SEGS operands; a batch the C side
    declines (QZ_ERR_FORMAT: a segment off its single call's one-launch plan) runs as single calls,
    which give the same bits."""
    lib = _lib.load()
    counts = []
    for i0 in range(0, len(ts), STATS_SEGS):
        t2 = [_rows2d(t) for t in ts[i0:i0 + STATS_SEGS]]
        o = outs[i0:i0 + STATS_SEGS]
        n, cols = len(t2), t2[0].shape[1]
        rows = (ctypes.c_int64 * n)(*[t.shape[0] for t in t2])
        lds = (ctypes.c_int64 * n)(*[t.stride(0) for t in t2])
        ptrs = (ctypes.c_void_p * n)(*[t.data_ptr() for t in t2])
        optrs = (ctypes.c_void_p * n)(*[x.data_ptr() for x in o])
        need = getattr(lib, fn_ws)(n, rows, cols, *extra)
        rc = _lib.QZ_ERR_FORMAT
        if need:
            ws = stats_workspace(need + 256, t2[0].device)
            rc = getattr(lib, fn_run)(n, ptrs, rows, cols, lds, *extra, optrs, _ptr(ws), ws.numel(), _stream())
        if rc == _lib.QZ_ERR_FORMAT:
            for t, x in zip(t2, o):
                single(t, x)
        else:
            _lib.check(rc, fn_run)
        counts += [t.shape[0] for t in t2]
    return counts


def awq_absmean_segments(xs: List[torch.Tensor], sums: List[torch.Tensor]) -> List[int]:
    """sums[i][c] += sum_t |xs[i][t, c]| for every i in ONE launch (qz_awq_absmean_accum_segments),
    bit-identical to awq_absmean_accum(xs[i], sums[i]) each; the sums must be distinct tensors and
    the operands non-empty bf16 device tensors of one channel count.  Returns the token counts."""
    if not xs:
        return []
    for x, o in zip(xs, sums):
        _check_dev(x, "activations")
        if x.dtype != torch.bfloat16 or x.numel() == 0 or o.dtype != torch.float32 or x.shape[-1] != xs[0].shape[-1] \
                or o.numel() != x.shape[-1] or not o.is_contiguous() or o.device != x.device:
            raise ValueError("awq_absmean_segments: non-empty bf16 operands of one width, contiguous float32 sums "
                             "of that width on the same device")
    return _segments("qz_awq_absmean_segments_workspace_size", "qz_awq_absmean_accum_segments",
                     awq_absmean_accum, xs, sums)


def awq_weight_mean_segments(ws: List[torch.Tensor], group_size: int, wsums: List[torch.Tensor]) -> List[int]:
    """wsums[i][c] += w_mean column sums of ws[i] for every i in ONE launch
    (qz_awq_weight_mean_accum_segments), bit-identical to awq_weight_mean_accum(ws[i], group_size,
    wsums[i]) each; distinct float64 sums, one column count.  Returns the row counts."""
    if not ws:
        return []
    for w, o in zip(ws, wsums):
        _check_dev(w, "weight")
        if w.dtype != torch.bfloat16 or w.numel() == 0 or o.dtype != torch.float64 or w.shape[-1] != ws[0].shape[-1] \
                or o.numel() != w.shape[-1] or not o.is_contiguous() or o.device != w.device:
            raise ValueError("awq_weight_mean_segments: non-empty bf16 weights of one width, contiguous float64 sums "
                             "of that width on the same device")
    g = int(group_size)
    return _segments("qz_awq_weight_mean_segments_workspace_size", "qz_awq_weight_mean_accum_segments",
                     lambda w, o: awq_weight_mean_accum(w, g, o), ws, wsums, g)


def awq_sq_err_accum(a: torch.Tensor, b: torch.Tensor, out: torch.Tensor) -> torch.Tensor:
    """out[0] += sum(f32(bf16(a - b))^2) (f64, deterministic): the AWQ grid loss numerator
    over two bf16 parent outputs of the same shape (qz_awq_sq_err_accum)."""
    _check_dev(a, "a")
    if a.shape != b.shape or a.dtype != torch.bfloat16 or b.dtype != torch.bfloat16:
        raise ValueError("awq_sq_err_accum: a and b must be bf16 tensors of the same shape")
    if out.dtype != torch.float64 or out.numel() < 1 or not out.is_cuda:
        raise ValueError("awq_sq_err_accum: out must be a float64 device tensor")
    a2 = a.reshape(-1, a.shape[-1]) if a.dim() != 1 else a.reshape(1, -1)
    b2 = b.reshape(-1, b.shape[-1]) if b.dim() != 1 else b.reshape(1, -1)
    if a2.stride(-1) != 1:
        a2 = a2.contiguous()
    if b2.stride(-1) != 1:
        b2 = b2.contiguous()
    r, c = a2.shape
    lib = _lib.load()
    ws = workspace(lib.qz_awq_sq_err_workspace_size(r, c) + 256, a.device)
    rc = lib.qz_awq_sq_err_accum(_ptr(a2), _ptr(b2), r, c, a2.stride(0), b2.stride(0), _ptr(out), _ptr(ws),
                                 ws.numel(), _stream())
    _lib.check(rc, "qz_awq_sq_err_accum")
    return out


def awq_sq_err_partials_count(shape) -> int:
    """Number of f64 partial sums one loss over a bf16 output of ``shape`` writes."""
    r = 1
    for d in shape[:-1]:
        r *= int(d)
    return int(_lib.load().qz_awq_sq_err_partials_count(r, int(shape[-1])))


def awq_sq_err_partials(a: torch.Tensor, b: torch.Tensor, part: torch.Tensor) -> None:
    """Stage 1 of ``awq_sq_err_accum`` into ``part`` (a float64 device row of at least
    ``awq_sq_err_partials_count(a.shape)`` entries); reduce later with ``awq_sq_err_reduce``."""
    _check_dev(a, "a")
    if a.shape != b.shape or a.dtype != torch.bfloat16 or b.dtype != torch.bfloat16:
        raise ValueError("awq_sq_err_partials: a and b must be bf16 tensors of the same shape")
    a2 = a.reshape(-1, a.shape[-1]) if a.dim() != 1 else a.reshape(1, -1)
    b2 = b.reshape(-1, b.shape[-1]) if b.dim() != 1 else b.reshape(1, -1)
    if a2.stride(-1) != 1:
        a2 = a2.contiguous()
    if b2.stride(-1) != 1:
        b2 = b2.contiguous()
    r, c = a2.shape
    lib = _lib.load()
    if part.dtype != torch.float64 or not part.is_cuda or part.stride(-1) != 1 or \
            part.numel() < lib.qz_awq_sq_err_partials_count(r, c):
        raise ValueError("awq_sq_err_partials: part must be a contiguous float64 device row of "
                         "awq_sq_err_partials_count(shape) entries")
    rc = lib.qz_awq_sq_err_partials(_ptr(a2), _ptr(b2), r, c, a2.stride(0), b2.stride(0), _ptr(part), _stream())
    _lib.check(rc, "qz_awq_sq_err_partials")


def awq_sq_err_partials_multi(a: torch.Tensor, bs: Sequence[torch.Tensor], part: torch.Tensor) -> None:
    """``awq_sq_err_partials(a, b)`` for up to 8 outputs ``bs`` against one reference ``a`` in one
    launch (``a`` read once): output g's partials go to row g of the 2-D float64 ``part``;
    bit-identical per output.  All tensors dense bf16 of one shape."""
    _check_dev(a, "a")
    if not 1 <= len(bs) <= 8:
        raise ValueError("awq_sq_err_partials_multi: 1 to 8 outputs")
    for b in bs:
        if b.shape != a.shape or b.dtype != torch.bfloat16 or not b.is_contiguous():
            raise ValueError("awq_sq_err_partials_multi: outputs must be contiguous bf16 tensors of a's shape")
    if a.dtype != torch.bfloat16 or not a.is_contiguous():
        raise ValueError("awq_sq_err_partials_multi: a must be a contiguous bf16 tensor")
    if part.dtype != torch.float64 or part.dim() != 2 or part.stride(1) != 1 or part.shape[0] < len(bs):
        raise ValueError("awq_sq_err_partials_multi: part must be a 2-D float64 tensor with a row per output")
    c = a.shape[-1]
    r = a.numel() // c
    lib = _lib.load()
    if part.shape[1] < lib.qz_awq_sq_err_partials_count(r, c):
        raise ValueError("awq_sq_err_partials_multi: part rows shorter than awq_sq_err_partials_count(shape)")
    ptrs = (ctypes.c_void_p * len(bs))(*[b.data_ptr() for b in bs])
    rc = lib.qz_awq_sq_err_partials_multi(_ptr(a), ptrs, len(bs), r, c, _ptr(part), part.stride(0), _stream())
    _lib.check(rc, "qz_awq_sq_err_partials_multi")


def awq_sq_err_reduce(part: torch.Tensor, nb: int, out: torch.Tensor) -> torch.Tensor:
    """out.view(-1)[i] += fixed-order sum of part[i, :nb] for every row i of the 2-D float64
    ``part`` (one launch; bit-identical to ``awq_sq_err_accum`` per loss)."""
    if part.dtype != torch.float64 or part.dim() != 2 or part.stride(1) != 1 or not part.is_cuda:
        raise ValueError("awq_sq_err_reduce: part must be a 2-D float64 device tensor with unit column stride")
    if out.dtype != torch.float64 or not out.is_contiguous() or out.numel() != part.shape[0]:
        raise ValueError("awq_sq_err_reduce: out must be a contiguous float64 tensor with one entry per row")
    if nb > part.shape[1]:
        raise ValueError("awq_sq_err_reduce: nb exceeds the partial rows")
    rc = _lib.load().qz_awq_sq_err_reduce(_ptr(part), part.shape[0], int(nb), part.stride(0), _ptr(out), _stream())
    _lib.check(rc, "qz_awq_sq_err_reduce")
    return out


def awq_grid_scales(x_mean: torch.Tensor, w_mean: Optional[torch.Tensor], ratio: float, duo_scaling: bool,
                    out: Optional[torch.Tensor] = None) -> torch.Tensor:
    x_mean = x_mean.to(torch.float32).contiguous()
    wm = w_mean.to(torch.float32).contiguous() if w_mean is not None else None
    if out is None:
        out = torch.empty_like(x_mean)
    rc = _lib.load().qz_awq_grid_scales(_ptr(x_mean), _ptr(wm), x_mean.numel(), float(ratio), int(duo_scaling),
                                        _ptr(out), _stream())
    _lib.check(rc, "qz_awq_grid_scales")
    return out


def awq_grid_scales_batched(x_mean: torch.Tensor, w_mean: Optional[torch.Tensor], ratio: float, duo_scaling: bool,
                            out: Optional[torch.Tensor] = None) -> torch.Tensor:
    """``awq_grid_scales`` for [B, C] stacks of independent mappings (one launch)."""
    x_mean = x_mean.to(torch.float32).contiguous()
    wm = w_mean.to(torch.float32).contiguous() if w_mean is not None else None
    if x_mean.dim() != 2 or (wm is not None and wm.shape != x_mean.shape):
        raise ValueError("awq_grid_scales_batched: x_mean / w_mean must be [B, C]")
    if out is None:
        out = torch.empty_like(x_mean)
    rc = _lib.load().qz_awq_grid_scales_batched(_ptr(x_mean), _ptr(wm), x_mean.shape[0], x_mean.shape[1],
                                                float(ratio), int(duo_scaling), _ptr(out), _stream())
    _lib.check(rc, "qz_awq_grid_scales_batched")
    return out


def scale_columns_(w: torch.Tensor, s: torch.Tensor, divide: bool = False) -> torch.Tensor:
    """In place W[:, c] *= s[c] (or /=), bf16-rounded (AWQ _apply_smoothing, balance layers)."""
    _check_dev(w, "weight")
    s = s.to(device=w.device, dtype=torch.float32).contiguous()
    if w.dim() == 3 and not (w.stride(0) == w.shape[1] * w.stride(1)):
        for wi in w:  # strided batch of slices (fused experts): one launch per slice, in place
            scale_columns_(wi, s, divide)
        return w
    w2 = w.view(-1, w.shape[-1]) if w.dim() == 3 else (w if w.dim() == 2 else w.reshape(1, -1))
    if w2.stride(-1) != 1:
        raise ValueError("scale_columns_: rows must be contiguous")
    rc = _lib.load().qz_scale_columns(_ptr(w2), w2.shape[0], w2.shape[1], w2.stride(0), _ptr(s), int(divide),
                                      _stream())
    _lib.check(rc, "qz_scale_columns")
    return w


def scale_rows_(w: torch.Tensor, s: torch.Tensor, divide: bool = True) -> torch.Tensor:
    """In place W[r, :] /= s[r] (or *=): smooth Linear's output rows, 1-D norm weights, biases."""
    _check_dev(w, "weight")
    w2 = w.reshape(-1, 1) if w.dim() == 1 else w
    s = s.to(device=w.device, dtype=torch.float32).contiguous()
    rc = _lib.load().qz_scale_rows(_ptr(w2), w2.shape[0], w2.shape[1], w2.stride(0), _ptr(s), int(divide),
                                   _stream())
    _lib.check(rc, "qz_scale_rows")
    return w


def moe_combine(expert_out: torch.Tensor, top_k_weights: torch.Tensor, perm: torch.Tensor, src: torch.Tensor,
                tokens: int, top_k: int, out: Optional[torch.Tensor] = None) -> torch.Tensor:
    """qz_moe_combine: the eager experts loop's weighting and ascending-expert bf16 accumulation
    in one pass.  ``expert_out`` [tokens * top_k, hidden] bf16 in expert-sorted order,
    ``top_k_weights`` the router's [tokens, top_k] weights (bf16 or f32), ``perm`` the sort
    permutation (sorted row -> flat (token, slot)), ``src`` the sorted row of each token's j-th
    expert in ascending id ([tokens * top_k]).  Returns [tokens, hidden] bf16."""
    _check_dev(expert_out, "expert_out")
    if expert_out.dtype != torch.bfloat16 or top_k_weights.dtype not in (torch.bfloat16, torch.float32):
        raise TypeError(f"qz_moe_combine: bf16 expert outputs and bf16/f32 weights, got {expert_out.dtype}, "
                        f"{top_k_weights.dtype}")
    d = expert_out.contiguous()
    w = top_k_weights.reshape(-1).contiguous()
    perm = perm.to(torch.int64).contiguous()
    src = src.to(torch.int64).contiguous()
    if d.dim() != 2 or d.shape[0] != tokens * top_k or w.numel() != tokens * top_k or perm.numel() != d.shape[0] \
            or src.numel() != d.shape[0]:
        raise ValueError(f"qz_moe_combine: shapes {tuple(d.shape)}, weights {w.numel()}, perm {perm.numel()}, "
                         f"src {src.numel()} for {tokens} tokens x top-{top_k}")
    if out is None:
        out = torch.empty(tokens, d.shape[1], dtype=torch.bfloat16, device=d.device)
    rc = _lib.load().qz_moe_combine(_ptr(d), d.shape[0], d.shape[1], _ptr(w), int(w.dtype == torch.float32),
                                    _ptr(perm), _ptr(src), tokens, top_k, _ptr(out), _stream())
    _lib.check(rc, "qz_moe_combine")
    return out


def moe_silu_mul(gate_up: torch.Tensor, out: Optional[torch.Tensor] = None) -> torch.Tensor:
    """qz_moe_silu_mul: ``silu(gate) * up`` for a [rows, 2 * inter] bf16 gate/up GEMM output
    (gate = the first half of the columns) into a dense [rows, inter] bf16 tensor."""
    _check_dev(gate_up, "gate_up")
    if gate_up.dtype != torch.bfloat16 or gate_up.dim() != 2 or gate_up.stride(1) != 1 or gate_up.shape[1] % 2:
        raise ValueError(f"qz_moe_silu_mul: a row-major [rows, 2 * inter] bf16 tensor, got {gate_up.dtype} "
                         f"{tuple(gate_up.shape)} strides {gate_up.stride()}")
    rows, inter = gate_up.shape[0], gate_up.shape[1] // 2
    if out is None:
        out = torch.empty(rows, inter, dtype=torch.bfloat16, device=gate_up.device)
    if out.dtype != torch.bfloat16 or tuple(out.shape) != (rows, inter) or not out.is_contiguous():
        raise ValueError(f"qz_moe_silu_mul: out must be a dense [{rows}, {inter}] bf16 tensor")
    rc = _lib.load().qz_moe_silu_mul(_ptr(gate_up), rows, inter, gate_up.stride(0), _ptr(out), _stream())
    _lib.check(rc, "qz_moe_silu_mul")
    return out


def silu_mul(gate: torch.Tensor, up: torch.Tensor, out: Optional[torch.Tensor] = None) -> torch.Tensor:
    """qz_silu_mul: ``silu(gate) * up`` for two bf16 [rows, inter] tensors (row-major, any row
    stride) into a dense [rows, inter] bf16 tensor (leading dims of the inputs are flattened)."""
    _check_dev(gate, "gate")
    if gate.dtype != torch.bfloat16 or up.dtype != torch.bfloat16 or gate.shape != up.shape:
        raise ValueError(f"qz_silu_mul: two bf16 tensors of one shape, got {gate.dtype} {tuple(gate.shape)}, "
                         f"{up.dtype} {tuple(up.shape)}")
    shape = gate.shape
    g2, u2 = gate.reshape(-1, shape[-1]), up.reshape(-1, shape[-1])
    if g2.stride(1) != 1 or u2.stride(1) != 1:
        raise ValueError("qz_silu_mul: rows must be contiguous")
    if out is None:
        out = torch.empty(shape, dtype=torch.bfloat16, device=gate.device)
    if out.dtype != torch.bfloat16 or out.shape != shape or not out.is_contiguous():
        raise ValueError(f"qz_silu_mul: out must be a dense {tuple(shape)} bf16 tensor")
    rc = _lib.load().qz_silu_mul(_ptr(g2), g2.stride(0), _ptr(u2), u2.stride(0), g2.shape[0], g2.shape[1],
                                 _ptr(out), _stream())
    _lib.check(rc, "qz_silu_mul")
    return out


def rmsnorm128(x: torch.Tensor, weight: torch.Tensor, eps: float, out: Optional[torch.Tensor] = None) -> torch.Tensor:
    """qz_rmsnorm128: Qwen3RMSNorm's forward over the last dim (128) of a bf16 tensor whose rows
    are contiguous (row stride a multiple of 4 elements, 8-B aligned), with a bf16 weight."""
    _check_dev(x, "x")
    if x.dtype != torch.bfloat16 or weight.dtype != torch.bfloat16 or x.shape[-1] != 128 or weight.numel() != 128:
        raise ValueError(f"qz_rmsnorm128: bf16 [..., 128] input and bf16 [128] weight, got {x.dtype} "
                         f"{tuple(x.shape)}, {weight.dtype} {tuple(weight.shape)}")
    x2 = x.reshape(-1, 128)
    if x2.stride(1) != 1:
        raise ValueError("qz_rmsnorm128: rows must be contiguous")
    w = weight.contiguous()
    if out is None:
        out = torch.empty(x.shape, dtype=torch.bfloat16, device=x.device)
    rc = _lib.load().qz_rmsnorm128(_ptr(x2), x2.shape[0], x2.stride(0), _ptr(w), float(eps), _ptr(out), _stream())
    _lib.check(rc, "qz_rmsnorm128")
    return out


def rotary128(x: torch.Tensor, cos: torch.Tensor, sin: torch.Tensor) -> torch.Tensor:
    """qz_rotary128: ``x * cos + rotate_half(x) * sin`` (apply_rotary_pos_emb with unsqueeze_dim=1)
    for a bf16 [B, H, T, 128] ``x`` at any strides and bf16 [B, T, 128] ``cos`` / ``sin``; the
    output has ``x``'s memory layout (as PyTorch's elementwise result would)."""
    _check_dev(x, "x")
    if (x.dim() != 4 or x.shape[-1] != 128 or cos.shape != sin.shape or cos.dim() != 3
            or cos.shape[0] not in (1, x.shape[0]) or cos.shape[1] != x.shape[2] or cos.shape[2] != 128
            or any(t.dtype != torch.bfloat16 for t in (x, cos, sin)) or x.stride(-1) != 1
            or cos.stride() != sin.stride() or cos.stride(-1) != 1):
        raise ValueError(f"qz_rotary128: bf16 x [B, H, T, 128] and cos / sin [B, T, 128], got {tuple(x.shape)} "
                         f"{x.dtype}, {tuple(cos.shape)} {cos.dtype}")
    out = torch.empty_like(x)
    B, H, T, _ = x.shape
    cb = cos.stride(0) if cos.shape[0] == B and B > 1 else 0
    rc = _lib.load().qz_rotary128(_ptr(x), B, H, T, x.stride(0), x.stride(1), x.stride(2), _ptr(cos), _ptr(sin),
                                  cb, cos.stride(1), _ptr(out), out.stride(0), out.stride(1), out.stride(2),
                                  _stream())
    _lib.check(rc, "qz_rotary128")
    return out


class PreparedQuantize:
    """A qz_quantize call with every argument marshalled once (bench / tight host loops):
    ``run(w)`` costs one ctypes call + one kernel launch.  Graph-capturable."""

    def __init__(self, w_like: torch.Tensor, a: QuantizationArgs, out: Dict[str, torch.Tensor],
                 out_fmt: Optional[int] = None):
        self.geom = _geom(w_like)
        b, r, c, _, _ = self.geom
        self.ca = a.to_c()
        self.out_fmt = default_out_fmt(a) if out_fmt is None else out_fmt
        self.lib = _lib.load()
        n = self.lib.qz_quantize_workspace_size(b, r, c, ctypes.byref(self.ca))
        self.ws = torch.empty(max(n, 256), dtype=torch.uint8, device=w_like.device)
        self.out = out
        self._args_tail = (ctypes.byref(self.ca), self.out_fmt, _ptr(out["codes"]), _ptr(out["scale"]),
                           _ptr(out.get("zero_point")), _ptr(out.get("global_scale")), _ptr(self.ws),
                           self.ws.numel())

    def run(self, w: torch.Tensor, stream=None) -> None:
        b, r, c, ld_r, ld_b = self.geom
        st = _P(stream.cuda_stream) if stream is not None else _stream()
        rc = self.lib.qz_quantize(_P(w.data_ptr()), b, r, c, ld_r, ld_b, *self._args_tail, st)
        if rc:
            _lib.check(rc, "qz_quantize")

    def prepare_many(self, ws: Sequence[torch.Tensor],
                     outs: Optional[Sequence[Dict[str, torch.Tensor]]] = None) -> Callable[..., None]:
        """Marshal a qz_quantize_many call over every weight of ``ws`` (same geometry as
        ``w_like``) into the prepared outputs (or into ``outs[i]`` for weight i); the returned
        ``go(stream=None)`` enqueues one launch per weight from ONE host call."""
        b, r, c, ld_r, ld_b = self.geom
        for w in ws:
            if _geom(w) != self.geom or not w.is_cuda:
                raise ValueError("prepare_many: every weight needs the prepared geometry and a device")
        n = len(ws)

        if outs is not None and len(outs) != n:
            raise ValueError("prepare_many: one output dict per weight")

        def arr(key):
            ts = [self.out.get(key)] * n if outs is None else [o.get(key) for o in outs]
            return None if ts[0] is None else (ctypes.c_void_p * n)(*[t.data_ptr() for t in ts])

        args = (n, (ctypes.c_void_p * n)(*[w.data_ptr() for w in ws]), arr("codes"),
                arr("scale"), arr("zero_point"), arr("global_scale"),
                b, r, c, ld_r, ld_b, ctypes.byref(self.ca), self.out_fmt, _P(self.ws.data_ptr()), self.ws.numel())
        keep = list(ws) + list(outs or [])  # the pointers stay valid while the closure lives

        def go(stream=None) -> None:
            st = _P(stream.cuda_stream) if stream is not None else _stream()
            rc = self.lib.qz_quantize_many(*args, st)
            if rc:
                _lib.check(rc, "qz_quantize_many")
        go.weights = keep
        return go


def unpack_zero_points(packed: torch.Tensor, num_bits: int, shape) -> torch.Tensor:
    """Inverse of pack_to_int32(zp, packed_dim=0): int32 [ceil(R*bits/32), C] -> int8 [R, C]."""
    pf = 32 // num_bits
    shifts = torch.arange(pf, device=packed.device, dtype=torch.int32).view(1, -1, 1) * num_bits
    u = (packed.unsqueeze(1) >> shifts) & ((1 << num_bits) - 1)
    u = u.reshape(-1, packed.shape[-1])[: int(shape[0])]
    return (u - (1 << (num_bits - 1))).to(torch.int8)
