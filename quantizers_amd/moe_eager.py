"""transformers' fused MoE experts in the reference's arithmetic, at grouped-GEMM speed.

The reference pins transformers 4.57, whose MoE blocks loop over per-expert Linear modules: per
routed expert, gather its tokens, gate / up GEMM, ``act(gate) * up``, down GEMM, times the
routing weight, ``index_add_`` into a bf16 accumulator -- so every token sums its top-k
contributions in ascending expert order with a bf16 rounding after each add.  transformers 5
keeps that loop as the experts' ``eager`` form (with two host syncs per expert) and defaults to
a ``grouped_mm`` form that sums the top-k contributions in f32 -- different bits in about half
of the outputs (``profiles/r02at_fast_eager.log``).

``FastEagerExperts`` computes the eager result with two grouped GEMMs (tokens sorted by expert:
hipBLASLt gives every row the same bits as the per-expert GEMM), the routing weight, and k
sequential bf16 adds in ascending expert order -- on the GPU ``act(gate) * up`` as one
qz_moe_silu_mul pass and the last three as one qz_moe_combine pass -- no host sync, ~10 launches instead of ~9 per expert.  The first call per input shape is checked bit for bit against the module's own eager
forward; a mismatch makes that module use the eager forward for the rest of the pass.
Decision D15: the AWQ pass runs MoE experts in this eager arithmetic."""
from __future__ import annotations

import contextlib
import inspect
import logging
import os
from typing import Callable, Dict, Optional, Tuple

import torch
from torch import nn

from . import ops

log = logging.getLogger(__name__)

FAST_EAGER = True  # False: the eager loop itself (same bits, ~2x slower)
PLANNED = os.environ.get("QZ_PLANNED_EXPERTS", "1") == "1"  # A/B knob: per-expert GEMMs from a grid's fixed routing
FUSED_COMBINE = os.environ.get("QZ_MOE_FUSED_COMBINE", "1") == "1"  # A/B knob: qz_moe_combine for the weighted adds


FUSED_ACT = os.environ.get("QZ_MOE_FUSED_ACT", "1") == "1"  # A/B knob: qz_moe_silu_mul for act_fn(gate) * up
_ACT_OK: Dict[torch.device, bool] = {}  # qz_moe_silu_mul verified against the composed ops (per device)


def _act_mul(m: nn.Module, gu: torch.Tensor, out: Optional[torch.Tensor] = None) -> torch.Tensor:
    """``act_fn(gate) * up`` of the [rows, 2 * inter] gate/up GEMM output.  For a SiLU on bf16 GPU
    tensors: one qz_moe_silu_mul pass instead of two strided ones -- compared bit for bit with
    the composed ops on the first non-empty call per device (its exp is the device library's),
    and never used again if they differ."""
    gate, up = gu.chunk(2, dim=-1)
    if (FUSED_ACT and gu.is_cuda and gu.dtype == torch.bfloat16 and gu.is_contiguous() and gu.numel()
            and type(m.act_fn).__name__ in ("SiLUActivation", "SiLU") and not getattr(m.act_fn, "inplace", False)):
        ok = _ACT_OK.get(gu.device)
        if ok is None:
            want = m.act_fn(gate) * up
            ok = _ACT_OK[gu.device] = _bits_equal(ops.moe_silu_mul(gu), want)
            if not ok:
                log.info("MoE: qz_moe_silu_mul differs from the composed silu * up on %s; composed ops kept", gu.device)
            return want if out is None else out.copy_(want)
        if ok:
            return ops.moe_silu_mul(gu, out=out)
    return m.act_fn(gate) * up if out is None else torch.mul(m.act_fn(gate), up, out=out)


def _fused(d: torch.Tensor, top_k_weights: torch.Tensor, hidden_states: torch.Tensor) -> bool:
    """The weighting, reorder and k bf16 adds as one qz_moe_combine pass (same roundings, same
    order: bit-identical to the composed ops, and checked against the eager loop like the rest of
    this form); the composed PyTorch ops otherwise (CPU tensors, other dtypes)."""
    return (FUSED_COMBINE and d.is_cuda and d.dtype == torch.bfloat16 and hidden_states.dtype == torch.bfloat16
            and top_k_weights.dtype in (torch.bfloat16, torch.float32))


def eager_forward(module: nn.Module) -> Optional[Callable]:
    """The experts class's eager forward (the function transformers' ``use_experts_implementation``
    wraps), or None for a module that is not a transformers fused-experts module."""
    if not (type(module).__name__.endswith("Experts") and hasattr(module, "gate_up_proj")
            and hasattr(module, "down_proj") and hasattr(module, "act_fn") and hasattr(module, "num_experts")):
        return None
    if getattr(module, "has_bias", False) or getattr(module, "is_transposed", False) \
            or not getattr(module, "is_concatenated", True) or not getattr(module, "has_gate", True):
        return None
    fwd = type(module).forward
    fwd = getattr(fwd, "__wrapped__", fwd)
    try:
        params = list(inspect.signature(fwd).parameters)
    except (TypeError, ValueError):
        return None
    return fwd if params[1:] == ["hidden_states", "top_k_index", "top_k_weights"] else None


def _bits_equal(a: torch.Tensor, b: torch.Tensor) -> bool:
    if a.dtype != b.dtype or a.shape != b.shape:
        return False
    if a.dtype in (torch.bfloat16, torch.float16):
        return torch.equal(a.view(torch.int16), b.view(torch.int16))
    return torch.equal(a, b)


def fast_eager(m: nn.Module, hidden_states: torch.Tensor, top_k_index: torch.Tensor,
               top_k_weights: torch.Tensor) -> torch.Tensor:
    """The eager experts result without host syncs (see the module docstring)."""
    t, k = top_k_index.shape
    flat = top_k_index.reshape(-1).to(torch.int64)
    _, perm = torch.sort(flat, stable=True)  # (token, slot) pairs grouped by expert
    counts = torch.zeros(m.num_experts, dtype=torch.int64, device=flat.device).scatter_add_(
        0, flat, torch.ones_like(flat))
    offs = counts.cumsum(0).to(torch.int32)
    xg = hidden_states[perm // k]
    h = _act_mul(m, nn.functional.grouped_mm(xg, m.gate_up_proj.transpose(-2, -1), offs=offs))
    d = nn.functional.grouped_mm(h, m.down_proj.transpose(-2, -1), offs=offs)
    order = torch.argsort(top_k_index, dim=-1)  # each token's experts in ascending id: the eager add order
    if _fused(d, top_k_weights, hidden_states):
        inv = torch.empty_like(perm)
        inv[perm] = torch.arange(perm.numel(), device=perm.device)
        base = torch.arange(t, device=perm.device)[:, None] * k
        return ops.moe_combine(d, top_k_weights, perm, inv[(base + order).reshape(-1)], t, k)
    d = d * top_k_weights.reshape(-1)[perm][:, None]
    contrib = torch.empty_like(d)
    contrib[perm] = d
    contrib = contrib.view(t, k, -1)
    contrib = torch.gather(contrib, 1, order[:, :, None].expand(-1, -1, contrib.shape[-1]))
    final = torch.zeros_like(hidden_states)
    for j in range(k):
        final = final + contrib[:, j].to(final.dtype)
    return final


# Routing plans of the active ``fixed_routing`` context: (module, input) -> host expert bounds
_FIXED: Optional[Dict[Tuple, Dict]] = None


@contextlib.contextmanager
def fixed_routing():
    """Inside, the experts' routing does not change between forwards: an AWQ grid whose balance
    layers are all expert weights re-runs the MoE block on the same cached inputs through the
    same router, so the routing of the first grid forward holds for all of them.  The first
    forward turns the routing into host-side expert bounds (one host sync per grid) and every
    forward then runs the per-expert GEMMs from those bounds (``planned_eager``) -- torch's
    ``grouped_mm`` on ROCm reads its group offsets on the host at every call, which drains the
    GPU twice per forward."""
    global _FIXED
    prev, _FIXED = _FIXED, {}
    try:
        yield
    finally:
        _FIXED = prev


def _plan(m: nn.Module, top_k_index: torch.Tensor) -> Dict:
    k = top_k_index.shape[1]
    flat = top_k_index.reshape(-1).to(torch.int64)
    _, perm = torch.sort(flat, stable=True)  # (token, slot) pairs grouped by expert
    counts = torch.zeros(m.num_experts, dtype=torch.int64, device=flat.device).scatter_add_(
        0, flat, torch.ones_like(flat))
    bounds = [0] + counts.cumsum(0).tolist()  # the one host sync
    # row of the expert-sorted output that lands in (token t, j-th expert in ascending id): the
    # scatter back to (token, slot) order and the gather into ascending-expert order composed
    # into ONE index, so the forward moves the [t * k, H] contributions once instead of twice
    order = torch.argsort(top_k_index, dim=-1)
    inv = torch.argsort(perm)
    base = torch.arange(top_k_index.shape[0], device=flat.device)[:, None] * k
    src = inv[(base + order).reshape(-1)]
    return {"perm": perm, "tok": perm // k, "bounds": bounds, "src": src}


EXPERT_STREAMS = int(os.environ.get("QZ_EXPERT_STREAMS", "4"))  # concurrent per-expert GEMM streams
_streams: Dict[torch.device, list] = {}


def _side_streams(dev: torch.device) -> list:
    ss = _streams.get(dev)
    if ss is None or len(ss) != EXPERT_STREAMS:
        ss = _streams[dev] = [torch.cuda.Stream(dev) for _ in range(EXPERT_STREAMS)]
    return ss


def _expert_mms(x: torch.Tensor, w: torch.Tensor, out: torch.Tensor, b, n: int) -> list:
    """The per-expert GEMM operands out[rows of e] = x[rows of e] @ w[e]^T of every routed expert,
    dealt round-robin into ``n`` lists (one per stream).  Built once per plan: the views stay
    valid because the plan's buffers and the expert parameters are rewritten in place."""
    lists = [[] for _ in range(n)]
    for e in range(w.shape[0]):
        if b[e + 1] > b[e]:
            lists[e % n].append((x[b[e]:b[e + 1]], w[e].t(), out[b[e]:b[e + 1]], b[e], b[e + 1], e))
    return lists


def _run_mms(lists: list, dev: torch.device) -> None:
    """Issue the GEMMs of ``_expert_mms``.  A routed expert's GEMM is small (~2k rows: a few dozen
    output tiles on a 256-CU part), so the lists run on EXPERT_STREAMS streams side by side, each
    list issued in one go from its stream; every GEMM is the same call on the same operands
    whichever stream runs it, so the bits do not change."""
    if len(lists) == 1:
        for x, wt, o, *_ in lists[0]:
            torch.mm(x, wt, out=o)
        return
    main = torch.cuda.current_stream(dev)
    ss = _side_streams(dev)
    for st in ss:
        st.wait_stream(main)
    for st, items in zip(ss, lists):
        with torch.cuda.stream(st):
            for x, wt, o, *_ in items:
                torch.mm(x, wt, out=o)
    for st in ss:
        main.wait_stream(st)


DIRECT_GEMMS = os.environ.get("QZ_DIRECT_EXPERT_GEMMS", "1") == "1"  # A/B knob: qz_expert_gemms for the planned GEMMs
# hipBLASLt workspace limit of the direct GEMMs: torch's (HIPBLASLT_WORKSPACE_SIZE / CUBLASLT_WORKSPACE_SIZE
# in KiB), else its ROCm default; the algorithm choice depends on it, and each plan verifies the bits
_WS_BYTES = int(os.environ.get("HIPBLASLT_WORKSPACE_SIZE", os.environ.get("CUBLASLT_WORKSPACE_SIZE", 76 * 1024))) * 1024
_ws: Dict[int, torch.Tensor] = {}  # stream handle -> its hipBLASLt workspace


def _direct_spec(bounds, n: int) -> list:
    """Per stream: the (first row, end row, expert) arrays of the routed experts' GEMMs for
    qz_expert_gemms, experts dealt round-robin over ``n`` streams as in ``_expert_mms``."""
    import numpy as np
    b = np.asarray(bounds, dtype=np.int64)
    es = np.nonzero(b[1:] > b[:-1])[0]
    spec = []
    for st in range(n):
        sel = es[es % n == st]
        spec.append((np.ascontiguousarray(b[sel]), np.ascontiguousarray(b[sel + 1]), sel.astype(np.int32)))
    return spec


_BOUND: list = []  # [True / False] once qz_expert_gemms_library has been called


def bind_hipblaslt(lib) -> bool:
    """Bind qz_expert_gemms to PyTorch's own hipBLASLt (torch/lib/libhipblaslt.so, already loaded
    by libtorch_hip) once per process; on refusal log why (qz_expert_gemms_status) and return
    False -- the callers then keep torch.mm per expert."""
    if not _BOUND:
        path = os.path.join(os.path.dirname(torch.__file__), "lib", "libhipblaslt.so")
        rc = lib.qz_expert_gemms_library(path.encode())
        _BOUND.append(rc == 0)
        if rc:
            log.warning("MoE: qz_expert_gemms cannot use torch's hipBLASLt: %s; torch.mm per expert",
                        lib.qz_expert_gemms_status().decode())
    return _BOUND[0]


def _run_direct(spec: list, x: torch.Tensor, w: torch.Tensor, out: torch.Tensor) -> None:
    """The GEMMs of ``_expert_mms`` through qz_expert_gemms: one C call per stream, GIL released."""
    from . import _lib
    lib, dev = _lib.load(), x.device
    if not bind_hipblaslt(lib):
        raise RuntimeError(lib.qz_expert_gemms_status().decode())
    main = torch.cuda.current_stream(dev)
    ss = _side_streams(dev) if len(spec) > 1 else [main]
    for st in ss:
        if st is not main:
            st.wait_stream(main)
    for st, (r0, r1, ex) in zip(ss, spec):
        if not len(r0):
            continue
        wsb = _ws.get(st.cuda_stream)  # one hipBLASLt workspace per stream (kernels on a stream serialise)
        if wsb is None:
            wsb = _ws[st.cuda_stream] = torch.empty(_WS_BYTES, dtype=torch.uint8, device=dev)
        rc = lib.qz_expert_gemms(x.data_ptr(), x.stride(0), w.data_ptr(), w.stride(0), w.stride(1), w.shape[1],
                                 w.shape[2], out.data_ptr(), out.stride(0), r0.ctypes.data, r1.ctypes.data,
                                 ex.ctypes.data, len(r0), wsb.data_ptr(), _WS_BYTES, st.cuda_stream)
        if rc:
            raise _lib.QzError(f"qz_expert_gemms: {lib.qz_strerror(rc).decode()} "
                               f"({lib.qz_expert_gemms_status().decode()})")
    for st in ss:
        if st is not main:
            main.wait_stream(st)


def _plan_buffers(m: nn.Module, hidden_states: torch.Tensor, p: Dict, streams: int) -> Dict:
    """The planned forward's intermediates, allocated once per plan.  The per-expert GEMMs run
    either as one ``torch.mm`` per routed expert on precomputed operand views (built on first
    use) or, on the GPU, as one qz_expert_gemms call per stream (verified against torch.mm for
    every GEMM problem it has not run before)."""
    rows, dev, dt = p["tok"].numel(), hidden_states.device, hidden_states.dtype
    n = streams if hidden_states.is_cuda else 1
    buf = {"xg": torch.empty(rows, hidden_states.shape[1], dtype=dt, device=dev),
           "gu": torch.empty(rows, m.gate_up_proj.shape[1], dtype=dt, device=dev),
           "h": torch.empty(rows, m.gate_up_proj.shape[1] // 2, dtype=dt, device=dev),
           "d": torch.empty(rows, m.down_proj.shape[1], dtype=dt, device=dev), "n": n, "bounds": p["bounds"]}
    buf["w1"], buf["w2"] = m.gate_up_proj, m.down_proj
    direct = (DIRECT_GEMMS and hidden_states.is_cuda and dt == torch.bfloat16
              and m.gate_up_proj.dtype == dt and m.down_proj.dtype == dt
              and all(t.stride(-1) == 1 for t in (m.gate_up_proj, m.down_proj)))
    buf["direct"] = None if direct else False  # None: to be verified on the first forward
    if direct:
        buf["spec1"] = buf["spec2"] = _direct_spec(p["bounds"], n)
    buf["key"] = (dev, dt, tuple(hidden_states.shape), n)
    return buf


def _torch_mms(buf: Dict, which: int) -> None:
    lists = buf.get(f"mm{which}")
    if lists is None:
        x, w, out = (buf["xg"], buf["w1"], buf["gu"]) if which == 1 else (buf["h"], buf["w2"], buf["d"])
        lists = buf[f"mm{which}"] = _expert_mms(x, w, out, buf["bounds"], buf["n"])
    _run_mms(lists, buf["xg"].device)


_DIRECT_LOGGED = [False]
_VERIFIED: set = set()  # (device, m, n, k, strides) GEMM problems whose qz_expert_gemms bits equal torch.mm's


def _problems(spec: list, x: torch.Tensor, w: torch.Tensor, out: torch.Tensor) -> set:
    base = (x.device, w.shape[1], w.shape[2], x.stride(0), w.stride(1), out.stride(0))
    return {base + (int(a1 - a0),) for r0, r1, _ in spec for a0, a1 in zip(r0, r1)}


def _gemms(buf: Dict, which: int, x: torch.Tensor, w: torch.Tensor, out: torch.Tensor) -> None:
    """GEMM set ``which`` (1: gate/up, 2: down) of the plan.  A GEMM problem (shape, strides) the
    direct path has not run before is verified first: the set runs both ways and the direct
    path is kept only if its output equals torch.mm's bit for bit (a GEMM's bits depend only on
    its problem and data, so one match per problem suffices)."""
    spec = buf.get(f"spec{which}")
    if buf["direct"] is None:
        new = _problems(spec, x, w, out) - _VERIFIED
        if not new:
            buf[f"ok{which}"] = True
        else:
            _torch_mms(buf, which)
            want = out.clone()
            try:
                _run_direct(spec, x, w, out)
                ok = _bits_equal(out, want)
            except RuntimeError as e:
                log.info("MoE: qz_expert_gemms unavailable (%s); torch.mm per expert", e)
                ok = False
            if not ok:
                out.copy_(want)
                log.info("MoE: qz_expert_gemms differs from torch.mm at %s; torch.mm per expert", tuple(out.shape))
                buf["direct"] = False
                return
            _VERIFIED.update(new)
            buf[f"ok{which}"] = True
            if which == 2 and not _DIRECT_LOGGED[0]:
                _DIRECT_LOGGED[0] = True
                log.info("MoE: per-expert GEMMs through qz_expert_gemms (each new GEMM problem checked bit for "
                         "bit against torch.mm first)")
            if buf.get("ok1") and buf.get("ok2"):
                buf["direct"] = True
            return
        if buf.get("ok1") and buf.get("ok2"):
            buf["direct"] = True
    if buf["direct"] is False:
        _torch_mms(buf, which)
        return
    _run_direct(spec, x, w, out)


def planned_eager(m: nn.Module, hidden_states: torch.Tensor, top_k_index: torch.Tensor,
                  top_k_weights: torch.Tensor, p: Dict, streams: Optional[int] = None) -> torch.Tensor:
    """``fast_eager`` with the expert bounds on the host: one GEMM per routed expert over its
    rows of the expert-sorted tokens (the eager loop's per-expert GEMM shapes), no host sync.
    ``streams``: the per-expert GEMMs spread over that many streams (default EXPERT_STREAMS; 1 =
    the caller's stream, for calls already running side by side on their own streams)."""
    t, k = top_k_index.shape
    n = EXPERT_STREAMS if streams is None else streams
    buf = p.get("buf")
    if buf is None or buf["key"] != (hidden_states.device, hidden_states.dtype, tuple(hidden_states.shape), n):
        buf = p["buf"] = _plan_buffers(m, hidden_states, p, n)
    xg, gu, h, d = buf["xg"], buf["gu"], buf["h"], buf["d"]
    torch.index_select(hidden_states, 0, p["tok"], out=xg)
    _gemms(buf, 1, xg, m.gate_up_proj, gu)
    _act_mul(m, gu, out=h)
    _gemms(buf, 2, h, m.down_proj, d)
    if _fused(d, top_k_weights, hidden_states):
        return ops.moe_combine(d, top_k_weights, p["perm"], p["src"], t, k)
    d = d * top_k_weights.reshape(-1)[p["perm"]][:, None]
    contrib = d.index_select(0, p["src"]).view(t, k, -1)
    final = torch.zeros_like(hidden_states)
    for j in range(k):
        final = final + contrib[:, j].to(final.dtype)
    return final


class FastEagerExperts:
    """Instance-level forward for one experts module (see the module docstring)."""

    checked: Dict[Tuple, bool] = {}  # (class, shape, dtype) -> fast path verified; shared per pass
    planned_checked: Dict[Tuple, bool] = {}  # the same for planned_eager (checked against fast_eager)

    def __init__(self, module: nn.Module, eager: Callable):
        self.m = module
        self.eager = eager

    def forward(self, hidden_states, top_k_index, top_k_weights):
        if not FAST_EAGER or not hasattr(nn.functional, "grouped_mm"):
            return self.eager(self.m, hidden_states, top_k_index, top_k_weights)
        key = (type(self.m).__name__, tuple(hidden_states.shape), tuple(top_k_index.shape), hidden_states.dtype,
               tuple(self.m.gate_up_proj.shape))
        ok = FastEagerExperts.checked.get(key)
        if ok is None:
            want = self.eager(self.m, hidden_states, top_k_index, top_k_weights)
            try:
                ok = _bits_equal(fast_eager(self.m, hidden_states, top_k_index, top_k_weights), want)
            except (RuntimeError, TypeError, ValueError) as e:  # e.g. grouped_mm unsupported for these operands
                log.info("MoE: grouped eager form unavailable for %s (%s)", type(self.m).__name__, e)
                ok = False
            FastEagerExperts.checked[key] = ok
            if not ok:
                log.info("MoE: using %s's eager loop at %s", type(self.m).__name__, key[1])
            return want
        if not ok:
            return self.eager(self.m, hidden_states, top_k_index, top_k_weights)
        if _FIXED is not None and PLANNED:
            pkey = (id(self.m), hidden_states.data_ptr(), tuple(hidden_states.shape), tuple(top_k_index.shape))
            plan = _FIXED.get(pkey)
            if plan is None:
                plan = _FIXED[pkey] = _plan(self.m, top_k_index)
            pok = FastEagerExperts.planned_checked.get(key)
            if pok is None:
                want = fast_eager(self.m, hidden_states, top_k_index, top_k_weights)
                pok = _bits_equal(planned_eager(self.m, hidden_states, top_k_index, top_k_weights, plan), want)
                FastEagerExperts.planned_checked[key] = pok
                if not pok:
                    log.info("MoE: per-expert planned form differs for %s at %s; grouped form kept",
                             type(self.m).__name__, key[1])
                return want
            if pok:
                return planned_eager(self.m, hidden_states, top_k_index, top_k_weights, plan)
        return fast_eager(self.m, hidden_states, top_k_index, top_k_weights)


@contextlib.contextmanager
def eager_experts(model: nn.Module):
    """Every transformers fused-experts module of ``model`` forwards in the eager arithmetic
    (``FastEagerExperts``) inside the context; the modules' own forwards are restored after."""
    patched = []
    FastEagerExperts.checked = {}
    FastEagerExperts.planned_checked = {}
    try:
        for mod in model.modules():
            fwd = eager_forward(mod)
            if fwd is not None:
                mod.forward = FastEagerExperts(mod, fwd).forward  # instance attribute: Module.__call__ uses it
                patched.append(mod)
        yield len(patched)
    finally:
        for mod in patched:
            if "forward" in mod.__dict__:
                del mod.forward
