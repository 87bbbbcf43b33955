"""NVFP4 fused path (qz_quantize_nvfp4 / qz_quantize_grouped_nvfp4: k_nv_absmax + k_nv_encode)
vs the C oracle and vs the two-pass qz_quantize path, bit for bit.

The reference's NVFP4 recipes (configs/recipes/recipe_MoE_RTN_NVFP4.yaml:16-21,
recipe_Dense_NVFP4.yaml:7-12) quantize every expert / dense linear with a per-tensor global scale
(compressed-tensors TENSOR_GROUP).  These tests cover the shapes of the reference's models
(Qwen3-30B-A3B fused experts as strided gate / up halves, dense linears of hundreds of 32 KiB
tiles), ragged and one-tile slices, all-zero groups and slices, a slice larger than the MALL,
two streams with their own sync regions, and the sync region's zero-after-call contract.
"""
import ctypes

import pytest
import torch

import qref
from quantizers_amd import _lib, ops
from quantizers_amd.quantization import QuantizationArgs

pytestmark = pytest.mark.gpu

NV = dict(num_bits=4, type="float", strategy="tensor_group", group_size=16, scale_dtype="float8_e4m3fn")


class _OA:  # oracle args (qref.compress_weight reads these attributes)
    num_bits, type, symmetric, strategy, group_size, block_structure, scale_dtype = 4, "float", True, \
        "tensor_group", 16, None, "fp8"


def _bits(t):
    return t.view(torch.uint8) if t.dtype in (torch.float8_e4m3fn, torch.uint8) else t.view(torch.int32)


def _same(a, b):
    a, b = _bits(a.cpu()), _bits(b.cpu())
    assert a.shape == b.shape
    bad = a != b
    assert not bad.any(), f"{int(bad.sum())} / {bad.numel()} differ; first {bad.nonzero()[:4].tolist()}"


def two_pass(w: torch.Tensor, a: QuantizationArgs):
    """The two-pass qz_quantize path (absmax pre-pass, then the group kernel) -- the comparator."""
    b, r, c, ld_r, ld_b = ops._geom(w)
    o = ops.alloc_outputs(tuple(w.shape), a, None, w.device)
    lib = _lib.load()
    ca = a.to_c()
    ws = torch.empty(lib.qz_quantize_workspace_size(b, r, c, ctypes.byref(ca)) + 256, dtype=torch.uint8,
                     device=w.device)
    rc = lib.qz_quantize(ops._ptr(w), b, r, c, ld_r, ld_b, ctypes.byref(ca), _lib.QZ_OUT_FP4_PACKED,
                         ops._ptr(o["codes"]), ops._ptr(o["scale"]), ops._ptr(None), ops._ptr(o["global_scale"]),
                         ops._ptr(ws), ws.numel(), ops._stream())
    _lib.check(rc, "qz_quantize")
    return o


def _rand(shape, seed, scale=0.02, device="cpu"):
    g = torch.Generator(device=device).manual_seed(seed)
    return (torch.randn(*shape, generator=g, device=device) * scale).to(torch.bfloat16)


def _sync_clean(dev):
    buf = ops.sync_workspace(1, dev)
    torch.cuda.synchronize()
    assert not buf.any(), "the sync region was not left zero"


def test_small_slices_match_oracle(cuda):
    """Several slices, each ONE item or a ragged tail item, vs the C oracle per slice."""
    a = QuantizationArgs(**NV)
    for shape in [(3, 32, 128), (2, 100, 48), (4, 640, 112), (1, 16, 16)]:
        w = torch.stack([_rand(shape[1:], seed=i, scale=0.01 * (i + 1)) for i in range(shape[0])])
        w[0, 0, :16] = 0  # an all-zero group
        got = ops.quantize_weight(w.to(cuda), a)
        for i in range(shape[0]):
            ref = qref.compress_weight(w[i], _OA)
            _same(got["codes"][i], ref["weight_packed"])
            _same(got["scale"][i], ref["weight_scale"])
            _same(got["global_scale"][i:i + 1], ref["weight_global_scale"])
    _sync_clean(cuda)


def test_extreme_magnitudes_match_oracle(cuda):
    """Slices scaled by 2^-120 .. 2^100 (global scales near the ends of the f32 range, group scales
    whose reciprocal leaves rcp's accurate range) and a slice whose groups span 60 binades: the
    encode's scale tables and e4m3 conversion vs the C oracle, slice by slice."""
    a = QuantizationArgs(**NV)
    base = _rand((6, 64, 256), seed=77, scale=1.0)
    mult = torch.tensor([2.0 ** -120, 2.0 ** -60, 1.0, 2.0 ** 40, 2.0 ** 100, 1.0]).view(6, 1, 1)
    w = (base.float() * mult).to(torch.bfloat16)
    w[5] = (base[5].float() * (2.0 ** torch.arange(-30, 34, dtype=torch.float32).view(64, 1))).to(torch.bfloat16)
    got = ops.quantize_weight(w.to(cuda), a)
    for i in range(w.shape[0]):
        ref = qref.compress_weight(w[i], _OA)
        _same(got["codes"][i], ref["weight_packed"])
        _same(got["scale"][i], ref["weight_scale"])
        _same(got["global_scale"][i:i + 1], ref["weight_global_scale"])
    _sync_clean(cuda)


def test_qwen3_30b_a3b_fused_experts(cuda):
    """One Qwen3-30B-A3B MoE layer: gate_up_proj [128, 1536, 2048] as its strided gate / up halves
    (48 tiles per slice) and down_proj [128, 2048, 768]: bit-identical to the two-pass path, and
    two slices of each checked against the C oracle."""
    a = QuantizationArgs(**NV)
    gu = _rand((128, 1536, 2048), seed=11, device=cuda)
    dn = _rand((128, 2048, 768), seed=12, device=cuda)
    gu[5] *= 40  # slices with very different global scales
    dn[7].zero_()  # an all-zero slice: global scale inf, as compressed-tensors computes it
    for w in (gu[:, :768], gu[:, 768:], dn):
        got = ops.quantize_weight(w, a)
        ref = two_pass(w, a)
        for k in ("codes", "scale", "global_scale"):
            _same(got[k], ref[k])
        for i in (0, 5):
            r = qref.compress_weight(w[i].cpu().contiguous(), _OA)
            _same(got["codes"][i], r["weight_packed"])
            _same(got["scale"][i], r["weight_scale"])
    _sync_clean(cuda)


@pytest.mark.parametrize("shape", [(9728, 2560), (2560, 9728), (4096, 2560), (1024, 2560)])
def test_grouped_dense_qwen3_4b_shapes(cuda, shape):
    """recipe_Dense_NVFP4 on Qwen3-4B linears: one grouped call of 6 same-shape weights (slices
    of up to 1520 tiles) == per-weight two-pass results; one weight also vs the C oracle."""
    a = QuantizationArgs(**NV)
    ws = [_rand(shape, seed=100 + i, scale=0.01 * (1 + i % 3), device=cuda) for i in range(6)]
    gq = ops.GroupedQuantize(ws, a)
    outs = gq.run()
    for w, o in zip(ws, outs):
        ref = two_pass(w, a)
        for k in ("codes", "scale", "global_scale"):
            _same(o[k], ref[k])
    r = qref.compress_weight(ws[2].cpu(), _OA)
    _same(outs[2]["codes"], r["weight_packed"])
    _same(outs[2]["scale"], r["weight_scale"])
    _same(outs[2]["global_scale"], r["weight_global_scale"])
    _sync_clean(cuda)


def test_slice_larger_than_mall(cuda):
    """One [65536, 2560] slice (320 MiB of bf16, more than the 256 MiB MALL; 10240 tiles whose
    maximum is one key): bit-identical to the two-pass path; the maximum sits in the last tile."""
    a = QuantizationArgs(**NV)
    w = _rand((65536, 2560), seed=3, device=cuda)
    w[-1, -1] = 3.0
    got = ops.quantize_weight(w, a)
    ref = two_pass(w, a)
    for k in ("codes", "scale", "global_scale"):
        _same(got[k], ref[k])
    del w, got, ref
    _sync_clean(cuda)


def test_two_streams_own_sync_regions(cuda):
    """Two batches quantized concurrently on two streams, each with the sync region of its own
    (device, stream): both bit-identical to the two-pass path, both regions left zero."""
    a = QuantizationArgs(**NV)
    ws = [_rand((64, 768, 2048), seed=40 + i, scale=0.01 * (i + 1), device=cuda) for i in range(2)]
    refs = [two_pass(w, a) for w in ws]
    torch.cuda.synchronize()
    sts = [torch.cuda.Stream(cuda) for _ in ws]
    outs = []
    for w, st in zip(ws, sts):
        st.wait_stream(torch.cuda.current_stream(cuda))
        with torch.cuda.stream(st):
            outs.append([ops.quantize_weight(w, a) for _ in range(3)][-1])
    torch.cuda.synchronize()
    for o, r in zip(outs, refs):
        for k in ("codes", "scale", "global_scale"):
            _same(o[k], r[k])
    for st in sts:
        assert not ops.sync_workspace(1, cuda, st).any()


def test_argument_errors(cuda):
    lib = _lib.load()
    a = QuantizationArgs(**NV)
    w = torch.zeros(64, 64, dtype=torch.bfloat16, device=cuda)
    o = ops.alloc_outputs((64, 64), a, None, cuda)
    sync = ops.sync_workspace(1, cuda)
    args = lambda ca, sz=sync.numel(), sy=sync: (ops._ptr(w), 1, 64, 64, 4096, ctypes.byref(ca),  # noqa: E731
                                                 ops._ptr(o["codes"]), ops._ptr(o["scale"]),
                                                 ops._ptr(o["global_scale"]), ops._ptr(sy), sz, ops._stream())
    assert lib.qz_quantize_nvfp4(*args(a.to_c(), sz=16)) == _lib.QZ_ERR_WORKSPACE
    assert lib.qz_quantize_nvfp4(*args(a.to_c(), sy=None)) == _lib.QZ_ERR_NULL
    mx = QuantizationArgs(num_bits=4, type="float", group_size=32, scale_dtype="uint8")
    assert lib.qz_quantize_nvfp4(*args(mx.to_c())) == _lib.QZ_ERR_FORMAT
    assert lib.qz_quantize_nvfp4(*args(a.to_c())) == 0
    torch.cuda.synchronize()


def test_many_on_two_streams(cuda):
    """ops.quantize_nvfp4_many (round-robin over 2 streams, as CompressionPlan issues NVFP4
    parameters) == one quantize_weight call per parameter on one stream, and a following
    default-stream read sees every output."""
    a = QuantizationArgs(**NV)
    gu = _rand((16, 512, 1024), seed=61, device=cuda)
    dn = _rand((16, 1024, 256), seed=62, device=cuda)
    ws = [gu[:, :256], gu[:, 256:], dn, gu[:, :256] * 3]
    refs = [ops.quantize_weight(w, a) for w in ws]
    outs = [ops.alloc_outputs(tuple(w.shape), a, None, cuda) for w in ws]
    for o in outs:
        for t in o.values():
            if t is not None:
                t.fill_(0) if t.dtype != torch.float8_e4m3fn else t.view(torch.uint8).fill_(0)
    ops.quantize_nvfp4_many(list(zip(ws, outs)), a, n_streams=2)
    for o, r in zip(outs, refs):  # read on the default stream right after (no synchronize)
        for k in ("codes", "scale", "global_scale"):
            _same(o[k], r[k])


def test_plan_stacked_experts_take_two_stream_call(cuda, monkeypatch):
    """a stacked NVFP4 unit (every expert of a fused Qwen3-MoE parameter) in
    CompressionPlan.run goes through ops.quantize_nvfp4_many (the two-stream call), and its
    on-disk tensors equal the per-expert quantize of each slice."""
    from test_oneshot_gpu import _qwen3_moe
    from quantizers_amd.compressor import CompressionPlan, compression_units
    from quantizers_amd.model import iter_linears
    from quantizers_amd.quantization import preset_scheme
    m = _qwen3_moe().to(cuda)
    nv = preset_scheme("NVFP4", ["Linear"])
    m.quantization_scheme_map = {r.name: nv for r in iter_linears(m) if r.index is not None}
    units, _ = compression_units(m)
    plan = CompressionPlan(units, cuda)
    stacked = [u for u in units if u.stacked]
    assert len(stacked) == 6 and len(plan.singles) == 6  # 2 layers x (gate, up, down)
    calls = []
    real = ops.quantize_nvfp4_many

    def spy(items, a, **kw):
        calls.append(len(items))
        return real(items, a, **kw)
    monkeypatch.setattr(ops, "quantize_nvfp4_many", spy)
    plan.run()
    torch.cuda.synchronize()
    assert sum(calls) == 6, calls
    got = plan.tensors()
    for u in stacked:
        for g in u.refs:
            want = ops.compress_weight(g.weight.contiguous(), nv.weights)
            for k, v in want.items():
                assert torch.equal(got[f"{g.name}.{k}"].cpu(), v.cpu()), (g.name, k)
