"""GPU parity: the HIP library (through the C ABI) vs the CPU oracle, bit for bit.

Bar (BASELINE.json north_star): packed int words, integer zero-points, scales and FP8/FP4 codes
identical to the CPU restatement (oracle/ct_torch.py, itself pinned by oracle/quant_ref.c and
the KATs).  Every scheme the reference's recipes use, plus edge cases (all-zero groups, ties at
+-7.5*s, outliers, ragged shapes, fused-expert batches, strided views).
"""
import pytest
import torch

import ct_torch as ct
from quantizers_amd import ops, _lib
from quantizers_amd.quantization import QuantizationArgs

pytestmark = pytest.mark.gpu


def _w(n, k, seed=0, scale=0.02, device="cpu"):
    g = torch.Generator().manual_seed(seed)
    w = (torch.randn(n, k, generator=g) * scale).to(torch.bfloat16)
    return w


def _edge_weight(n, k, g, seed=1):
    w = _w(n, k, seed).float()
    gen = torch.Generator().manual_seed(seed + 100)
    m = torch.rand(n, k, generator=gen) < 0.001
    w[m] *= 20  # outliers
    w[0, :g] = 0  # an all-zero group
    if n > 2 and k >= g:  # exact ties at +-7.5*s and +-0.5*s
        w[2, :g] = 0.0
        w[2, 0] = 0.75
        w[2, 1] = -0.75
        w[2, 2] = 0.05
        w[2, 3] = -0.05
        w[2, 4] = 0.15
    return w.to(torch.bfloat16)


def _oracle_args(a: QuantizationArgs) -> ct.QArgs:
    sd = {None: None, "float8_e4m3fn": "fp8", "uint8": "e8m0"}[a.scale_dtype]
    return ct.QArgs(num_bits=a.num_bits, type=a.type, symmetric=a.symmetric, strategy=a.strategy,
                    group_size=a.group_size, block_structure=tuple(a.block_structure) if a.block_structure else None,
                    scale_dtype=sd)


def _eq(a: torch.Tensor, b: torch.Tensor):
    a = a.cpu()
    b = b.cpu()
    assert a.shape == b.shape, (a.shape, b.shape)
    if a.dtype in (torch.bfloat16, torch.float8_e4m3fn):
        a = a.view(torch.uint8 if a.dtype == torch.float8_e4m3fn else torch.int16)
        b = b.view(torch.uint8 if b.dtype == torch.float8_e4m3fn else torch.int16)
    bad = (a != b)
    assert not bad.any(), f"{int(bad.sum())} / {bad.numel()} mismatches; first at {bad.nonzero()[:5].tolist()}"


SCHEMES = [
    dict(num_bits=4, type="int", symmetric=True, group_size=128),
    dict(num_bits=4, type="int", symmetric=True, group_size=32),
    dict(num_bits=4, type="int", symmetric=True, group_size=64),
    dict(num_bits=4, type="int", symmetric=False, group_size=128),
    dict(num_bits=4, type="int", symmetric=False, group_size=32),
    dict(num_bits=8, type="int", symmetric=True, group_size=128),
    dict(num_bits=8, type="int", symmetric=False, group_size=64),
    dict(num_bits=4, type="int", symmetric=True, strategy="channel"),
    dict(num_bits=8, type="int", symmetric=True, strategy="channel"),
    dict(num_bits=4, type="int", symmetric=False, strategy="channel"),
    dict(num_bits=4, type="int", symmetric=True, strategy="tensor"),
    dict(num_bits=8, type="float", group_size=32),
    dict(num_bits=8, type="float", group_size=128),
    dict(num_bits=8, type="float", strategy="channel"),
    dict(num_bits=8, type="float", strategy="tensor"),
    dict(num_bits=8, type="float", strategy="block", block_structure=[128, 128]),
    dict(num_bits=8, type="float", strategy="block", block_structure=[64, 32]),
    dict(num_bits=4, type="float", group_size=32, scale_dtype="uint8"),  # MXFP4
    dict(num_bits=4, type="float", strategy="tensor_group", group_size=16, scale_dtype="float8_e4m3fn"),  # NVFP4
    dict(num_bits=4, type="int", symmetric=True, group_size=256),
    dict(num_bits=4, type="int", symmetric=True, group_size=512),
    dict(num_bits=4, type="int", symmetric=True, group_size=16),
]


def _id(d):
    return "-".join(f"{k}{v}" for k, v in d.items() if k not in ("type",)) + "-" + d["type"]


@pytest.mark.parametrize("scheme", SCHEMES, ids=_id)
@pytest.mark.parametrize("shape", [(256, 512), (384, 1024)])
def test_compress_matches_oracle(cuda, scheme, shape):
    a = QuantizationArgs(**scheme)
    n, k = shape
    gsz = a.group_size or (a.block_structure[1] if a.block_structure else k)
    w = _edge_weight(n, k, max(1, min(gsz, k)))
    ref = ct.compress_weight(w, _oracle_args(a))
    got = ops.compress_weight(w.to(cuda), a)
    assert set(got) == set(ref), (set(got), set(ref))
    for key in ref:
        _eq(got[key], ref[key])


@pytest.mark.parametrize("scheme", SCHEMES[:8] + SCHEMES[11:19], ids=_id)
def test_fake_quantize_matches_oracle(cuda, scheme):
    a = QuantizationArgs(**scheme)
    w = _edge_weight(128, 512, 32)
    oa = _oracle_args(a)
    gs = None
    if oa.strategy == "tensor_group":
        gs = ct.generate_gparam(w.amin().reshape(1), w.amax().reshape(1))
    mn, mx = ct.observe_minmax(w, oa)
    s, z = ct.calculate_qparams(mn, mx, oa, global_scale=gs)
    ref = ct.fake_quantize(w, s, z, oa, global_scale=gs)
    got = ops.fake_quantize(w.to(cuda), a)
    _eq(got, ref)


@pytest.mark.parametrize("scheme", [SCHEMES[0], SCHEMES[1], SCHEMES[3], SCHEMES[11], SCHEMES[17], SCHEMES[18],
                                    SCHEMES[7]], ids=_id)
def test_awq_fake_quant_scaled(cuda, scheme):
    a = QuantizationArgs(**scheme)
    w = _w(96, 512, seed=3)
    g = torch.Generator().manual_seed(7)
    s = (torch.rand(512, generator=g) * 3 + 0.05).float()
    ref = ct.awq_fake_quant_scaled(w, s, _oracle_args(a))
    got = ops.fake_quantize(w.to(cuda), a, col_scales=s.to(cuda))
    _eq(got, ref)


@pytest.mark.parametrize("scheme", [SCHEMES[i] for i in (0, 1, 3, 4, 5, 6, 11, 17, 19, 20, 21)], ids=_id)
@pytest.mark.parametrize("shape", [(333, 768), (7, 4608), (66, 1536)])
def test_awq_fake_quant_scaled_ragged(cuda, scheme, shape):
    """The column-tiled fake-quant kernel (k_fq_cols: 4-row tiles, 64-lane column chunks) on
    shapes whose rows are not a multiple of the tile and whose column units end mid-chunk
    (768 / 8 = 96 units), with scales spanning several binades and a few tiny/huge columns
    (the IEEE-division fallback)."""
    a = QuantizationArgs(**scheme)
    n, k = shape
    if k % a.group_size:
        pytest.skip("columns not divisible by the group size (a ValueError in both)")
    w = _w(n, k, seed=5)
    g = torch.Generator().manual_seed(13)
    s = (2.0 ** (torch.rand(k, generator=g) * 8 - 4)).float()
    s[3] = 2.0 ** -110
    s[k // 2] = 2.0 ** 105
    ref = ct.awq_fake_quant_scaled(w, s, _oracle_args(a))
    got = ops.fake_quantize(w.to(cuda), a, col_scales=s.to(cuda))
    _eq(got, ref)


def test_awq_fake_quant_scaled_headline_shape(cuda):
    """Q(W*s)/s of the bench weight [11008, 4096], int4 sym g128, compared in full."""
    a = QuantizationArgs(num_bits=4, type="int", symmetric=True, group_size=128)
    w = _w(11008, 4096, seed=0)
    g = torch.Generator().manual_seed(3)
    s = (torch.rand(4096, generator=g) * 3 + 0.05).float()
    ref = ct.awq_fake_quant_scaled(w, s, _oracle_args(a))
    got = ops.fake_quantize(w.to(cuda), a, col_scales=s.to(cuda))
    _eq(got, ref)


def test_headline_shape_int4_g128(cuda):
    """The bench workload: bf16 [11008, 4096], int4 sym g128 (compared in full)."""
    w = _w(11008, 4096, seed=0)
    a = QuantizationArgs(num_bits=4, type="int", symmetric=True, group_size=128)
    import qref
    ref_p, ref_s = qref.int_sym_group_pack(w, 4, 128)
    got = ops.quantize_weight(w.to(cuda), a)
    _eq(got["codes"], ref_p)
    _eq(got["scale"], ref_s)


def test_batched_experts_and_strided(cuda):
    a = QuantizationArgs(num_bits=4, type="int", symmetric=True, group_size=32)
    e = torch.stack([_w(64, 256, seed=i) for i in range(5)])
    got = ops.compress_weight(e.to(cuda), a)
    for i in range(5):
        ref = ct.compress_weight(e[i], _oracle_args(a))
        _eq(got["weight_packed"][i], ref["weight_packed"])
        _eq(got["weight_scale"][i], ref["weight_scale"])
    # strided view (columns of a wider buffer) -> generic path, same answer
    big = _w(64, 384, seed=9)
    view = big.to(cuda)[:, 64:320]
    ref = ct.compress_weight(big[:, 64:320].contiguous(), _oracle_args(a))
    got = ops.compress_weight(view, a)
    _eq(got["weight_packed"], ref["weight_packed"])
    _eq(got["weight_scale"], ref["weight_scale"])


def test_nvfp4_batched_global_scale(cuda):
    a = QuantizationArgs(num_bits=4, type="float", strategy="tensor_group", group_size=16,
                         scale_dtype="float8_e4m3fn")
    e = torch.stack([_w(32, 128, seed=i, scale=0.01 * (i + 1)) for i in range(3)])
    got = ops.compress_weight(e.to(cuda), a)
    for i in range(3):
        ref = ct.compress_weight(e[i], _oracle_args(a))
        _eq(got["weight_packed"][i], ref["weight_packed"])
        _eq(got["weight_scale"][i], ref["weight_scale"])
        _eq(got["weight_global_scale"][i:i + 1], ref["weight_global_scale"])


@pytest.mark.parametrize("scheme", [SCHEMES[0], SCHEMES[3], SCHEMES[11], SCHEMES[15], SCHEMES[17], SCHEMES[18]],
                         ids=_id)
def test_dequantize_roundtrip(cuda, scheme):
    """dequantize(stored codes) == compressed-tensors dequantize of the oracle's codes."""
    a = QuantizationArgs(**scheme)
    w = _w(256, 256, seed=5)
    q = ops.quantize_weight(w.to(cuda), a)
    d = ops.dequantize(q["codes"], w.shape, a, q["scale"], q["zero_point"], q.get("global_scale"))
    oa = _oracle_args(a)
    gs = None
    if oa.strategy == "tensor_group":
        gs = ct.generate_gparam(w.amin().reshape(1), w.amax().reshape(1))
    mn, mx = ct.observe_minmax(w, oa)
    s, z = ct.calculate_qparams(mn, mx, oa, global_scale=gs)
    if oa.type == "int":
        codes = ct.quantize(w, s, z, oa, dtype=torch.int8)
    elif oa.num_bits == 8:
        codes = ct.quantize(w, s, z, oa, dtype=torch.float8_e4m3fn)
    else:
        codes = ct.quantize(w, s, z, oa, global_scale=gs)
    _eq(d, ct.dequantize(codes, s, z, oa, dtype=torch.bfloat16, global_scale=gs))


def test_observe_qparams_quantize_pipeline(cuda):
    """observe -> calculate_qparams -> quantize(given qparams) == fused qz_quantize."""
    for scheme in (SCHEMES[0], SCHEMES[3], SCHEMES[11], SCHEMES[15], SCHEMES[17]):
        a = QuantizationArgs(**scheme)
        w = _edge_weight(256, 512, 32).to(cuda)
        mn, mx = ops.observe_minmax(w, a)
        s, z = ops.calculate_qparams(mn, mx, a)
        codes = ops.quantize(w, s, z, a)
        fused = ops.quantize_weight(w, a)
        _eq(codes, fused["codes"])
        _eq(s, fused["scale"])


def test_pack_to_int32_both_dims(cuda):
    g = torch.Generator().manual_seed(0)
    for bits in (2, 3, 4, 8):
        v = torch.randint(-(1 << (bits - 1)), 1 << (bits - 1), (37, 53), generator=g).to(torch.int8)
        for dim in (0, 1):
            _eq(ops.pack_to_int32(v.to(cuda), bits, dim), ct.pack_to_int32(v, bits, dim))


def test_errors_are_value_errors(cuda):
    w = _w(16, 100).to(cuda)
    with pytest.raises(ValueError):
        ops.quantize_weight(w, QuantizationArgs(num_bits=4, group_size=128))
    with pytest.raises(ValueError):
        ops.quantize_weight(_w(100, 128).to(cuda), QuantizationArgs(num_bits=8, type="float", strategy="block",
                                                                     block_structure=[128, 128]))


def test_awq_stats(cuda):
    g = torch.Generator().manual_seed(0)
    x = torch.randn(3, 257, 2560, generator=g).to(torch.bfloat16)
    sums = torch.zeros(2560, dtype=torch.float32, device=cuda)
    n = ops.awq_absmean_accum(x.to(cuda), sums)
    assert n == 3 * 257
    ref, cnt = ct.awq_accumulate_mean(x)
    torch.testing.assert_close(sums.cpu(), ref, rtol=1e-5, atol=1e-4)
    ws = [_w(320, 512, seed=i) for i in range(2)]
    wsum = torch.zeros(512, dtype=torch.float64, device=cuda)
    rows = sum(ops.awq_weight_mean_accum(w.to(cuda), 32, wsum) for w in ws)
    ref = ct.awq_layer_means(ws, ct.QArgs(group_size=32))
    torch.testing.assert_close(wsum.cpu() / rows, ref, rtol=1e-12, atol=1e-12)
    xm = (ref.float() + 0.1)
    for ratio in (0.0, 0.35, 0.95):
        got = ops.awq_grid_scales(xm.to(cuda), ref.to(cuda), ratio, True)
        torch.testing.assert_close(got.cpu(), ct.awq_grid_scales(xm, ref, ratio, True), rtol=2e-6, atol=1e-7)


@pytest.mark.parametrize("tokens,ch", [(1, 8), (7, 264), (333, 1032), (4099, 520)])
def test_absmean_ragged_windows(cuda, tokens, ch):
    """Channel counts that leave a 512-column window partly empty (the stage-1 lanes past the
    last column load clamped addresses and their sums are discarded) and token counts that
    leave waves with a partial batch: equal to the oracle's accumulation (f32, order-dependent
    -> rtol), and the sums outside [0, ch) untouched."""
    g = torch.Generator().manual_seed(tokens)
    x = torch.randn(tokens, ch, generator=g).to(torch.bfloat16)
    sums = torch.full((ch + 16,), 7.0, dtype=torch.float32, device=cuda)
    n = ops.awq_absmean_accum(x.to(cuda), sums[:ch])
    assert n == tokens
    ref, _ = ct.awq_accumulate_mean(x.unsqueeze(0))
    torch.testing.assert_close(sums[:ch].cpu(), ref + 7.0, rtol=1e-5, atol=1e-4)
    assert torch.equal(sums[ch:].cpu(), torch.full((16,), 7.0))


@pytest.mark.parametrize("rows,cols,g", [(1, 32, 32), (9, 96, 32), (45, 640, 128), (1001, 1088, 64),
                                         (700, 1024, 256), (300, 2048, 512), (5000, 136, 8), (11008, 4096, 128),
                                         (40000, 512, 32)])
def test_weight_mean_ragged_windows(cuda, rows, cols, g):
    """w_mean with a partly empty last column window, row counts that are not multiples of the
    row slots per workgroup, and every window width (128 / 256 / 512 columns): the fixed-order
    tree, bit for bit."""
    w = _w(rows, cols, seed=rows)
    wsum = torch.zeros(cols, dtype=torch.float64, device=cuda)
    assert ops.awq_weight_mean_accum(w.to(cuda), g, wsum) == rows
    assert torch.equal(wsum.cpu(), _wmean_tree(w, g))


def _stats_tree(v, lay, dtype=None) -> "np.ndarray":
    """Fixed-order restatement of the AWQ statistics reduction (ops.awq_stats_layout, terms ``v``
    [R, C]).  Per row chunk, slot s sums rows s, s + S, ... in order and the chunk partial is
    ((slot 0 + slot 1) + ...).  One-launch plan: chunks form groups of CPG; a group's partial and
    then the final sum (over the groups; skipped with one group) are each, over TF thread
    groups f, ((sum_0 + sum_1) + ...) where sum_f adds items f, f + TF, ... in order.  Two-launch
    plan: the final sum alone, over all chunks, with TF = 16."""
    import numpy as np
    R, C = v.shape
    dt = v.dtype if dtype is None else dtype
    rc, nch, S, TF, cpg = (lay["rows_per_chunk"], lay["chunks"], lay["slots"], lay["final_groups"],
                           lay["chunks_per_group"])
    part = np.zeros((nch, C), dtype=dt)
    for k in range(nch):
        r0, r1 = k * rc, min(R, (k + 1) * rc)
        t = None
        for j in range(S):
            acc = np.zeros(C, dtype=dt)
            for r in range(r0 + j, r1, S):
                acc = acc + v[r]
            t = acc if t is None else t + acc
        part[k] = t

    def reduce(items):
        red = []
        for f in range(TF):
            acc = np.zeros(C, dtype=dt)
            for i in range(f, len(items), TF):
                acc = acc + items[i]
            red.append(acc)
        t = red[0]
        for f in range(1, TF):
            t = t + red[f]
        return t

    if not cpg:
        return np.zeros(C, dtype=dt) + reduce(list(part))
    groups = [reduce(list(part[g:g + cpg])) for g in range(0, nch, cpg)]
    return np.zeros(C, dtype=dt) + (groups[0] if len(groups) == 1 else reduce(groups))


@pytest.mark.parametrize("tokens,ch", [(2048, 2560), (16384, 4096), (333, 1032), (7, 264), (100000, 520)])
def test_absmean_fixed_order_bit_exact(cuda, tokens, ch):
    """absmean's f32 sums equal the restated fixed-order tree bit for bit (one launch: the
    last-arriving workgroup of each window adds the chunk partials), and the statistics
    workspace's arrival counters are zero again after the call."""
    import numpy as np
    g = torch.Generator().manual_seed(tokens + ch)
    x = torch.randn(tokens, ch, generator=g).to(torch.bfloat16)
    sums = torch.zeros(ch, dtype=torch.float32, device=cuda)
    ops.awq_absmean_accum(x.to(cuda), sums)
    lay = ops.awq_stats_layout("absmean", tokens, ch)
    want = _stats_tree(x.float().abs().numpy(), lay, np.float32)
    assert torch.equal(sums.cpu(), torch.from_numpy(want))
    torch.cuda.synchronize()
    for buf in ops._stats_ws_cache.values():
        assert not buf[:lay["head_bytes"]].any()


def _wmean_tree(w: torch.Tensor, g: int) -> torch.Tensor:
    """qz_awq_weight_mean_accum's sum for one call into a zero wsum: terms
    bf16(|w| / bf16(group absmax + 1e-6)) (the oracle's elementwise values) summed in f64 in the
    kernel's fixed order (``_stats_tree``)."""
    R, C = w.shape
    v = w.reshape(-1, g).abs()
    v = (v / (v.amax(dim=1, keepdim=True) + 1e-6)).reshape(R, C).double().numpy()
    return torch.from_numpy(_stats_tree(v, ops.awq_stats_layout("wmean", R, C, g)))


@pytest.mark.parametrize("shape,g", [((320, 512), 32), ((2000, 1536), 128), ((37, 4096), 64)])
def test_weight_mean_deterministic_fixed_order(cuda, shape, g):
    """w_mean is a fixed-order one-launch reduction: bit-identical to the restated tree, and
    identical across repeated calls while other work runs concurrently on another stream (the
    last-arriving workgroup differs from call to call; the order does not)."""
    w = _w(*shape, seed=11)
    wc = w.to(cuda)
    want = _wmean_tree(w, g)
    outs = []
    side = torch.cuda.Stream()
    junk = torch.randn(4096, 4096, device=cuda)
    for i in range(4):
        wsum = torch.zeros(shape[1], dtype=torch.float64, device=cuda)
        if i % 2:
            with torch.cuda.stream(side):
                for _ in range(3):
                    junk = junk @ junk.T / 4096  # concurrent load on the card
        ops.awq_weight_mean_accum(wc, g, wsum)
        torch.cuda.synchronize()
        outs.append(wsum.cpu())
    for o in outs:
        assert torch.equal(o, want), (o - want).abs().max()


def test_stats_segments_bit_identical_to_single_calls(cuda):
    """Segmented statistics (one launch over many operands) == one single call per operand, bit
    for bit: absmean over 17 calibration samples of a batched forward (two launches of <= 16
    segments; ragged, strided and 1-token samples) into zero sums and into sums holding an earlier
    total; w_mean over a Qwen3-4B mapping's balance layers (q / k / v, gate / up: the 2560-column
    plans) at group 128 and 32, and over an unaligned operand (the whole batch then runs as single
    calls).  The arrival counters are zero afterwards."""
    g = torch.Generator(device=cuda).manual_seed(21)
    base = torch.randn(17 * 2048 + 301, 3072, device=cuda, generator=g).to(torch.bfloat16)
    xs = [base[i * 2048:(i + 1) * 2048, :2560] for i in range(16)] + [base[16 * 2048:16 * 2048 + 300, :2560]]
    xs[3] = base[-1:, :2560]
    for pre in (0.0, 3.5):
        seg = [torch.full((2560,), pre, dtype=torch.float32, device=cuda) for _ in xs]
        one = [t.clone() for t in seg]
        assert ops.awq_absmean_segments(xs, seg) == [x.shape[0] for x in xs]
        for x, o in zip(xs, one):
            ops.awq_absmean_accum(x, o)
        for a, b in zip(seg, one):
            assert torch.equal(a, b)
    ws = [(torch.randn(r, 2560, device=cuda, generator=g) * 0.02).to(torch.bfloat16) for r in (4096, 1024, 1024)]
    ws += [(torch.randn(9728, 2560, device=cuda, generator=g) * 0.02).to(torch.bfloat16) for _ in range(2)]
    for gs in (128, 32):
        seg = [torch.zeros(2560, dtype=torch.float64, device=cuda) for _ in ws]
        one = [t.clone() for t in seg]
        assert ops.awq_weight_mean_segments(ws, gs, seg) == [w.shape[0] for w in ws]
        for w, o in zip(ws, one):
            ops.awq_weight_mean_accum(w, gs, o)
        for a, b in zip(seg, one):
            assert torch.equal(a, b)
    odd = torch.empty(300 * 2568 + 8, dtype=torch.bfloat16, device=cuda)[1:1 + 300 * 2568].view(300, 2568)[:, :2560]
    odd.copy_(ws[0][:300])
    seg = [torch.zeros(2560, dtype=torch.float64, device=cuda) for _ in range(2)]
    one = [t.clone() for t in seg]
    ops.awq_weight_mean_segments([ws[1], odd], 128, seg)
    ops.awq_weight_mean_accum(ws[1], 128, one[0])
    ops.awq_weight_mean_accum(odd, 128, one[1])
    for a, b in zip(seg, one):
        assert torch.equal(a, b)
    torch.cuda.synchronize()
    for buf in ops._stats_ws_cache.values():
        assert not buf[:32768].any()


def test_smoothing_ops(cuda):
    w = _w(64, 128, seed=2)
    s = torch.rand(128, generator=torch.Generator().manual_seed(1)) + 0.5
    got = ops.scale_columns_(w.clone().to(cuda), s.to(cuda))
    _eq(got, (w.float() * s.view(1, -1)).to(torch.bfloat16))
    n = _w(1, 128, seed=4).reshape(-1)
    got = ops.scale_rows_(n.clone().to(cuda), s.to(cuda), divide=True)
    _eq(got, (n.float() / s).to(torch.bfloat16))


@pytest.mark.parametrize("scheme", [SCHEMES[1], SCHEMES[17], SCHEMES[18], SCHEMES[11]], ids=_id)
def test_fused_expert_strided_slices(cuda, scheme):
    """[E, 2I, H] fused gate_up parameter: the gate half [:, :I] is a strided batch view."""
    a = QuantizationArgs(**scheme)
    g = torch.Generator().manual_seed(3)
    fused = (torch.randn(6, 2 * 64, 128, generator=g) * 0.02).to(torch.bfloat16)
    view = fused.to(cuda)[:, :64, :]
    got = ops.compress_weight(view, a)
    for e in range(6):
        ref = ct.compress_weight(fused[e, :64].contiguous(), _oracle_args(a))
        for k, v in ref.items():
            if k == "weight_shape":
                continue
            gv = got[k][e] if got[k].dim() > 1 or k != "weight_global_scale" else got[k][e:e + 1]
            _eq(gv, v)


def _all_bf16(limit):
    bits = torch.arange(0, 65536, dtype=torch.int32)
    bits = torch.where(bits >= 32768, bits - 65536, bits).to(torch.int16)
    x = bits.view(torch.bfloat16)
    keep = torch.isfinite(x.float()) & (x.float().abs() <= limit)
    return x[keep]


def _rows_with_anchor(vals, anchor, width):
    """rows of `width` = [anchor, 511 values...] so every group's scale is fixed by the anchor."""
    per = width - 1
    n = (vals.numel() + per - 1) // per
    pad = torch.zeros(n * per - vals.numel(), dtype=torch.bfloat16)
    body = torch.cat([vals, pad]).reshape(n, per)
    return torch.cat([torch.full((n, 1), anchor, dtype=torch.bfloat16), body], dim=1)


def test_fp8_encode_exhaustive_fast_path(cuda):
    """Every finite bf16 with |x| <= 448 through the single-pass FP8 kernel with scale 1."""
    w = _rows_with_anchor(_all_bf16(448.0), 448.0, 512)
    a = QuantizationArgs(num_bits=8, type="float", group_size=512)
    got = ops.compress_weight(w.to(cuda), a)
    assert torch.all(got["weight_scale"].cpu().float() == 1.0)
    ref = torch.clamp(w, -448, 448).to(torch.float8_e4m3fn)
    _eq(got["weight"], ref)


@pytest.mark.parametrize("anchor", [4.0, 5.96875])
def test_mxfp4_encode_exhaustive_fast_path(cuda, anchor):
    """Every finite bf16 with |x| <= anchor through the MXFP4 kernel with E8M0 scale 2^0."""
    vals = _all_bf16(anchor)
    w = _rows_with_anchor(vals, anchor, 32)
    a = QuantizationArgs(num_bits=4, type="float", group_size=32, scale_dtype="uint8")
    got = ops.compress_weight(w.to(cuda), a)
    assert torch.all(got["weight_scale"].cpu() == 127)
    ref = ct.compress_weight(w, _oracle_args(a))
    _eq(got["weight_packed"], ref["weight_packed"])


@pytest.mark.parametrize("scheme", [SCHEMES[i] for i in (1, 3, 7, 11, 17, 18)], ids=_id)
def test_batched_col_scales_match_per_slice(cuda, scheme):
    """qz_awq_fake_quant_batched (one scale vector per slice, the per-expert AWQ grid step) and
    qz_awq_grid_scales_batched are bit-identical to per-slice calls."""
    a = QuantizationArgs(**scheme)
    g = torch.Generator().manual_seed(11)
    fused = (torch.randn(5, 64, 256, generator=g) * 0.02).to(torch.bfloat16).to(cuda)
    xm = (torch.rand(5, 256, generator=g) + 0.01).to(cuda)
    wm = (torch.rand(5, 256, generator=g) + 0.01).to(cuda)
    for ratio in (0.0, 0.35, 0.95):
        s = ops.awq_grid_scales_batched(xm, wm, ratio, True)
        got = ops.fake_quantize_batched(fused, a, s)
        for e in range(5):
            s_e = ops.awq_grid_scales(xm[e], wm[e], ratio, True)
            _eq(s[e].view(torch.int32), s_e.view(torch.int32))
            _eq(got[e], ops.fake_quantize(fused[e], a, col_scales=s_e))


def test_batched_col_scales_expert_shape(cuda):
    """The per-expert AWQ grid step at a real expert shape (Qwen3-30B-A3B down_proj chunk:
    16 x [2048, 768], int4 g128): batched launch == per-slice launches."""
    a = QuantizationArgs(num_bits=4, type="int", symmetric=True, group_size=128)
    g = torch.Generator(device=cuda).manual_seed(5)
    w = (torch.randn(16, 2048, 768, device=cuda, generator=g) * 0.02).to(torch.bfloat16)
    xm = torch.rand(16, 768, device=cuda, generator=g) + 0.01
    wm = torch.rand(16, 768, device=cuda, generator=g) + 0.01
    s = ops.awq_grid_scales_batched(xm, wm, 0.5, True)
    got = ops.fake_quantize_batched(w, a, s)
    torch.cuda.synchronize()
    for e in (0, 7, 15):
        _eq(got[e], ops.fake_quantize(w[e], a, col_scales=s[e].clone()))


@pytest.mark.parametrize("shape,strided", [((4096, 2048), False), ((333, 100), False), ((512, 768), True)])
def test_awq_sq_err_accum(cuda, shape, strided):
    """qz_awq_sq_err_accum == sum(f32(bf16(a - b))^2) (f64), dense and strided rows."""
    g = torch.Generator().manual_seed(3)
    a = torch.randn(*shape, generator=g).to(torch.bfloat16)
    b = (a.float() + torch.randn(*shape, generator=g) * 0.01).to(torch.bfloat16)
    want = (a - b).float().pow(2).double().sum().item()
    ac, bc = a.to(cuda), b.to(cuda)
    if strided:
        big = torch.zeros(shape[0], shape[1] + 64, dtype=torch.bfloat16, device=cuda)
        big[:, :shape[1]] = ac
        ac = big[:, :shape[1]]
    out = torch.full((1,), 0.5, dtype=torch.float64, device=cuda)
    ops.awq_sq_err_accum(ac, bc, out)
    assert abs(out.item() - 0.5 - want) <= 1e-12 * max(want, 1.0)


def test_awq_sq_err_two_phase_matches_accum(cuda):
    """qz_awq_sq_err_partials into rows of one buffer + ONE qz_awq_sq_err_reduce == one
    qz_awq_sq_err_accum per loss, bit for bit (the same fixed-order tree), for several output
    shapes (each reduce call has one partial count), strided rows, and the out[] accumulation."""
    g = torch.Generator().manual_seed(5)
    for shape, strided in (((2048, 768), False), ((333, 100), False), ((512, 768), True), ((1, 8), False)):
        n = 6
        pairs = []
        for _ in range(n):
            a = torch.randn(*shape, generator=g).to(torch.bfloat16).to(cuda)
            b = (a.float() + torch.randn(*shape, generator=g).to(cuda) * 0.01).to(torch.bfloat16)
            if strided:
                big = torch.zeros(shape[0], shape[1] + 64, dtype=torch.bfloat16, device=cuda)
                big[:, :shape[1]] = a
                a = big[:, :shape[1]]
            pairs.append((a, b))
        nb = ops.awq_sq_err_partials_count(shape)
        assert nb >= 1
        part = torch.full((n, nb + 3), float("nan"), dtype=torch.float64, device=cuda)  # padded rows
        for i, (a, b) in enumerate(pairs):
            ops.awq_sq_err_partials(a, b, part[i])
        got = torch.full((n,), 0.25, dtype=torch.float64, device=cuda)
        ops.awq_sq_err_reduce(part, nb, got)
        want = torch.full((n,), 0.25, dtype=torch.float64, device=cuda)
        for i, (a, b) in enumerate(pairs):
            ops.awq_sq_err_accum(a, b, want[i:i + 1])
        assert torch.equal(got.cpu(), want.cpu()), (shape, got, want)
    with pytest.raises(ValueError):
        ops.awq_sq_err_reduce(part, nb + 4, got)


@pytest.mark.parametrize("n_b", [1, 3, 8])
def test_awq_sq_err_partials_multi_matches_single(cuda, n_b):
    """One launch over n_b outputs sharing a reference == n_b single-output partial launches, bit
    for bit (rows of the partial table, then the reduced losses)."""
    g = torch.Generator(device=cuda).manual_seed(n_b)
    shape = (1000, 264)
    a = torch.randn(*shape, device=cuda, generator=g).to(torch.bfloat16)
    bs = [(a.float() + torch.randn(*shape, device=cuda, generator=g) * 0.01).to(torch.bfloat16) for _ in range(n_b)]
    nb = ops.awq_sq_err_partials_count(shape)
    got = torch.full((n_b, nb + 2), float("nan"), dtype=torch.float64, device=cuda)
    want = torch.full_like(got, float("nan"))
    ops.awq_sq_err_partials_multi(a, bs, got)
    for i, b in enumerate(bs):
        ops.awq_sq_err_partials(a, b, want[i])
    assert torch.equal(got[:, :nb].cpu(), want[:, :nb].cpu())
    assert torch.isnan(got[:, nb:]).all()  # nothing written past the partial count
    with pytest.raises(ValueError):
        ops.awq_sq_err_partials_multi(a, bs * 9, got)


@pytest.mark.parametrize("scheme", [SCHEMES[i] for i in (0, 3, 11, 15, 17, 18)], ids=_id)
def test_large_launch_nontemporal_path(cuda, scheme):
    """Launches above 256 MiB take the non-temporal load/store variants (group, tile and NVFP4
    absmax kernels): one [9, 4096, 4096] launch == nine per-slice launches (which take the
    oracle-checked default path)."""
    a = QuantizationArgs(**scheme)
    g = torch.Generator(device=cuda).manual_seed(9)
    w = (torch.randn(9, 4096, 4096, device=cuda, generator=g) * 0.02).to(torch.bfloat16)
    assert w.numel() * 2 > 256 << 20
    big = ops.compress_weight(w, a)
    for e in (0, 4, 8):
        one = ops.compress_weight(w[e], a)
        for k, v in one.items():
            if k == "weight_shape":
                continue
            gv = big[k][e] if big[k].dim() > 1 or k != "weight_global_scale" else big[k][e:e + 1]
            _eq(gv.reshape(v.shape), v)
    if not a.is_nvfp4:  # AWQ fake-quant with column scales, non-temporal variant
        s = torch.rand(4096, device=cuda, generator=g) + 0.5
        fq = ops.fake_quantize(w, a, col_scales=s)
        _eq(fq[5], ops.fake_quantize(w[5], a, col_scales=s))


FULL = [dict(num_bits=4, type="int", symmetric=False, group_size=128),
        dict(num_bits=4, type="int", symmetric=True, group_size=32),
        dict(num_bits=8, type="float", group_size=32),
        dict(num_bits=8, type="float", strategy="block", block_structure=[128, 128]),
        dict(num_bits=4, type="float", group_size=32, scale_dtype="uint8"),
        dict(num_bits=4, type="float", strategy="tensor_group", group_size=16, scale_dtype="float8_e4m3fn")]


@pytest.mark.parametrize("scheme", FULL, ids=_id)
def test_full_size_parity_c_oracle(cuda, scheme):
    """BASELINE shape [11008, 4096] (with 0.1 % x20 outliers and an all-zero group row):
    every on-disk tensor bit-identical to the plain-C oracle (oracle/quant_ref.c)."""
    import qref
    a = QuantizationArgs(**scheme)
    g = torch.Generator().manual_seed(21)
    w = torch.randn(11008, 4096, generator=g) * 0.02
    mask = torch.rand(11008, 4096, generator=g) < 1e-3
    w[mask] *= 20
    w[5, :256] = 0.0  # all-zero groups (D1)
    w = w.to(torch.bfloat16)
    want = qref.compress_weight(w, _oracle_args(a))
    got = ops.compress_weight(w.to(cuda), a)
    want = {k: v for k, v in want.items() if not k.startswith("_")}
    assert set(got) == set(want), (set(got), set(want))
    for k, v in want.items():
        _eq(got[k], v)


def test_quantize_many_equals_single_calls(cuda):
    """qz_quantize_many (one host call, one launch per weight) == qz_quantize per weight, with
    distinct output buffers per item; and the bench's prepare_many (shared outputs) leaves the
    last weight's result."""
    import ctypes
    a = QuantizationArgs(num_bits=4, type="int", symmetric=True, group_size=128)
    ws = [_edge_weight(96, 1024, 128, seed=s).to(cuda) for s in range(3)]
    ref = [ops.compress_weight(w, a) for w in ws]
    outs = [ops.quantize_weight(torch.zeros_like(w), a) for w in ws]
    lib = _lib.load()
    n = len(ws)
    arr = lambda ts: (ctypes.c_void_p * n)(*[t.data_ptr() for t in ts])
    ca = a.to_c()
    nb = lib.qz_quantize_workspace_size(1, 96, 1024, ctypes.byref(ca))
    wsp = torch.empty(max(nb, 256), dtype=torch.uint8, device=cuda)
    rc = lib.qz_quantize_many(n, arr(ws), arr([o["codes"] for o in outs]), arr([o["scale"] for o in outs]), None,
                              None, 1, 96, 1024, 1024, 96 * 1024, ctypes.byref(ca), ops.default_out_fmt(a),
                              ctypes.c_void_p(wsp.data_ptr()), wsp.numel(),
                              ctypes.c_void_p(torch.cuda.current_stream().cuda_stream))
    assert rc == 0
    torch.cuda.synchronize()
    for o, r in zip(outs, ref):
        assert torch.equal(o["codes"].cpu(), r["weight_packed"].cpu())
        assert torch.equal(o["scale"].cpu().view(torch.int16), r["weight_scale"].cpu().view(torch.int16))
    assert lib.qz_quantize_many(-1, None, None, None, None, None, 1, 96, 1024, 1024, 96 * 1024, ctypes.byref(ca),
                                0, None, 0, None) == _lib.QZ_ERR_SHAPE
    prep = ops.PreparedQuantize(ws[0], a, {"codes": outs[0]["codes"], "scale": outs[0]["scale"],
                                           "zero_point": outs[0]["zero_point"]})
    prep.prepare_many(ws)()
    torch.cuda.synchronize()
    assert torch.equal(outs[0]["codes"].cpu(), ref[-1]["weight_packed"].cpu())


FP8_BLOCK = dict(num_bits=8, type="float", strategy="block", block_structure=[128, 128])


@pytest.mark.parametrize("shape", [(128, 128), (256, 256), (384, 384), (128, 640), (256, 768), (512, 2560),
                                   (1024, 4096)])
def test_fp8_block_strip_widths_c_oracle(cuda, shape):
    """FP8_BLOCK's strip kernel (qz_block.hip) at every strip width it picks -- 1, 2 or 4 blocks per
    workgroup from cols / 128 = 1, 2, 3, 5, 6, 20, 32 -- and on a row-strided view (the same
    weight's columns inside a wider tensor, ld_row > cols): codes and block scales bit-identical to
    the plain-C oracle (edge weight: outliers, an all-zero block row start, exact ties)."""
    import qref
    a = QuantizationArgs(**FP8_BLOCK)
    r, c = shape
    w = _edge_weight(r, c, 128, seed=r + c)
    want = qref.compress_weight(w, _oracle_args(a))
    got = ops.compress_weight(w.to(cuda), a)
    _eq(got["weight"], want["weight"])
    _eq(got["weight_scale"], want["weight_scale"])
    wide = torch.zeros(r, c + 256, dtype=torch.bfloat16, device=cuda)
    wide[:, 64:64 + c] = w.to(cuda)
    q = ops.quantize_weight(wide[:, 64:64 + c], a)  # ld_row = c + 256, 128-B aligned start
    _eq(q["codes"], want["weight"])
    _eq(q["scale"], want["weight_scale"])


def test_fp8_block_batch_and_zero_blocks(cuda):
    """A strided [E, r, c] batch (every other slice of a stack) through the strip kernel == per
    slice; an all-zero block gets the eps scale (D1) and zero codes, a block holding +-448 * s ties
    rounds as the oracle does."""
    import qref
    a = QuantizationArgs(**FP8_BLOCK)
    g = torch.Generator(device=cuda).manual_seed(12)
    stack = (torch.randn(6, 256, 512, device=cuda, generator=g) * 0.02).to(torch.bfloat16)
    stack[2, :128, :128] = 0
    stack[4, 128:, 384:] *= 1000
    view = stack[::2]  # ld_batch = 2 * 256 * 512
    got = ops.quantize_weight(view, a)
    for i in range(3):
        want = qref.compress_weight(view[i].cpu(), _oracle_args(a))
        _eq(got["codes"][i], want["weight"])
        _eq(got["scale"][i], want["weight_scale"])
    assert got["scale"][1, 0, 0].float().item() == 0.0078125 and not got["codes"][1, :128, :128].view(torch.uint8).any()


def test_fp8_block_store_policies_agree(cuda):
    """A large batch launch and small per-slice launches of the strip kernel agree (the store
    policy was once chosen by launch size, qz_block.hip): a [9, 8192, 4096] batch (906 MB moved)
    == its nine per-slice launches (135 MB each), and slice 4 == the plain-C oracle."""
    import qref
    a = QuantizationArgs(**FP8_BLOCK)
    g = torch.Generator(device=cuda).manual_seed(14)
    w = (torch.randn(9, 8192, 4096, device=cuda, generator=g) * 0.02).to(torch.bfloat16)
    assert w.numel() * 3 > 768 << 20 and w[0].numel() * 3 < 768 << 20
    big = ops.quantize_weight(w, a)
    for e in range(9):
        one = ops.quantize_weight(w[e], a)
        _eq(big["codes"][e], one["codes"])
        _eq(big["scale"][e], one["scale"])
    want = qref.compress_weight(w[4].cpu(), _oracle_args(a))
    _eq(big["codes"][4], want["weight"])
    _eq(big["scale"][4], want["weight_scale"])


@pytest.mark.parametrize("scheme", ["int4_g128_sym", "int4_g32_asym", "int8_g64_sym", "fp8_g32", "mxfp4_g32",
                                    "fp8_block128"])
def test_quantize_grouped_equals_single_calls(cuda, scheme):
    """qz_quantize_grouped (n weights, ONE launch, per-weight pointer table) == quantize_weight per
    weight, bit for bit, in the small-launch path (3 weights) and in the large-launch path
    (nt loads, UNROLL 4 tiles: 9 x [4096, 4096] = 302 MB > 256 MiB).  FP8_BLOCK: the strip kernel
    in table mode (shapes divisible by its 128 x 128 blocks)."""
    a = {"int4_g128_sym": QuantizationArgs(num_bits=4, type="int", symmetric=True, group_size=128),
         "int4_g32_asym": QuantizationArgs(num_bits=4, type="int", symmetric=False, group_size=32),
         "int8_g64_sym": QuantizationArgs(num_bits=8, type="int", symmetric=True, group_size=64),
         "fp8_g32": QuantizationArgs(num_bits=8, type="float", symmetric=True, group_size=32),
         "mxfp4_g32": QuantizationArgs(num_bits=4, type="float", group_size=32, scale_dtype="uint8"),
         "fp8_block128": QuantizationArgs(**FP8_BLOCK)}[scheme]
    block = scheme == "fp8_block128"
    gsz = 128 if block else a.group_size
    for n, (r, c) in ((3, (128, 1024) if block else (96, 1024)), (9, (4096, 4096))):
        ws = [_edge_weight(r, c, gsz, seed=s).to(cuda) for s in range(n)]
        ref = [ops.quantize_weight(w, a) for w in ws]
        got = ops.GroupedQuantize(ws, a).run()
        torch.cuda.synchronize()
        for o, rf in zip(got, ref):
            assert torch.equal(o["codes"].cpu(), rf["codes"].cpu())
            assert torch.equal(o["scale"].cpu().view(torch.uint8), rf["scale"].cpu().view(torch.uint8))
            if not a.symmetric:
                assert torch.equal(o["zero_point"].cpu(), rf["zero_point"].cpu())
        del ws, ref, got
    # quantize_weights: grouped per shape + per-weight launches for the rest, same results
    shp = ((128, 256), (256, 512)) if block else ((64, 256), (32, 512))
    mix = [_edge_weight(*shp[0], gsz, seed=7).to(cuda), _edge_weight(*shp[1], gsz, seed=8).to(cuda),
           _edge_weight(*shp[0], gsz, seed=9).to(cuda)]
    for o, w in zip(ops.quantize_weights(mix, a), mix):
        rf = ops.quantize_weight(w, a)
        assert torch.equal(o["codes"].cpu(), rf["codes"].cpu())


@pytest.mark.parametrize("scheme", ["int4_g128_sym", "int4_g32_asym", "fp8_g32", "mxfp4_g32"])
def test_quantize_grouped_mixed_shapes(cuda, scheme):
    """qz_quantize_grouped_var: weights of different shapes (Qwen3-style q/k/o/gate/down, ragged
    row counts, a weight smaller than one tile) in ONE launch == quantize_weight per weight."""
    a = {"int4_g128_sym": QuantizationArgs(num_bits=4, type="int", symmetric=True, group_size=128),
         "int4_g32_asym": QuantizationArgs(num_bits=4, type="int", symmetric=False, group_size=32),
         "fp8_g32": QuantizationArgs(num_bits=8, type="float", symmetric=True, group_size=32),
         "mxfp4_g32": QuantizationArgs(num_bits=4, type="float", group_size=32, scale_dtype="uint8")}[scheme]
    shapes = [(512, 2560), (128, 2560), (320, 512), (2560, 1024), (3, 256), (1023, 768), (128, 2560)]
    ws = [_edge_weight(r, c, a.group_size, seed=s).to(cuda) for s, (r, c) in enumerate(shapes)]
    gq = ops.GroupedQuantize(ws, a)
    assert gq.mixed
    got = gq.run()
    for w, o in zip(ws, got):
        rf = ops.quantize_weight(w, a)
        assert torch.equal(o["codes"].cpu(), rf["codes"].cpu())
        assert torch.equal(o["scale"].cpu().view(torch.uint8), rf["scale"].cpu().view(torch.uint8))
        if not a.symmetric:
            assert torch.equal(o["zero_point"].cpu(), rf["zero_point"].cpu())


def test_quantize_grouped_rejects(cuda):
    import ctypes
    nv = QuantizationArgs(num_bits=4, type="float", strategy="tensor_group", group_size=16)
    w = _edge_weight(32, 256, 16, seed=1).to(cuda)
    w2 = _edge_weight(64, 256, 16, seed=2).to(cuda)
    with pytest.raises(ValueError):  # NVFP4 groups one shape per call (qz_quantize_grouped_nvfp4)
        ops.GroupedQuantize([w, w2], nv)
    a = QuantizationArgs(num_bits=4, type="int", symmetric=True, group_size=128)
    lib = _lib.load()
    tab = torch.zeros(4, dtype=torch.int64, device=cuda)
    st = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
    assert lib.qz_quantize_grouped(1, ctypes.c_void_p(tab.data_ptr()), 32, 256, ctypes.byref(nv.to_c()), 3,
                                   st) == _lib.QZ_ERR_FORMAT
    assert lib.qz_quantize_grouped(-1, ctypes.c_void_p(tab.data_ptr()), 32, 256, ctypes.byref(a.to_c()), 0,
                                   st) == _lib.QZ_ERR_SHAPE
    assert lib.qz_quantize_grouped(0, None, 32, 256, ctypes.byref(a.to_c()), 0, st) == 0
    with pytest.raises(ValueError):  # output aliasing a weight
        ops.GroupedQuantize([w], a, outs=[{"codes": w.view(torch.int32)[:, :32], "scale": w[:, :2],
                                           "zero_point": None}])


def test_reentrant_from_host_threads(cuda):
    """The ABI is stateless and reentrant (include/quantizers_amd.h): four host threads, each on
    its own stream, quantize / fake-quantize / grouped-quantize concurrently -- every result equals
    the serial one."""
    import threading
    a = QuantizationArgs(num_bits=4, type="int", symmetric=True, group_size=128)
    ws = [_edge_weight(512, 1024, 128, seed=40 + i).to(cuda) for i in range(4)]
    s = (torch.rand(1024, generator=torch.Generator().manual_seed(2)) + 0.5).to(cuda)
    ref = [(ops.quantize_weight(w, a), ops.fake_quantize(w, a, col_scales=s)) for w in ws]
    ref_g = ops.GroupedQuantize(ws, a).run()
    torch.cuda.synchronize()
    got, errs = [None] * 4, []

    def work(i):
        try:
            st = torch.cuda.Stream(cuda)
            with torch.cuda.stream(st):
                outs = []
                for _ in range(5):
                    outs.append((ops.quantize_weight(ws[i], a), ops.fake_quantize(ws[i], a, col_scales=s),
                                 ops.GroupedQuantize(ws, a).run(st)))
            st.synchronize()
            got[i] = outs
        except Exception as e:  # noqa: BLE001 -- reported below
            errs.append(e)

    th = [threading.Thread(target=work, args=(i,)) for i in range(4)]
    for t in th:
        t.start()
    for t in th:
        t.join(timeout=120)
    assert not errs, errs
    for i in range(4):
        for q, fq, g in got[i]:
            _eq(q["codes"], ref[i][0]["codes"])
            _eq(q["scale"], ref[i][0]["scale"])
            _eq(fq, ref[i][1])
            for o, r in zip(g, ref_g):
                _eq(o["codes"], r["codes"])


def test_whole_model_plan_equals_per_weight(cuda):
    """The headline workload in full: the product's CompressionPlan over all 252 Qwen3-4B linears
    (5 grouped launches, the bench's step) gives every on-disk tensor bit-identical to the
    per-weight launch of the same weight (itself oracle-checked at full size above), and one
    weight per shape matches the plain-C oracle outright."""
    import os
    import sys
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    import bench
    import qref
    from quantizers_amd.compressor import CompressionPlan, compression_units
    torch.manual_seed(3)
    model = bench.build_model(cuda)
    units, _ = compression_units(model)
    plan = CompressionPlan(units, cuda)
    assert plan.launches == 5 and len(units) == 252
    plan.run()
    got = plan.tensors()
    seen = set()
    for u in units:
        w = u.refs[0].weight
        ref = ops.compress_weight(w, u.scheme.weights)
        for k, v in ref.items():
            _eq(got[f"{u.refs[0].name}.{k}"], v)
        if tuple(w.shape) not in seen:
            seen.add(tuple(w.shape))
            want = qref.compress_weight(w.cpu(), _oracle_args(u.scheme.weights))
            for k, v in want.items():
                if not k.startswith("_"):
                    _eq(got[f"{u.refs[0].name}.{k}"], v)
    assert len(seen) == 5
    del model, plan, got
    torch.cuda.empty_cache()


def test_whole_model_plan_mixed_fp8_block_int4(cuda):
    """BASELINE.json configs[2] through the product: the mixed recipe (FP8_BLOCK q/k/v/o + int4 g32
    gate/up/down, configs/recipes/mixed_fp8_block_awq_int4.yaml = the reference's
    recipe_mixed_fp8_int4.yaml, quirk M1 corrected) on the Qwen3-4B model is 5 grouped launches --
    q, k+v and o through the FP8_BLOCK strip kernel, gate+up and down through the group kernel --
    and every on-disk tensor equals the per-weight launch; one weight per shape also vs the
    plain-C oracle."""
    import os
    import sys
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    import bench
    import qref
    from quantizers_amd.compressor import CompressionPlan, compression_units
    torch.manual_seed(6)
    model = bench.build_model(cuda, bench.MIXED_RECIPE)
    units, _ = compression_units(model)
    plan = CompressionPlan(units, cuda)
    assert len(units) == 252 and plan.launches == 5 and not plan.singles
    assert sum(1 for gq, *_ in plan.grouped if ops.is_fp8_block128(gq.a)) == 3
    plan.run()
    got = plan.tensors()
    seen = set()
    for u in units:
        w = u.refs[0].weight
        ref = ops.compress_weight(w, u.scheme.weights)
        for k, v in ref.items():
            _eq(got[f"{u.refs[0].name}.{k}"], v)
        if tuple(w.shape) not in seen:
            seen.add(tuple(w.shape))
            want = qref.compress_weight(w.cpu(), _oracle_args(u.scheme.weights))
            for k, v in want.items():
                if not k.startswith("_"):
                    _eq(got[f"{u.refs[0].name}.{k}"], v)
    assert len(seen) == 5
    del model, plan, got
    torch.cuda.empty_cache()


def test_whole_model_plan_nvfp4_two_streams(cuda):
    """recipe_Dense_NVFP4 on the Qwen3-4B model: the CompressionPlan's 7 grouped NVFP4 calls, run
    over two streams (ops.nvfp4_streams), give every on-disk tensor bit-identical to the per-weight
    call; one weight per shape also vs the plain-C oracle."""
    import os
    import sys
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    import bench
    import qref
    from quantizers_amd.compressor import CompressionPlan, compression_units
    from quantizers_amd.quantization import preset_scheme
    torch.manual_seed(4)
    model = bench.build_model(cuda)
    nv = preset_scheme("NVFP4", ["Linear"])
    model.quantization_scheme_map = {n: nv for n in model.quantization_scheme_map}
    units, _ = compression_units(model)
    plan = CompressionPlan(units, cuda)
    assert sum(1 for gq, *_ in plan.grouped if gq.nvfp4) == 5 and len(units) == 252
    plan.run()
    got = plan.tensors()
    seen = set()
    for u in units:
        w = u.refs[0].weight
        ref = ops.compress_weight(w, u.scheme.weights)
        for k, v in ref.items():
            _eq(got[f"{u.refs[0].name}.{k}"], v)
        if tuple(w.shape) not in seen:
            seen.add(tuple(w.shape))
            want = qref.compress_weight(w.cpu(), _oracle_args(u.scheme.weights))
            for k, v in want.items():
                if not k.startswith("_"):
                    _eq(got[f"{u.refs[0].name}.{k}"], v)
    del model, plan, got
    torch.cuda.empty_cache()


def test_stats_one_launch_stress_many_grids(cuda):
    """the one-launch statistics reductions hand partials between workgroups through
    agent-coherent stores / loads and counters (no release / acquire fence).  Over 24 grid shapes
    (1 to 64 chunks per window, ragged windows, both statistics), each call repeated while a GEMM
    stream loads the card, every result equals the restated fixed-order tree bit for bit and the
    counters are left zero."""
    import numpy as np
    rng = np.random.default_rng(7)
    side = torch.cuda.Stream()
    junk = torch.randn(2048, 2048, device=cuda)
    for case in range(24):
        which = "absmean" if case % 2 == 0 else "wmean"
        cols = int(rng.choice([264, 520, 1032, 2048, 2560, 4096]))
        g = int(rng.choice([32, 64, 128])) if which == "wmean" else 0
        cols -= cols % max(g, 8)
        rows = int(rng.integers(8, 9000))
        x = _w(rows, cols, seed=1000 + case, scale=0.02 if which == "wmean" else 1.0)
        xd = x.to(cuda)
        if which == "absmean":
            lay = ops.awq_stats_layout("absmean", rows, cols)
            want = torch.from_numpy(_stats_tree(x.float().abs().numpy(), lay, np.float32))
        else:
            want = _wmean_tree(x, g)
        for rep in range(3):
            with torch.cuda.stream(side):
                for _ in range(2):
                    junk = junk @ junk.T / 2048
            out = torch.zeros(cols, dtype=torch.float32 if which == "absmean" else torch.float64, device=cuda)
            if which == "absmean":
                ops.awq_absmean_accum(xd, out)
            else:
                ops.awq_weight_mean_accum(xd, g, out)
            torch.cuda.synchronize()
            assert torch.equal(out.cpu(), want), (case, which, rows, cols, g, rep)
    for buf in ops._stats_ws_cache.values():
        assert not buf[:32768].any()


def _slices_vs_single_and_oracle(stack_view, a, out, oracle_slices):
    """Every slice of a batched launch's outputs == the per-slice launch; ``oracle_slices`` of them
    also == the plain-C oracle."""
    import qref
    for e in range(stack_view.shape[0]):
        one = ops.quantize_weight(stack_view[e], a)
        _eq(out["codes"][e], one["codes"])
        _eq(out["scale"][e], one["scale"])
    for e in oracle_slices:
        want = qref.compress_weight(stack_view[e].cpu(), _oracle_args(a))
        codes = want.get("weight_packed", want.get("weight"))
        _eq(out["codes"][e], codes)
        _eq(out["scale"][e], want["weight_scale"])


def test_bench_config4_mxfp4_expert_halves_full_size(cuda):
    """VERDICT r04 item 3, BASELINE.json configs[3] exactly as bench.py times it: MXFP4 over the
    strided gate / up halves gu[:, :768], gu[:, 768:] of one Qwen3-30B-A3B fused parameter
    [128, 1536, 2048] and over the down projections [128, 2048, 768] -- one launch each through the
    non-temporal path (403 MB / 201 MB per launch) -- every slice equals its own launch, two slices
    per launch equal the plain-C oracle (reference configs/test-quantize_qwen3_30b_a3b_nvfp4.yaml:18-25
    names the model; MXFP4 is BASELINE's scheme)."""
    mx = QuantizationArgs(num_bits=4, type="float", group_size=32, scale_dtype="uint8")
    g = torch.Generator(device=cuda).manual_seed(31)
    gu = (torch.randn(128, 1536, 2048, device=cuda, generator=g) * 0.02).to(torch.bfloat16)
    gu[7, 100, :64] *= 300  # outliers in one slice
    dn = (torch.randn(128, 2048, 768, device=cuda, generator=g) * 0.02).to(torch.bfloat16)
    for view in (gu[:, :768], gu[:, 768:], dn):
        assert view.numel() * 2 > 200 << 20
        out = ops.quantize_weight(view, mx)
        _slices_vs_single_and_oracle(view, mx, out, (7, 127))
        del out


def test_bench_config5_minimax_full_size(cuda):
    """VERDICT r04 item 3, BASELINE.json configs[4] as bench.py's minimax_pass times it
    (recipe_Minimax-M2.1-AWQ-MixedPrec.yaml:24-48): int4 sym g32 over the strided w1 / w3 halves of
    a fused [256, 3072, 3072] parameter and the w2 [256, 3072, 1536] stack, FP8 g32 over the
    attention q [6144, 3072] and o [3072, 6144]: every slice == its own launch, two slices per
    launch and both attention weights == the plain-C oracle."""
    import qref
    i4 = QuantizationArgs(num_bits=4, type="int", symmetric=True, group_size=32)
    f8 = QuantizationArgs(num_bits=8, type="float", symmetric=True, group_size=32)
    g = torch.Generator(device=cuda).manual_seed(32)
    gu = (torch.randn(256, 3072, 3072, device=cuda, generator=g) * 0.02).to(torch.bfloat16)
    for view in (gu[:, :1536], gu[:, 1536:]):
        out = ops.quantize_weight(view, i4)
        _slices_vs_single_and_oracle(view, i4, out, (0, 255))
        del out
    del gu
    dn = (torch.randn(256, 3072, 1536, device=cuda, generator=g) * 0.02).to(torch.bfloat16)
    out = ops.quantize_weight(dn, i4)
    _slices_vs_single_and_oracle(dn, i4, out, (3, 200))
    del dn, out
    for r, c in ((6144, 3072), (3072, 6144)):
        w = (torch.randn(r, c, device=cuda, generator=g) * 0.02).to(torch.bfloat16)
        got = ops.compress_weight(w, f8)
        want = qref.compress_weight(w.cpu(), _oracle_args(f8))
        _eq(got["weight"], want["weight"])
        _eq(got["weight_scale"], want["weight_scale"])
    torch.cuda.empty_cache()


def test_write_through_tail_gate_and_alignment(cuda):
    """Round 6's write-through tail rules (qz_device.h wt_tail_from, qz_quant.hip encode_store):
    a grouped int4 g128 launch writing >= 64 MiB of codes takes the tail, smaller launches do not,
    and a table entry whose codes are only 4-B aligned keeps the 4-B stores inside a tail launch --
    every case bit-identical to per-weight launches.  The misaligned table goes through the C ABI
    (GroupedQuantize refuses codes that are not 16-B aligned, the header's contract)."""
    import ctypes
    from quantizers_amd import _lib
    a = QuantizationArgs(num_bits=4, type="int", symmetric=True, group_size=128)
    r, c = 4096, 4096  # 8 MiB of codes per weight: 9 weights = 72 MiB (tail), 3 = 24 MiB (no tail)
    ws = [_edge_weight(r, c, 128, seed=40 + s).to(cuda) for s in range(9)]
    ref = [ops.quantize_weight(w, a) for w in ws]
    for n in (3, 9):
        got = ops.GroupedQuantize(ws[:n], a).run()
        torch.cuda.synchronize()
        for o, rf in zip(got, ref):
            assert torch.equal(o["codes"], rf["codes"]) and torch.equal(o["scale"].view(torch.int16),
                                                                         rf["scale"].view(torch.int16))
    # codes of every other weight 4 bytes past a 16-B boundary
    nw = r * c // 8
    bufs = [torch.zeros(nw + 4, dtype=torch.int32, device=cuda) for _ in ws]
    codes = [b[1:1 + nw].view(r, c // 8) if i % 2 else b[:nw].view(r, c // 8) for i, b in enumerate(bufs)]
    scales = [torch.empty(r, c // 128, dtype=torch.bfloat16, device=cuda) for _ in ws]
    assert all(codes[i].data_ptr() % 16 == 4 for i in range(1, 9, 2))
    with pytest.raises(ValueError):
        ops.GroupedQuantize(ws, a, outs=[{"codes": cd, "scale": sc, "zero_point": None}
                                         for cd, sc in zip(codes, scales)])
    table = torch.tensor([[w.data_ptr() for w in ws], [cd.data_ptr() for cd in codes],
                          [sc.data_ptr() for sc in scales], [0] * 9], dtype=torch.int64).reshape(-1).to(cuda)
    lib, ca = _lib.load(), a.to_c()
    rc = lib.qz_quantize_grouped(9, ctypes.c_void_p(table.data_ptr()), r, c, ctypes.byref(ca),
                                 _lib.QZ_OUT_PACKED_INT32, ops._stream())
    assert rc == 0
    torch.cuda.synchronize()
    for cd, sc, rf in zip(codes, scales, ref):
        assert torch.equal(cd, rf["codes"]) and torch.equal(sc.view(torch.int16), rf["scale"].view(torch.int16))


@pytest.mark.parametrize("scheme", ["int4_g128_sym", "int4_g32_asym", "int8_channel_sym", "fp8_g32", "fp8_block128"])
def test_kernel_scales_match_torch_affine_quantization(cuda, scheme):
    """The kernels' bf16 scales (and int zero points) against torch's own quantization code directly
    (torch.ao.quantization.pt2e._affine_quantization._choose_qparams_affine, torchao's algorithm;
    the oracle-side pin is tests/test_torchao_pin.py): scales bit for bit; asymmetric zero points
    equal wherever compressed-tensors' extra bf16 rounding of qmin - min / s does not cross a
    half-integer."""
    from torch.ao.quantization.pt2e._affine_quantization import _choose_qparams_affine
    a, block, tdt = {
        "int4_g128_sym": (QuantizationArgs(num_bits=4, type="int", symmetric=True, group_size=128), [1, 128], torch.int8),
        "int4_g32_asym": (QuantizationArgs(num_bits=4, type="int", symmetric=False, group_size=32), [1, 32], torch.int8),
        "int8_channel_sym": (QuantizationArgs(num_bits=8, type="int", symmetric=True, strategy="channel"), [1, 2048],
                             torch.int8),
        "fp8_g32": (QuantizationArgs(num_bits=8, type="float", symmetric=True, group_size=32), [1, 32],
                    torch.float8_e4m3fn),
        "fp8_block128": (QuantizationArgs(**FP8_BLOCK), [128, 128], torch.float8_e4m3fn)}[scheme]
    g = torch.Generator().manual_seed(77)
    w = (torch.randn(512, 2048, generator=g) * (torch.rand(512, 1, generator=g) * 0.05 + 1e-3)).to(torch.bfloat16)
    got = ops.quantize_weight(w.to(cuda), a)
    torch.cuda.synchronize()
    qmin, qmax = (-8, 7) if a.num_bits == 4 else (-128, 127)
    kw = {} if tdt == torch.float8_e4m3fn else {"quant_min": qmin, "quant_max": qmax}
    s_ao, z_ao = _choose_qparams_affine(w, "SYMMETRIC" if a.symmetric else "ASYMMETRIC", block, tdt,
                                        eps=torch.finfo(torch.bfloat16).tiny, **kw)
    assert torch.equal(got["scale"].cpu().reshape(-1).view(torch.int16), s_ao.reshape(-1).view(torch.int16))
    if not a.symmetric:
        zp = got["zero_point"].cpu().reshape(-1).float()
        mn = torch.min(w.reshape(-1, block[1]).amin(-1), torch.zeros(1, dtype=torch.bfloat16))
        q = mn / s_ao.reshape(-1)
        same = (qmin - torch.round(q.float())) == torch.round((qmin - q).float())
        assert torch.equal(zp[same], z_ao.reshape(-1).float()[same])
        assert (~same).sum() <= max(2, same.numel() // 1000)
