"""AWQ golden fixture (tests/golden/awq_int4_g128.safetensors, made by make_awq_golden.py from
the oracle): a cross-round pin of the AWQ statistics, the 20 grid-scale vectors, the grid losses
and their argmin, Q(W*s)/s at the best ratio and the applied smoothing.

CPU: the oracle still reproduces the fixture (bit for bit; losses to 1e-9, CPU bf16 GEMM).
GPU: the HIP kernels on the fixture inputs -- statistics to the f32/f64 summation-order
tolerance, scales to 4 ulps, Q(W*s)/s and the smoothing bit for bit, losses (device GEMM) to
2e-3 and the same argmin."""
import os

import pytest
import torch
from safetensors.torch import load_file

import ct_torch as ct

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
FIX = os.path.join(ROOT, "tests", "golden", "awq_int4_g128.safetensors")
FIX_BF16 = os.path.join(ROOT, "tests", "golden", "awq_int4_g128_bf16.safetensors")  # D8 bf16 reading
OA = ct.QArgs(num_bits=4, type="int", symmetric=True, group_size=128)


def _bits_eq(a, b):
    assert a.shape == b.shape and a.dtype == b.dtype
    if a.dtype == torch.bfloat16:
        a, b = a.view(torch.int16), b.view(torch.int16)
    elif a.dtype == torch.float32:
        a, b = a.view(torch.int32), b.view(torch.int32)
    elif a.dtype == torch.float64:
        a, b = a.view(torch.int64), b.view(torch.int64)
    assert torch.equal(a, b)


@pytest.mark.parametrize("literal", [False, True], ids=["fp32", "bf16"])
def test_oracle_reproduces_awq_fixture(literal):
    import importlib.util
    spec = importlib.util.spec_from_file_location("make_awq_golden", os.path.join(ROOT, "tests", "golden",
                                                                                 "make_awq_golden.py"))
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    got = mod.build(literal)
    want = load_file(FIX_BF16 if literal else FIX)
    for k in ("x", "w", "x_mean", "w_mean", "scales", "best", "fq_best", "smoothed"):
        _bits_eq(got[k], want[k])
    torch.testing.assert_close(got["losses"], want["losses"], rtol=1e-9, atol=0)


@pytest.mark.gpu
def test_hip_awq_pipeline_matches_fixture(cuda):
    from quantizers_amd import ops
    from quantizers_amd.quantization import QuantizationArgs
    f = load_file(FIX)
    x, w = f["x"].to(cuda), f["w"].to(cuda)
    a = QuantizationArgs(num_bits=4, type="int", symmetric=True, group_size=128)
    sums = torch.zeros(x.shape[1], dtype=torch.float32, device=cuda)
    n = ops.awq_absmean_accum(x, sums)
    x_mean = sums / n
    torch.testing.assert_close(x_mean.cpu(), f["x_mean"], rtol=2e-6, atol=0)
    wsum = torch.zeros(x.shape[1], dtype=torch.float64, device=cuda)
    rows = ops.awq_weight_mean_accum(w, 128, wsum)
    torch.testing.assert_close((wsum / rows).cpu(), f["w_mean"], rtol=1e-13, atol=0)
    ref = torch.nn.functional.linear(x, w)
    losses = torch.zeros(20, dtype=torch.float64, device=cuda)
    xm_fix, wm_fix = f["x_mean"].to(cuda), f["w_mean"].float().to(cuda)
    for i in range(20):
        # the kernels' own statistics -> scales close to the fixture's
        s_dev = ops.awq_grid_scales(x_mean, (wsum / rows).float(), i / 20, True)
        torch.testing.assert_close(s_dev.cpu(), f["scales"][i], rtol=1e-5, atol=0)
        # the fixture's statistics -> the fixture's scales to 4 ulps (device powf / sqrtf vs torch)
        s = ops.awq_grid_scales(xm_fix, wm_fix, i / 20, True)
        torch.testing.assert_close(s.cpu(), f["scales"][i], rtol=4.8e-7, atol=0)
        # Q(W*s)/s with the fixture's exact scales: bit for bit
        fq = ops.fake_quantize(w, a, col_scales=f["scales"][i].to(cuda))
        if i == int(f["best"]):
            _bits_eq(fq.cpu(), f["fq_best"])
        out = torch.nn.functional.linear(x, fq)
        ops.awq_sq_err_accum(ref, out, losses[i:i + 1])
    losses = losses.cpu() / ref.numel()
    torch.testing.assert_close(losses, f["losses"], rtol=2e-3, atol=0)
    assert int(torch.argmin(losses)) == int(f["best"])
    best = f["scales"][int(f["best"])].to(cuda)
    sm = w.clone()
    ops.scale_columns_(sm, best, divide=False)
    _bits_eq(sm.cpu(), f["smoothed"])


def _ulps_bf16(a, b):
    """|a - b| in bf16 units of the last place (same-sign finite values)."""
    return (a.view(torch.int16).to(torch.int32) - b.view(torch.int16).to(torch.int32)).abs()


@pytest.mark.gpu
def test_hip_awq_pipeline_matches_bf16_fixture(cuda):
    """D8's bf16 reading through the product's own pieces (awq._AbsMean(bf16=True), awq._w_mean,
    awq._grid_scales_bf16, the fake-quant and smoothing kernels with bf16 scales): statistics and
    scale vectors within 1 bf16 ulp of the literal oracle (device vs CPU summation order / powf;
    almost all equal), Q(W*s)/s and the smoothing bit for bit for the fixture's scales, the 20
    losses to 2e-3 with the same argmin."""
    from quantizers_amd import awq, ops
    from quantizers_amd.model import LinearRef
    from quantizers_amd.quantization import QuantizationArgs
    f = load_file(FIX_BF16)
    x, w = f["x"].to(cuda), f["w"].to(cuda)
    a = QuantizationArgs(num_bits=4, type="int", symmetric=True, group_size=128)
    am = awq._AbsMean(bf16=True)
    am.add(x)
    xm = am.mean()
    assert xm.dtype == torch.bfloat16
    d = _ulps_bf16(xm.cpu(), f["x_mean"])
    assert d.max() <= 1 and (d > 0).float().mean() < 0.01, (int(d.max()), float((d > 0).float().mean()))
    lin = torch.nn.Linear(w.shape[1], w.shape[0], bias=False, dtype=torch.bfloat16, device=cuda)
    lin.weight.data = w
    ref_lin = LinearRef("w", lin, "weight", None)
    wm = awq._w_mean([[ref_lin]], {"w": a}, w.shape[1], True, cuda)
    d = _ulps_bf16(wm.cpu(), f["w_mean"])
    assert d.max() <= 1 and (d > 0).float().mean() < 0.01, (int(d.max()), float((d > 0).float().mean()))
    ref = torch.nn.functional.linear(x, w)
    losses = torch.zeros(20, dtype=torch.float64, device=cuda)
    for i in range(20):
        s = awq._grid_scales_bf16(f["x_mean"].to(cuda), f["w_mean"].to(cuda), i / 20, True)
        d = _ulps_bf16(s.cpu().to(torch.bfloat16), f["scales"][i])
        assert d.max() <= 1 and (d > 0).float().mean() < 0.01, (i, int(d.max()))
        fq = ops.fake_quantize(w, a, col_scales=f["scales"][i].float().to(cuda))
        if i == int(f["best"]):
            _bits_eq(fq.cpu(), f["fq_best"])
        ops.awq_sq_err_accum(ref, torch.nn.functional.linear(x, fq), losses[i:i + 1])
    losses = losses.cpu() / ref.numel()
    torch.testing.assert_close(losses, f["losses"], rtol=2e-3, atol=0)
    assert int(torch.argmin(losses)) == int(f["best"])
    sm = w.clone()
    ops.scale_columns_(sm, f["scales"][int(f["best"])].float().to(cuda), divide=False)
    _bits_eq(sm.cpu(), f["smoothed"])


@pytest.mark.gpu
def test_running_means_batched_equals_per_operand_gpu():
    """awq._running_means_bf16 (all experts of an expert search at once) == awq._running_mean_bf16
    per expert on the device, bit for bit: ragged token counts, batches an expert never saw
    (count 0, incl. its first batches), sums across many binades."""
    from quantizers_amd import awq
    dev = torch.device("cuda:0")
    g = torch.Generator().manual_seed(8)
    E, P, C = 37, 16, 768
    counts = torch.randint(0, 300, (E, P), generator=g)
    counts[counts < 60] = 0
    counts[3, :5] = 0
    counts[5, :] = 0
    counts[5, 9] = 1
    scale = 10.0 ** torch.empty(E, P, C).uniform_(-3, 2, generator=g)
    parts = (torch.rand(E, P, C, generator=g) * scale * counts[:, :, None].clamp(min=1)).float().to(dev)
    cl = counts.tolist()
    got = awq._running_means_bf16(parts, cl)
    for e in range(E):
        want = awq._running_mean_bf16([(parts[e, j], cl[e][j]) for j in range(P)])
        assert torch.equal(got[e].view(torch.int16), want.view(torch.int16)), e
