"""D8, bf16 reading (awq.AWQ_DTYPE = "bf16"): the product's host-side helpers restate the literal
oracle (oracle/ct_torch.*_literal) -- CPU, no GPU: the bf16 running mean over per-batch f32 sums
and the bf16 grid-scale formula ([C] and batched [B, C]) are torch ops whose bits this checks."""
import pytest
import torch

import ct_torch as ct
from quantizers_amd import awq


def test_running_mean_bf16_matches_literal_oracle():
    g = torch.Generator().manual_seed(3)
    xs = [(torch.randn(n, 256, generator=g) * 10.0 ** torch.empty(256).uniform_(-2, 1, generator=g)).to(torch.bfloat16)
          for n in (64, 17, 1, 128)]
    prev = None
    for x in xs:
        prev = ct.awq_accumulate_mean_literal(x, prev)
    parts = [(x.abs().float().sum(0), x.shape[0]) for x in xs]
    got = awq._running_mean_bf16(parts)
    # against the CPU reading (true division) and f32 batch sums in another order: within 1 ulp
    d = (got.view(torch.int16).int() - prev[0].view(torch.int16).int()).abs()
    assert d.max() <= 1 and (d > 0).float().mean() < 0.02
    # torch's own batch sums: bit for bit with the device reading (reciprocal division)
    dev_prev = None
    for x in xs:
        dev_prev = ct.awq_accumulate_mean_literal(x, dev_prev, device_division=True)
    exact = awq._running_mean_bf16([(x.abs().sum(0).float(), x.shape[0]) for x in xs])
    assert torch.equal(exact.view(torch.int16), dev_prev[0].view(torch.int16))
    assert awq._running_mean_bf16([(torch.zeros(4), 0)]) is None


def test_oracle_from_kernel_sums_reproduces_product():
    """fed the statistics kernels' own sums (absmean: f32 per calibration
    batch; w_mean: f64 per balance layer), the literal oracle's combination steps
    (ct_torch.awq_running_mean_from_sums_literal / awq_layer_means_from_sums_literal, device
    semantics) give the product's bf16 x_mean and w_mean bit for bit -- single operand
    (_running_mean_bf16, _layer_means_bf16) and batched over experts (_running_means_bf16).  What
    is left between the product and the fully literal oracle is the kernels' summation order
    (f32 / f64 vs torch's bf16 sum) and the device powf of the grid formula."""
    g = torch.Generator().manual_seed(11)
    C = 512
    for trial in range(6):
        nb = 1 + trial * 3
        counts = [int(v) for v in torch.randint(0, 2049, (nb,), generator=g)]
        counts[0] = max(counts[0], 1)
        scale = 10.0 ** torch.empty(C).uniform_(-3, 2, generator=g)
        sums = [(torch.rand(C, generator=g) * scale * n).float() for n in counts]
        want = ct.awq_running_mean_from_sums_literal(list(zip(sums, counts)), device_division=True)[0]
        got = awq._running_mean_bf16(list(zip(sums, counts)))
        assert torch.equal(got.view(torch.int16), want.view(torch.int16)), trial
        batched = awq._running_means_bf16(torch.stack(sums)[None], [counts])[0]
        assert torch.equal(batched.view(torch.int16), want.view(torch.int16)), trial
        rows = [int(v) for v in torch.randint(1, 20000, (1 + trial % 4,), generator=g)]
        wsums = [(torch.rand(C, generator=g, dtype=torch.float64) * r * 0.6) for r in rows]
        want_w = ct.awq_layer_means_from_sums_literal(list(zip(wsums, rows)), device_division=True)
        got_w = awq._layer_means_bf16(list(zip(wsums, rows)))
        assert got_w.dtype == torch.bfloat16
        assert torch.equal(got_w.view(torch.int16), want_w.view(torch.int16)), trial


def test_device_and_cpu_division_rarely_differ_on_bf16():
    """D8's one device-dependent op, bf16 tensor / count: torch's GPU form (product with the f32
    reciprocal) and its CPU form (true division) differ by at most 1 ulp and almost never -- an
    8-bit dividend over an integer count lands within the reciprocal's error of a bf16 rounding
    midpoint only for rare (mantissa, count) pairs, at every exponent of such a mantissa (243 of
    325,120,000 (bf16, count) pairs over every positive normal bf16 and the counts 1, 8, ...,
    69994; 241 here, where three of the eleven counts are such counts: 49351, 54503, 65535).
    Every positive normal bf16 against these counts: the departure of the product's device form
    from the CPU reading."""
    import numpy as np
    u = np.arange(0x0080, 0x7F80, dtype=np.uint32)
    t = torch.from_numpy((u << 16).view(np.float32)).to(torch.bfloat16)
    diff = 0
    counts = (1, 3, 7, 100, 2047, 2048, 16383, 32768, 49351, 54503, 65535)
    for n in counts:
        a = ct.div_scalar_bf16(t, n, True).view(torch.int16).int()
        b = ct.div_scalar_bf16(t, n, False).view(torch.int16).int()
        assert (a - b).abs().max() <= 1
        diff += int((a != b).sum())
    assert 0 < diff < 1e-3 * t.numel() * len(counts), diff


@pytest.mark.parametrize("duo", [True, False])
def test_grid_scales_bf16_matches_literal_oracle(duo):
    g = torch.Generator().manual_seed(4)
    xm = (torch.rand(4, 512, generator=g) * 3).to(torch.bfloat16)
    wm = (torch.rand(4, 512, generator=g)).to(torch.bfloat16)
    xm[1, 7] = 0.0  # a dead channel: 0^r, clamp
    for r in (0.0, 0.05, 0.5, 0.95):
        got = awq._grid_scales_bf16(xm, wm, r, duo)
        assert got.dtype == torch.float32
        for b in range(4):
            want = ct.awq_grid_scales_literal(xm[b], wm[b], r, duo)
            assert torch.equal(got[b].to(torch.bfloat16).view(torch.int16), want.view(torch.int16)), (r, b)
            assert torch.equal(got[b], awq._grid_scales_bf16(xm[b], wm[b], r, duo))
        out = torch.empty(4, 512)
        assert awq._grid_scales_bf16(xm, wm, r, duo, out=out) is out and torch.equal(out, got)


def test_awq_dtype_validated():
    with pytest.raises(ValueError):
        awq.awq_layer(torch.nn.Module(), "x", [], [], {}, awq_dtype="fp16")


def test_stats_segments_validate_arguments():
    """The segmented statistics wrappers reject operands the C side must never see (checked on
    the host before any launch)."""
    from quantizers_amd import ops
    x = torch.zeros(4, 64, dtype=torch.bfloat16)
    with pytest.raises(ValueError):  # host tensors
        ops.awq_absmean_segments([x], [torch.zeros(64)])
    assert ops.awq_absmean_segments([], []) == [] and ops.awq_weight_mean_segments([], 128, []) == []


def test_running_means_batched_cpu_semantics():
    """awq._running_means_bf16 takes, per operand and batch, bf16(f32(m) * c), the bf16 sum and
    the product with the f32 reciprocal of the running count -- restated here step by step with
    NumPy f32 reciprocals (the GPU test compares it with the per-operand device loop)."""
    import numpy as np
    g = torch.Generator().manual_seed(5)
    E, P, C = 6, 7, 32
    counts = torch.randint(0, 6, (E, P), generator=g)
    counts[2] = 0
    counts[2, 5] = 4
    counts[4] = 0  # an operand that never saw a token: 0
    parts = torch.rand(E, P, C, generator=g) * 300
    got = awq._running_means_bf16(parts, counts.tolist())
    for e in range(E):
        m, c = torch.zeros(C, dtype=torch.bfloat16), 0
        for j in range(P):
            n = int(counts[e, j])
            if n == 0:
                continue
            sb = parts[e, j].to(torch.bfloat16)
            inv = float(np.float32(1.0) / np.float32(c + n))
            t = sb if c == 0 else (m.float() * float(c)).to(torch.bfloat16) + sb
            m = (t.float() * inv).to(torch.bfloat16)
            c += n
        assert torch.equal(got[e].view(torch.int16), m.view(torch.int16)), e
