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
    d = (got.view(torch.int16).int() - prev[0].view(torch.int16).int()).abs()
    assert d.max() <= 1 and (d > 0).float().mean() < 0.02  # per-batch sums: f32 order vs torch's bf16 sum
    exact = awq._running_mean_bf16([(x.abs().sum(0).float(), x.shape[0]) for x in xs])  # torch's own batch sums
    assert torch.equal(exact.view(torch.int16), prev[0].view(torch.int16))
    assert awq._running_mean_bf16([(torch.zeros(4), 0)]) is None


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
