"""D8, bf16 reading (the default): the statistics kernels' own sums fed to the literal oracle's
combination steps reproduce the product's bf16 x_mean and w_mean bit for bit.

The product computes each calibration batch's sum |x| per channel in f32 (``k_absmean_1l`` /
``k_absmean_seg``) and each balance layer's column sum of the group-normalised |W| in f64
(``k_wmean_1l`` / ``k_wmean_seg``); llmcompressor's ``_accumulate_mean`` / ``_compute_layer_means``
then combine them in bf16 (oracle/ct_torch.awq_running_mean_from_sums_literal /
awq_layer_means_from_sums_literal, device semantics).  Given the kernels' sums, the only freedom
left is none: bit-identical.  Against the fully literal oracle (torch's bf16 sums on the CPU, CPU
division) the product differs by summation order only: within 1 bf16 ulp on a few channels.
"""
import pytest
import torch

import ct_torch as ct
from quantizers_amd import awq

pytestmark = pytest.mark.gpu


def _ulp(a, b):
    return (a.view(torch.int16).int() - b.view(torch.int16).int()).abs()


@pytest.mark.parametrize("segmented", [False, True])
def test_x_mean_from_kernel_sums(cuda, segmented):
    g = torch.Generator().manual_seed(21)
    C = 2560
    xs = [(torch.randn(n, C, generator=g) * 10.0 ** torch.empty(C).uniform_(-2, 1, generator=g)).to(torch.bfloat16)
          for n in (2048, 2048, 17, 1, 1000, 2048)]
    am = awq._AbsMean(bf16=True)
    if segmented:
        am.add_samples([x.to(cuda) for x in xs])
    else:
        for x in xs:
            am.add(x.to(cuda))
    got = am.mean().cpu()
    sums = [(p.cpu(), n) for p, n in am.parts]
    assert [n for _, n in sums] == [x.shape[0] for x in xs]
    want = ct.awq_running_mean_from_sums_literal(sums, device_division=True)[0]
    assert torch.equal(got.view(torch.int16), want.view(torch.int16))
    lit = None
    for x in xs:
        lit = ct.awq_accumulate_mean_literal(x, lit)
    d = _ulp(got, lit[0])
    assert d.max() <= 1 and (d > 0).float().mean() < 0.02, (int(d.max()), float((d > 0).float().mean()))


def test_w_mean_from_kernel_sums(cuda):
    g = torch.Generator().manual_seed(22)
    ws = [(torch.randn(r, 2560, generator=g) * 0.02).to(torch.bfloat16) for r in (9728, 9728, 1024)]
    parts = awq._w_mean_parts([(w.to(cuda), 128) for w in ws], 2560, cuda)
    assert [n for _, n in parts] == [w.shape[0] for w in ws]
    assert all(p.dtype == torch.float64 for p, _ in parts)
    got = awq._layer_means_bf16(parts).cpu()
    want = ct.awq_layer_means_from_sums_literal([(p.cpu(), n) for p, n in parts], device_division=True)
    assert torch.equal(got.view(torch.int16), want.view(torch.int16))
    lit = ct.awq_layer_means_literal(ws, ct.QArgs(group_size=128))
    d = _ulp(got, lit)
    assert d.max() <= 1 and (d > 0).float().mean() < 0.02, (int(d.max()), float((d > 0).float().mean()))
