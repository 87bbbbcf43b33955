"""Guard bands around kernel outputs: every byte outside a kernel's output (and workspace) ranges
must be untouched.  Follows up the hipBLASLt/rocBLAS failure recorded in DESIGN.md (§6: bf16
bmm [16, 2048, 768] x [16, 768, 2048] right after the batched AWQ grid kernels ran on the same
buffers): the batched fake-quant / grid-scale kernels are run at exactly that shape into
buffers carved out of one canary-filled allocation, and the canaries are checked afterwards,
as are the weights they read.

Result on MI355X (profiles/r02a_guard_band.txt): canaries, inputs and per-slice outputs all
intact after the batched kernels (synchronised and checked), and the NEXT call -- torch.bmm of
a fresh bf16 [16, 2048, 768] tensor with these outputs transposed -- raised
hipErrorIllegalAddress.  Round 3 reproduced that fault with the same torch.bmm on plain
allocations in a process that never loaded this library (scripts/bmm_fault_probe.py stage A,
profiles/r03b_bmm_probe.log): a defect of torch's bundled hipBLASLt at that shape (DESIGN.md
§9).  The product's expert search uses one 2-D GEMM per expert (awq.search_experts), which the
test runs instead."""
import ctypes

import pytest
import torch

from quantizers_amd import _lib, ops
from quantizers_amd.quantization import QuantizationArgs

pytestmark = pytest.mark.gpu

CANARY = 0xA5
PAD = 1 << 16  # bytes of canary before and after every buffer


class Arena:
    """One device allocation; ``take`` carves a 256-B aligned buffer with PAD canary bytes on
    both sides; ``intact`` checks every byte outside the carved buffers."""

    def __init__(self, nbytes, dev):
        self.buf = torch.full((nbytes,), CANARY, dtype=torch.uint8, device=dev)
        self.off = PAD
        self.used = []

    def take(self, shape, dtype):
        n = 1
        for d in shape:
            n *= d
        nb = n * torch.empty((), dtype=dtype).element_size()
        start = (self.off + 255) // 256 * 256
        if start + nb + PAD > self.buf.numel():
            raise ValueError("arena too small")
        self.used.append((start, start + nb))
        self.off = start + nb + PAD
        return self.buf[start:start + nb].view(dtype).view(*shape)

    def intact(self):
        torch.cuda.synchronize()
        mask = torch.ones(self.buf.numel(), dtype=torch.bool, device=self.buf.device)
        for a, b in self.used:
            mask[a:b] = False
        bad = (self.buf[mask] != CANARY).nonzero()
        return bad.numel() == 0, bad[:8].flatten().tolist()


def _weights(e, n, k, dev, seed=5):
    g = torch.Generator(device=dev).manual_seed(seed)
    return (torch.randn(e, n, k, device=dev, generator=g) * 0.02).to(torch.bfloat16)


@pytest.mark.parametrize("bits,group", [(4, 128), (4, 32), (8, 32)])
def test_batched_awq_grid_guard_band(cuda, bits, group):
    E, N, K = 16, 2048, 768
    a = QuantizationArgs(num_bits=bits, type="int", symmetric=True, group_size=group)
    ar = Arena(E * N * K * 2 * 2 + E * K * 4 * 3 + (64 << 20), cuda)
    w = ar.take((E, N, K), torch.bfloat16)
    w.copy_(_weights(E, N, K, cuda))
    w_before = w.clone()
    xm = ar.take((E, K), torch.float32)
    wm = ar.take((E, K), torch.float32)
    xm.copy_(torch.rand(E, K, device=cuda) + 0.01)
    wm.copy_(torch.rand(E, K, device=cuda) + 0.01)
    s = ar.take((E, K), torch.float32)
    out = ar.take((E, N, K), torch.bfloat16)
    ca = a.to_c()
    lib = _lib.load()
    ws_n = lib.qz_quantize_workspace_size(E, N, K, ctypes.byref(ca)) + 4 * E + 256
    ws = ar.take((ws_n,), torch.uint8)
    st = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
    P = lambda t: ctypes.c_void_p(t.data_ptr())  # noqa: E731
    for ratio in (0.0, 0.35, 0.95):
        rc = lib.qz_awq_grid_scales_batched(P(xm), P(wm), E, K, ctypes.c_float(ratio), 1, P(s), st)
        assert rc == 0
        rc = lib.qz_awq_fake_quant_batched(P(w), E, N, K, K, N * K, ctypes.byref(ca), P(s), K, P(out), P(ws),
                                           ws.numel(), st)
        assert rc == 0
    ok, where = ar.intact()
    assert ok, f"bytes outside the outputs were written at arena offsets {where}"
    assert torch.equal(w.view(torch.int16), w_before.view(torch.int16)), "the weights (inputs) were modified"
    # the outputs are the per-slice results (sanity: the kernels did run)
    ref = ops.fake_quantize(w[3], a, col_scales=s[3].clone())
    assert torch.equal(out[3].view(torch.int16), ref.view(torch.int16))
    # the product's expert-search GEMMs (2-D, one per expert) on these buffers
    x = torch.randn(N, K, device=cuda, dtype=torch.bfloat16)
    for e in (0, 7, 15):
        y = torch.nn.functional.linear(x, out[e])
        torch.cuda.synchronize()
        assert torch.isfinite(y).all()


def test_grouped_quantize_guard_band(cuda):
    a = QuantizationArgs(num_bits=4, type="int", symmetric=True, group_size=128)
    n, R, C = 7, 1024, 2560
    ar = Arena(n * R * C * 3 + (32 << 20), cuda)
    ws = [ar.take((R, C), torch.bfloat16) for _ in range(n)]
    for i, w in enumerate(ws):
        w.copy_(_weights(1, R, C, cuda, seed=i)[0])
    outs = [{"codes": ar.take((R, C // 8), torch.int32), "scale": ar.take((R, C // 128), torch.bfloat16),
             "zero_point": None} for _ in range(n)]
    ops.GroupedQuantize(ws, a, outs=outs).run()
    ok, where = ar.intact()
    assert ok, where
    one = ops.quantize_weight(ws[4], a)
    assert torch.equal(one["codes"], outs[4]["codes"])


def test_grouped_mixed_shapes_guard_band(cuda):
    """The mixed-shape grouped launch (workgroup -> weight map): nothing outside the outputs."""
    a = QuantizationArgs(num_bits=4, type="int", symmetric=True, group_size=128)
    shapes = [(1024, 2560), (96, 1024), (2560, 512), (8, 128), (640, 2560)]
    ar = Arena(sum(r * c for r, c in shapes) * 3 + (32 << 20), cuda)
    ws = [ar.take(shp, torch.bfloat16) for shp in shapes]
    for i, (w, (r, c)) in enumerate(zip(ws, shapes)):
        w.copy_(_weights(1, r, c, cuda, seed=i)[0])
    outs = [{"codes": ar.take((r, c // 8), torch.int32), "scale": ar.take((r, c // 128), torch.bfloat16),
             "zero_point": None} for r, c in shapes]
    ops.GroupedQuantize(ws, a, outs=outs).run()
    torch.cuda.synchronize()
    ok, where = ar.intact()
    assert ok, where
    for i in (0, 3, 4):
        one = ops.quantize_weight(ws[i], a)
        assert torch.equal(one["codes"], outs[i]["codes"])


def test_awq_stat_kernels_guard_band(cuda):
    T, Cc = 3000, 2560
    ar = Arena(T * Cc * 2 + (32 << 20), cuda)
    x = ar.take((T, Cc), torch.bfloat16)
    x.copy_(torch.randn(T, Cc, device=cuda).to(torch.bfloat16))
    sums = ar.take((Cc,), torch.float32)
    sums.zero_()
    lib = _lib.load()
    wsn = lib.qz_awq_absmean_workspace_size(T, Cc)
    wsp = ar.take((wsn,), torch.uint8)
    wsp.zero_()  # statistics workspace contract: arrival counters zero before the first call
    st = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
    P = lambda t: ctypes.c_void_p(t.data_ptr())  # noqa: E731
    assert lib.qz_awq_absmean_accum(P(x), T, Cc, Cc, P(sums), P(wsp), wsp.numel(), st) == 0
    wsum = ar.take((Cc,), torch.float64)
    wsum.zero_()
    wmn = lib.qz_awq_weight_mean_workspace_size(T, Cc, 128)
    wmw = ar.take((max(wmn, 16),), torch.uint8)
    wmw.zero_()
    assert lib.qz_awq_weight_mean_accum(P(x), T, Cc, Cc, 128, P(wsum), P(wmw), wmw.numel(), st) == 0
    ok, where = ar.intact()
    assert ok, where
    assert torch.allclose(sums.double(), x.float().abs().sum(0).double(), rtol=1e-5)
    head = 32768  # QZ_STATS_HEAD_BYTES: every call leaves the arrival counters zero
    assert not wsp[:head].any() and not wmw[:head].any()
