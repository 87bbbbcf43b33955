"""D16 forward swaps on the pinned transformers: all three engage on a Qwen3 model (a transformers
upgrade that changes the restated code makes this fail, not just the AWQ pass slower), and
oneshot's log names a swap that did not engage (CPU)."""
import logging

import torch


def test_all_three_dense_swaps_engage_on_qwen3():
    from test_dense_norm import _qwen3
    from quantizers_amd.dense_mlp import fused_mlps
    from quantizers_amd.dense_norm import fused_rmsnorms
    from quantizers_amd.rotary import fused_rotary
    m = _qwen3()
    n_layers = m.config.num_hidden_layers
    with fused_mlps(m) as n_mlp, fused_rmsnorms(m) as n_norm, fused_rotary(m) as n_rot:
        assert n_mlp == n_layers  # one Qwen3MLP per layer
        assert n_norm == 4 * n_layers + 1  # every Qwen3RMSNorm: 4 per layer + the final norm
        assert n_rot == 1  # apply_rotary_pos_emb of the Qwen3 modeling module


def test_swap_log_warns_when_a_swap_does_not_engage(caplog):
    from test_dense_norm import _qwen3
    from quantizers_amd.oneshot import _log_swaps
    m = _qwen3()
    with caplog.at_level(logging.INFO, logger="quantizers_amd.oneshot"):
        _log_swaps(m, {"SiLU·up (dense_mlp)": 2, "rotary embedding (rotary)": 0})
    warn = [r for r in caplog.records if r.levelno == logging.WARNING]
    assert len(warn) == 1 and "rotary" in warn[0].getMessage() and "did NOT engage" in warn[0].getMessage()
    caplog.clear()
    m.config.model_type = "minimax_m2"
    with caplog.at_level(logging.INFO, logger="quantizers_amd.oneshot"):
        _log_swaps(m, {"rotary embedding (rotary)": 0})
    assert not [r for r in caplog.records if r.levelno == logging.WARNING]
    assert torch.is_tensor(next(m.parameters()))


def test_bmm_guard_routes_only_the_pinned_fault_class(monkeypatch):
    """Inside bmm_guard a bf16 batched NT product with K = 768 (the class of the pinned hipBLASLt
    fault) runs as per-batch 2-D GEMMs with the same result; any other product,
    and anything outside the context, is the original function (CPU: routing enabled for the
    test through patching._ROUTE_DEVICES)."""
    from quantizers_amd import patching
    monkeypatch.setattr(patching, "_ROUTE_DEVICES", ("cuda", "cpu"))
    g = torch.Generator().manual_seed(0)
    x = torch.randn(3, 40, 768, generator=g).to(torch.bfloat16)
    o = torch.randn(3, 24, 768, generator=g).to(torch.bfloat16)
    nt = o.transpose(1, 2)  # [3, 768, 24], stride(-2) == 1: F.linear's NT layout
    want = torch.stack([x[i].float() @ nt[i].float() for i in range(3)]).to(torch.bfloat16)
    assert patching.pinned_bmm_defect(x, nt)
    assert not patching.pinned_bmm_defect(x, nt.contiguous())  # NN layout: untouched
    assert not patching.pinned_bmm_defect(x.float(), nt.float())  # f32: untouched
    assert not patching.pinned_bmm_defect(x[..., :512], nt[:, :512])  # other K: untouched
    orig = torch.bmm
    calls = []
    monkeypatch.setattr(patching, "_per_batch_mm", lambda a, b: calls.append(1) or orig(a, b.contiguous()))
    with patching.bmm_guard():
        assert torch.bmm is not orig
        for got in (torch.bmm(x, nt), torch.matmul(x, nt), x @ nt, x.matmul(nt)):
            assert got.shape == (3, 40, 24)
        torch.bmm(x, nt.contiguous())
    assert len(calls) == 4 and torch.bmm is orig
    monkeypatch.undo()
    monkeypatch.setattr(patching, "_ROUTE_DEVICES", ("cuda", "cpu"))
    with patching.bmm_guard():  # the real routing: per-batch torch.mm, same values as a float product
        got = torch.bmm(x, nt)
    assert torch.allclose(got.float(), want.float(), rtol=2e-2, atol=2e-2)


def test_bmm_guard_grad_and_rmatmul(monkeypatch):
    """the guard's per-batch route is autograd-safe (no ``out=``), and a ``tensor @
    non-tensor`` product still reaches the other operand's __rmatmul__ inside the guard."""
    from quantizers_amd import patching
    monkeypatch.setattr(patching, "_ROUTE_DEVICES", ("cuda", "cpu"))
    g = torch.Generator().manual_seed(1)
    x = torch.randn(2, 8, 768, generator=g).to(torch.bfloat16).requires_grad_(True)
    nt = torch.randn(2, 4, 768, generator=g).to(torch.bfloat16).transpose(1, 2)

    class R:
        def __rmatmul__(self, other):
            return "rmatmul"
    with patching.bmm_guard():
        y = torch.bmm(x, nt)
        y.float().sum().backward()
        assert x @ R() == "rmatmul"
    assert x.grad is not None and x.grad.shape == x.shape
