"""D15 on the CPU: moe_eager.fast_eager (two grouped GEMMs + k ordered bf16 adds) is bit-identical
to transformers' eager fused-experts forward (the reference's 4.57 per-expert loop), and the
eager_experts context patches and restores every experts module."""
import pytest
import torch

import quantizers_amd.moe_eager as me


def _models():
    from test_oneshot_gpu import _minimax, _qwen3_moe
    return {"qwen3_moe": _qwen3_moe, "minimax": _minimax}


@pytest.mark.parametrize("arch", ["qwen3_moe", "minimax"])
@pytest.mark.parametrize("tokens,k", [(300, 2), (64, 1), (1, 2)])
def test_fast_eager_bit_identical(arch, tokens, k):
    m = _models()[arch]()
    ex = next(mod for mod in m.modules() if me.eager_forward(mod) is not None)
    g = torch.Generator().manual_seed(tokens)
    x = torch.randn(tokens, ex.gate_up_proj.shape[-1], generator=g).to(torch.bfloat16)
    w, idx = torch.topk(torch.rand(tokens, ex.num_experts, generator=g).softmax(-1), k, dim=-1)
    w = (w / w.sum(-1, keepdim=True)).to(torch.bfloat16)
    with torch.no_grad():
        got = me.fast_eager(ex, x, idx, w)
        want = me.eager_forward(ex)(ex, x, idx, w)
    assert torch.equal(got.view(torch.int16), want.view(torch.int16))


def test_context_patches_and_restores():
    m = _models()["qwen3_moe"]()
    mods = [mod for mod in m.modules() if me.eager_forward(mod) is not None]
    assert mods and all("forward" not in mod.__dict__ for mod in mods)
    ids = torch.randint(0, 256, (1, 16))
    with torch.no_grad(), me.eager_experts(m) as n:
        assert n == len(mods) and all("forward" in mod.__dict__ for mod in mods)
        m(ids)
        m(ids)  # second call: the verified fast path
        assert all(me.FastEagerExperts.checked.values())
    assert all("forward" not in mod.__dict__ for mod in mods)


@pytest.mark.parametrize("arch", ["qwen3_moe", "minimax"])
@pytest.mark.parametrize("tokens,k", [(300, 2), (1, 2)])
def test_planned_eager_bit_identical(arch, tokens, k):
    """The fixed-routing form (host expert bounds from one plan, one GEMM per routed expert) is
    bit-identical to the eager forward, and one plan serves repeated forwards with new expert
    weights (the AWQ grid writes its fake-quantized weights into the parameters in place)."""
    m = _models()[arch]()
    ex = next(mod for mod in m.modules() if me.eager_forward(mod) is not None)
    g = torch.Generator().manual_seed(tokens + 7)
    x = torch.randn(tokens, ex.gate_up_proj.shape[-1], generator=g).to(torch.bfloat16)
    w, idx = torch.topk(torch.rand(tokens, ex.num_experts, generator=g).softmax(-1), k, dim=-1)
    w = (w / w.sum(-1, keepdim=True)).to(torch.bfloat16)
    with torch.no_grad():
        plan = me._plan(ex, idx)
        for step in range(2):
            got = me.planned_eager(ex, x, idx, w, plan)
            want = me.eager_forward(ex)(ex, x, idx, w)
            assert torch.equal(got.view(torch.int16), want.view(torch.int16)), step
            ex.gate_up_proj.mul_(1.5)  # new weights, same routing


def test_fixed_routing_context_uses_plans():
    """Inside fixed_routing the patched experts forward takes the planned form (checked once
    against the grouped form) and equals the forward outside the context."""
    m = _models()["qwen3_moe"]()
    ids = torch.randint(0, 256, (1, 16), generator=torch.Generator().manual_seed(3))
    with torch.no_grad(), me.eager_experts(m):
        want = m(ids).logits
        m(ids)
        with me.fixed_routing():
            got1 = m(ids).logits
            got2 = m(ids).logits
            assert me._FIXED  # plans were recorded
        assert me._FIXED is None
        assert all(me.FastEagerExperts.planned_checked.values())
    assert torch.equal(got1, want) and torch.equal(got2, want)


def _composed(d, w, perm, src, t, k):
    """The composed PyTorch tail of fast_eager / planned_eager (the eager loop's arithmetic)."""
    d = d * w.reshape(-1)[perm][:, None]
    contrib = d.index_select(0, src).view(t, k, d.shape[1])
    final = torch.zeros(t, d.shape[1], dtype=torch.bfloat16, device=d.device)
    for j in range(k):
        final = final + contrib[:, j].to(final.dtype)
    return final


@pytest.mark.gpu
@pytest.mark.parametrize("hidden", [2048, 3072, 100, 8])
@pytest.mark.parametrize("wdtype", [torch.bfloat16, torch.float32])
@pytest.mark.parametrize("tokens,k", [(300, 8), (257, 2), (1, 1), (0, 4)])
def test_moe_combine_bit_identical(cuda, hidden, wdtype, tokens, k):
    """qz_moe_combine == the composed weighting / reorder / k bf16 adds, bit for bit: wide and
    narrow rows (16-B and scalar kernels), bf16 and f32 routing weights, signed zeros, infinities
    and values whose bf16 sums round."""
    from quantizers_amd import ops
    g = torch.Generator().manual_seed(hidden * 31 + tokens * 7 + k)
    n_exp = 16
    idx = torch.stack([torch.randperm(n_exp, generator=g)[:k] for _ in range(tokens)]) if tokens else \
        torch.empty(0, k, dtype=torch.int64)
    w = torch.rand(tokens, k, generator=g).to(wdtype)
    d = (torch.randn(tokens * k, hidden, generator=g) * 3).to(torch.bfloat16)
    if d.numel():
        d.view(-1)[::97] = -0.0
        d.view(-1)[5::1013] = float("inf")
        d.view(-1)[7::2039] = 65504.0
    idx, w, d = idx.to(cuda), w.to(cuda), d.to(cuda)
    flat = idx.reshape(-1)
    _, perm = torch.sort(flat, stable=True)
    order = torch.argsort(idx, dim=-1)
    inv = torch.argsort(perm)
    src = inv[(torch.arange(tokens, device=cuda)[:, None] * k + order).reshape(-1)]
    got = ops.moe_combine(d, w, perm, src, tokens, k)
    want = _composed(d, w, perm, src, tokens, k)
    assert got.shape == want.shape == (tokens, hidden)
    assert torch.equal(got.view(torch.int16), want.view(torch.int16))
    if tokens:  # unaligned expert outputs (a 1-element offset view) take the scalar kernel
        big = torch.empty(d.numel() + 1, dtype=torch.bfloat16, device=cuda)
        du = big[1:].view_as(d)
        du.copy_(d)
        got_u = ops.moe_combine(du, w, perm, src, tokens, k)
        assert torch.equal(got_u.view(torch.int16), want.view(torch.int16))
        with pytest.raises(ValueError):
            ops.moe_combine(d[:-1], w, perm, src, tokens, k)


@pytest.mark.gpu
@pytest.mark.parametrize("arch", ["qwen3_moe", "minimax"])
def test_fused_forms_bit_identical_gpu(cuda, arch):
    """On the GPU (qz_moe_combine tail): the grouped and the planned forms equal transformers'
    eager fused-experts forward bit for bit."""
    m = _models()[arch]().to(cuda)
    ex = next(mod for mod in m.modules() if me.eager_forward(mod) is not None)
    g = torch.Generator().manual_seed(11)
    tokens, k = 300, 2
    x = torch.randn(tokens, ex.gate_up_proj.shape[-1], generator=g).to(torch.bfloat16).to(cuda)
    w, idx = torch.topk(torch.rand(tokens, ex.num_experts, generator=g).softmax(-1), k, dim=-1)
    w, idx = (w / w.sum(-1, keepdim=True)).to(torch.bfloat16).to(cuda), idx.to(cuda)
    with torch.no_grad():
        want = me.eager_forward(ex)(ex, x, idx, w)
        got = me.fast_eager(ex, x, idx, w)
        planned = me.planned_eager(ex, x, idx, w, me._plan(ex, idx))
    assert torch.equal(got.view(torch.int16), want.view(torch.int16))
    assert torch.equal(planned.view(torch.int16), want.view(torch.int16))


@pytest.mark.gpu
@pytest.mark.parametrize("rows,inter", [(300, 768), (257, 1536), (5, 12), (0, 64)])
def test_moe_silu_mul_bit_identical(cuda, rows, inter):
    """qz_moe_silu_mul == F.silu(gate) * up over the gate/up GEMM output, bit for bit (16-B and
    scalar kernels; large, tiny, signed-zero and infinite inputs).  The product path also
    re-checks this on its first call (moe_eager._act_mul)."""
    from quantizers_amd import ops
    g = torch.Generator().manual_seed(rows + inter)
    gu = (torch.randn(rows, 2 * inter, generator=g) * 4).to(torch.bfloat16)
    if gu.numel():
        gu.view(-1)[::53] = -0.0
        gu.view(-1)[3::101] = float("inf")
        gu.view(-1)[4::103] = -float("inf")
        gu.view(-1)[6::107] = -90.0
        gu.view(-1)[8::109] = 1e-38
    gu = gu.to(cuda)
    gate, up = gu.chunk(2, dim=-1)
    want = torch.nn.functional.silu(gate) * up
    got = ops.moe_silu_mul(gu)
    assert got.shape == want.shape
    nan = torch.isnan(want)
    assert torch.equal(torch.isnan(got), nan)
    assert torch.equal(got.view(torch.int16)[~nan], want.view(torch.int16)[~nan])


@pytest.mark.gpu
@pytest.mark.parametrize("n,k", [(1536, 2048), (2048, 768), (96, 64)])
def test_expert_gemms_bit_identical(cuda, n, k):
    """qz_expert_gemms (hipBLASLt called from C, one call per stream) == torch.mm(x[rows],
    w[e].t()) per expert, bit for bit: expert row counts from 0 to a few thousand, experts out of
    order, one stream."""
    import numpy as np
    from quantizers_amd import _lib
    import quantizers_amd.moe_eager as me_
    g = torch.Generator().manual_seed(n + k)
    E = 9
    counts = [0, 1, 7, 64, 300, 2049, 17, 128, 5]
    b = [0]
    for c in counts:
        b.append(b[-1] + c)
    x = (torch.randn(b[-1], k, generator=g) * 0.5).to(torch.bfloat16).to(cuda)
    w = (torch.randn(E, n, k, generator=g) * 0.05).to(torch.bfloat16).to(cuda)
    want = torch.zeros(b[-1], n, dtype=torch.bfloat16, device=cuda)
    for e in range(E):
        if counts[e]:
            torch.mm(x[b[e]:b[e + 1]], w[e].t(), out=want[b[e]:b[e + 1]])
    order = [4, 0, 8, 2, 6, 1, 3, 5, 7]
    r0 = np.array([b[e] for e in order], dtype=np.int64)
    r1 = np.array([b[e + 1] for e in order], dtype=np.int64)
    ex = np.array(order, dtype=np.int32)
    got = torch.full_like(want, float("nan"))
    ws = torch.empty(me_._WS_BYTES, dtype=torch.uint8, device=cuda)
    rc = _lib.load().qz_expert_gemms(x.data_ptr(), x.stride(0), w.data_ptr(), w.stride(0), w.stride(1), n, k,
                                     got.data_ptr(), got.stride(0), r0.ctypes.data, r1.ctypes.data, ex.ctypes.data,
                                     len(order), ws.data_ptr(), me_._WS_BYTES, torch.cuda.current_stream().cuda_stream)
    assert rc == 0, _lib.load().qz_strerror(rc)
    torch.cuda.synchronize()
    assert torch.equal(got.view(torch.int16), want.view(torch.int16))


@pytest.mark.gpu
def test_expert_gemms_four_threads(cuda):
    """qz_expert_gemms called from 4 host threads at once, each on its own stream (the round-3 host
    crash came from concurrent callers on one shared hipBLASLt handle; the library now serialises
    them): threads 0-1 run the SAME problems, threads 2-3 different ones, 8 rounds each; every
    output is bit-identical to torch.mm per expert."""
    import threading
    import numpy as np
    from quantizers_amd import _lib
    import quantizers_amd.moe_eager as me_
    lib = _lib.load()
    assert me_.bind_hipblaslt(lib), lib.qz_expert_gemms_status()
    shapes = [(1536, 2048), (1536, 2048), (2048, 768), (96, 64)]
    jobs = []
    for t, (n, k) in enumerate(shapes):
        g = torch.Generator().manual_seed(1000 + (t if t >= 2 else 0))
        counts = [0, 3, 129, 700, 64, 1]
        b = np.cumsum([0] + counts)
        x = (torch.randn(int(b[-1]), k, generator=g) * 0.5).to(torch.bfloat16).to(cuda)
        w = (torch.randn(len(counts), n, k, generator=g) * 0.05).to(torch.bfloat16).to(cuda)
        want = torch.zeros(int(b[-1]), n, dtype=torch.bfloat16, device=cuda)
        for e, c in enumerate(counts):
            if c:
                torch.mm(x[b[e]:b[e + 1]], w[e].t(), out=want[b[e]:b[e + 1]])
        order = np.array([3, 1, 5, 0, 2, 4], dtype=np.int32)
        jobs.append(dict(x=x, w=w, want=want, r0=np.ascontiguousarray(b[order]).astype(np.int64),
                         r1=np.ascontiguousarray(b[order + 1]).astype(np.int64), ex=order, n=n, k=k,
                         out=[torch.full_like(want, float("nan")) for _ in range(8)],
                         ws=torch.empty(me_._WS_BYTES, dtype=torch.uint8, device=cuda),
                         stream=torch.cuda.Stream(cuda)))
    torch.cuda.synchronize()
    errs = []
    start = threading.Barrier(len(jobs))

    def run(j):
        try:
            start.wait()
            for o in j["out"]:
                rc = lib.qz_expert_gemms(j["x"].data_ptr(), j["x"].stride(0), j["w"].data_ptr(), j["w"].stride(0),
                                         j["w"].stride(1), j["n"], j["k"], o.data_ptr(), o.stride(0),
                                         j["r0"].ctypes.data, j["r1"].ctypes.data, j["ex"].ctypes.data, len(j["ex"]),
                                         j["ws"].data_ptr(), me_._WS_BYTES, j["stream"].cuda_stream)
                if rc:
                    errs.append((rc, lib.qz_expert_gemms_status()))
        except Exception as e:  # noqa: BLE001
            errs.append(e)

    ths = [threading.Thread(target=run, args=(j,)) for j in jobs]
    for th in ths:
        th.start()
    for th in ths:
        th.join(timeout=120)
    torch.cuda.synchronize()
    assert not errs, errs
    for j in jobs:
        for o in j["out"]:
            assert torch.equal(o.view(torch.int16), j["want"].view(torch.int16))
