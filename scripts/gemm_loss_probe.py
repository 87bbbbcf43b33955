"""Prototype A/B: the fused GEMM -> grid loss kernel (quantizers_amd/csrc/proto/
qz_gemm_loss.hip, built into csrc/proto/libqz_proto.so) against the product's per-grid-point path
(torch's bf16 linear = hipBLASLt, then ops.awq_sq_err_accum) on the Qwen3-30B-A3B expert w2 problem:
X [32768, 768] x W [2048, 768]^T, loss against R [32768, 2048].

1. layout check with exact small-integer data (every product exact in f32): C must equal torch's;
2. random data: C vs torch's (fraction of bf16 outputs that differ; GEMM rounding order only);
3. timing (HIP events, median of 7 passes of 20 launches): hipBLASLt GEMM, loss kernel, the two
   together (the product's per-grid-point cost), the prototype's GEMM core (bf16 store) and its
   fused loss mode; PFLOP/s of each GEMM; the fused loss vs the reference loss.
"""
import ctypes
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from quantizers_amd import ops  # noqa: E402

P = ctypes.c_void_p
I64 = ctypes.c_int64


def main():
    lib = ctypes.CDLL(os.environ.get("PROTO_LIB", os.path.join(ROOT, "quantizers_amd/csrc/proto/libqz_proto.so")))
    lib.qzp_gemm_nt.argtypes = [P, P, P, P, P, I64, I64, I64, I64, I64, I64, ctypes.c_int, P]
    dev = torch.device("cuda:0")
    st = torch.cuda.current_stream()
    T, N, K = int(os.environ.get("T", 32768)), int(os.environ.get("N", 2048)), int(os.environ.get("K", 768))
    g = torch.Generator(device=dev).manual_seed(0)

    def run(x, w, r, c, part, mode):
        rc = lib.qzp_gemm_nt(P(x.data_ptr()), P(w.data_ptr()), P(r.data_ptr()), P(c.data_ptr()), P(part.data_ptr()),
                             T, N, K, x.stride(0), w.stride(0), r.stride(0), mode, P(st.cuda_stream))
        assert rc == 0, rc

    nparts = (T // 256) * (N // 256)
    part = torch.zeros(nparts, dtype=torch.float64, device=dev)
    # 1. exact layout check, both MFMA shapes
    xi = torch.randint(-3, 4, (T, K), device=dev, generator=g).to(torch.bfloat16)
    wi = torch.randint(-3, 4, (N, K), device=dev, generator=g).to(torch.bfloat16)
    ci = torch.empty(T, N, dtype=torch.bfloat16, device=dev)
    ref = (xi.float() @ wi.float().t()).to(torch.bfloat16)
    for mode in (0, 2, 8, 10):
        ci.zero_()
        run(xi, wi, ci, ci, part, mode)
        exact = torch.equal(ci.view(torch.int16), ref.view(torch.int16))
        print(f"layout check mode {mode} (exact integer data): {'OK' if exact else 'MISMATCH'}", flush=True)
        if not exact:
            bad = (ci.float() != ref.float()).nonzero()[:5].tolist()
            print("first mismatches", bad, flush=True)
            return
    del xi, wi, ci, ref
    # 2. random data
    x = (torch.randn(T, K, device=dev, generator=g)).to(torch.bfloat16)
    w = (torch.randn(N, K, device=dev, generator=g) * 0.05).to(torch.bfloat16)
    w2 = (w.float() + torch.randn(N, K, device=dev, generator=g) * 0.002).to(torch.bfloat16)  # "grid point"
    r = torch.nn.functional.linear(x, w)
    c = torch.empty_like(r)
    c_bl = torch.nn.functional.linear(x, w2)
    loss_ref = torch.zeros(1, dtype=torch.float64, device=dev)
    ops.awq_sq_err_accum(c_bl, r, loss_ref)
    for mode in (0, 2, 8, 10):
        run(x, w2, r, c, part, mode)
        diff = (c.view(torch.int16) != c_bl.view(torch.int16)).float().mean().item()
        rel = ((c.float() - c_bl.float()).abs().max() / c_bl.float().abs().max()).item()
        print(f"random data mode {mode}: {diff * 100:.3f} % of bf16 outputs differ from hipBLASLt's (max rel {rel:.2e})",
              flush=True)
        run(x, w2, r, c, part, mode | 1)
        torch.cuda.synchronize()
        lf, lr = part.sum().item(), loss_ref.item()
        print(f"loss mode {mode | 1}: fused {lf:.9e}  hipBLASLt+k_sqdiff {lr:.9e}  rel diff {(lf - lr) / lr:.2e}",
              flush=True)
    # 3. timing
    flop = 2 * T * N * K
    out = torch.empty_like(r)
    lsum = torch.zeros(1, dtype=torch.float64, device=dev)

    def t_of(fn, n=20, passes=7):
        for _ in range(3):
            fn()
        torch.cuda.synchronize()
        ts = []
        for _ in range(passes):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(st)
            for _ in range(n):
                fn()
            e1.record(st)
            torch.cuda.synchronize()
            ts.append(e0.elapsed_time(e1) * 1e3 / n)
        return sorted(ts)[len(ts) // 2]
    legs = [
        ("hipBLASLt linear", lambda: torch.mm(x, w2.t(), out=out), True),
        ("k_sqdiff loss", lambda: ops.awq_sq_err_accum(out, r, lsum), False),
        ("hipBLASLt + k_sqdiff", lambda: (torch.mm(x, w2.t(), out=out), ops.awq_sq_err_accum(out, r, lsum)), False),
    ]
    for mode, name in ((0, "16x16x32"), (4, "16x16x32 prio"), (2, "32x32x16"), (6, "32x32x16 prio"),
                       (8, "pipe 16x16x32"), (10, "pipe 32x32x16")):
        legs.append((f"proto core {name}", lambda mode=mode: run(x, w2, r, c, part, mode), True))
        legs.append((f"proto fused {name}", lambda mode=mode: run(x, w2, r, c, part, mode | 1), False))
    for name, fn, gemm in legs:
        us = t_of(fn)
        extra = f"  {flop / (us * 1e-6) / 1e15:.3f} PFLOP/s" if gemm else ""
        print(f"{name:32s} {us:9.2f} us{extra}", flush=True)


if __name__ == "__main__":
    main()
