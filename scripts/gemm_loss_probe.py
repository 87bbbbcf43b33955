"""Prototype A/B: the fused GEMM -> grid loss kernel (quantizers_amd/csrc/proto/
qz_gemm_loss.hip, built into csrc/proto/libqz_proto.so) against the product's expert-search path
(awq._batched_losses: torch's bf16 mm = hipBLASLt per grid point, MULTI_LOSS = 8 outputs per
ops.awq_sq_err_partials_multi launch, one ordered reduce) on the Qwen3-30B-A3B expert w2 problem:
X [32768, 768] x W [2048, 768]^T, losses against R [32768, 2048].

1. layout check with exact small-integer data (every product exact in f32), both orientations;
2. losses on random data, single items, ragged rows and a batch of 8 grid points, vs the product's;
3. timing (HIP events, median of 7 passes): per grid point, the product's path and the fused
   launch (one item, and 8 grid points x E experts per launch).
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
    lib.qzp_gemm_sqerr.argtypes = [P, I64, I64, I64, I64, P, ctypes.c_int, P]
    lib.qzp_gemm_sqerr_tiles.argtypes = [I64, I64]
    lib.qzp_gemm_sqerr_tiles.restype = I64
    dev = torch.device("cuda:0")
    st = torch.cuda.current_stream()
    T, N, K = int(os.environ.get("T", 32768)), int(os.environ.get("N", 2048)), int(os.environ.get("K", 768))
    g = torch.Generator(device=dev).manual_seed(0)

    def table(items, nb):
        """items: [(x, w, r, rows)] -> (device table, part [n, nb])"""
        part = torch.zeros(len(items), nb, dtype=torch.float64, device=dev)
        rows = [[x.data_ptr(), w.data_ptr(), r.data_ptr(), part[i].data_ptr(), nr] for i, (x, w, r, nr) in enumerate(items)]
        return torch.tensor(rows, dtype=torch.int64, device=dev), part

    def launch(tab, n, rows_max, c, mode):
        rc = lib.qzp_gemm_sqerr(P(tab.data_ptr()), n, rows_max, N, K, P(c.data_ptr() if c is not None else 0), mode,
                                P(st.cuda_stream))
        assert rc == 0, rc

    nb = lib.qzp_gemm_sqerr_tiles(T, N)
    parts = lambda m: nb * 8 if m & 64 else nb  # noqa: E731  (the persistent form: 8 partials per tile)
    # 1. exact layout check, both orientations
    xi = torch.randint(-3, 4, (T, K), device=dev, generator=g).to(torch.bfloat16)
    wi = torch.randint(-3, 4, (N, K), device=dev, generator=g).to(torch.bfloat16)
    ci = torch.empty(T, N, dtype=torch.bfloat16, device=dev)
    ref = (xi.float() @ wi.float().t()).to(torch.bfloat16)
    env_modes = lambda k, d: [int(v) for v in os.environ.get(k, d).split(",")]  # noqa: E731
    for mode in env_modes("LAYOUT_MODES", "0,2,4,6,8,16"):
        ci.zero_()
        tab, _ = table([(xi, wi, ci, T)], parts(mode))
        launch(tab, 1, T, ci, mode)
        exact = torch.equal(ci.view(torch.int16), ref.view(torch.int16))
        print(f"layout check mode {mode} (exact integer data): {'OK' if exact else 'MISMATCH'}", flush=True)
        if not exact:
            print("first mismatches", (ci.float() != ref.float()).nonzero()[:5].tolist(), flush=True)
            return
        reps = int(os.environ.get("RACE_REPS", 0))  # race screen: the same launch again and again
        if reps and mode & 96:
            bad = 0
            for _ in range(reps):
                ci.zero_()
                launch(tab, 1, T, ci, mode)
                bad += int(not torch.equal(ci.view(torch.int16), ref.view(torch.int16)))
            print(f"  race screen mode {mode}: {bad} of {reps} launches differ", flush=True)
            if bad:
                return
    del xi, wi, ci, ref
    # 2. losses
    x = torch.randn(T, K, device=dev, generator=g).to(torch.bfloat16)
    w = (torch.randn(N, K, device=dev, generator=g) * 0.05).to(torch.bfloat16)
    r = torch.nn.functional.linear(x, w)
    ws = [(w.float() + torch.randn(N, K, device=dev, generator=g) * 0.002 * (1 + i)).to(torch.bfloat16)
          for i in range(8)]

    def ref_loss(x_, w_, r_):
        acc = torch.zeros(1, dtype=torch.float64, device=dev)
        ops.awq_sq_err_accum(torch.nn.functional.linear(x_, w_), r_.contiguous(), acc)
        return acc.item()
    for mode in env_modes("LOSS_MODES", "7,17"):
        tab, part = table([(x, ws[0], r, T)], parts(mode))
        launch(tab, 1, T, None, mode)
        torch.cuda.synchronize()
        lf, lr = part.sum().item(), ref_loss(x, ws[0], r)
        print(f"loss mode {mode}: fused {lf:.9e} product {lr:.9e} rel {(lf - lr) / lr:.2e}", flush=True)
        for tr in (1000, 4097, 300):  # ragged rows
            tab, part = table([(x, ws[1], r, tr)], parts(mode))
            launch(tab, 1, T, None, mode)
            torch.cuda.synchronize()
            lf, lr = part.sum().item(), ref_loss(x[:tr], ws[1], r[:tr])
            print(f"  ragged rows {tr}: fused {lf:.9e} product {lr:.9e} rel {(lf - lr) / lr:.2e}", flush=True)
        tab, part = table([(x, wq, r, T) for wq in ws], parts(mode))
        launch(tab, 8, T, None, mode)
        torch.cuda.synchronize()
        rel = max(abs(part[i].sum().item() / ref_loss(x, ws[i], r) - 1) for i in range(8))
        print(f"  batch of 8 grid points: max rel {rel:.2e}", flush=True)

    # 3. timing per grid point
    def t_of(fn, per, n=5, passes=7):
        for _ in range(2):
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
            ts.append(e0.elapsed_time(e1) * 1e3 / n / per)
        return sorted(ts)[len(ts) // 2]
    E = int(os.environ.get("E", 4))
    xs = [torch.randn(T, K, device=dev, generator=g).to(torch.bfloat16) for _ in range(E)]
    rs = [torch.nn.functional.linear(xe, w) for xe in xs]
    wq_all = torch.stack([torch.stack([wq] * E) for wq in ws])  # [8, E, N, K]
    outs = [torch.empty_like(rs[0]) for _ in range(8)]
    npart = ops.awq_sq_err_partials_count(rs[0].shape)
    ppart = torch.empty(E, 8, npart, dtype=torch.float64, device=dev)
    tot = torch.zeros(E * 8, dtype=torch.float64, device=dev)

    def product():  # awq._batched_losses with MULTI_LOSS = 8
        for k in range(E):
            for j in range(8):
                torch.mm(xs[k], wq_all[j, k].t(), out=outs[j])
            ops.awq_sq_err_partials_multi(rs[k], outs, ppart[k])
        ops.awq_sq_err_reduce(ppart.view(E * 8, npart), npart, tot)
    flop = 2 * T * N * K
    us = t_of(product, 8 * E)
    print(f"{'product (mm + multi-loss + reduce)':40s} {us:9.2f} us per grid point", flush=True)
    us_mm = t_of(lambda: torch.mm(xs[0], ws[0].t(), out=outs[0]), 1)
    print(f"{'  of which hipBLASLt mm':40s} {us_mm:9.2f} us  {flop / (us_mm * 1e-6) / 1e15:.3f} PFLOP/s", flush=True)
    cbuf = torch.empty_like(rs[0])
    for mode in env_modes("TIME_MODES", "6,16,7,17"):
        tab1, _ = table([(xs[0], ws[0], rs[0] if mode & 1 else cbuf, T)], parts(mode))
        us1 = t_of(lambda: launch(tab1, 1, T, cbuf, mode), 1)
        line = f"mode {mode} ({'fused loss' if mode & 1 else 'core, bf16 store'}, BK {64 if mode & 28 else 32}" \
               f"{', 4 waves' if mode & 8 else ''}{', 4 waves pipelined' if mode & 16 else ''}" \
               f"{', staggered phases' if mode & 32 else ''}{', persistent staggered' if mode & 64 else ''}): one item " \
               f"{us1:9.2f} us ({flop / (us1 * 1e-6) / 1e15:.3f} PFLOP/s)"
        if mode & 1:
            tabn, partn = table([(xs[k], wq_all[j, k], rs[k], T) for k in range(E) for j in range(8)], parts(mode))
            usn = t_of(lambda: launch(tabn, 8 * E, T, None, mode), 8 * E)
            line += f", {8 * E} items per launch {usn:9.2f} us per grid point ({flop / (usn * 1e-6) / 1e15:.3f} PFLOP/s)"
        print(line, flush=True)

if __name__ == "__main__":
    main()
