"""Sustained-load behaviour of the headline kernel: per-launch durations over long back-to-back
runs (grouped launches of K weights, and single-weight launches), after idle gaps.
usage: python scripts/sustain.py   (env: K=200 REPS=10)"""
import os
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from quantizers_amd import ops  # noqa: E402
from quantizers_amd.quantization import QuantizationArgs  # noqa: E402

ROWS, COLS = 11008, 4096
ALG = ROWS * COLS * 2 + ROWS * COLS // 2 + ROWS * COLS // 128 * 2


def main():
    K = int(os.environ.get("K", 200))
    reps = int(os.environ.get("REPS", 10))
    dev = torch.device("cuda:0")
    a = QuantizationArgs(num_bits=4, type="int", symmetric=True, group_size=128)
    copies = [(torch.randn(ROWS, COLS, device=dev) * 0.02).to(torch.bfloat16) for _ in range(12)]
    gq = ops.GroupedQuantize([copies[i % 12] for i in range(K)], a)
    st = torch.cuda.current_stream()
    o = ops.quantize_weight(copies[0], a)
    prep = ops.PreparedQuantize(copies[0], a, {"codes": o["codes"], "scale": o["scale"], "zero_point": None})

    def series(fn, n, label):
        ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(n)]
        for i in range(n):
            ev[i][0].record(st)
            fn(i)
            ev[i][1].record(st)
        torch.cuda.synchronize()
        d = [s.elapsed_time(e) for s, e in ev]
        return d

    for phase in range(2):
        g = series(lambda i: gq.run(st), reps, "grouped")
        print(f"phase {phase} grouped K={K}: " + " ".join(f"{x * 1e3 / K:.2f}" for x in g) + " us/weight  "
              + " ".join(f"{ALG * K / (x * 1e-3) / 1e12:.2f}" for x in g) + " TB/s", flush=True)
        s = series(lambda i: prep.run(copies[i % 12], st), 400, "single")
        chunks = [sum(s[i:i + 40]) / 40 * 1e3 for i in range(0, 400, 40)]
        print(f"phase {phase} single (per 40 launches, event pairs): " + " ".join(f"{x:.2f}" for x in chunks) + " us",
              flush=True)
        time.sleep(2.0)
    # long run: 60 grouped launches (~250 ms) then single launches
    g = series(lambda i: gq.run(st), 60, "grouped")
    print("long grouped: " + " ".join(f"{ALG * K / (x * 1e-3) / 1e12:.2f}" for x in g[::5]) + " TB/s (every 5th)",
          flush=True)
    # same bytes, different launch shapes: grouped 4 weights / one [44032, 4096] weight / a [4, 11008, 4096] batch
    g4 = ops.GroupedQuantize([copies[i % 12] for i in range(4)], a)
    big = [(torch.randn(4 * ROWS, COLS, device=dev) * 0.02).to(torch.bfloat16) for _ in range(3)]
    ob = ops.quantize_weight(big[0], a)
    pb = ops.PreparedQuantize(big[0], a, {"codes": ob["codes"], "scale": ob["scale"], "zero_point": None})
    stk = [torch.stack([copies[(4 * j + i) % 12] for i in range(4)]) for j in range(3)]
    os_ = ops.quantize_weight(stk[0], a)
    ps = ops.PreparedQuantize(stk[0], a, {"codes": os_["codes"], "scale": os_["scale"], "zero_point": None})
    # grouped K=200 writing 12 rotating output sets (step i -> outputs i % 12, same input copy i % 12)
    outs12 = [{"codes": torch.empty_like(o["codes"]), "scale": torch.empty_like(o["scale"]), "zero_point": None}
              for _ in range(12)]
    gq12 = ops.GroupedQuantize([copies[i % 12] for i in range(K)], a, outs=[outs12[i % 12] for i in range(K)])
    g12 = ops.GroupedQuantize([copies[i % 12] for i in range(12)], a, outs=outs12)
    # distinct outputs carved from ONE allocation (fragment / TLB test) and 48 rotating output sets
    nc, ns = o["codes"].numel(), o["scale"].numel()
    big_c = torch.empty(K, nc, dtype=o["codes"].dtype, device=dev)
    big_s = torch.empty(K, ns, dtype=o["scale"].dtype, device=dev)
    gqb = ops.GroupedQuantize([copies[i % 12] for i in range(K)], a,
                              outs=[{"codes": big_c[i].view(o["codes"].shape), "scale": big_s[i].view(o["scale"].shape),
                                     "zero_point": None} for i in range(K)])
    outs48 = [{"codes": torch.empty_like(o["codes"]), "scale": torch.empty_like(o["scale"]), "zero_point": None}
              for _ in range(48)]
    gq48 = ops.GroupedQuantize([copies[i % 12] for i in range(K)], a, outs=[outs48[i % 48] for i in range(K)])
    for rnd in range(3):
        for name, fn, nw in (("grouped200/12out", lambda i: gq12.run(st), K), ("grouped200", lambda i: gq.run(st), K),
                             ("grouped200/onealloc", lambda i: gqb.run(st), K),
                             ("grouped200/48out", lambda i: gq48.run(st), K),
                             ("grouped12", lambda i: g12.run(st), 12)):
            d = series(fn, 10 if nw == K else 100, name)
            d = sorted(d)[len(d) // 2]
            print(f"round {rnd} {name:17s} median {d * 1e3 / nw:.2f} us/weight = {ALG * nw / (d * 1e-3) / 1e12:.2f} TB/s",
                  flush=True)
    for rnd in range(3):
        for name, fn in (("grouped4", lambda i: g4.run(st)), ("one[44032]", lambda i: pb.run(big[i % 3], st)),
                         ("batch[4,11008]", lambda i: ps.run(stk[i % 3], st))):
            d = series(fn, 40, name)
            d = sorted(d)[len(d) // 2]
            print(f"round {rnd} {name:15s} median {d * 1e3:.2f} us = {ALG * 4 / (d * 1e-3) / 1e12:.2f} TB/s", flush=True)


if __name__ == "__main__":
    main()
