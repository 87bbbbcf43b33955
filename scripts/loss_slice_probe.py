"""Probe: the expert search's per-(expert, grid point) GEMM + loss, with the token rows in S
slices (GEMM slice -> loss slice while the slice's output and reference are still in the 256 MiB
Infinity Cache) vs one pass (S = 1).  Qwen3-30B-A3B w2 shape: h [32768, 768], W [2048, 768],
20 grid weights per expert, 8 experts, expert-major.  Prints ms per expert search (20 points)."""
import sys

import torch

sys.path.insert(0, __import__("os").path.dirname(__import__("os").path.dirname(__import__("os").path.abspath(__file__))))
from quantizers_amd import ops  # noqa: E402

T, I, H, G, E = 32768, 768, 2048, 20, 8


def main():
    dev = torch.device("cuda:0")
    hs = [torch.randn(T, I, device=dev).to(torch.bfloat16) for _ in range(E)]
    w0 = [(torch.randn(H, I, device=dev) * 0.02).to(torch.bfloat16) for _ in range(E)]
    wq = [[(w + torch.randn_like(w) * 1e-3).to(torch.bfloat16) for _ in range(G)] for w in w0]
    refs = [torch.nn.functional.linear(h, w) for h, w in zip(hs, w0)]
    out = torch.empty(T, H, dtype=torch.bfloat16, device=dev)
    losses = {}
    for S in (1, 2, 4, 1, 2, 4):
        rows = T // S
        nb = ops.awq_sq_err_partials_count((rows, H))
        part = torch.empty(E, G, S, nb, dtype=torch.float64, device=dev)
        tot = torch.zeros(E * G * S, dtype=torch.float64, device=dev)

        def run():
            for k in range(E):
                for g in range(G):
                    for s in range(S):
                        hsl = hs[k][s * rows:(s + 1) * rows]
                        o = out[:rows]
                        torch.mm(hsl, wq[k][g].t(), out=o)
                        ops.awq_sq_err_partials(refs[k][s * rows:(s + 1) * rows], o, part[k, g, s])
            tot.zero_()
            ops.awq_sq_err_reduce(part.view(E * G * S, nb), nb, tot)

        run()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(3):
            run()
        e1.record()
        torch.cuda.synchronize()
        ms = e0.elapsed_time(e1) / 3 / E
        lo = tot.view(E, G, S).sum(-1)
        if S in losses:
            same = torch.equal(lo, losses[S])
        else:
            losses[S] = lo.clone()
            same = None
        rel = ((lo - losses[1]).abs() / losses[1]).max().item()
        print(f"S={S}: {ms:7.3f} ms per expert search (20 GEMM+loss), max rel loss diff vs S=1 {rel:.2e}, "
              f"argmin equal {torch.equal(lo.argmin(1), losses[1].argmin(1))}, repeat-identical {same}", flush=True)


if __name__ == "__main__":
    main()
