#!/usr/bin/env python3
"""Per-layer GPU busy fraction and kernel-time breakdown of an AWQ oneshot kernel trace
(rocprofv3 --kernel-trace; a rocpd .db converted with rocpd2csv):

  python scripts/e2e_breakdown.py <kernel_trace.csv> <layers> [plain-run log] [header]

The oneshot region starts at the first embedding gather (layer-0 input capture); a layer starts
at its first activation-statistics kernel (k_absmean_1l, or k_absmean_partial on the two-launch
path)."""
import collections
import csv
import sys


def _busy(seg):
    span = seg[-1][1] - seg[0][0]
    busy, end = 0, seg[0][0]
    for s, e, _ in seg:
        busy += max(0, e - max(s, end))
        end = max(end, e)
    return span, busy


def _key(name):
    return name.replace("(anonymous namespace)::", "").split("(")[0].replace("void ", "")[:110]


def _category(k):
    if "Cijk" in k:
        return "hipBLASLt GEMM"
    if k.startswith("attn_fwd"):
        return "attention (attn_fwd)"
    if k.startswith("k_"):
        return "this repo's kernels"
    return "torch elementwise / reduce / copy"


def main(path, layers, plain=None, header=None):
    print("# " + (header or f"scripts/awq_e2e.py {layers} 16 2048 (Qwen3-4B dims, {layers} layers, 16 x 2048 "
                  "calibration tokens, int4 g128 AWQ, model resident on the device)"))
    print("# rocprofv3 --kernel-trace --output-format csv; scripts/e2e_breakdown.py")
    if plain:
        print("# plain run of the same command: " + open(plain).read().strip().splitlines()[-1])
    rows = list(csv.DictReader(open(path)))
    iv = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]) for r in rows)
    i0 = next(i for i, x in enumerate(iv) if "vectorized_gather_kernel" in x[2])
    sub = iv[i0:]
    ab = [i for i, x in enumerate(sub) if "k_absmean_1l" in x[2] or "k_absmean_partial" in x[2]]
    per = len(ab) // layers
    marks = [ab[k] for k in range(0, per * layers, per)]
    span, busy = _busy(sub[:marks[0]])
    print(f"\ncapture of layer-0 inputs + first-call setup: {span / 1e6:.1f} ms, GPU busy {busy / 1e6:.1f} ms")
    bounds = marks + [len(sub)]
    print("per layer (first statistics kernel of the layer to the next layer's):")
    for j in range(layers):
        span, busy = _busy(sub[bounds[j]:bounds[j + 1]])
        print(f"  layer {j}: span {span / 1e6:7.1f} ms  GPU busy {busy / 1e6:7.1f} ms ({busy / span:.3f})")
    steady = sub[marks[1]:]
    span, busy = _busy(steady)
    print(f"layers 1-{layers - 1}: {span / 1e6:.1f} ms, GPU busy {busy / span:.3f}")
    tot, cnt = collections.Counter(), collections.Counter()
    for s, e, n in steady:
        tot[_key(n)] += e - s
        cnt[_key(n)] += 1
    T = sum(tot.values())
    cat = collections.Counter()
    for k, v in tot.items():
        cat[_category(k)] += v
    print(f"\nkernel time over layers 1-{layers - 1}: {T / 1e6:.1f} ms ({T / 1e6 / (layers - 1):.1f} ms per layer)")
    for c, v in cat.most_common():
        print(f"  {c:36s} {v / 1e6:8.1f} ms {v / T:6.1%}")
    print(f"\ntop kernels, layers 1-{layers - 1}:")
    for k, v in tot.most_common(32):
        print(f"{v / 1e6:8.1f} ms {v / T:6.1%} {cnt[k]:6d}  {k}")


if __name__ == "__main__":
    main(sys.argv[1], int(sys.argv[2]), sys.argv[3] if len(sys.argv) > 3 and sys.argv[3] else None,
         sys.argv[4] if len(sys.argv) > 4 else None)
