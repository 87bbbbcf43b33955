"""Leg-by-leg comparison of two bench.py lines (the JSON line of each log): every numeric timing
field (ms / us / value / frac), the relative difference, and the largest difference.
usage: python scripts/bench_compare.py a.log b.log"""
import json
import sys


def line(path):
    for l in open(path):
        if l.startswith("{"):
            return json.loads(l)
    raise SystemExit(f"{path}: no JSON line")


KEYS = ("value", "ms", "us", "us_per_weight", "frac", "ms_per_step", "event_ms_per_step", "ms_max_rank",
        "us_per_copy_max_rank", "s_total")


def walk(a, b, path, out):
    if isinstance(a, dict) and isinstance(b, dict):
        for k in a:
            if k in b:
                walk(a[k], b[k], f"{path}.{k}" if path else k, out)
    elif isinstance(a, list) and isinstance(b, list) and len(a) == len(b) and all(isinstance(x, dict) for x in a):
        for i, (x, y) in enumerate(zip(a, b)):
            walk(x, y, f"{path}[{i}]", out)
    elif isinstance(a, (int, float)) and isinstance(b, (int, float)) and not isinstance(a, bool):
        if path.split(".")[-1] in KEYS and a:
            out.append((path, a, b, (b - a) / a))


def main(pa, pb):
    out = []
    walk(line(pa), line(pb), "", out)
    for p, a, b, r in out:
        print(f"{r * 100:+7.2f} %  {p}: {a:.6g} -> {b:.6g}")
    skip = ("awq_oneshot", "pcie_inclusive", "cpu_baseline", "end_to_end", "steady_state")
    core = [x for x in out if not any(s in x[0] for s in skip)]
    worst = max(core, key=lambda x: abs(x[3]))
    print(f"largest difference over the kernel legs: {worst[3] * 100:+.2f} % ({worst[0]})")


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2])
