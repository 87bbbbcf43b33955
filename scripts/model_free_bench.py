#!/usr/bin/env python3
"""model_free_ptq end to end, as the reference calls it
(/root/reference/scripts/quant_GLM-4.7-Flash-FP8.py:11-24: scheme FP8_BLOCK, its ignore list,
max_workers=16, device cuda:0), on a synthetic multi-shard bf16 checkpoint of Qwen3-4B dims written
to the box's local disk.

Prints, as one JSON line: the checkpoint, the ceilings -- a read-only pass over the same files with
the same reader (cold: pages dropped with posix_fadvise(DONTNEED) after an fsync; warm: from the page
cache), the H2D rate of the product's pinned staging (pageable host tensors -> device) and of a
pinned DMA, the D2H rate, a write-only pass of the outputs -- and model_free_ptq's wall time and
per-phase busy times (model_free.run_summary) for cold and warm inputs.

usage: python scripts/model_free_bench.py [--dir DIR] [--shards 4] [--reps 2]
"""
import argparse
import json
import os
import shutil
import sys
import time
from concurrent.futures import ThreadPoolExecutor

import torch
from safetensors.torch import save_file

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from quantizers_amd import model_free  # noqa: E402
from quantizers_amd.staging import H2DStager  # noqa: E402

IGNORE = ["lm_head", "re:.*mlp\\.gate$", "re:.*kv_a_proj_with_mqa$", "re:.*q_a_proj$", "model.embed_tokens"]
H, I, Q, KV, L, V = 2560, 9728, 4096, 1024, 36, 151936  # Qwen3-4B public dims


def layer_tensors(i, dev, gen):
    p = f"model.layers.{i}."
    shapes = {"self_attn.q_proj.weight": (Q, H), "self_attn.k_proj.weight": (KV, H), "self_attn.v_proj.weight": (KV, H),
              "self_attn.o_proj.weight": (H, Q), "mlp.gate_proj.weight": (I, H), "mlp.up_proj.weight": (I, H),
              "mlp.down_proj.weight": (H, I), "input_layernorm.weight": (H,), "post_attention_layernorm.weight": (H,),
              "self_attn.q_norm.weight": (128,), "self_attn.k_norm.weight": (128,)}
    return {p + k: (torch.randn(s, device=dev, generator=gen) * 0.02).to(torch.bfloat16).cpu() for k, s in shapes.items()}


def evict(path):
    """Drop a file's pages from the page cache (dirty pages flushed first)."""
    fd = os.open(path, os.O_RDWR)
    try:
        os.fsync(fd)
        os.posix_fadvise(fd, 0, 0, os.POSIX_FADV_DONTNEED)
    finally:
        os.close(fd)


def make_checkpoint(d, n_shards, dev):
    os.makedirs(d, exist_ok=True)
    gen = torch.Generator(device=dev).manual_seed(0)
    per = -(-L // n_shards)
    files, wmap, total = [], {}, 0
    for s in range(n_shards):
        fn = f"model-{s + 1:05d}-of-{n_shards:05d}.safetensors"
        t = {}
        if s == 0:
            t["model.embed_tokens.weight"] = (torch.randn(V, H, device=dev, generator=gen) * 0.02).to(torch.bfloat16).cpu()
        if s == n_shards - 1:
            t["model.norm.weight"] = torch.ones(H, dtype=torch.bfloat16)
        for i in range(s * per, min((s + 1) * per, L)):
            t.update(layer_tensors(i, dev, gen))
        save_file(t, os.path.join(d, fn), {"format": "pt"})
        for k, v in t.items():
            wmap[k] = fn
            total += v.numel() * 2
        files.append(fn)
        del t
    with open(os.path.join(d, "model.safetensors.index.json"), "w") as f:
        json.dump({"metadata": {"total_size": total}, "weight_map": wmap}, f)
    shutil.copy(os.path.join(ROOT, "configs", "models", "qwen3-4b", "config.json"), os.path.join(d, "config.json"))
    return files, total


def read_pass(d, files, workers, chunk=64 << 20):
    """Every byte of the files read once with os.preadv in ``chunk`` pieces by ``workers`` threads
    (each into its own scratch buffer): the disk (cold) / page-cache (warm) read ceiling."""
    import threading
    local = threading.local()
    fds = {f: os.open(os.path.join(d, f), os.O_RDONLY) for f in files}
    jobs = [(f, off, min(chunk, os.path.getsize(os.path.join(d, f)) - off))
            for f in files for off in range(0, os.path.getsize(os.path.join(d, f)), chunk)]

    def job(j):
        f, off, n = j
        if not hasattr(local, "buf"):
            local.buf = bytearray(chunk)
        return os.preadv(fds[f], [memoryview(local.buf)[:n]], off)
    t0 = time.perf_counter()
    with ThreadPoolExecutor(max_workers=workers) as pool:
        nb = sum(pool.map(job, jobs))
    s = time.perf_counter() - t0
    for fd in fds.values():
        os.close(fd)
    return nb, s


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--dir", default=os.path.join(os.environ.get("TMPDIR", "/tmp"), "qz_model_free"))
    ap.add_argument("--shards", type=int, default=4)
    ap.add_argument("--reps", type=int, default=2)
    ap.add_argument("--workers", type=int, default=16)
    args = ap.parse_args()
    dev = torch.device("cuda:0")
    src, dst = os.path.join(args.dir, "in"), os.path.join(args.dir, "out")
    shutil.rmtree(args.dir, ignore_errors=True)
    os.makedirs(args.dir)
    du = shutil.disk_usage(args.dir)
    print(f"disk at {args.dir}: {du.free / 1e9:.1f} GB free of {du.total / 1e9:.1f}", flush=True)
    t0 = time.perf_counter()
    files, total = make_checkpoint(src, args.shards, dev)
    for f in files:
        evict(os.path.join(src, f))
    res = {"checkpoint": {"dims": "Qwen3-4B (36 layers, hidden 2560, inter 9728, vocab 151936), random bf16",
                          "shards": len(files), "bytes": total, "write_s": time.perf_counter() - t0,
                          "dir": args.dir, "disk_free_GB": du.free / 1e9},
           "call": "model_free_ptq(ckpt, out, scheme='FP8_BLOCK', ignore=<reference list>, max_workers=%d, "
                   "device='cuda:0')" % args.workers}
    print(json.dumps(res["checkpoint"]), flush=True)
    # ceilings
    nb, s = read_pass(src, files, args.workers)
    res["read_only_cold"] = {"bytes": nb, "s": s, "GBps": nb / s / 1e9}
    nb, s = read_pass(src, files, args.workers)
    res["read_only_warm"] = {"bytes": nb, "s": s, "GBps": nb / s / 1e9}
    print(json.dumps({k: res[k] for k in ("read_only_cold", "read_only_warm")}), flush=True)
    host = model_free._read(os.path.join(src, files[1]))
    ws = [t for t in host.values() if t.dim() == 2]
    hb = sum(t.numel() * 2 for t in ws)
    st = H2DStager(dev)
    for rep in range(3):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        outs = [st.copy(t) for t in ws]
        st.synchronize()
        s = time.perf_counter() - t0
        del outs
    res["h2d_staged"] = {"bytes": hb, "s": s, "GBps": hb / s / 1e9, "how": "H2DStager (pageable -> pinned -> device)"}
    pin = torch.empty(hb, dtype=torch.uint8, pin_memory=True)
    dbuf = torch.empty(hb, dtype=torch.uint8, device=dev)
    for rep in range(3):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        dbuf.copy_(pin, non_blocking=True)
        torch.cuda.synchronize()
        s = time.perf_counter() - t0
    res["h2d_pinned_dma"] = {"bytes": hb, "s": s, "GBps": hb / s / 1e9}
    ob = hb // 2
    for rep in range(3):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        pin[:ob].copy_(dbuf[:ob], non_blocking=True)
        torch.cuda.synchronize()
        s = time.perf_counter() - t0
    res["d2h_pinned_dma"] = {"bytes": ob, "s": s, "GBps": ob / s / 1e9}
    del pin, dbuf, host, ws
    print(json.dumps({k: res[k] for k in ("h2d_staged", "h2d_pinned_dma", "d2h_pinned_dma")}), flush=True)
    # the call, cold and warm inputs
    runs = []
    for rep in range(args.reps * 2):
        cold = rep % 2 == 0
        shutil.rmtree(dst, ignore_errors=True)
        if cold:
            for f in files:
                evict(os.path.join(src, f))
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        model_free.model_free_ptq(src, dst, scheme="FP8_BLOCK", ignore=IGNORE, max_workers=args.workers,
                                  device="cuda:0")
        wall = time.perf_counter() - t0
        summ = model_free.run_summary()
        out_bytes = sum(os.path.getsize(os.path.join(dst, f)) for f in os.listdir(dst) if f.endswith(".safetensors"))
        r = {"inputs": "cold" if cold else "warm", "wall_s": wall, "in_GBps": total / wall / 1e9,
             "out_bytes": out_bytes, "phases": summ}
        runs.append(r)
        print(json.dumps(r), flush=True)
    res["runs"] = runs
    # write-only ceiling: the last run's output files written again from memory
    outs = {f: model_free._read(os.path.join(dst, f)) for f in sorted(os.listdir(dst)) if f.endswith(".safetensors")}
    wdir = os.path.join(args.dir, "wonly")
    os.makedirs(wdir)
    t0 = time.perf_counter()
    with ThreadPoolExecutor(max_workers=args.workers) as pool:
        list(pool.map(lambda kv: save_file(kv[1], os.path.join(wdir, kv[0]), {"format": "pt"}), outs.items()))
    s = time.perf_counter() - t0
    for f in outs:
        evict(os.path.join(wdir, f))  # the flush to disk, timed apart (the product does not fsync)
    s_sync = time.perf_counter() - t0
    res["write_only"] = {"bytes": out_bytes, "s": s, "GBps": out_bytes / s / 1e9,
                         "s_with_fsync": s_sync, "GBps_with_fsync": out_bytes / s_sync / 1e9,
                         "how": "save_file of the outputs from memory, as many threads as workers (as the product "
                                "writes: into the page cache); then fsync"}
    print(json.dumps(res["write_only"]), flush=True)
    shutil.rmtree(args.dir, ignore_errors=True)
    print("RESULT " + json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
