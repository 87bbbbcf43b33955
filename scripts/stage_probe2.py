#!/usr/bin/env python3
"""Which side makes the whole-model host -> device move slow (stage_probe.py): the host tensors
the GPU-initialised model was copied into, or the device blocks it freed?

  model_src   : the model's host tensors -> device blocks already written by earlier copies
  filled_src  : freshly filled host tensors of the same shapes -> the blocks the model freed
  (each twice, alternating)"""
import json
import os
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from quantizers_amd.staging import H2DStager  # noqa: E402


def host_model(dev):
    from transformers import AutoConfig, AutoModelForCausalLM
    cfg = AutoConfig.from_pretrained(os.path.join(ROOT, "configs", "models", "qwen3-4b"))
    torch.manual_seed(0)
    with torch.device(dev):
        m = AutoModelForCausalLM.from_config(cfg, dtype=torch.bfloat16)
    return m.to("cpu")


def run(st, srcs):
    for k in st.stats:
        st.stats[k] = 0 if k == "bytes" else 0.0
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    per = []
    outs = []
    for name, t in srcs:
        t1 = time.perf_counter()
        outs.append(st.copy(t))
        st.synchronize()
        per.append((time.perf_counter() - t1, name, t.numel() * t.element_size()))
    dt = time.perf_counter() - t0
    per.sort(reverse=True)
    return outs, {"s": round(dt, 3), "GBps": round(st.stats["bytes"] / dt / 1e9, 1),
                  "slowest": [(round(a * 1e3, 1), n, b) for a, n, b in per[:4]]}


def main():
    dev = torch.device("cuda", 0)
    st = H2DStager(dev)
    res = {}
    for rnd in range(2):
        m = host_model(dev)  # its device blocks are now free in the caching allocator
        srcs = [(n, p.data) for n, p in m.named_parameters()]
        filled = [(n, torch.empty(t.shape, dtype=t.dtype).fill_(0.5)) for n, t in srcs]
        # filled host tensors into the blocks the model freed
        outs, res[f"filled_src_into_model_blocks_{rnd}"] = run(st, filled)
        del outs
        # the model's host tensors into blocks just written by copies
        outs, res[f"model_src_into_copied_blocks_{rnd}"] = run(st, srcs)
        del outs, m, srcs, filled
        torch.cuda.empty_cache()
        print(json.dumps({k: v for k, v in res.items() if k.endswith(str(rnd))}), flush=True)


if __name__ == "__main__":
    main()
