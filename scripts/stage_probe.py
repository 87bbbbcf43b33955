#!/usr/bin/env python3
"""Where the time of a whole-model host -> device move goes (H2DStager.stats: device
allocation, waits for a staging buffer, host memcpy into it, DMA enqueue), for the model as the
CLI's --random-init builds it (GPU init, copied to the host), moved whole (oneshot's resident
placement) vs decoder layer by layer (layerwise), in both orders.

  python scripts/stage_probe.py [config dir]"""
import json
import os
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def build(cfg_dir, dev):
    from transformers import AutoConfig, AutoModelForCausalLM
    cfg = AutoConfig.from_pretrained(cfg_dir)
    torch.manual_seed(0)
    with torch.device(dev):
        m = AutoModelForCausalLM.from_config(cfg, dtype=torch.bfloat16)
    return m.to("cpu")


def main():
    from quantizers_amd import oneshot as os_mod
    from quantizers_amd.model import decoder_layers
    from quantizers_amd.staging import H2DStager
    cfg = sys.argv[1] if len(sys.argv) > 1 else os.path.join(ROOT, "configs", "models", "qwen3-4b")
    dev = torch.device("cuda", 0)
    torch.empty(1, device=dev)
    for mode in ("whole_keep", "whole", "whole_keep", "whole", "layerwise"):
        m = build(cfg, dev)
        torch.cuda.synchronize()
        st = H2DStager(dev)
        t0 = time.perf_counter()
        per = []
        keep = []
        if mode.startswith("whole"):
            for mn, mod in m.named_modules():
                for store in (mod._parameters, mod._buffers):
                    for name, t in list(store.items()):
                        if t is not None and t.device.type == "cpu":
                            t1 = time.perf_counter()
                            d = st.copy(t)
                            if mode == "whole_synced":
                                st.synchronize()
                                per.append((time.perf_counter() - t1, t.numel() * t.element_size(), f"{mn}.{name}"))
                            if mode == "whole_keep":
                                keep.append(t.data)
                            if isinstance(t, torch.nn.Parameter):
                                t.data = d
                            else:
                                store[name] = d
            st.synchronize()
            t_copy = time.perf_counter() - t0
            keep.clear()  # the host tensors are freed here, after the copies
        else:
            for layer in decoder_layers(m):
                host = os_mod._onload(layer, st)
                torch.cuda.synchronize()
                os_mod._offload(layer, host)
        dt = time.perf_counter() - t0
        if mode.startswith("whole"):
            st.stats["copy_phase_s"] = t_copy
        print(json.dumps({"mode": mode, "s": round(dt, 3), "GBps": round(st.stats["bytes"] / dt / 1e9, 1),
                          **{k: (round(v, 3) if isinstance(v, float) else v) for k, v in st.stats.items()}}), flush=True)
        if per:
            per.sort(reverse=True)
            print(json.dumps({"slowest": [(round(a * 1e3, 2), b, c) for a, b, c in per[:8]],
                              "median_GBps": round(sorted(b / a for a, b, _ in per if b > 1 << 20)[len(per) // 2] / 1e9, 1)}))
        del m, st
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
