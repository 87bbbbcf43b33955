#!/usr/bin/env python3
"""D8 measurement: what the oracle's AWQ dtype decision
changes.  TEST INFRASTRUCTURE (CPU only, imports oracle/): the oracle's reading (x_mean f32 sums,
w_mean f64 sums, grid scales f32, smoothing products f32 -> bf16, loss an f64 sum) against the
literal reading of SURVEY A.6 (ct_torch.*_literal: x_mean, w_mean and the grid scales in bf16,
W * s and the smoothing in bf16, the loss an f32 sum per calibration batch), on

  1. the AWQ golden fixture's mapping (tests/golden/awq_int4_g128.safetensors inputs), and
  2. a 2-layer Qwen3-4B-shaped model (public dims, random bf16 weights, non-trivial norms), the
     reference's W4A16 AWQ mappings (input_layernorm -> q/k/v, post_attention_layernorm ->
     gate/up, up -> down; v -> o skipped, D9), int4 symmetric g128, N_SEQ x SEQ random tokens,
     layer-sequential: calibrate, search, smooth, propagate, then quantize every linear.

Reported: argmins changed (of the mappings searched), smoothed-weight bf16 elements that differ,
and ``weight_packed`` int32 words that differ.  Both modes run the same driver; only the D8
dtypes differ.  usage: python tests/golden/d8_probe.py [N_SEQ SEQ]  (writes nothing; the numbers
are recorded in profiles/r05_d8_probe.txt and DESIGN.md)."""
import json
import os
import sys
import time

import torch
from safetensors.torch import load_file

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, os.path.join(ROOT, "oracle"))
import ct_torch as ct  # noqa: E402

A = ct.QArgs(num_bits=4, type="int", symmetric=True, group_size=128)


class Mode:
    """The D8 dtypes of one reading."""

    def __init__(self, literal: bool):
        self.literal = literal

    def x_mean(self, xs):
        prev = None
        if self.literal:
            for x in xs:
                prev = ct.awq_accumulate_mean_literal(x, prev)
            return prev[0]
        for x in xs:
            prev = ct.awq_accumulate_mean(x, prev)
        return prev[0] / prev[1]

    def w_mean(self, ws):
        return ct.awq_layer_means_literal(ws, A) if self.literal else ct.awq_layer_means(ws, A).float()

    def scales(self, xm, wm, r):
        return ct.awq_grid_scales_literal(xm, wm, r) if self.literal else ct.awq_grid_scales(xm, wm, r)

    def fq(self, w, s):
        return ct.awq_fake_quant_scaled_literal(w, s, A) if self.literal else ct.awq_fake_quant_scaled(w, s, A)

    def loss(self, refs, outs):
        if self.literal:  # llmcompressor _compute_loss: an f32 sum per batch, summed as Python floats
            tot = sum((r - o).view(-1).float().pow(2).sum().item() for r, o in zip(refs, outs))
        else:  # the product: f64 sum of f32(bf16(a - b))^2 (k_sqdiff, D8)
            tot = sum((r - o).double().pow(2).sum().item() for r, o in zip(refs, outs))
        return tot / sum(r.numel() for r in refs)

    def mul_cols(self, w, s):  # balance W[:, c] *= s[c]
        return w * s.view(1, -1) if self.literal else (w.float() * s.float().view(1, -1)).to(w.dtype)

    def div(self, t, s):  # smooth layer: norm weight / s, or Linear rows / s
        sv = s.view(-1, *([1] * (t.dim() - 1)))
        return t / sv if self.literal else (t.float() / sv.float()).to(t.dtype)


def search(mode: Mode, xs, balance, run_parent):
    """One mapping: (best index, best scale vector).  ``balance`` = list of nn.Linear,
    ``run_parent()`` = the parent's outputs over the cached batches."""
    xm = mode.x_mean(xs)
    wm = mode.w_mean([m.weight.data for m in balance])
    refs = run_parent()
    orig = [m.weight.data.clone() for m in balance]
    best, best_loss, best_s = -1, float("inf"), None
    for i in range(20):
        s = mode.scales(xm, wm, i / 20)
        for m, w0 in zip(balance, orig):
            m.weight.data = mode.fq(w0, s)
        loss = mode.loss(refs, run_parent())
        if loss < best_loss:
            best, best_loss, best_s = i, loss, s
    for m, w0 in zip(balance, orig):
        m.weight.data = w0
    return best, best_s


def fixture_level():
    f = load_file(os.path.join(HERE, "awq_int4_g128.safetensors"))
    x, w = f["x"], f["w"]
    res = {}
    for name, mode in (("oracle", Mode(False)), ("literal", Mode(True))):
        lin = torch.nn.Linear(w.shape[1], w.shape[0], bias=False, dtype=torch.bfloat16)
        lin.weight.data = w.clone()
        best, s = search(mode, [x], [lin], lambda: [lin(x)])
        sm = mode.mul_cols(w, s)
        res[name] = (best, sm, ct.compress_weight(sm, A)["weight_packed"])
    (b0, s0, p0), (b1, s1, p1) = res["oracle"], res["literal"]
    return {"argmin_oracle": b0, "argmin_literal": b1,
            "smoothed_bf16_diff": int((s0.view(torch.int16) != s1.view(torch.int16)).sum()), "smoothed_numel": s0.numel(),
            "packed_words_diff": int((p0 != p1).sum()), "packed_words": p0.numel()}


def model_level(n_seq: int, seq: int):
    from transformers import AutoConfig, AutoModelForCausalLM
    out = {}
    for name, literal in (("oracle", False), ("literal", True)):
        mode = Mode(literal)
        cfg = AutoConfig.from_pretrained(os.path.join(ROOT, "configs", "models", "qwen3-4b"))
        cfg.num_hidden_layers = 2
        torch.manual_seed(0)
        model = AutoModelForCausalLM.from_config(cfg, dtype=torch.bfloat16).eval()
        with torch.no_grad():
            for n, p in model.named_parameters():
                if n.endswith("layernorm.weight"):
                    p.copy_((torch.rand_like(p.float()) * 1.5 + 0.25).to(p.dtype))
        g = torch.Generator().manual_seed(42)
        ids = [torch.randint(0, cfg.vocab_size, (1, seq), generator=g) for _ in range(n_seq)]
        layers = model.model.layers
        inputs = []

        def cap(mod, args, kwargs):
            kw = {n: v for n, v in kwargs.items() if n != "hidden_states"}
            inputs.append((args[0] if args else kwargs["hidden_states"], kw))
            raise StopIteration
        h = layers[0].register_forward_pre_hook(cap, with_kwargs=True)
        with torch.no_grad():
            for t in ids:
                try:
                    model(input_ids=t)
                except StopIteration:
                    pass
        h.remove()
        argmins = []
        with torch.no_grad():
            for li, layer in enumerate(layers):
                at, ml, dn = [], [], []
                hooks = [layer.self_attn.register_forward_pre_hook(
                    lambda m, a, k: at.append((k["hidden_states"], {n: v for n, v in k.items() if n != "hidden_states"})),
                    with_kwargs=True),
                    layer.mlp.register_forward_pre_hook(lambda m, a: ml.append(a[0])),
                    layer.mlp.down_proj.register_forward_pre_hook(lambda m, a: dn.append(a[0]))]
                for hs, kw in inputs:
                    layer(hs, **kw)
                for hk in hooks:
                    hk.remove()
                sa, mlp = layer.self_attn, layer.mlp
                maps = [(layer.input_layernorm, [sa.q_proj, sa.k_proj, sa.v_proj], [x for x, _ in at],
                         lambda: [sa(hidden_states=x, **k)[0] for x, k in at]),
                        (layer.post_attention_layernorm, [mlp.gate_proj, mlp.up_proj], ml,
                         lambda: [mlp(x) for x in ml]),
                        (mlp.up_proj, [mlp.down_proj], dn, lambda: [mlp.down_proj(x) for x in dn])]
                for smooth, bal, xs, run in maps:
                    best, s = search(mode, xs, bal, run)
                    argmins.append(best)
                    for m in bal:
                        m.weight.data = mode.mul_cols(m.weight.data, s)
                    smooth.weight.data = mode.div(smooth.weight.data, s)
                inputs = [(layer(hs, **kw), kw) for hs, kw in inputs]
                print(f"  {name}: layer {li} argmins {argmins[-3:]}", file=sys.stderr, flush=True)
        lin = {n: m.weight.data.clone() for n, m in model.named_modules()
               if isinstance(m, torch.nn.Linear) and ".layers." in n}
        out[name] = (argmins, lin, {n: ct.compress_weight(w, A)["weight_packed"] for n, w in lin.items()})
    (a0, w0, p0), (a1, w1, p1) = out["oracle"], out["literal"]
    per = {}
    for n in w0:
        per[n] = {"smoothed_bf16_diff_frac": float((w0[n].view(torch.int16) != w1[n].view(torch.int16)).float().mean()),
                  "packed_words_diff_frac": float((p0[n] != p1[n]).float().mean())}
    return {"argmins_oracle": a0, "argmins_literal": a1, "argmins_changed": sum(x != y for x, y in zip(a0, a1)),
            "mappings": len(a0),
            "smoothed_bf16_diff": sum(int((w0[n].view(torch.int16) != w1[n].view(torch.int16)).sum()) for n in w0),
            "smoothed_numel": sum(w.numel() for w in w0.values()),
            "packed_words_diff": sum(int((p0[n] != p1[n]).sum()) for n in p0),
            "packed_words": sum(p.numel() for p in p0.values()), "per_linear": per}


if __name__ == "__main__":
    n_seq, seq = (int(sys.argv[1]), int(sys.argv[2])) if len(sys.argv) > 2 else (4, 256)
    torch.set_num_threads(os.cpu_count() or 8)
    t0 = time.time()
    fx = fixture_level()
    print(json.dumps({"fixture_mapping": fx}), flush=True)
    md = model_level(n_seq, seq)
    print(json.dumps({"qwen3_4b_2layers": md, "calibration": f"{n_seq} x {seq} tokens",
                      "seconds": round(time.time() - t0, 1)}), flush=True)
