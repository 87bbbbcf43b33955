"""End-to-end on the GPU: oneshot (RTN + AWQ) on small random-weight Qwen3 / Qwen3-MoE models,
save_compressed -> compressed-tensors checkpoint, bit-exact against the CPU oracle applied to the
same (smoothed) weights; AWQ checked against an oracle restatement of the search."""
import json
import os

import pytest
import torch

import ct_torch as ct
from quantizers_amd import ops
from quantizers_amd.awq import DEFAULT_MAPPINGS, resolve_mappings
from quantizers_amd.compressor import compressed_state_dict, load_decompressed, save_compressed
from quantizers_amd.oneshot import oneshot

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _qwen3(layers=2, hidden=256, inter=512):
    from transformers import AutoModelForCausalLM, Qwen3Config
    cfg = Qwen3Config(hidden_size=hidden, intermediate_size=inter, num_hidden_layers=layers, num_attention_heads=4,
                      num_key_value_heads=2, head_dim=64, vocab_size=512, max_position_embeddings=256)
    torch.manual_seed(0)
    m = AutoModelForCausalLM.from_config(cfg, dtype=torch.bfloat16)
    with torch.no_grad():  # non-trivial norms so smoothing has something to move
        for n, p in m.named_parameters():
            if n.endswith("layernorm.weight"):
                p.copy_((torch.rand_like(p.float()) * 1.5 + 0.25).to(p.dtype))
    return m


def _qwen3_moe():
    from transformers import AutoModelForCausalLM, Qwen3MoeConfig
    cfg = Qwen3MoeConfig(hidden_size=128, intermediate_size=256, moe_intermediate_size=64, num_hidden_layers=2,
                         num_attention_heads=4, num_key_value_heads=2, head_dim=32, vocab_size=256, num_experts=8,
                         num_experts_per_tok=2)
    torch.manual_seed(0)
    return AutoModelForCausalLM.from_config(cfg, dtype=torch.bfloat16)


def _calib(n=4, s=64, vocab=512):
    g = torch.Generator().manual_seed(42)
    return [{"input_ids": torch.randint(0, vocab, (s,), generator=g)} for _ in range(n)]


def _oa(a):
    sd = {None: None, "float8_e4m3fn": "fp8", "uint8": "e8m0"}[a.scale_dtype]
    return ct.QArgs(num_bits=a.num_bits, type=a.type, symmetric=a.symmetric, strategy=a.strategy,
                    group_size=a.group_size, block_structure=tuple(a.block_structure) if a.block_structure else None,
                    scale_dtype=sd)


def _eq(a, b, key=""):
    a, b = a.cpu(), b.cpu()
    assert a.shape == b.shape, (key, a.shape, b.shape)
    if a.dtype in (torch.bfloat16, torch.float8_e4m3fn):
        a = a.view(torch.int16 if a.dtype == torch.bfloat16 else torch.uint8)
        b = b.view(torch.int16 if b.dtype == torch.bfloat16 else torch.uint8)
    assert torch.equal(a, b), key


def _check_against_oracle(model, sd):
    """Every targeted module's on-disk tensors == oracle compress of its current bf16 weight."""
    from quantizers_amd.model import iter_linears
    n = 0
    for ref in iter_linears(model):
        sch = model.quantization_scheme_map.get(ref.name)
        if sch is None:
            assert f"{ref.name}.weight" in sd
            continue
        want = ct.compress_weight(ref.weight.detach().cpu().contiguous(), _oa(sch.weights))
        for k, v in want.items():
            _eq(sd[f"{ref.name}.{k}"], v, f"{ref.name}.{k}")
        n += 1
    return n


def test_rtn_w4a16_save_roundtrip(cuda, tmp_path):
    m = _qwen3().to(cuda)
    recipe = {"s": {"m": {"QuantizationModifier": {"scheme": "W4A16", "targets": "Linear", "ignore": ["lm_head"]}}}}
    oneshot(m, recipe)
    out = save_compressed(m, str(tmp_path / "w4a16"))
    cfg = json.load(open(os.path.join(out, "config.json")))["quantization_config"]
    assert cfg["quant_method"] == "compressed-tensors" and cfg["format"] == "pack-quantized"
    assert cfg["quantization_status"] == "compressed" and cfg["ignore"] == ["lm_head"]
    g = cfg["config_groups"]["group_0"]["weights"]
    assert (g["num_bits"], g["group_size"], g["strategy"], g["symmetric"]) == (4, 128, "group", True)
    sd = compressed_state_dict(m)
    assert _check_against_oracle(m, sd) == 14
    # decompress and compare with the oracle fake-quant
    dec = load_decompressed(out)
    w = m.model.layers[0].mlp.down_proj.weight.detach().cpu()
    oa = ct.QArgs(num_bits=4, group_size=128)
    mn, mx = ct.observe_minmax(w, oa)
    s, z = ct.calculate_qparams(mn, mx, oa)
    q = ct.quantize(w, s, z, oa, dtype=torch.int8)
    _eq(dec["model.layers.0.mlp.down_proj.weight"], ct.dequantize(q, s, None, oa, dtype=torch.bfloat16))


@pytest.mark.parametrize("moe", [False, True], ids=["dense", "moe"])
def test_rtn_host_resident_model_staged(cuda, monkeypatch, moe):
    """A host-resident model (RTN recipe: oneshot moves nothing): save-time compression stages the
    weights through the pinned buffers, in several plan chunks sharing one stager (fused expert
    parameters staged whole and sliced on the device), and gives the same tensors as the
    device-resident model and the oracle."""
    import quantizers_amd.compressor as comp
    build = _qwen3_moe if moe else _qwen3
    recipe = {"s": {"m": {"QuantizationModifier": {"scheme": "W4A16", "targets": "Linear", "ignore": ["lm_head"]}}}}
    if moe:  # int4 g32 on the experts only (the other linears stay bf16)
        recipe = {"s": {"m": {"QuantizationModifier": {"config_groups": {"g": {
            "targets": ["re:.*mlp\\.experts\\.\\d+\\.(down_proj|gate_proj|up_proj)$"],
            "weights": {"num_bits": 4, "type": "int", "symmetric": True, "strategy": "group", "group_size": 32}}}}}}}
    m = build()
    oneshot(m, recipe, device=cuda)
    assert next(m.parameters()).device.type == "cpu"
    monkeypatch.setattr(comp, "STAGE_BYTES", 300 << 10)  # several plans
    host_sd = compressed_state_dict(m, cuda)
    assert _check_against_oracle(m, host_sd) == (2 * 8 * 3 if moe else 14)
    md = build().to(cuda)
    oneshot(md, recipe)
    dev_sd = compressed_state_dict(md)
    assert set(host_sd) == set(dev_sd)
    for k in host_sd:
        _eq(host_sd[k], dev_sd[k], k)


@pytest.mark.parametrize("resident", [True, False], ids=["device", "host"])
def test_streamed_shards_match_state_dict(cuda, tmp_path, resident):
    """save_compressed streams shards while it compresses: with a small shard size the files
    (model-XXXXX-of-NNNNN + index) hold exactly compressed_state_dict's tensors, in unit order,
    and no temporary file is left."""
    from safetensors.torch import load_file
    recipe = {"s": {"m": {"QuantizationModifier": {"scheme": "W4A16", "targets": "Linear", "ignore": ["lm_head"]}}}}
    m = _qwen3()
    if resident:
        m = m.to(cuda)
    oneshot(m, recipe, device=cuda)
    out = save_compressed(m, str(tmp_path / "ck"), max_shard_bytes=200 << 10, device=cuda)
    files = sorted(os.listdir(out))
    shards = [f for f in files if f.endswith(".safetensors")]
    assert len(shards) > 3 and not any(f.endswith(".tmp") for f in files)
    assert all(f.endswith(f"-of-{len(shards):05d}.safetensors") for f in shards)
    idx = json.load(open(os.path.join(out, "model.safetensors.index.json")))
    got = {}
    for f in shards:
        part = load_file(os.path.join(out, f))
        assert all(idx["weight_map"][k] == f for k in part)
        got.update(part)
    want = compressed_state_dict(m, cuda)
    assert set(got) == set(want) == set(idx["weight_map"])
    for k in want:
        _eq(got[k], want[k], k)


def test_documented_patch_keeps_quantization_config(cuda, tmp_path):
    """INTEGRATION.md's do_oneshot.py patch: save_compressed(model, dir) and then the
    reference's own model.config.save_pretrained(dir) (e.g. left in by a maintainer) -- the
    rewritten config.json still carries the compressed-tensors quantization_config."""
    m = _qwen3(layers=1).to(cuda)
    oneshot(m, {"s": {"m": {"QuantizationModifier": {"scheme": "W4A16", "targets": "Linear",
                                                        "ignore": ["lm_head"]}}}})
    out = str(tmp_path / "ckpt")
    save_compressed(m, out)
    want = json.load(open(os.path.join(out, "config.json")))["quantization_config"]
    m.config.save_pretrained(out)
    got = json.load(open(os.path.join(out, "config.json")))
    assert got.get("quantization_config") == want
    assert want["quant_method"] == "compressed-tensors"


def test_host_model_resident_vs_layer_onload(cuda):
    """A host-resident model: moved to the device once (device_resident=True, the default when it
    fits) or onloaded layer by layer and returned to the host (False, the reference's placement)
    -- the smoothed weights and the compressed tensors are identical either way."""
    recipe = os.path.join(ROOT, "configs", "recipes", "awq_w4a16_g32.yaml")
    out = {}
    for resident in (True, False):
        m = _qwen3()
        oneshot(m, recipe, dataset=_calib(), max_seq_length=64, device=cuda, device_resident=resident)
        dev = next(m.model.layers[0].parameters()).device
        assert dev.type == ("cuda" if resident else "cpu")
        out[resident] = compressed_state_dict(m)
    assert out[True].keys() == out[False].keys()
    for k in out[True]:
        _eq(out[True][k], out[False][k], k)


def test_awq_int4_g32_end_to_end(cuda, tmp_path):
    torch.manual_seed(0)
    m = _qwen3().to(cuda)
    calib = _calib()
    ids = torch.stack([c["input_ids"] for c in calib]).to(cuda)
    with torch.no_grad():
        ref_logits = m(ids).logits.float()
    recipe = os.path.join(ROOT, "configs", "recipes", "awq_w4a16_g32.yaml")
    oneshot(m, recipe, dataset=calib, max_seq_length=64)
    rep = m.awq_report
    assert len(rep) == 2
    for layer, maps in rep.items():
        # v_proj -> o_proj skipped for GQA (D9): 3 mappings per layer
        assert len(maps) == 3, maps.keys()
        for smooth, r in maps.items():
            assert 0.0 <= r["best_ratio"] < 1.0 and len(r["history"]) == 20
            assert r["best_loss"] <= r["history"][0] + 1e-12
    # smoothing preserves the function (up to bf16 rounding of the rescaled weights)
    with torch.no_grad():
        new_logits = m(ids).logits.float()
    rel = (new_logits - ref_logits).norm() / ref_logits.norm()
    assert rel < 0.05, rel
    out = save_compressed(m, str(tmp_path / "awq"))
    sd = compressed_state_dict(m)
    assert _check_against_oracle(m, sd) == 14
    assert os.path.exists(os.path.join(out, "model.safetensors"))
    assert open(os.path.join(out, "recipe.yaml")).read() == open(recipe).read()


@pytest.mark.parametrize("arch", ["qwen2", "llama"])
def test_awq_mha_with_biases(cuda, arch):
    """Other llama-family decoders: full multi-head attention (so the v_proj -> o_proj mapping
    runs: four mappings per layer) with q/k/v biases set to non-zero values.  Smoothing v_proj
    must divide its bias too, or the smoothed model's output moves by W_o (s - 1) b; the check is
    that smoothing preserves the function, and the checkpoint matches the oracle."""
    from transformers import AutoModelForCausalLM, LlamaConfig, Qwen2Config
    kw = dict(hidden_size=256, intermediate_size=512, num_hidden_layers=2, num_attention_heads=4,
              num_key_value_heads=4, vocab_size=512, max_position_embeddings=256)
    cfg = Qwen2Config(**kw) if arch == "qwen2" else LlamaConfig(attention_bias=True, **kw)
    torch.manual_seed(0)
    m = AutoModelForCausalLM.from_config(cfg, dtype=torch.bfloat16)
    with torch.no_grad():
        for n, p in m.named_parameters():
            if n.endswith("layernorm.weight"):
                p.copy_((torch.rand_like(p.float()) * 1.5 + 0.25).to(p.dtype))
            elif n.endswith(".bias"):
                p.copy_((torch.rand_like(p.float()) - 0.5).to(p.dtype))
    m = m.to(cuda)
    calib = _calib()
    ids = torch.stack([c["input_ids"] for c in calib]).to(cuda)
    with torch.no_grad():
        ref_logits = m(ids).logits.float()
    v_bias0 = m.model.layers[0].self_attn.v_proj.bias.detach().clone()
    oneshot(m, os.path.join(ROOT, "configs", "recipes", "awq_w4a16_g32.yaml"), dataset=calib, max_seq_length=64)
    for layer, maps in m.awq_report.items():
        assert len(maps) == 4, maps.keys()  # v_proj -> o_proj included (no GQA)
    assert not torch.equal(m.model.layers[0].self_attn.v_proj.bias, v_bias0)  # the bias was rescaled
    with torch.no_grad():
        new_logits = m(ids).logits.float()
    rel = (new_logits - ref_logits).norm() / ref_logits.norm()
    assert rel < 0.05, rel
    sd = compressed_state_dict(m)
    assert _check_against_oracle(m, sd) == 14
    assert "model.layers.0.self_attn.v_proj.bias" in sd


def test_awq_layer_matches_oracle_search(cuda):
    """Layer-0 AWQ: statistics, w_mean and grid losses from the GPU path vs a CPU restatement."""
    from quantizers_amd.quantization import QuantizationArgs
    m = _qwen3(layers=1).to(cuda)
    calib = _calib(n=2, s=32)
    a = QuantizationArgs(num_bits=4, type="int", symmetric=True, group_size=32)
    layer = m.model.layers[0]
    names = [f"model.layers.0.mlp.{p}" for p in ("gate_proj", "up_proj", "down_proj")]
    quantized = {n: a for n in names}
    (r,) = [x for x in resolve_mappings(layer, "model.layers.0", DEFAULT_MAPPINGS, quantized)
            if x.smooth_name.endswith("post_attention_layernorm")]
    # inputs of the MLP for each sample
    xs = []
    h = layer.mlp.register_forward_pre_hook(lambda mod, args: xs.append(args[0].detach().clone()))
    with torch.no_grad():
        for c in calib:
            m(c["input_ids"].unsqueeze(0).to(cuda))
    h.remove()
    gw, uw = layer.mlp.gate_proj.weight.detach(), layer.mlp.up_proj.weight.detach()
    # GPU statistics
    sums = torch.zeros(gw.shape[1], dtype=torch.float32, device=cuda)
    cnt = sum(ops.awq_absmean_accum(x, sums) for x in xs)
    x_mean = sums / cnt
    wsum = torch.zeros(gw.shape[1], dtype=torch.float64, device=cuda)
    rows = ops.awq_weight_mean_accum(gw, 32, wsum) + ops.awq_weight_mean_accum(uw, 32, wsum)
    w_mean = wsum / rows
    # CPU restatement
    xc = [x.cpu() for x in xs]
    s_ref, n_ref = None, 0
    for x in xc:
        s_ref = ct.awq_accumulate_mean(x, None if s_ref is None else (s_ref, n_ref))
        s_ref, n_ref = s_ref
    torch.testing.assert_close(x_mean.cpu(), s_ref / n_ref, rtol=1e-5, atol=1e-6)
    wm_ref = ct.awq_layer_means([gw.cpu(), uw.cpu()], ct.QArgs(group_size=32))
    torch.testing.assert_close(w_mean.cpu(), wm_ref, rtol=1e-12, atol=1e-12)
    # grid points: scale vectors and the fused Q(W*s)/s step vs the restatement
    for ratio in (0.0, 0.45, 0.9):
        s = ops.awq_grid_scales(x_mean, w_mean.float(), ratio, True)
        s_c = ct.awq_grid_scales(s_ref / n_ref, wm_ref, ratio, True)
        torch.testing.assert_close(s.cpu(), s_c, rtol=1e-5, atol=1e-7)
        g_fq = ops.fake_quantize(gw, a, col_scales=s)
        g_ref = ct.awq_fake_quant_scaled(gw.cpu(), s.cpu(), ct.QArgs(group_size=32))
        _eq(g_fq, g_ref, f"fake-quant ratio {ratio}")


def test_dense_mlp_awq_all_ratios_and_argmin(cuda):
    """post_attention_layernorm -> {gate, up} (parent: the MLP) through awq_layer: all 20 grid
    losses against a restatement (oracle statistics, oracle grid scales, oracle Q(W*s)/s, the
    same MLP forward on the device), the chosen ratio is the restated argmin, and the applied
    smoothing is bf16(W * s) on gate/up and bf16(w / s) on the norm."""
    import copy
    from quantizers_amd.awq import awq_layer
    from quantizers_amd.oneshot import _batches, _capture_layer0_inputs
    from quantizers_amd.quantization import QuantizationArgs
    from quantizers_amd.recipe import AWQMapping
    m = _qwen3(layers=1).to(cuda)
    layer = m.model.layers[0]
    a = QuantizationArgs(num_bits=4, type="int", symmetric=True, group_size=128)
    quantized = {f"model.layers.0.mlp.{p}": a for p in ("gate_proj", "up_proj", "down_proj")}
    inputs = _capture_layer0_inputs(m, m.model.layers, _batches(_calib(n=3, s=64), None, None, cuda))
    xs = []
    h = layer.mlp.register_forward_pre_hook(lambda mod, args: xs.append(args[0].detach().clone()))
    with torch.no_grad():
        for args, kw in inputs:
            layer(*args, **kw)
    h.remove()
    mlp0 = copy.deepcopy(layer.mlp)
    norm0 = layer.post_attention_layernorm.weight.detach().clone()
    gw, uw = mlp0.gate_proj.weight.detach().cpu(), mlp0.up_proj.weight.detach().cpu()
    rep = awq_layer(layer, "model.layers.0", inputs,
                    [AWQMapping("re:.*post_attention_layernorm$", ["re:.*gate_proj$", "re:.*up_proj$"])], quantized,
                    awq_dtype="fp32")
    r = rep["model.layers.0.post_attention_layernorm"]
    # restatement
    oa = ct.QArgs(group_size=128)
    s_ref, n_ref = None, 0
    for x in xs:
        (s_ref, n_ref) = ct.awq_accumulate_mean(x.cpu(), None if s_ref is None else (s_ref, n_ref))
    x_mean = s_ref / n_ref
    w_mean = ct.awq_layer_means([gw, uw], oa).float()
    xcat = torch.cat([x.reshape(-1, x.shape[-1]) for x in xs])
    with torch.no_grad():
        ref_out = mlp0(xcat)
        hist = []
        probe = copy.deepcopy(mlp0)
        for i in range(20):
            s = ct.awq_grid_scales(x_mean, w_mean, i / 20, True)
            probe.gate_proj.weight.copy_(ct.awq_fake_quant_scaled(gw, s, oa))
            probe.up_proj.weight.copy_(ct.awq_fake_quant_scaled(uw, s, oa))
            hist.append((ref_out - probe(xcat)).double().pow(2).sum().item() / ref_out.numel())
    torch.testing.assert_close(torch.tensor(r["history"]), torch.tensor(hist), rtol=2e-3, atol=1e-12)
    best_i = int(round(r["best_ratio"] * 20))
    want_i = min(range(20), key=lambda i: (hist[i], i))
    srt = sorted(hist)
    if srt[1] > srt[0] * 1.002:  # the restated argmin is unambiguous at this tolerance
        assert best_i == want_i, (best_i, want_i, hist)
    assert hist[best_i] <= min(hist) * 1.002
    # the applied smoothing, from the device statistics awq_layer used (same kernels, same order)
    sums = torch.zeros(x_mean.numel(), dtype=torch.float32, device=cuda)
    cnt = sum(ops.awq_absmean_accum(x, sums) for x in xs)
    wsum = torch.zeros(x_mean.numel(), dtype=torch.float64, device=cuda)
    rows = sum(ops.awq_weight_mean_accum(w.to(cuda), 128, wsum) for w in (gw, uw))
    torch.testing.assert_close((sums / cnt).cpu(), x_mean, rtol=1e-5, atol=1e-7)
    s = ops.awq_grid_scales(sums / cnt, (wsum / rows).float(), best_i / 20, True).cpu()
    _eq(layer.mlp.gate_proj.weight, (gw.float() * s.view(1, -1)).to(torch.bfloat16), "gate smoothed")
    _eq(layer.mlp.up_proj.weight, (uw.float() * s.view(1, -1)).to(torch.bfloat16), "up smoothed")
    _eq(layer.post_attention_layernorm.weight, (norm0.cpu().float() / s).to(torch.bfloat16), "norm smoothed")


def test_dense_mlp_awq_bf16_matches_literal_oracle(cuda):
    """D8, bf16 reading (the default since round 5): post_attention_layernorm -> {gate, up} through
    awq_layer vs the literal restatement (ct_torch.*_literal: the bf16 running mean over the
    calibration batches, bf16 w_mean per layer, bf16 grid formula, Q(W*s)/s with bf16 scales): all
    20 losses, the argmin, and the applied smoothing -- bf16(W * s) on gate / up and bf16(w / s) on
    the norm with the product's own bf16 scale vector (itself within 1 ulp of the restatement's)."""
    import copy
    from quantizers_amd import awq as awq_mod
    from quantizers_amd.awq import awq_layer
    from quantizers_amd.oneshot import _batches, _capture_layer0_inputs
    from quantizers_amd.quantization import QuantizationArgs
    from quantizers_amd.recipe import AWQMapping
    m = _qwen3(layers=1).to(cuda)
    layer = m.model.layers[0]
    a = QuantizationArgs(num_bits=4, type="int", symmetric=True, group_size=128)
    quantized = {f"model.layers.0.mlp.{p}": a for p in ("gate_proj", "up_proj", "down_proj")}
    inputs = _capture_layer0_inputs(m, m.model.layers, _batches(_calib(n=3, s=64), None, None, cuda))
    xs = []
    h = layer.mlp.register_forward_pre_hook(lambda mod, args: xs.append(args[0].detach().clone()))
    with torch.no_grad():
        for args, kw in inputs:
            layer(*args, **kw)
    h.remove()
    mlp0 = copy.deepcopy(layer.mlp)
    norm0 = layer.post_attention_layernorm.weight.detach().clone()
    gw, uw = mlp0.gate_proj.weight.detach().cpu(), mlp0.up_proj.weight.detach().cpu()
    rep = awq_layer(layer, "model.layers.0", inputs,
                    [AWQMapping("re:.*post_attention_layernorm$", ["re:.*gate_proj$", "re:.*up_proj$"])], quantized,
                    awq_dtype="bf16")
    r = rep["model.layers.0.post_attention_layernorm"]
    oa = ct.QArgs(group_size=128)
    prev = None
    for x in xs:
        prev = ct.awq_accumulate_mean_literal(x.cpu().reshape(-1, x.shape[-1]), prev)
    x_mean = prev[0]
    w_mean = ct.awq_layer_means_literal([gw, uw], oa)
    xcat = torch.cat([x.reshape(-1, x.shape[-1]) for x in xs])
    with torch.no_grad():
        ref_out = mlp0(xcat)
        hist = []
        probe = copy.deepcopy(mlp0)
        for i in range(20):
            s = ct.awq_grid_scales_literal(x_mean, w_mean, i / 20, True)
            probe.gate_proj.weight.copy_(ct.awq_fake_quant_scaled_literal(gw, s, oa))
            probe.up_proj.weight.copy_(ct.awq_fake_quant_scaled_literal(uw, s, oa))
            hist.append((ref_out - probe(xcat)).double().pow(2).sum().item() / ref_out.numel())
    torch.testing.assert_close(torch.tensor(r["history"]), torch.tensor(hist), rtol=5e-3, atol=1e-12)
    best_i = int(round(r["best_ratio"] * 20))
    assert hist[best_i] <= min(hist) * 1.005
    # the product's own statistics (bf16) -> its scale vector; within 1 ulp of the restatement's
    am = awq_mod._AbsMean(bf16=True)
    for x in xs:
        am.add(x)
    parts = []
    for w_ in (gw, uw):
        ws_ = torch.zeros(w_.shape[1], dtype=torch.float64, device=cuda)
        parts.append((ws_, ops.awq_weight_mean_accum(w_.to(cuda), 128, ws_)))
    wm_dev = (parts[0][0].to(torch.bfloat16) + parts[1][0].to(torch.bfloat16)) / (parts[0][1] + parts[1][1])
    s_dev = awq_mod._grid_scales_bf16(am.mean(), wm_dev, best_i / 20, True).cpu()
    s_lit = ct.awq_grid_scales_literal(x_mean, w_mean, best_i / 20, True)
    d = (s_dev.to(torch.bfloat16).view(torch.int16).int() - s_lit.view(torch.int16).int()).abs()
    assert d.max() <= 1 and (d > 0).float().mean() < 0.02, (int(d.max()), float((d > 0).float().mean()))
    _eq(layer.mlp.gate_proj.weight, (gw.float() * s_dev.view(1, -1)).to(torch.bfloat16), "gate smoothed")
    _eq(layer.mlp.up_proj.weight, (uw.float() * s_dev.view(1, -1)).to(torch.bfloat16), "up smoothed")
    _eq(layer.post_attention_layernorm.weight, (norm0.cpu().float() / s_dev).to(torch.bfloat16), "norm smoothed")


@pytest.mark.parametrize("observer", ["minmax", "static_minmax"])
def test_stateful_observer_grid(cuda, observer):
    """D7, stateful reading: a balance layer whose scheme names ``minmax`` (moving average,
    averaging_constant 0.01) or ``static_minmax`` (running extremes) keeps the observer memory
    across the grid points.  (1) the device step (W*s -> observe -> state update -> qparams ->
    fake-quant -> /s) is bit-identical to the oracle over a run of updates; (2) awq_layer's 20
    losses match a restatement that threads the same state through the grid."""
    import copy
    from quantizers_amd.awq import _ObserverState, _fake_quant_stateful, awq_layer
    from quantizers_amd.oneshot import _batches, _capture_layer0_inputs
    from quantizers_amd.quantization import QuantizationArgs
    from quantizers_amd.recipe import AWQMapping
    a = QuantizationArgs(num_bits=4, type="int", symmetric=True, group_size=32, observer=observer)
    oa = ct.QArgs(group_size=32)

    def step_ref(w, s, past):
        ws = (w.float() * s.view(1, -1)).to(torch.bfloat16)
        mn, mx = ct.observe_minmax(ws, oa)
        if observer == "minmax":
            mn, mx = ct.moving_average_minmax(mn, mx, *(past or (None, None)))
        elif past is not None:
            mn, mx = torch.minimum(past[0], mn), torch.maximum(past[1], mx)
        sc, zp = ct.calculate_qparams(mn, mx, oa)
        return (ct.fake_quantize(ws, sc, zp, oa).float() / s.view(1, -1)).to(torch.bfloat16), (mn, mx)

    g = torch.Generator().manual_seed(4)
    w = (torch.randn(96, 256, generator=g) * 0.02).to(torch.bfloat16)
    st, past = _ObserverState(a), None
    out = torch.empty(96, 256, dtype=torch.bfloat16, device=cuda)
    for i in range(5):
        s = (torch.rand(256, generator=g) * 2 + 0.2).float()
        _fake_quant_stateful(w.to(cuda), a, s.to(cuda), out, st)
        want, past = step_ref(w, s, past)
        _eq(out, want, f"stateful step {i}")
        _eq(st.mn, past[0], f"state min {i}")
    # (2) through awq_layer: post_attention_layernorm -> gate/up, parent the MLP
    m = _qwen3(layers=1).to(cuda)
    layer = m.model.layers[0]
    quantized = {f"model.layers.0.mlp.{p}": a for p in ("gate_proj", "up_proj", "down_proj")}
    inputs = _capture_layer0_inputs(m, m.model.layers, _batches(_calib(n=2, s=64), None, None, cuda))
    xs = []
    h = layer.mlp.register_forward_pre_hook(lambda mod, args: xs.append(args[0].detach().clone()))
    with torch.no_grad():
        for args, kw in inputs:
            layer(*args, **kw)
    h.remove()
    mlp0 = copy.deepcopy(layer.mlp)
    gw, uw = mlp0.gate_proj.weight.detach().cpu(), mlp0.up_proj.weight.detach().cpu()
    rep = awq_layer(layer, "model.layers.0", inputs,
                    [AWQMapping("re:.*post_attention_layernorm$", ["re:.*gate_proj$", "re:.*up_proj$"])], quantized,
                    stateful_observers=True, awq_dtype="fp32")
    r = rep["model.layers.0.post_attention_layernorm"]
    sums = torch.zeros(gw.shape[1], dtype=torch.float32, device=cuda)
    cnt = sum(ops.awq_absmean_accum(x, sums) for x in xs)
    wsum = torch.zeros(gw.shape[1], dtype=torch.float64, device=cuda)
    rows = sum(ops.awq_weight_mean_accum(t.to(cuda), 32, wsum) for t in (gw, uw))
    xcat = torch.cat([x.reshape(-1, x.shape[-1]) for x in xs])
    hist, pg, pu = [], None, None
    with torch.no_grad():
        ref_out = mlp0(xcat)
        probe = copy.deepcopy(mlp0)
        for i in range(20):
            s = ops.awq_grid_scales(sums / cnt, (wsum / rows).float(), i / 20, True).cpu()
            fg, pg = step_ref(gw, s, pg)
            fu, pu = step_ref(uw, s, pu)
            probe.gate_proj.weight.copy_(fg)
            probe.up_proj.weight.copy_(fu)
            hist.append((ref_out - probe(xcat)).double().pow(2).sum().item() / ref_out.numel())
    torch.testing.assert_close(torch.tensor(r["history"]), torch.tensor(hist), rtol=1e-3, atol=1e-12)


def test_mixed_fp8_block_and_awq(cuda, tmp_path):
    m = _qwen3().to(cuda)
    oneshot(m, os.path.join(ROOT, "configs/recipes/mixed_fp8_block_awq_int4.yaml"), dataset=_calib(),
            max_seq_length=64)
    sd = compressed_state_dict(m)
    assert _check_against_oracle(m, sd) == 14
    assert sd["model.layers.0.self_attn.q_proj.weight"].dtype == torch.float8_e4m3fn
    assert sd["model.layers.0.self_attn.q_proj.weight_scale"].shape == (2, 2)
    save_compressed(m, str(tmp_path / "mixed"))
    cfg = json.load(open(tmp_path / "mixed" / "config.json"))["quantization_config"]
    assert cfg["format"] == "mixed-precision"
    assert {g["format"] for g in cfg["config_groups"].values()} == {"float-quantized", "pack-quantized"}


@pytest.mark.parametrize("recipe,key", [("moe_experts_nvfp4.yaml", "weight_global_scale"),
                                        ("moe_experts_mxfp4.yaml", "weight_packed")])
def test_moe_fused_experts(cuda, tmp_path, recipe, key):
    m = _qwen3_moe().to(cuda)
    oneshot(m, os.path.join(ROOT, "configs/recipes", recipe))
    names = sorted(m.quantization_scheme_map)
    assert len(names) == 2 * 8 * 3  # layers x experts x {gate, up, down}
    assert "model.layers.1.mlp.experts.7.down_proj" in names
    sd = compressed_state_dict(m)
    assert _check_against_oracle(m, sd) == 48
    assert f"model.layers.0.mlp.experts.3.gate_proj.{key}" in sd
    assert not any(k.endswith("experts.gate_up_proj") for k in sd)
    save_compressed(m, str(tmp_path / "moe"))


def _minimax(layers=2, experts=8):
    import warnings
    from transformers import AutoModelForCausalLM, MiniMaxM2Config
    cfg = MiniMaxM2Config(hidden_size=128, intermediate_size=64, num_hidden_layers=layers, num_attention_heads=4,
                          num_key_value_heads=2, head_dim=32, vocab_size=256, num_local_experts=experts,
                          num_experts_per_tok=2, bos_token_id=1, eos_token_id=2)
    torch.manual_seed(0)
    with warnings.catch_warnings():
        warnings.simplefilter("ignore")
        m = AutoModelForCausalLM.from_config(cfg, dtype=torch.bfloat16)
    with torch.no_grad():
        for n, p in m.named_parameters():
            if n.endswith("layernorm.weight"):
                p.copy_((torch.rand_like(p.float()) * 1.5 + 0.25).to(p.dtype))
    return m


@pytest.mark.parametrize("arch", ["qwen3_moe", "minimax"])
def test_moe_fast_eager_experts(cuda, monkeypatch, arch):
    """D15: the AWQ pass runs transformers' fused experts in their eager arithmetic (the
    reference's 4.57 per-expert loop).  moe_eager.fast_eager is bit-identical to the modules'
    eager forward (direct check), and a whole AWQ pass through it gives the same loss histories
    and parameters as one through the eager loop itself."""
    import quantizers_amd.moe_eager as me
    m = (_qwen3_moe() if arch == "qwen3_moe" else _minimax()).to(cuda)
    ex = next(mod for mod in m.modules() if me.eager_forward(mod) is not None)
    g = torch.Generator(device=cuda).manual_seed(1)
    x = torch.randn(300, ex.gate_up_proj.shape[-1], device=cuda, generator=g).to(torch.bfloat16)
    probs = torch.rand(300, ex.num_experts, device=cuda, generator=g).softmax(-1)
    w, idx = torch.topk(probs, 2, dim=-1)
    w = (w / w.sum(-1, keepdim=True)).to(torch.bfloat16)
    with torch.no_grad():
        _eq(me.fast_eager(ex, x, idx, w), me.eager_forward(ex)(ex, x, idx, w), "fast eager")
    recipe = os.path.join(ROOT, "configs", "recipes",
                          "awq_w4a16_g32.yaml" if arch == "qwen3_moe" else "minimax_awq_mixedprec.yaml")
    out = {}
    for fast in (True, False):
        monkeypatch.setattr(me, "FAST_EAGER", fast)
        mm = (_qwen3_moe() if arch == "qwen3_moe" else _minimax()).to(cuda)
        oneshot(mm, recipe, dataset=_calib(vocab=256), max_seq_length=64)
        assert all(me.eager_forward(mod) is None or "forward" not in mod.__dict__ for mod in mm.modules())
        out[fast] = (mm.awq_report, {n: p.detach().clone() for n, p in mm.named_parameters()})
    (rep1, p1), (rep0, p0) = out[True], out[False]
    assert rep1.keys() == rep0.keys()
    for layer in rep1:
        for smooth, r in rep1[layer].items():
            assert r.get("history") == rep0[layer][smooth].get("history"), (layer, smooth)
    for n in p1:
        _eq(p1[n], p0[n], n)


@pytest.mark.parametrize("knob", ["EXPERT_MAJOR", "CONCAT_EXPERT_INPUTS", "OVERLAP_LOSS", "BATCHED_LOSS", "moe_eager.PLANNED", "moe_eager.EXPERT_STREAMS",
                                  "moe_eager.FUSED_COMBINE", "moe_eager.FUSED_ACT", "moe_eager.DIRECT_GEMMS",
                                  "MULTI_LOSS"])
def test_expert_search_knobs_bit_identical(cuda, monkeypatch, knob):
    """The expert-search speed knobs (experts-outer order; one GEMM for the per-expert inputs)
    change nothing: loss histories and smoothed parameters equal with the knob on and off."""
    import quantizers_amd.awq as awq_mod
    import quantizers_amd.moe_eager as moe_mod
    target, name = (moe_mod, knob.split(".", 1)[1]) if knob.startswith("moe_eager.") else (awq_mod, knob)
    values = {"EXPERT_STREAMS": {True: 4, False: 1}, "MULTI_LOSS": {True: 8, False: 1}}.get(
        name, {True: True, False: False})
    out = {}
    for on in (True, False):
        monkeypatch.setattr(target, name, values[on])
        m = _minimax(layers=1, experts=4).to(cuda)
        oneshot(m, os.path.join(ROOT, "configs/recipes/minimax_awq_mixedprec.yaml"), dataset=_calib(vocab=256),
                max_seq_length=64)
        out[on] = (m.awq_report, {n: p.detach().clone() for n, p in m.named_parameters()})
    (r1, p1), (r0, p0) = out[True], out[False]
    assert r1.keys() == r0.keys() and sum(len(v) for v in r1.values()) >= 4
    for layer in r1:
        for smooth, r in r1[layer].items():
            assert r.get("history") == r0[layer][smooth].get("history"), (layer, smooth)
    for n in p1:
        _eq(p1[n], p0[n], n)


@pytest.mark.parametrize("arch", ["qwen3", "qwen3_moe", "minimax"])
def test_batched_layer_calls_bit_identical(cuda, monkeypatch, arch):
    """The calibration and propagation passes run the stacked samples as one layer call (hooks
    split it back per sample): loss histories, smoothed parameters and the checkpoint tensors
    equal the per-sample passes."""
    import quantizers_amd.oneshot as os_mod
    build = {"qwen3": _qwen3, "qwen3_moe": _qwen3_moe, "minimax": _minimax}[arch]
    recipe = os.path.join(ROOT, "configs", "recipes",
                          "minimax_awq_mixedprec.yaml" if arch == "minimax" else "awq_w4a16_g32.yaml")
    out = {}
    for on in (True, False):
        monkeypatch.setattr(os_mod, "BATCH_LAYER_CALLS", on)
        m = build().to(cuda)
        oneshot(m, recipe, dataset=_calib(vocab=256), max_seq_length=64)
        out[on] = (m.awq_report, {n: p.detach().clone() for n, p in m.named_parameters()}, compressed_state_dict(m))
    (r1, p1, s1), (r0, p0, s0) = out[True], out[False]
    assert r1.keys() == r0.keys()
    for layer in r1:
        for smooth, r in r1[layer].items():
            assert r.get("history") == r0[layer][smooth].get("history"), (layer, smooth)
    for n in p1:
        _eq(p1[n], p0[n], n)
    assert s1.keys() == s0.keys()
    for k in s1:
        _eq(s1[k], s0[k], k)


def test_minimax_awq_mixedprec_end_to_end(cuda, tmp_path):
    """recipe_Minimax-M2.1-AWQ-MixedPrec semantics on a tiny random MiniMax-M2: FP8 g32 attention,
    int4 g32 experts, AWQ over attention, all experts' w1/w3 and each expert's w3 -> w2."""
    m = _minimax().to(cuda)
    calib = _calib(vocab=256)
    ids = torch.stack([c["input_ids"] for c in calib]).to(cuda)
    with torch.no_grad():
        ref_logits = m(ids).logits.float()
    oneshot(m, os.path.join(ROOT, "configs/recipes/minimax_awq_mixedprec.yaml"), dataset=calib, max_seq_length=64)
    for layer, maps in m.awq_report.items():
        assert len(maps) == 10, sorted(maps)  # input_ln, post_attn_ln, 8 x w3 (v->o dropped, D9)
        moe = maps[f"{layer}.post_attention_layernorm"]
        assert moe["parent"] == f"{layer}.block_sparse_moe" and len(moe["balance"]) == 16
        for r in maps.values():
            assert 0.0 <= r["best_ratio"] < 1.0 and len(r["history"]) == 20
            assert r["best_loss"] <= r["history"][0]
    with torch.no_grad():
        new_logits = m(ids).logits.float()
    rel = (new_logits - ref_logits).norm() / ref_logits.norm()
    assert rel < 0.06, rel  # smoothing is exact up to bf16 rounding (0.050 with D8's bf16 scales, 0.04 with f32)
    sd = compressed_state_dict(m)
    assert _check_against_oracle(m, sd) == 2 * (4 + 24)
    assert sd["model.layers.1.block_sparse_moe.experts.7.w2.weight_packed"].dtype == torch.int32
    assert sd["model.layers.0.self_attn.q_proj.weight"].dtype == torch.float8_e4m3fn
    assert "model.layers.0.block_sparse_moe.gate.weight" in sd
    assert "model.layers.0.block_sparse_moe.e_score_correction_bias" in sd
    assert not any(".mlp." in k for k in sd)
    out = save_compressed(m, str(tmp_path / "mm"))
    cfg = json.load(open(os.path.join(out, "config.json")))["quantization_config"]
    assert cfg["format"] == "mixed-precision" and cfg["ignore"] == ["lm_head"]


@pytest.mark.parametrize("calibrate_all", [True, False])
def test_expert_w3_w2_awq_matches_oracle(cuda, calibrate_all):
    """One expert's w3 -> w2 mapping: statistics over the expert's w2 inputs (all tokens, or the
    routed ones), w_mean, grid losses and the applied smoothing vs a CPU restatement."""
    import torch.nn.functional as F
    from quantizers_amd.awq import awq_layer
    from quantizers_amd.recipe import AWQMapping
    from quantizers_amd.quantization import QuantizationArgs
    m = _minimax(layers=1, experts=4).to(cuda)
    layer = m.model.layers[0]
    experts = layer.mlp.experts
    a = QuantizationArgs(num_bits=4, type="int", symmetric=True, group_size=32)
    pre = "model.layers.0.block_sparse_moe.experts"
    quantized = {f"{pre}.{e}.{p}": a for e in range(4) for p in ("w1", "w2", "w3")}
    calib = _calib(n=2, s=48, vocab=256)
    from quantizers_amd.oneshot import _capture_layer0_inputs, _batches
    inputs = _capture_layer0_inputs(m, m.model.layers, _batches(calib, None, None, cuda))
    seen = []
    h = experts.register_forward_pre_hook(lambda mod, args: seen.append((args[0].clone(), args[1].clone())))
    with torch.no_grad():
        for args, kw in inputs:
            layer(*args, **kw)
    h.remove()
    gu0, down0 = experts.gate_up_proj.data.clone(), experts.down_proj.data.clone()
    rep = awq_layer(layer, "model.layers.0", inputs, [AWQMapping("re:.*w3$", ["re:.*w2$"])], quantized,
                    mtype="minimax_m2", calibrate_all_experts=calibrate_all, awq_dtype="fp32")
    assert len(rep) == 4
    oa = ct.QArgs(group_size=32)
    for e in range(4):
        with torch.no_grad():
            hs = []
            for x, topk in seen:
                if not calibrate_all:
                    x = x[(topk == e).any(-1)]
                g, u = F.linear(x, gu0[e]).chunk(2, dim=-1)
                hs.append(experts.act_fn(g) * u)
        s_ref, n_ref = None, 0
        for t in hs:
            (s_ref, n_ref) = ct.awq_accumulate_mean(t.cpu(), None if s_ref is None else (s_ref, n_ref))
        x_mean = s_ref / n_ref
        w2 = down0[e].cpu()
        w_mean = ct.awq_layer_means([w2], oa)
        ref_out = [F.linear(t, down0[e]) for t in hs]
        cpu_hist = []
        for i in range(20):
            s = ct.awq_grid_scales(x_mean, w_mean, i / 20, True)
            wq = ct.awq_fake_quant_scaled(w2, s, oa).to(cuda)
            got = [F.linear(t, wq) for t in hs]
            cpu_hist.append(sum((p - q).float().pow(2).sum().item() for p, q in zip(ref_out, got)) /
                            sum(p.numel() for p in ref_out))
        r = rep[f"{pre}.{e}.w3"]
        torch.testing.assert_close(torch.tensor(r["history"]), torch.tensor(cpu_hist), rtol=1e-3, atol=1e-12)
        best = r["best_ratio"]
        assert cpu_hist[int(round(best * 20))] <= min(cpu_hist) * 1.001
        s = ct.awq_grid_scales(x_mean, w_mean, best, True)
        _eq(experts.down_proj.data[e], (w2.float() * s.view(1, -1)).to(torch.bfloat16), f"w2 smoothed {e}")
        up0 = gu0[e, 64:].cpu()
        _eq(experts.gate_up_proj.data[e, 64:], (up0.float() / s.view(-1, 1)).to(torch.bfloat16), f"w3 smoothed {e}")
        _eq(experts.gate_up_proj.data[e, :64], gu0[e, :64], "w1 untouched")


@pytest.mark.parametrize("calibrate_all", [True, False])
def test_expert_w3_w2_awq_bf16_batched_statistics(cuda, calibrate_all):
    """D8 bf16 reading on the expert w3 -> w2 searches, whose statistics are computed for all
    experts of a search at once (segmented absmean over every expert's per-batch token runs, the
    batched bf16 running mean, segmented w_mean): each expert's smoothing equals bf16(w2 * s) with s
    from the per-expert computation (one absmean call per batch, the per-expert running mean, one
    w_mean call), and the 20 losses follow the literal restatement."""
    import torch.nn.functional as F
    from quantizers_amd import awq as awq_mod
    from quantizers_amd.awq import awq_layer
    from quantizers_amd.recipe import AWQMapping
    from quantizers_amd.quantization import QuantizationArgs
    m = _minimax(layers=1, experts=4).to(cuda)
    layer = m.model.layers[0]
    experts = layer.mlp.experts
    a = QuantizationArgs(num_bits=4, type="int", symmetric=True, group_size=32)
    pre = "model.layers.0.block_sparse_moe.experts"
    quantized = {f"{pre}.{e}.{p}": a for e in range(4) for p in ("w1", "w2", "w3")}
    from quantizers_amd.oneshot import _capture_layer0_inputs, _batches
    inputs = _capture_layer0_inputs(m, m.model.layers, _batches(_calib(n=3, s=48, vocab=256), None, None, cuda))
    seen = []
    h = experts.register_forward_pre_hook(lambda mod, args: seen.append((args[0].clone(), args[1].clone())))
    with torch.no_grad():
        for args, kw in inputs:
            layer(*args, **kw)
    h.remove()
    gu0, down0 = experts.gate_up_proj.data.clone(), experts.down_proj.data.clone()
    rep = awq_layer(layer, "model.layers.0", inputs, [AWQMapping("re:.*w3$", ["re:.*w2$"])], quantized,
                    mtype="minimax_m2", calibrate_all_experts=calibrate_all, awq_dtype="bf16")
    oa = ct.QArgs(group_size=32)
    for e in range(4):
        with torch.no_grad():
            hs = []
            for x, topk in seen:
                if not calibrate_all:
                    x = x[(topk == e).any(-1)]
                g, u = F.linear(x, gu0[e]).chunk(2, dim=-1)
                hs.append(experts.act_fn(g) * u)
        am = awq_mod._AbsMean(bf16=True)
        for t in hs:
            am.add(t)
        ws = torch.zeros(down0.shape[2], dtype=torch.float64, device=cuda)
        n = ops.awq_weight_mean_accum(down0[e], 32, ws)
        wm = ws.to(torch.bfloat16) / n
        r = rep[f"{pre}.{e}.w3"]
        s = awq_mod._grid_scales_bf16(am.mean(), wm, r["best_ratio"], True)
        _eq(experts.down_proj.data[e], (down0[e].float() * s.view(1, -1)).to(torch.bfloat16), f"w2 smoothed {e}")
        prev = None
        for t in hs:
            if t.shape[0]:
                prev = ct.awq_accumulate_mean_literal(t.cpu(), prev)
        w2 = down0[e].cpu()
        w_lit = ct.awq_layer_means_literal([w2], oa)
        ref_out = [F.linear(t, down0[e]) for t in hs]
        hist = []
        for i in range(20):
            sl = ct.awq_grid_scales_literal(prev[0], w_lit, i / 20, True)
            wq = ct.awq_fake_quant_scaled_literal(w2, sl, oa).to(cuda)
            got = [F.linear(t, wq) for t in hs]
            hist.append(sum((p - q).float().pow(2).sum().item() for p, q in zip(ref_out, got)) /
                        sum(p.numel() for p in ref_out))
        torch.testing.assert_close(torch.tensor(r["history"]), torch.tensor(hist), rtol=5e-3, atol=1e-12)


@pytest.mark.parametrize("dtype", [torch.float16, torch.float32])
def test_non_bf16_model_rejected_up_front(cuda, dtype):
    """an fp16 / fp32 MoE model under the AWQ recipe.  Every kernel reads bf16 weights
    (the reference loads bf16, do_oneshot.py:88), so oneshot refuses it before any work with a
    ValueError that names the fix, instead of failing inside the expert searches or the save; the
    statistics wrappers refuse non-bf16 weights too (awq_weight_mean_accum used to read them as
    bf16), while activations of another dtype are converted (awq_absmean_accum, add_samples and the
    expert searches' token runs)."""
    m = _minimax(layers=1, experts=4).to(cuda, dtype)
    with pytest.raises(ValueError, match="bfloat16"):
        oneshot(m, os.path.join(ROOT, "configs/recipes/minimax_experts_awq.yaml"), dataset=_calib(vocab=256),
                max_seq_length=64)
    w = torch.randn(64, 256, device=cuda, dtype=dtype)
    with pytest.raises(ValueError, match="bfloat16"):
        ops.awq_weight_mean_accum(w, 32, torch.zeros(256, dtype=torch.float64, device=cuda))
    x = torch.randn(40, 256, device=cuda, dtype=dtype)
    s1, s2 = torch.zeros(256, device=cuda), torch.zeros(256, device=cuda)
    assert ops.awq_absmean_accum(x, s1) == 40 and ops.awq_absmean_accum(x.to(torch.bfloat16), s2) == 40
    assert torch.equal(s1, s2)


def _awq_rank(rank, world, port, out):
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        m = _minimax(experts=8).to("cuda:0")
        oneshot(m, os.path.join(ROOT, "configs/recipes/minimax_experts_awq.yaml"), dataset=_calib(vocab=256),
                max_seq_length=64)
        if rank == 1:
            torch.save({k: v.detach().cpu() for k, v in m.state_dict().items()}, out)
    finally:
        dist.destroy_process_group()


def test_expert_awq_sharded_two_ranks(cuda, tmp_path):
    """Per-expert w3 -> w2 searches sharded over 2 ranks (gloo control plane, one card): the
    smoothed model is bit-identical to the one-process run."""
    import socket
    import torch.multiprocessing as mp
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    out = str(tmp_path / "rank1.pt")
    mp.spawn(_awq_rank, args=(2, port, out), nprocs=2, join=True)
    m = _minimax(experts=8).to(cuda)
    oneshot(m, os.path.join(ROOT, "configs/recipes/minimax_experts_awq.yaml"), dataset=_calib(vocab=256),
            max_seq_length=64)
    two = torch.load(out, weights_only=True)
    for k, v in m.state_dict().items():
        _eq(v, two[k], k)
    assert len(m.awq_report["model.layers.0"]) == 9


def test_moe_norm_to_all_experts_matches_oracle(cuda):
    """post_attention_layernorm -> every expert's w1/w3 (parent = the MoE block): the scales
    applied (from x_mean over the MoE block input and w_mean over all 2E balance slices) and
    the smoothing of the norm and of every expert slice vs a CPU restatement."""
    from quantizers_amd.awq import awq_layer
    from quantizers_amd.recipe import AWQMapping
    from quantizers_amd.quantization import QuantizationArgs
    from quantizers_amd.oneshot import _capture_layer0_inputs, _batches
    m = _minimax(layers=1, experts=4).to(cuda)
    layer = m.model.layers[0]
    experts = layer.mlp.experts
    a = QuantizationArgs(num_bits=4, type="int", symmetric=True, group_size=32)
    pre = "model.layers.0.block_sparse_moe.experts"
    quantized = {f"{pre}.{e}.{p}": a for e in range(4) for p in ("w1", "w2", "w3")}
    inputs = _capture_layer0_inputs(m, m.model.layers, _batches(_calib(n=3, s=40, vocab=256), None, None, cuda))
    seen = []
    h = layer.mlp.register_forward_pre_hook(lambda mod, args: seen.append(args[0].detach().clone()))
    with torch.no_grad():
        for args, kw in inputs:
            layer(*args, **kw)
    h.remove()
    norm0 = layer.post_attention_layernorm.weight.detach().cpu().clone()
    gu0 = experts.gate_up_proj.detach().cpu().clone()
    rep = awq_layer(layer, "model.layers.0", inputs,
                    [AWQMapping("re:.*post_attention_layernorm$", ["re:.*w1$", "re:.*w3$"])], quantized,
                    mtype="minimax_m2", awq_dtype="fp32")
    r = rep["model.layers.0.post_attention_layernorm"]
    assert len(r["balance"]) == 8 and r["parent"] == "model.layers.0.block_sparse_moe"
    s_ref, n_ref = None, 0
    for x in seen:
        (s_ref, n_ref) = ct.awq_accumulate_mean(x.cpu(), None if s_ref is None else (s_ref, n_ref))
    x_mean = s_ref / n_ref
    w_mean = ct.awq_layer_means([gu0[e, :64] for e in range(4)] + [gu0[e, 64:] for e in range(4)],
                                ct.QArgs(group_size=32))
    s = ct.awq_grid_scales(x_mean, w_mean, r["best_ratio"], True)
    _eq(layer.post_attention_layernorm.weight, (norm0.float() / s).to(torch.bfloat16), "norm smoothed")
    _eq(experts.gate_up_proj.data, (gu0.float() * s.view(1, 1, -1)).to(torch.bfloat16), "w1/w3 smoothed")


def test_moe_norm_to_all_experts_bf16(cuda):
    """D8 bf16 reading on the MoE-block mapping (post_attention_layernorm -> every expert's w1/w3):
    w_mean is a bf16 sum over the 2E expert slices in the mapping's balance order; the norm and
    every slice are smoothed with the product's bf16 scale vector (recomputed here from its own
    statistics helpers on a pre-search copy), which is within 1 ulp of the literal restatement's."""
    import copy
    from quantizers_amd import awq as awq_mod
    from quantizers_amd.awq import awq_layer, resolve_mappings
    from quantizers_amd.recipe import AWQMapping
    from quantizers_amd.quantization import QuantizationArgs
    from quantizers_amd.oneshot import _capture_layer0_inputs, _batches
    m = _minimax(layers=1, experts=4).to(cuda)
    layer = m.model.layers[0]
    experts = layer.mlp.experts
    a = QuantizationArgs(num_bits=4, type="int", symmetric=True, group_size=32)
    pre = "model.layers.0.block_sparse_moe.experts"
    quantized = {f"{pre}.{e}.{p}": a for e in range(4) for p in ("w1", "w2", "w3")}
    inputs = _capture_layer0_inputs(m, m.model.layers, _batches(_calib(n=3, s=40, vocab=256), None, None, cuda))
    seen = []
    h = layer.mlp.register_forward_pre_hook(lambda mod, args: seen.append(args[0].detach().clone()))
    with torch.no_grad():
        for args, kw in inputs:
            layer(*args, **kw)
    h.remove()
    layer0 = copy.deepcopy(layer)
    norm0 = layer.post_attention_layernorm.weight.detach().cpu().clone()
    gu0 = experts.gate_up_proj.detach().cpu().clone()
    mp = [AWQMapping("re:.*post_attention_layernorm$", ["re:.*w1$", "re:.*w3$"])]
    rep = awq_layer(layer, "model.layers.0", inputs, mp, quantized, mtype="minimax_m2", awq_dtype="bf16")
    r = rep["model.layers.0.post_attention_layernorm"]
    (r0,) = resolve_mappings(layer0, "model.layers.0", mp, quantized, "minimax_m2")
    assert r0.balance_names == r["balance"]
    am = awq_mod._AbsMean(bf16=True)
    for x in seen:
        am.add(x)
    wm = awq_mod._w_mean(None, quantized, gu0.shape[-1], True, cuda, r0.balance)
    s = awq_mod._grid_scales_bf16(am.mean(), wm, r["best_ratio"], True).cpu()
    prev = None
    for x in seen:
        prev = ct.awq_accumulate_mean_literal(x.cpu(), prev)
    w_lit = ct.awq_layer_means_literal([gu0[e, :64] for e in range(4)] + [gu0[e, 64:] for e in range(4)],
                                       ct.QArgs(group_size=32))
    s_lit = ct.awq_grid_scales_literal(prev[0], w_lit, r["best_ratio"], True)
    d = (s.to(torch.bfloat16).view(torch.int16).int() - s_lit.view(torch.int16).int()).abs()
    assert d.max() <= 1 and (d > 0).float().mean() < 0.05, (int(d.max()), float((d > 0).float().mean()))
    _eq(layer.post_attention_layernorm.weight, (norm0.float() / s).to(torch.bfloat16), "norm smoothed")
    _eq(experts.gate_up_proj.data, (gu0.float() * s.view(1, 1, -1)).to(torch.bfloat16), "w1/w3 smoothed")


def _awq_rank_dense(rank, world, port, out):
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        m = _qwen3().to("cuda:0")
        oneshot(m, os.path.join(ROOT, "configs/recipes/awq_w4a16_g32.yaml"), dataset=_calib(), max_seq_length=64)
        if rank == world - 1:
            torch.save({k: v.detach().cpu() for k, v in m.state_dict().items()}, out)
    finally:
        dist.destroy_process_group()


def test_dense_awq_grid_split_three_ranks(cuda, tmp_path):
    """Dense AWQ with the 20 grid ratios split over 3 ranks (gloo control plane, one card):
    bit-identical smoothed model to the one-process run."""
    import socket
    import torch.multiprocessing as mp
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    out = str(tmp_path / "rank2.pt")
    mp.spawn(_awq_rank_dense, args=(3, port, out), nprocs=3, join=True)
    m = _qwen3().to(cuda)
    oneshot(m, os.path.join(ROOT, "configs/recipes/awq_w4a16_g32.yaml"), dataset=_calib(), max_seq_length=64)
    other = torch.load(out, weights_only=True)
    for k, v in m.state_dict().items():
        _eq(v, other[k], k)


@pytest.mark.parametrize("arch", ["qwen3", "qwen3_moe", "minimax"])
def test_concurrent_sample_calls_bit_identical(cuda, monkeypatch, arch):
    """QZ_CALIB_THREADS: the per-sample calibration and propagation calls on 3 host threads /
    streams (the hooks file their observations per sample and combine them in sample order)
    give the loss histories and smoothed parameters of the sequential calls, bit for bit."""
    import quantizers_amd.awq as awq_mod
    import quantizers_amd.oneshot as os_mod
    build = {"qwen3": _qwen3, "qwen3_moe": _qwen3_moe, "minimax": _minimax}[arch]
    recipe = os.path.join(ROOT, "configs", "recipes",
                          {"qwen3": "awq_w4a16_g32.yaml", "qwen3_moe": "awq_w4a16_g32.yaml",
                           "minimax": "minimax_awq_mixedprec.yaml"}[arch])
    monkeypatch.setattr(os_mod, "BATCH_LAYER_CALLS", False)  # the per-sample path is what runs threaded
    out = {}
    for threads in (1, 3):
        monkeypatch.setattr(awq_mod, "CALIB_THREADS", threads)
        m = build().to(cuda)
        oneshot(m, recipe, dataset=_calib(n=5, vocab=256), max_seq_length=64)
        out[threads] = (m.awq_report, {n: p.detach().clone() for n, p in m.named_parameters()})
    (r1, p1), (r3, p3) = out[1], out[3]
    assert r1.keys() == r3.keys()
    for layer in r1:
        for smooth, r in r1[layer].items():
            assert r.get("history") == r3[layer][smooth].get("history"), (layer, smooth)
    for n in p1:
        _eq(p1[n], p3[n], n)


@pytest.mark.parametrize("arch", ["qwen3_moe", "minimax"])
def test_grid_graph_replay_bit_identical(cuda, monkeypatch, arch):
    """QZ_GRID_GRAPHS: the fixed-routing MoE-block grids replay their forward from one HIP graph
    (checked against the eager forward on first use); the loss histories and smoothed
    parameters equal the eager-forward run's bit for bit, and the replay path was the one taken."""
    import quantizers_amd.awq as awq_mod
    build = _qwen3_moe if arch == "qwen3_moe" else _minimax
    recipe = os.path.join(ROOT, "configs", "recipes",
                          "awq_w4a16_g32.yaml" if arch == "qwen3_moe" else "minimax_awq_mixedprec.yaml")
    states = []
    close = awq_mod._GraphedForward.close

    def spy(self):
        states.append(self.state)
        close(self)
    monkeypatch.setattr(awq_mod._GraphedForward, "close", spy)
    out = {}
    for on in (False, True):
        monkeypatch.setattr(awq_mod, "GRID_GRAPHS", on)
        m = build().to(cuda)
        oneshot(m, recipe, dataset=_calib(n=5, vocab=256), max_seq_length=64)
        out[on] = (m.awq_report, {n: p.detach().clone() for n, p in m.named_parameters()})
    assert states and all(s is True for s in states), states
    (r0, p0), (r1, p1) = out[False], out[True]
    assert r0.keys() == r1.keys()
    for layer in r0:
        for smooth, r in r0[layer].items():
            assert r.get("history") == r1[layer][smooth].get("history"), (layer, smooth)
    for n in p0:
        _eq(p0[n], p1[n], n)
