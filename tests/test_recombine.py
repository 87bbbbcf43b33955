"""MiniMax-style recombine (FP8 source + compressed experts -> mixed-precision), CPU only:
tensor routing, renames, config (scripts/recombine_weights_MiniMax-M2.1.py semantics)."""
import json
import os

import torch
from safetensors.torch import load_file, save_file

import ct_torch as ct
from quantizers_amd.recombine import recombine


def _fp8_ckpt(d):
    g = torch.Generator().manual_seed(0)
    os.makedirs(d)
    L = "model.layers.0"
    f1 = {f"{L}.self_attn.q_proj.weight": torch.randn(256, 128, generator=g).to(torch.float8_e4m3fn),
          f"{L}.self_attn.q_proj.weight_scale_inv": torch.rand(2, 1, generator=g),
          f"{L}.input_layernorm.weight": torch.ones(128, dtype=torch.bfloat16),
          f"{L}.post_attention_layernorm.weight": torch.ones(128, dtype=torch.bfloat16),
          f"{L}.block_sparse_moe.gate.weight": torch.randn(2, 128, generator=g).to(torch.bfloat16)}
    f2 = {}
    for e in range(2):
        for w, shp in (("w1", (64, 128)), ("w3", (64, 128)), ("w2", (128, 64))):
            f2[f"{L}.block_sparse_moe.experts.{e}.{w}.weight"] = torch.randn(*shp, generator=g).to(torch.float8_e4m3fn)
            f2[f"{L}.block_sparse_moe.experts.{e}.{w}.weight_scale_inv"] = torch.rand(1, 1, generator=g)
    save_file(f1, os.path.join(d, "model-00001-of-00002.safetensors"))
    save_file(f2, os.path.join(d, "model-00002-of-00002.safetensors"))
    wm = {k: "model-00001-of-00002.safetensors" for k in f1} | {k: "model-00002-of-00002.safetensors" for k in f2}
    json.dump({"weight_map": wm}, open(os.path.join(d, "model.safetensors.index.json"), "w"))
    json.dump({"model_type": "minimax_m2", "quantization_config": {"quant_method": "fp8"}},
              open(os.path.join(d, "config.json"), "w"))
    (open(os.path.join(d, "tokenizer.json"), "w")).write("{}")
    return f1, f2


def _compressed_ckpt(d):
    g = torch.Generator().manual_seed(1)
    os.makedirs(d)
    L = "model.layers.0"
    sd = {f"{L}.post_attention_layernorm.weight": (torch.rand(128, generator=g) + 0.5).to(torch.bfloat16),
          f"{L}.input_layernorm.weight": torch.full((128,), 3.0, dtype=torch.bfloat16)}
    a = ct.QArgs(num_bits=4, group_size=32)
    for e in range(2):
        for w, shp in (("w1", (64, 128)), ("w3", (64, 128)), ("w2", (128, 64))):
            wt = (torch.randn(*shp, generator=g) * 0.02).to(torch.bfloat16)
            for k, v in ct.compress_weight(wt, a).items():
                sd[f"{L}.block_sparse_moe.experts.{e}.{w}.{k}"] = v
    save_file(sd, os.path.join(d, "model.safetensors"))
    json.dump({"quantization_config": {"config_groups": {"group_0": {
        "targets": ["re:.*block_sparse_moe\\.experts\\.\\d+\\.(w1|w2|w3)$"],
        "weights": {"num_bits": 4, "type": "int", "group_size": 32, "strategy": "group", "symmetric": True},
        "format": "pack-quantized"}}, "ignore": ["lm_head"]}}, open(os.path.join(d, "config.json"), "w"))
    return sd


def test_recombine(tmp_path):
    f1, f2 = _fp8_ckpt(str(tmp_path / "fp8"))
    comp = _compressed_ckpt(str(tmp_path / "comp"))
    st = recombine(str(tmp_path / "fp8"), str(tmp_path / "comp"), str(tmp_path / "out"))
    assert (st.experts_replaced, st.smoothing_replaced, st.scale_inv_renamed, st.scale_inv_dropped) == (6, 1, 1, 6)
    out = {}
    for fn in ("model-00001-of-00002.safetensors", "model-00002-of-00002.safetensors"):
        out.update(load_file(str(tmp_path / "out" / fn)))
    L = "model.layers.0"
    assert torch.equal(out[f"{L}.self_attn.q_proj.weight"].view(torch.uint8), f1[f"{L}.self_attn.q_proj.weight"].view(torch.uint8))
    assert torch.equal(out[f"{L}.self_attn.q_proj.weight_scale"], f1[f"{L}.self_attn.q_proj.weight_scale_inv"])
    assert not any(k.endswith("_scale_inv") for k in out)
    assert torch.equal(out[f"{L}.post_attention_layernorm.weight"], comp[f"{L}.post_attention_layernorm.weight"])
    assert torch.equal(out[f"{L}.input_layernorm.weight"], f1[f"{L}.input_layernorm.weight"])  # FP8 side kept
    for e in range(2):
        for w in ("w1", "w2", "w3"):
            b = f"{L}.block_sparse_moe.experts.{e}.{w}"
            assert f"{b}.weight" not in out
            for s in ("weight_packed", "weight_scale", "weight_shape"):
                assert torch.equal(out[f"{b}.{s}"], comp[f"{b}.{s}"])
    idx = json.load(open(tmp_path / "out" / "model.safetensors.index.json"))
    assert set(idx["weight_map"]) == set(out)
    cfg = json.load(open(tmp_path / "out" / "config.json"))
    qc = cfg["quantization_config"]
    assert cfg["model_type"] == "minimax_m2" and qc["format"] == "mixed-precision" and qc["ignore"] == ["lm_head"]
    assert qc["config_groups"]["group_0"]["weights"]["block_structure"] == [128, 128]
    assert qc["config_groups"]["group_1"]["targets"][0] == "Linear"
    assert (tmp_path / "out" / "tokenizer.json").exists()


def test_recombine_dry_run(tmp_path):
    _fp8_ckpt(str(tmp_path / "fp8"))
    _compressed_ckpt(str(tmp_path / "comp"))
    st = recombine(str(tmp_path / "fp8"), str(tmp_path / "comp"), str(tmp_path / "out"), dry_run=True)
    assert st.experts_replaced == 6 and not (tmp_path / "out").exists()


def test_output_shard_names_follow_reference(tmp_path):
    """recombine_weights_MiniMax-M2.1.py:68-72: MiniMax-M2.1's ``-of-00130`` FP8 shards are
    written as ``-of-00125``; the index points at the renamed files; other names are kept."""
    from quantizers_amd.recombine import output_file_name
    assert output_file_name("model-00007-of-00130.safetensors") == "model-00007-of-00125.safetensors"
    assert output_file_name("model-00001-of-00002.safetensors") == "model-00001-of-00002.safetensors"
    src = tmp_path / "fp8"
    _fp8_ckpt(str(src))
    idx = json.load(open(src / "model.safetensors.index.json"))
    for old in ("model-00001-of-00002.safetensors", "model-00002-of-00002.safetensors"):
        os.rename(src / old, src / old.replace("of-00002", "of-00130"))
    idx["weight_map"] = {k: v.replace("of-00002", "of-00130") for k, v in idx["weight_map"].items()}
    json.dump(idx, open(src / "model.safetensors.index.json", "w"))
    comp = tmp_path / "comp"
    _compressed_ckpt(str(comp))
    recombine(str(src), str(comp), str(tmp_path / "out"))
    files = sorted(f for f in os.listdir(tmp_path / "out") if f.endswith(".safetensors"))
    assert files == ["model-00001-of-00125.safetensors", "model-00002-of-00125.safetensors"]
    out_idx = json.load(open(tmp_path / "out" / "model.safetensors.index.json"))
    assert set(out_idx["weight_map"].values()) == set(files)

