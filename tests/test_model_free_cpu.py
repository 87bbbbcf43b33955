"""model_free_ptq host logic on CPU (no kernels): target selection, shard discovery, refusal of a
CPU device (no CPU fallback)."""
import json
import os

import pytest
import torch
from safetensors.torch import save_file

from quantizers_amd.model_free import _shard_files, is_target, model_free_ptq


def test_is_target():
    ig = ["lm_head", "re:.*mlp\\.gate$", "model.embed_tokens"]
    assert is_target("model.layers.0.self_attn.q_proj.weight", (8, 8), torch.bfloat16, ig)
    assert not is_target("model.layers.0.mlp.gate.weight", (8, 8), torch.bfloat16, ig)
    assert not is_target("model.embed_tokens.weight", (8, 8), torch.bfloat16, ig)
    assert not is_target("model.norm.weight", (8,), torch.bfloat16, ig)
    assert not is_target("x.weight_scale", (8, 8), torch.bfloat16, ig)
    assert not is_target("x.weight", (8, 8), torch.float8_e4m3fn, ig)


def test_shard_files(tmp_path):
    save_file({"a": torch.zeros(2)}, str(tmp_path / "m-1.safetensors"))
    save_file({"b": torch.zeros(2)}, str(tmp_path / "m-2.safetensors"))
    assert _shard_files(str(tmp_path)) == ["m-1.safetensors", "m-2.safetensors"]
    json.dump({"weight_map": {"a": "m-1.safetensors"}}, open(tmp_path / "model.safetensors.index.json", "w"))
    assert _shard_files(str(tmp_path)) == ["m-1.safetensors"]


def test_refuses_cpu(tmp_path):
    save_file({"a.weight": torch.zeros(8, 128, dtype=torch.bfloat16)}, str(tmp_path / "model.safetensors"))
    with pytest.raises(ValueError, match="no CPU fallback"):
        model_free_ptq(str(tmp_path), str(tmp_path / "out"), "W4A16", device="cpu")
