"""The do_oneshot CLI end to end (random-init tiny Qwen3, synthetic calibration) on the GPU."""
import json
import os

import pytest

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_do_oneshot_cli(cuda, tmp_path, monkeypatch):
    from transformers import Qwen3Config
    cfg = Qwen3Config(hidden_size=256, intermediate_size=512, num_hidden_layers=2, num_attention_heads=4,
                      num_key_value_heads=2, head_dim=64, vocab_size=512)
    cdir = tmp_path / "model_cfg"
    cfg.save_pretrained(cdir)
    run = tmp_path / "run.yaml"
    recipe = os.path.join(ROOT, "configs", "recipes", "awq_w4a16_g128.yaml")
    run.write_text(f"model: {{name: 'Qwen/Qwen3-4B'}}\nquantization: {{recipe: '{recipe}'}}\n")
    monkeypatch.chdir(tmp_path)
    from quantizers_amd.cli import main
    out = main(["--config", str(run), "--random-init", str(cdir), "--calib-random", "4,64",
                "--output", str(tmp_path / "out")])
    qc = json.load(open(os.path.join(out, "config.json")))["quantization_config"]
    assert qc["format"] == "pack-quantized" and qc["config_groups"]["group_0"]["weights"]["group_size"] == 128
    assert os.path.exists(os.path.join(out, "model.safetensors"))
