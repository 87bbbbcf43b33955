"""The do_oneshot CLI end to end (random-init tiny Qwen3, synthetic calibration) on the GPU."""
import json
import os

import pytest
import torch

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


def _cli_rank(rank, world, port, argv, cwd):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), WORLD_SIZE=str(world), RANK=str(rank),
                      LOCAL_RANK=str(rank), QZ_DIST_BACKEND="gloo")
    os.chdir(cwd)
    from quantizers_amd.cli import main
    main(argv)


def test_do_oneshot_cli_two_ranks(cuda, tmp_path, monkeypatch):
    """The CLI under a 2-rank launch (torchrun's env; gloo with both ranks on one card): it joins
    the process group, splits the AWQ work, shards the compression, rank 0 alone writes -- and
    the checkpoint is byte-identical to the one-process CLI run."""
    import socket
    import torch.multiprocessing as mp
    from safetensors.torch import load_file
    from transformers import Qwen3Config
    cfg = Qwen3Config(hidden_size=256, intermediate_size=512, num_hidden_layers=2, num_attention_heads=4,
                      num_key_value_heads=2, head_dim=64, vocab_size=512)
    cdir = tmp_path / "model_cfg"
    cfg.save_pretrained(cdir)
    run = tmp_path / "run.yaml"
    recipe = os.path.join(ROOT, "configs", "recipes", "awq_w4a16_g128.yaml")
    run.write_text(f"model: {{name: 'Qwen/Qwen3-4B'}}\nquantization: {{recipe: '{recipe}'}}\n")
    base = ["--config", str(run), "--random-init", str(cdir), "--calib-random", "4,64"]
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    mp.spawn(_cli_rank, args=(2, port, base + ["--output", str(tmp_path / "two")], str(tmp_path)), nprocs=2,
             join=True)
    monkeypatch.chdir(tmp_path)
    from quantizers_amd.cli import main
    main(base + ["--output", str(tmp_path / "one")])
    a, b = load_file(str(tmp_path / "one" / "model.safetensors")), load_file(str(tmp_path / "two" / "model.safetensors"))
    assert a.keys() == b.keys()
    for k in a:
        assert a[k].dtype == b[k].dtype and a[k].shape == b[k].shape, k
        assert a[k].view(-1).view(torch.uint8).equal(b[k].view(-1).view(torch.uint8)), k
    assert json.load(open(tmp_path / "one" / "config.json")) == json.load(open(tmp_path / "two" / "config.json"))

