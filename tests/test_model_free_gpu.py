"""Data-free checkpoint quantization (model_free_ptq, scripts/quant_GLM-4.7-Flash-FP8.py:11-24)
on the GPU, every output tensor checked bit-exact against the CPU oracle."""
import json
import os

import pytest
import torch
from safetensors.torch import load_file, save_file

import ct_torch as ct
from quantizers_amd.compressor import load_decompressed
from quantizers_amd.model_free import model_free_ptq
from quantizers_amd.quantization import preset_scheme

pytestmark = pytest.mark.gpu


def _oa(a):
    sd = {None: None, "float8_e4m3fn": "fp8", "uint8": "e8m0"}[a.scale_dtype]
    return ct.QArgs(num_bits=a.num_bits, type=a.type, symmetric=a.symmetric, strategy=a.strategy,
                    group_size=a.group_size, block_structure=tuple(a.block_structure) if a.block_structure else None,
                    scale_dtype=sd)


def _eq(a, b, key):
    a, b = a.cpu(), b.cpu()
    assert a.shape == b.shape and a.dtype == b.dtype, (key, a.shape, b.shape, a.dtype, b.dtype)
    if a.dtype in (torch.bfloat16, torch.float8_e4m3fn):
        a, b = a.view(torch.uint8), b.view(torch.uint8)
    assert torch.equal(a, b), key


def _load_dir(d):
    sd = {}
    for f in sorted(os.listdir(d)):
        if f.endswith(".safetensors"):
            sd.update(load_file(os.path.join(d, f)))
    return sd


@pytest.mark.parametrize("scheme", ["FP8_BLOCK", "W4A16", "MXFP4A16"])
def test_model_free_qwen3_sharded(cuda, tmp_path, scheme):
    from transformers import AutoModelForCausalLM, Qwen3Config
    cfg = Qwen3Config(hidden_size=256, intermediate_size=512, num_hidden_layers=2, num_attention_heads=4,
                      num_key_value_heads=2, head_dim=64, vocab_size=512, tie_word_embeddings=False)
    torch.manual_seed(0)
    m = AutoModelForCausalLM.from_config(cfg, dtype=torch.bfloat16)
    src, dst = tmp_path / "src", tmp_path / "dst"
    m.save_pretrained(str(src), max_shard_size="400KB")
    (src / "tokenizer_config.json").write_text("{}")
    files = [f for f in os.listdir(src) if f.endswith(".safetensors")]
    assert len(files) > 1
    ignore = ["lm_head", "model.embed_tokens"]
    model_free_ptq(str(src), str(dst), scheme=scheme, ignore=ignore, max_workers=2, device=cuda)
    orig = _load_dir(src)
    got = _load_dir(dst)
    a = preset_scheme(scheme, ["Linear"]).weights
    n = 0
    for k, t in orig.items():
        mod = k[:-len(".weight")]
        if k.endswith(".weight") and t.dim() == 2 and mod not in ignore:
            for kk, v in ct.compress_weight(t, _oa(a)).items():
                _eq(got[f"{mod}.{kk}"], v, f"{mod}.{kk}")
            n += 1
        else:
            _eq(got[k], t, k)
    assert n == 14
    idx = json.load(open(dst / "model.safetensors.index.json"))
    assert set(idx["weight_map"]) == set(got) and set(idx["weight_map"].values()) == set(files)
    qc = json.load(open(dst / "config.json"))["quantization_config"]
    assert qc["quant_method"] == "compressed-tensors" and qc["ignore"] == ["lm_head", "model.embed_tokens"]
    assert (dst / "tokenizer_config.json").exists()
    dec = load_decompressed(str(dst))
    assert dec["model.layers.1.mlp.down_proj.weight"].shape == (256, 512)


def test_model_free_skips_nondivisible(cuda, tmp_path):
    g = torch.Generator().manual_seed(0)
    src, dst = tmp_path / "src", tmp_path / "dst"
    os.makedirs(src)
    t = {"a.weight": (torch.randn(64, 256, generator=g) * 0.02).to(torch.bfloat16),
         "b.weight": (torch.randn(64, 200, generator=g) * 0.02).to(torch.bfloat16),
         "norm.weight": torch.ones(256, dtype=torch.bfloat16),
         "emb.weight": torch.randn(32, 256, generator=g).to(torch.bfloat16)}
    save_file(t, str(src / "model.safetensors"))
    model_free_ptq(str(src), str(dst), scheme="W4A16", ignore=["emb"], device=cuda)
    got = load_file(str(dst / "model.safetensors"))
    assert "a.weight_packed" in got and "b.weight" in got and "b.weight_packed" not in got
    _eq(got["emb.weight"], t["emb.weight"], "emb")
    qc = json.load(open(dst / "config.json"))["quantization_config"]
    assert qc["ignore"] == ["b", "emb"]
    want = ct.compress_weight(t["a.weight"], ct.QArgs(num_bits=4, group_size=128))
    for k, v in want.items():
        _eq(got[f"a.{k}"], v, k)


def _rank_main(rank, world, port, src, dst):
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        model_free_ptq(src, dst, scheme="W4A16", ignore=["lm_head", "model.embed_tokens"], device="cuda:0")
    finally:
        dist.destroy_process_group()


def test_model_free_two_ranks(cuda, tmp_path):
    """Two processes (gloo control plane, one card): files split by size across ranks, each rank
    writes its own shards, rank 0 writes index + config; identical to the one-process output."""
    import socket
    import torch.multiprocessing as mp
    from transformers import AutoModelForCausalLM, Qwen3Config
    cfg = Qwen3Config(hidden_size=256, intermediate_size=512, num_hidden_layers=2, num_attention_heads=4,
                      num_key_value_heads=2, head_dim=64, vocab_size=512, tie_word_embeddings=False)
    torch.manual_seed(1)
    src = tmp_path / "src"
    AutoModelForCausalLM.from_config(cfg, dtype=torch.bfloat16).save_pretrained(str(src), max_shard_size="400KB")
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    mp.spawn(_rank_main, args=(2, port, str(src), str(tmp_path / "two")), nprocs=2, join=True)
    model_free_ptq(str(src), str(tmp_path / "one"), scheme="W4A16", ignore=["lm_head", "model.embed_tokens"],
                   device=cuda)
    one, two = _load_dir(tmp_path / "one"), _load_dir(tmp_path / "two")
    assert set(one) == set(two)
    for k in one:
        _eq(two[k], one[k], k)
    for f in ("config.json", "model.safetensors.index.json"):
        assert json.load(open(tmp_path / "one" / f)) == json.load(open(tmp_path / "two" / f))


def test_model_free_torn_shard_raises_and_closes(cuda, tmp_path):
    """A shard shorter than its header says (a torn download) stops the call with the short read,
    and every input file is closed afterwards -- the failing one and those queued ahead of it."""
    g = torch.Generator().manual_seed(2)
    src = tmp_path / "src"
    os.makedirs(src)
    names = [f"model-{i + 1:05d}-of-00004.safetensors" for i in range(4)]
    wmap = {}
    for i, fn in enumerate(names):
        save_file({f"l{i}.{p}.weight": (torch.randn(128, 256, generator=g) * 0.02).to(torch.bfloat16)
                   for p in ("q", "k")}, str(src / fn))
        wmap.update({f"l{i}.{p}.weight": fn for p in ("q", "k")})
    (src / "model.safetensors.index.json").write_text(json.dumps({"metadata": {}, "weight_map": wmap}))
    os.truncate(src / names[0], os.path.getsize(src / names[0]) - 4096)
    with pytest.raises(IOError, match="short read"):
        model_free_ptq(str(src), str(tmp_path / "dst"), scheme="W4A16", max_workers=4, device=cuda)
    assert _open_under(src) == []


def _open_under(d):
    """This process's open file descriptors on files under directory ``d``."""
    out = []
    for fd in os.listdir("/proc/self/fd"):
        try:
            t = os.readlink(f"/proc/self/fd/{fd}")
        except OSError:
            continue
        if t.startswith(str(d) + os.sep):
            out.append(t)
    return out
