"""Multi-rank product path on one card: ``oneshot`` (AWQ) + ``save_compressed`` under
torch.distributed (2 ranks, gloo control plane sharing cuda:0) -- each rank compressing and
writing its own shards of the save plan (``compressor.save_plan``), rank 0 adding the index and
config -- produces a checkpoint byte-identical to the one-process run, with one shard or with
several (both ranks writing)."""
import filecmp
import os
import socket

import pytest
import torch

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
RECIPE = os.path.join(ROOT, "configs", "recipes", "awq_w4a16_g32.yaml")


def _model_and_data():
    from test_oneshot_gpu import _calib, _qwen3
    return _qwen3(layers=2), _calib()


SHARD = 200 << 10  # the 2-layer model (about 1.3 MB of tensors) in several shards


def _rank(rank, world, port, out_dir):
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    torch.cuda.set_device(0)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from quantizers_amd.compressor import save_compressed
        from quantizers_amd.oneshot import oneshot
        m, data = _model_and_data()
        m = m.to("cuda:0")
        oneshot(m, RECIPE, dataset=data, max_seq_length=64)
        save_compressed(m, out_dir)
        save_compressed(m, out_dir + "_sharded", max_shard_bytes=SHARD)
    finally:
        dist.destroy_process_group()


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def test_save_compressed_two_ranks_byte_identical(cuda, tmp_path):
    import torch.multiprocessing as mp
    from quantizers_amd.compressor import save_compressed
    from quantizers_amd.oneshot import oneshot
    multi = str(tmp_path / "two_ranks")
    mp.spawn(_rank, args=(2, _port(), multi), nprocs=2, join=True)
    m, data = _model_and_data()
    m = m.to(cuda)
    oneshot(m, RECIPE, dataset=data, max_seq_length=64)
    one = save_compressed(m, str(tmp_path / "one_process"))
    for fn in ("model.safetensors", "config.json", "recipe.yaml"):
        assert filecmp.cmp(os.path.join(one, fn), os.path.join(multi, fn), shallow=False), fn
    one = save_compressed(m, str(tmp_path / "one_process_sharded"), max_shard_bytes=SHARD)
    files = sorted(os.listdir(one))
    assert files == sorted(os.listdir(multi + "_sharded")) and "model.safetensors.index.json" in files
    assert len([f for f in files if f.endswith(".safetensors")]) >= 2
    for fn in files:
        assert filecmp.cmp(os.path.join(one, fn), os.path.join(multi + "_sharded", fn), shallow=False), fn


def _rank_skeleton(rank, world, port, out_dir):
    """Rank 0 holds the model on the host (layer-by-layer onload), rank 1 a meta skeleton:
    every decoder layer reaches rank 1 by broadcast, rank 1 keeps only its shards' tensors."""
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    torch.cuda.set_device(0)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from transformers import AutoModelForCausalLM
        from quantizers_amd.compressor import save_compressed
        from quantizers_amd.oneshot import oneshot
        m, data = _model_and_data()
        if rank != 0:
            with torch.device("meta"):
                m = AutoModelForCausalLM.from_config(m.config, dtype=torch.bfloat16)
        oneshot(m, RECIPE, dataset=data, max_seq_length=64, device="cuda:0", device_resident=False,
                max_shard_bytes=SHARD)
        if rank != 0:
            n_meta = sum(p.is_meta for p in m.parameters())
            assert 0 < n_meta < len(list(m.parameters())), n_meta
        save_compressed(m, out_dir, max_shard_bytes=SHARD)
    finally:
        dist.destroy_process_group()


def test_skeleton_rank_save_byte_identical(cuda, tmp_path):
    """One host copy of the model for two ranks (residency.Residency): the checkpoint equals the
    one-process run's, byte for byte."""
    import torch.multiprocessing as mp
    from quantizers_amd.compressor import save_compressed
    from quantizers_amd.oneshot import oneshot
    multi = str(tmp_path / "skeleton")
    mp.spawn(_rank_skeleton, args=(2, _port(), multi), nprocs=2, join=True)
    m, data = _model_and_data()
    m = m.to(cuda)
    oneshot(m, RECIPE, dataset=data, max_seq_length=64)
    one = save_compressed(m, str(tmp_path / "one"), max_shard_bytes=SHARD)
    files = sorted(os.listdir(one))
    assert files == sorted(os.listdir(multi)) and len([f for f in files if f.endswith(".safetensors")]) >= 2
    for fn in files:
        assert filecmp.cmp(os.path.join(one, fn), os.path.join(multi, fn), shallow=False), fn


def test_materialise_outside_keeps_ties(cuda):
    """rank 0's host-resident non-layer tensors moved to the device keep their ties --
    tie_word_embeddings' lm_head.weight stays the very Parameter embed_tokens holds, so the
    broadcast sends it once and the checkpoint gets no untied copy."""
    from transformers import AutoModelForCausalLM, Qwen3Config
    from quantizers_amd import residency
    cfg = Qwen3Config(hidden_size=128, intermediate_size=256, num_hidden_layers=1, num_attention_heads=2,
                      num_key_value_heads=1, head_dim=64, vocab_size=256, tie_word_embeddings=True)
    m = AutoModelForCausalLM.from_config(cfg, dtype=torch.bfloat16)  # host-resident, as rank 0's RTN model
    assert m.lm_head.weight is m.model.embed_tokens.weight
    res = residency.Residency(m, cuda, 1 << 30)
    res.materialise_outside(m, m.model.layers)
    assert m.model.embed_tokens.weight.is_cuda
    assert m.lm_head.weight is m.model.embed_tokens.weight
    ss = residency.slots(m, exclude=m.model.layers)
    alias = residency._alias_groups(ss)
    assert sum(1 for i, a in enumerate(alias) if a != i) == 1  # one tied slot, sent once
