"""The streaming safetensors shard writer of save_compressed (CPU): shards in the order tensors
are added, at most max_shard_bytes each (a larger tensor alone), renamed model-XXXXX-of-NNNNN
+ index at close (or model.safetensors for one shard), no temporary file left."""
import json
import os

import torch
from safetensors.torch import load_file

from quantizers_amd.compressor import _ShardWriter


def _tensors():
    g = torch.Generator().manual_seed(0)
    return [(f"m.{i}.weight_packed", torch.randint(-100, 100, (16, 8 + i), dtype=torch.int32, generator=g))
            for i in range(10)] + [("m.big", torch.randn(64, 64, generator=g).to(torch.bfloat16))]


def test_multi_shard(tmp_path):
    items = _tensors()
    w = _ShardWriter(str(tmp_path), max_shard_bytes=1200)
    w.add(items[:4])
    w.add(items[4:])
    n, total = w.close()
    assert n == len(items) and total == sum(t.numel() * t.element_size() for _, t in items)
    files = sorted(os.listdir(tmp_path))
    shards = [f for f in files if f.endswith(".safetensors")]
    assert len(shards) > 2 and not any(f.endswith(".tmp") for f in files)
    idx = json.load(open(tmp_path / "model.safetensors.index.json"))
    assert idx["metadata"]["total_size"] == total
    got, order = {}, []
    for f in shards:
        assert f.endswith(f"-of-{len(shards):05d}.safetensors")
        part = load_file(str(tmp_path / f))
        assert sum(t.numel() * t.element_size() for t in part.values()) <= 1200 or len(part) == 1
        for k in part:
            assert idx["weight_map"][k] == f
        got.update(part)
        order.append(sorted(part))
    for name, t in items:
        assert torch.equal(got[name], t)
    # shards follow the order tensors were added
    first = [min(items.index(next(it for it in items if it[0] == k)) for k in names) for names in order]
    assert first == sorted(first)


def test_single_shard(tmp_path):
    items = _tensors()
    w = _ShardWriter(str(tmp_path), max_shard_bytes=1 << 30)
    w.add(items)
    w.close()
    assert sorted(os.listdir(tmp_path)) == ["model.safetensors"]
    got = load_file(str(tmp_path / "model.safetensors"))
    assert all(torch.equal(got[k], t) for k, t in items)
