"""Owner-keeps residency (CPU, gloo world 2): rank 0 holds the model, rank 1 a meta skeleton;
the non-layer tensors and each decoder layer are broadcast, rank 1 keeps only the tensors of its
own checkpoint shards, and the per-rank save is byte-identical to one process's.  The compress
step is the CPU oracle stand-in of test_distributed_cpu (test infrastructure); on GPUs the same
logic drives the HIP kernels (tests/test_multirank_save_gpu.py)."""
import filecmp
import os
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp
from torch import nn

SHARD = 6000


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _model(meta=False, tied=False):
    from quantizers_amd.quantization import QuantizationArgs, QuantizationScheme
    torch.manual_seed(0)
    ctx = torch.device("meta") if meta else torch.device("cpu")
    with ctx:
        m = nn.Module()
        m.model = nn.Module()
        m.model.embed = nn.Embedding(50, 64)
        m.model.layers = nn.ModuleList()
        for _ in range(3):
            blk = nn.Module()
            blk.q_proj = nn.Linear(64, 96, bias=False)
            blk.up_proj = nn.Linear(64, 128, bias=True)
            blk.norm = nn.LayerNorm(64)
            m.model.layers.append(blk)
        m.lm_head = nn.Linear(64, 50 if tied else 32, bias=False)
        if tied:  # tie_word_embeddings: lm_head.weight IS embed.weight (one Parameter)
            m.lm_head.weight = m.model.embed.weight
    m.to(torch.bfloat16)
    sch = QuantizationScheme(targets=["Linear"], weights=QuantizationArgs(num_bits=4, type="int", symmetric=True,
                                                                          group_size=32))
    m.quantization_scheme_map = {f"model.layers.{i}.{p}": sch for i in range(3) for p in ("q_proj", "up_proj")}
    return m


def _worker(rank, world, port, out_dir, q, tied=False):
    import sys
    sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__))))
    sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "oracle"))
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from test_distributed_cpu import _OraclePlan
        from quantizers_amd import compressor, residency
        compressor.CompressionPlan = _OraclePlan
        m = _model(meta=rank != 0, tied=tied)
        assert residency.skeleton_mode(m)
        res = residency.Residency(m, "cpu", SHARD)
        m.quantization_residency = res
        layers = m.model.layers
        res.materialise_outside(m, layers)
        res.distribute(m, layers, onload=lambda layer: None, offload=lambda layer, host: None)
        res.release_outside(m, layers)
        if tied:  # the tie survives the broadcasts and the release on every rank
            assert m.lm_head.weight is m.model.embed.weight
        n_meta = sum(p.is_meta for p in m.parameters())
        compressor.save_compressed(m, out_dir, max_shard_bytes=SHARD, device="cpu")
        with pytest.raises(ValueError, match="save plan"):
            compressor.save_compressed(m, out_dir + "_x", max_shard_bytes=SHARD * 2, device="cpu")
        q.put((rank, n_meta, len(list(m.parameters()))))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world,tied", [(2, False), (2, True), (4, True), (8, False)])
def test_skeleton_rank_keeps_its_shards_and_save_matches_one_process(tmp_path, world, tied):
    """World 2 / 4 / 8 (more ranks than some shard counts: ranks that own no file, units whose
    tensors straddle two ranks' files), tied and untied embeddings: every rank writes its own
    shards and the directory is byte-identical to one process's."""
    import sys
    sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "oracle"))
    sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
    from test_distributed_cpu import _OraclePlan
    from quantizers_amd import compressor
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    multi = str(tmp_path / "multi")
    port = _port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, multi, q, tied)) for r in range(world)]
    for p in procs:
        p.start()
    res = dict((r, (a, b)) for r, a, b in (q.get(timeout=300) for _ in range(world)))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert res[0][0] == 0  # rank 0 keeps the whole model
    assert all(0 < res[r][0] <= res[r][1] for r in range(1, world))  # helpers hold a part, the rest is meta
    assert any(res[r][0] < res[r][1] for r in range(1, world))
    saved = compressor.CompressionPlan
    compressor.CompressionPlan = _OraclePlan
    try:
        one = compressor.save_compressed(_model(tied=tied), str(tmp_path / "one"), max_shard_bytes=SHARD, device="cpu")
    finally:
        compressor.CompressionPlan = saved
    files = sorted(os.listdir(one))
    assert files == sorted(os.listdir(multi)) and len([f for f in files if f.endswith(".safetensors")]) > 2
    for fn in files:
        assert filecmp.cmp(os.path.join(one, fn), os.path.join(multi, fn), shallow=False), fn


def _dir_worker(rank, world, port, base, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from quantizers_amd.compressor import _check_shared_dir
        _check_shared_dir(os.path.join(base, "same"), rank)  # one directory: passes
        try:
            _check_shared_dir(os.path.join(base, f"rank{rank}"), rank)  # per-rank directories: refused
            q.put((rank, "no error"))
        except RuntimeError as e:
            q.put((rank, "refused" if "not one shared directory" in str(e) else str(e)))
    finally:
        dist.destroy_process_group()


def test_save_refuses_unshared_output_dir(tmp_path):
    """Each rank writes its own shards, so save_compressed checks that every rank sees rank 0's
    output directory (a multi-node run without a shared filesystem stops before writing)."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _port()
    procs = [ctx.Process(target=_dir_worker, args=(r, 2, port, str(tmp_path), q)) for r in range(2)]
    for p in procs:
        p.start()
    got = dict(q.get(timeout=120) for _ in range(2))
    for p in procs:
        p.join(timeout=60)
    assert got == {0: "refused", 1: "refused"}, got
    assert not [f for f in os.listdir(tmp_path / "same") if f.startswith(".qz_rank_probe")]
