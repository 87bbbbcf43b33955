"""Multi-process (world_size 2, gloo, CPU) coverage of the sharded-quantize + all-gather path.
The compress function is the CPU oracle here (the gather logic is what is under test); on GPUs
the same code runs with backend nccl (RCCL) and the HIP kernels."""
import os
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from quantizers_amd.distributed import gather_state, plan_shards, sharded_compress


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _weights():
    g = torch.Generator().manual_seed(0)
    shapes = {"a.q_proj": (64, 128), "a.k_proj": (32, 128), "a.down_proj": (128, 256), "b.up_proj": (256, 128),
              "b.gate_proj": (256, 128)}
    return {k: (torch.randn(*s, generator=g) * 0.02).to(torch.bfloat16) for k, s in shapes.items()}


def _worker(rank, world, port, q):
    import sys
    sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "oracle"))
    import ct_torch as ct
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    a = ct.QArgs(num_bits=4, group_size=32)
    calls = []

    def compress(name, w):
        calls.append(name)
        return ct.compress_weight(w, a)

    out = sharded_compress(_weights(), compress, device=torch.device("cpu"))
    # tensors travel as serialized bytes: a tensor put on the queue is shared through a file
    # descriptor of this process, which may have exited before the parent unpickles it
    import io
    buf = io.BytesIO()
    torch.save({k: v.clone() for k, v in out.items()}, buf)
    q.put((rank, calls, buf.getvalue()))
    dist.barrier()
    dist.destroy_process_group()


def test_plan_is_balanced_and_deterministic():
    items = [(f"w{i}", (i % 7 + 1) * 100) for i in range(50)]
    p1 = plan_shards(items, 4)
    p2 = plan_shards(list(reversed(items)), 4)
    assert p1 == p2
    assert sorted(sum(p1, [])) == sorted(k for k, _ in items)
    loads = [sum(dict(items)[k] for k in s) for s in p1]
    assert max(loads) - min(loads) <= 700


def test_sharded_compress_gloo_world2():
    import sys
    sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "oracle"))
    import ct_torch as ct
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = [q.get(timeout=120) for _ in range(2)]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    import io
    res = sorted((r, c, torch.load(io.BytesIO(b), weights_only=True)) for r, c, b in res)
    calls0, calls1 = res[0][1], res[1][1]
    assert not set(calls0) & set(calls1) and sorted(calls0 + calls1) == sorted(_weights())
    ref = {}
    for k, w in _weights().items():
        for kk, v in ct.compress_weight(w, ct.QArgs(num_bits=4, group_size=32)).items():
            ref[f"{k}.{kk}"] = v
    for _, _, out in res:
        assert set(out) == set(ref)
        for k in ref:
            a, b = out[k], ref[k]
            if a.dtype == torch.bfloat16:
                a, b = a.view(torch.int16), b.view(torch.int16)
            assert torch.equal(a, b), k


def test_gather_single_process_passthrough():
    t = {"x": torch.arange(5)}
    assert gather_state(t) == t


# ---------------------------------------------------------------- save_compressed, 2 ranks
class _OraclePlan:
    """Stand-in for compressor.CompressionPlan on a CPU-only host (test infrastructure): the
    units are compressed by the CPU oracle, so the sharding / gather / rank-0 write logic of
    save_compressed runs here; on GPUs the same logic drives the HIP kernels (tests/
    test_multirank_save_gpu.py)."""

    def __init__(self, units, device, stager=None):
        import ct_torch as ct
        self.out = {}
        for u in units:
            a = u.scheme.weights
            oa = ct.QArgs(num_bits=a.num_bits, type=a.type, symmetric=a.symmetric, strategy=a.strategy,
                          group_size=a.group_size)
            for ref in u.refs:
                for k, v in ct.compress_weight(ref.weight.detach().contiguous(), oa).items():
                    self.out[f"{ref.name}.{k}"] = v

    def run(self, stream=None):
        pass

    def tensors(self):
        return dict(self.out)


def _tiny_model():
    from torch import nn
    from quantizers_amd.quantization import QuantizationArgs, QuantizationScheme
    torch.manual_seed(0)
    m = nn.Module()
    m.model = nn.Module()
    m.model.layers = nn.ModuleList()
    for _ in range(3):
        blk = nn.Module()
        blk.q_proj = nn.Linear(64, 96, bias=False)
        blk.up_proj = nn.Linear(64, 128, bias=True)
        blk.norm = nn.LayerNorm(64)
        m.model.layers.append(blk)
    m.lm_head = nn.Linear(64, 32, bias=False)
    m.to(torch.bfloat16)
    sch = QuantizationScheme(targets=["Linear"], weights=QuantizationArgs(num_bits=4, type="int", symmetric=True,
                                                                          group_size=32))
    m.quantization_scheme_map = {f"model.layers.{i}.{p}": sch for i in range(3) for p in ("q_proj", "up_proj")}
    return m


def _save_worker(rank, world, port, out_dir, shard_bytes, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        import sys
        sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "oracle"))
        from quantizers_amd import compressor
        compressor.CompressionPlan = _OraclePlan
        written = []
        real = compressor._write_shard_file

        def spy(shard, path, ready):
            written.append(os.path.basename(path))
            real(shard, path, ready)
        compressor._write_shard_file = spy
        compressor.save_compressed(_tiny_model(), out_dir, max_shard_bytes=shard_bytes, device="cpu")
        q.put((rank, sorted(os.listdir(out_dir)), sorted(written)))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("shard_bytes", [5 << 30, 6000])
def test_save_compressed_gloo_world2_matches_one_process(tmp_path, shard_bytes):
    """Each rank writes its own shards of the plan (no gather); the files are byte-identical to
    one process, and with several shards both ranks write."""
    import filecmp
    import sys
    sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "oracle"))
    from quantizers_amd import compressor
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    multi = str(tmp_path / "multi")
    procs = [ctx.Process(target=_save_worker, args=(r, 2, port, multi, shard_bytes, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = sorted(q.get(timeout=120) for _ in range(2))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert res[0][1] == res[1][1]
    saved = compressor.CompressionPlan
    compressor.CompressionPlan = _OraclePlan
    try:
        one = compressor.save_compressed(_tiny_model(), str(tmp_path / "one"), max_shard_bytes=shard_bytes,
                                         device="cpu")
    finally:
        compressor.CompressionPlan = saved
    files = sorted(os.listdir(one))
    assert files == res[0][1]
    shards = [f for f in files if f.endswith(".safetensors")]
    assert sorted(res[0][2] + res[1][2]) == shards and not set(res[0][2]) & set(res[1][2])
    if shard_bytes < 1 << 20:
        assert len(shards) > 2 and res[0][2] and res[1][2]  # both ranks wrote
        assert "model.safetensors.index.json" in files
    else:
        assert shards == ["model.safetensors"]
    for fn in files:
        assert filecmp.cmp(os.path.join(one, fn), os.path.join(multi, fn), shallow=False), fn


def _gather_worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        local = {f"r{rank}.t{i}": torch.arange(i * 7 + rank * 3 + 1, dtype=torch.int16) for i in range(5)}
        local[f"r{rank}.e"] = torch.empty(0, dtype=torch.float32)
        res = []
        # tiny buckets: several rounds, ragged per-rank sizes; big buckets: one collective
        # received in place; gather to one rank (dst) and all-gather to every rank (dst=None)
        for dst, to_host, bucket in MODES:
            out = gather_state(local, dst=dst, to_host=to_host, bucket_bytes=bucket)
            res.append({k: v.tolist() for k, v in out.items()})
        q.put((rank, res))
    finally:
        dist.destroy_process_group()


MODES = [(1, True, 64), (None, False, 64), (None, False, 1 << 20), (2, False, 1 << 20), (0, False, 64)]


def test_gather_state_buckets_and_dst():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_gather_worker, args=(r, 3, port, q)) for r in range(3)]
    for p in procs:
        p.start()
    res = dict(q.get(timeout=120) for _ in range(3))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    want = {f"r{r}.t{i}": list(range(i * 7 + r * 3 + 1)) for r in range(3) for i in range(5)}
    want.update({f"r{r}.e": [] for r in range(3)})
    for m, (dst, _, _) in enumerate(MODES):
        for r in range(3):
            assert res[r][m] == (want if dst is None or dst == r else {}), (MODES[m], r)
