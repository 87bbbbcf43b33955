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
    q.put((rank, calls, {k: v.clone() for k, v in out.items()}))
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
    res.sort()
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
