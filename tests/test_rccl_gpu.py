"""The RCCL (backend ``nccl``) collectives of the product path, executed on the MI355X.

An 8-GPU node is the driver's, and RCCL refuses two ranks on one device, so this runs the same
calls in a 1-rank RCCL communicator on cuda:0: ``gather_state``'s packed all-gather path
(``distributed._gather_packed``: flat byte buffers, bucketed ``all_gather_into_tensor`` rounds,
pinned-host receive) and the AWQ grid's loss all-reduce (``awq._all_reduce_sum``).  The
multi-rank arithmetic (padding, per-rank offsets, dst-only receive) is covered by the gloo
world-2 tests (tests/test_distributed_cpu.py); this pins that the RCCL calls themselves run on
device tensors and move the bytes unchanged."""
import socket

import pytest
import torch

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def rccl():
    import torch.distributed as dist
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    torch.cuda.set_device(0)
    dist.init_process_group("nccl", init_method=f"tcp://127.0.0.1:{port}", rank=0, world_size=1,
                            device_id=torch.device("cuda", 0))
    assert dist.get_backend() == "nccl"
    yield dist
    dist.destroy_process_group()


def _state(dev):
    g = torch.Generator(device=dev).manual_seed(3)
    return {"a.weight_packed": torch.randint(-2**31, 2**31 - 1, (96, 40), dtype=torch.int32, device=dev, generator=g),
            "a.weight_scale": torch.randn(96, 10, device=dev, generator=g).to(torch.bfloat16),
            "b.weight": torch.randn(33, 17, device=dev, generator=g).to(torch.float8_e4m3fn),
            "b.weight_scale": torch.rand(1, 1, device=dev, generator=g),
            "c.weight_shape": torch.tensor([96, 320], dtype=torch.int32, device=dev),
            "d.empty": torch.empty(0, 8, dtype=torch.bfloat16, device=dev)}


def _same(a, b):
    assert a.dtype == b.dtype and a.shape == b.shape
    assert torch.equal(a.reshape(-1).view(torch.uint8).cpu(), b.reshape(-1).view(torch.uint8).cpu())


@pytest.mark.parametrize("to_host", [False, True])
@pytest.mark.parametrize("bucket", [1 << 30, 4096, 16])
def test_packed_all_gather_rccl(rccl, to_host, bucket):
    from quantizers_amd.distributed import _gather_packed
    dev = torch.device("cuda", 0)
    local = _state(dev)
    out = _gather_packed(local, None, None, to_host, bucket)
    assert set(out) == set(local)
    for k, v in local.items():
        assert out[k].device.type == ("cpu" if to_host else "cuda")
        _same(out[k], v)


def test_packed_all_gather_rccl_dst(rccl):
    from quantizers_amd.distributed import _gather_packed
    local = _state(torch.device("cuda", 0))
    out = _gather_packed(local, None, 0, True, 1 << 20)
    for k, v in local.items():
        _same(out[k], v)


def test_grid_loss_all_reduce_rccl(rccl):
    from quantizers_amd.awq import _all_reduce_sum
    t = torch.arange(20, dtype=torch.float32, device="cuda") * 0.5
    ref = t.clone()
    _all_reduce_sum(t)
    torch.cuda.synchronize()
    assert torch.equal(t, ref)  # one rank: the sum is the rank's own losses, bit for bit
