"""Pinned, double-buffered host -> device staging (quantizers_amd/staging.py): every byte lands,
across chunk boundaries, for non-contiguous / pinned / empty sources, and a consumer on the
caller's stream sees the data after ``wait``."""
import pytest
import torch

from quantizers_amd.staging import H2DStager

pytestmark = pytest.mark.gpu


def _srcs():
    g = torch.Generator().manual_seed(5)
    a = torch.randn(3001, 17, generator=g).to(torch.bfloat16)  # 102 KB: many 4 KB chunks, ragged tail
    b = torch.randint(-2**31, 2**31 - 1, (64, 33), dtype=torch.int32, generator=g).t()  # non-contiguous
    c = torch.randn(4096, generator=g).pin_memory()  # pinned: direct DMA
    d = torch.empty(0, 8, dtype=torch.bfloat16)
    e = torch.randn(3, generator=g).to(torch.float8_e4m3fn)
    return [a, b, c, d, e]


@pytest.mark.parametrize("chunk", [4096, 1 << 20])
def test_stager_copies_every_byte(cuda, chunk):
    st = H2DStager(cuda, chunk_bytes=chunk)
    srcs = _srcs()
    outs = [st.copy(s) for s in srcs]
    st.wait()
    # a consumer on the caller's stream, ordered after the copies by the event
    sums = [o.float().sum() if o.numel() and o.dtype != torch.float8_e4m3fn else None for o in outs]
    torch.cuda.synchronize()
    for s, o, sm in zip(srcs, outs, sums):
        assert o.device.type == "cuda" and o.shape == s.shape and o.dtype == s.dtype
        assert torch.equal(o.cpu().reshape(-1).view(torch.uint8), s.contiguous().reshape(-1).view(torch.uint8))
        if sm is not None:
            assert sm.item() == o.float().sum().item()  # same reduction after the sync
