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


@pytest.mark.parametrize("slots,slot_bytes", [(2, 4096), (8, 1 << 20)])
def test_disk_stager_loads_every_byte(cuda, tmp_path, slots, slot_bytes):
    """staging.DiskStager (model_free_ptq's reader): every selected tensor of a safetensors file
    lands on the device byte for byte -- tensors spanning many slots, ragged tails, tiny and empty
    ones, several files in flight on one pool -- and a consumer on the caller's stream sees them
    after ``wait``."""
    from concurrent.futures import ThreadPoolExecutor
    from safetensors.torch import save_file
    from quantizers_amd.staging import DiskStager, safetensors_header
    g = torch.Generator().manual_seed(6)
    files = []
    for f in range(3):
        t = {f"w{f}.big": torch.randn(257, 129, generator=g).to(torch.bfloat16),
             f"w{f}.small": torch.randn(3, generator=g).to(torch.bfloat16),
             f"w{f}.i32": torch.randint(-9, 9, (40, 7), dtype=torch.int32, generator=g),
             f"w{f}.empty": torch.empty(0, 4, dtype=torch.bfloat16),
             f"w{f}.skip": torch.randn(11, generator=g)}
        p = str(tmp_path / f"f{f}.safetensors")
        save_file(t, p)
        files.append((p, t))
    with ThreadPoolExecutor(max_workers=5) as pool:
        st = DiskStager(cuda, pool, slots=slots, slot_bytes=slot_bytes)
        loads = []
        for p, t in files:
            hdr = safetensors_header(p)
            assert set(hdr[1]) == set(t)
            names = [k for k in t if not k.endswith(".skip")]
            loads.append((t, names, st.load(p, names, hdr)))
        for t, names, fl in loads:
            dev = st.wait(fl)
            assert set(dev) == set(names) and fl.nbytes == sum(t[k].numel() * t[k].element_size() for k in names)
            sums = {k: v.double().sum() for k, v in dev.items()}  # on the caller's stream
            torch.cuda.synchronize()
            for k in names:
                assert dev[k].dtype == t[k].dtype and dev[k].shape == t[k].shape
                assert torch.equal(dev[k].cpu().reshape(-1).view(torch.uint8), t[k].reshape(-1).view(torch.uint8)), k
                assert sums[k].item() == t[k].double().sum().item()


def test_disk_stager_truncated_file_fails_and_closes(cuda, tmp_path):
    """A file shorter than its header says (a torn copy): ``wait`` raises the short read, and the
    file is closed only after every other chunk of the load has finished -- also for a load that is
    released without being waited on (model_free_ptq's files queued ahead of a failure)."""
    import os
    from concurrent.futures import ThreadPoolExecutor
    from safetensors.torch import save_file
    from quantizers_amd.staging import DiskStager, safetensors_header
    g = torch.Generator().manual_seed(7)
    p = str(tmp_path / "torn.safetensors")
    save_file({"a.weight": torch.randn(64, 256, generator=g).to(torch.bfloat16),
               "b.weight": torch.randn(64, 256, generator=g).to(torch.bfloat16)}, p)
    hdr = safetensors_header(p)
    os.truncate(p, os.path.getsize(p) - 1000)

    def fds():  # open descriptors on the torn file
        n = 0
        for fd in os.listdir("/proc/self/fd"):
            try:
                n += os.readlink(f"/proc/self/fd/{fd}") == p
            except OSError:
                pass
        return n
    with ThreadPoolExecutor(max_workers=4) as pool:
        st = DiskStager(cuda, pool, slots=2, slot_bytes=4096)
        assert fds() == 0
        fl = st.load(p, ["a.weight", "b.weight"], hdr)
        with pytest.raises(IOError, match="short read"):
            st.wait(fl)
        assert fl.fd == -1 and all(f.done() for f in fl.futures) and fds() == 0
        fl2 = st.load(p, ["a.weight", "b.weight"], hdr)
        st.release(fl2)
        assert fl2.fd == -1 and all(f.done() for f in fl2.futures) and fds() == 0
        st.release(fl2)  # idempotent
        # the stager keeps working after a failed load
        good = str(tmp_path / "good.safetensors")
        w = torch.randn(33, 65, generator=g).to(torch.bfloat16)
        save_file({"w.weight": w}, good)
        dev = st.wait(st.load(good, ["w.weight"]))
        torch.cuda.synchronize()
        assert torch.equal(dev["w.weight"].cpu().view(torch.int16), w.view(torch.int16))
