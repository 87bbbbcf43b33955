"""Host -> device staging through pinned bounce buffers.

A pageable ``tensor.to(device)`` is a synchronous copy through the driver's own small staging
area (the Qwen3-4B model's 8 GB took 7.8 s as ``model.to``).  ``H2DStager`` copies host tensors
in chunks through two pinned buffers: the host memcpy of chunk k+1 overlaps the DMA of chunk k,
which runs on a side stream; the caller's stream waits for the DMAs with one event
(``wait(stream)``) before it uses the device tensors."""
from __future__ import annotations

import json
import os
import queue
import struct
import time
from typing import Dict, List, Optional, Tuple

import torch


class H2DStager:
    def __init__(self, device, chunk_bytes: int = 256 << 20):
        self.device = torch.device(device)
        self.chunk = chunk_bytes
        self.stream = torch.cuda.Stream(self.device)
        self._stage: Optional[List[torch.Tensor]] = None
        self._done: List[Optional[torch.cuda.Event]] = [None, None]
        self._k = 0
        self.stats = {"bytes": 0, "alloc_s": 0.0, "wait_s": 0.0, "memcpy_s": 0.0, "enqueue_s": 0.0}

    def _buffers(self) -> List[torch.Tensor]:
        if self._stage is None:
            self._stage = [torch.empty(self.chunk, dtype=torch.uint8, pin_memory=True) for _ in range(2)]
        return self._stage

    def copy(self, src: torch.Tensor) -> torch.Tensor:
        """Enqueue the copy of host tensor ``src``; returns its (not yet filled) device tensor."""
        src = src.detach()
        t0 = time.perf_counter()
        dst = torch.empty(src.shape, dtype=src.dtype, device=self.device)
        self.stats["alloc_s"] += time.perf_counter() - t0
        if src.numel() == 0:
            return dst
        self.stats["bytes"] += src.numel() * src.element_size()
        dst.record_stream(self.stream)  # not reused by the allocator before its DMA has run
        # dst may be a block the caller's stream freed while its kernels still read it: the DMA
        # that overwrites it runs after the caller's stream's work so far
        self.stream.wait_stream(torch.cuda.current_stream(self.device))
        if src.is_pinned() and src.is_contiguous():  # DMA straight from the caller's pinned memory
            with torch.cuda.stream(self.stream):
                dst.copy_(src, non_blocking=True)
                ev = torch.cuda.Event()
                ev.record(self.stream)
            self._done[self._k % 2] = ev  # keeps ordering for wait(); no staging buffer used
            self._k += 1
            return dst
        src = src.contiguous()
        sb, db = src.reshape(-1).view(torch.uint8), dst.reshape(-1).view(torch.uint8)
        stage = self._buffers()
        for off in range(0, sb.numel(), self.chunk):
            n = min(self.chunk, sb.numel() - off)
            i = self._k % 2
            t0 = time.perf_counter()
            if self._done[i] is not None:
                self._done[i].synchronize()  # the DMA that last read this staging buffer
            t1 = time.perf_counter()
            stage[i][:n].copy_(sb[off:off + n])
            t2 = time.perf_counter()
            with torch.cuda.stream(self.stream):
                db[off:off + n].copy_(stage[i][:n], non_blocking=True)
                ev = torch.cuda.Event()
                ev.record(self.stream)
            self.stats["wait_s"] += t1 - t0
            self.stats["memcpy_s"] += t2 - t1
            self.stats["enqueue_s"] += time.perf_counter() - t2
            self._done[i] = ev
            self._k += 1
        return dst

    def wait(self, stream=None) -> None:
        """Make ``stream`` (default: the device's current stream) wait for every copy so far."""
        ev = torch.cuda.Event()
        ev.record(self.stream)
        (stream if stream is not None else torch.cuda.current_stream(self.device)).wait_event(ev)

    def synchronize(self) -> None:
        self.stream.synchronize()


_ST_DTYPES = {"BF16": torch.bfloat16, "F16": torch.float16, "F32": torch.float32, "F64": torch.float64,
              "I8": torch.int8, "U8": torch.uint8, "I16": torch.int16, "I32": torch.int32, "I64": torch.int64,
              "BOOL": torch.bool, "F8_E4M3": torch.float8_e4m3fn}


def safetensors_header(path: str) -> Tuple[int, Dict[str, Tuple[str, Tuple[int, ...], Tuple[int, int]]]]:
    """(data section offset, {name: (dtype tag, shape, (begin, end) within the data section)}) of a
    safetensors file, from its 8-byte little-endian header length and JSON header."""
    with open(path, "rb") as f:
        n = struct.unpack("<Q", f.read(8))[0]
        hdr = json.loads(f.read(n))
    hdr.pop("__metadata__", None)
    return 8 + n, {k: (v["dtype"], tuple(v["shape"]), tuple(v["data_offsets"])) for k, v in hdr.items()}


class FileLoad:
    """The pending disk -> device load of one file's tensors (``DiskStager.load``)."""

    def __init__(self, fd: int, tensors: Dict[str, torch.Tensor], futures: list, nbytes: int):
        self.fd, self.tensors, self.futures, self.nbytes = fd, tensors, futures, nbytes


class DiskStager:
    """Disk -> device for tensors of safetensors files, for the data-free driver: worker threads
    (``pool``) read each tensor's byte range with ``os.preadv`` straight into one of ``slots``
    pinned buffers of ``slot_bytes`` and issue its DMA on the stager's stream; a slot is reused
    once its DMA has completed.  So the disk reads run on many threads beside the GPU work, and
    the host never copies the bytes again (H2DStager, fed from a memory map, reads the file on the
    caller's thread in its page-cache -> pinned memcpy: 7.7 GB/s cold, profiles/r06h_model_free.log)."""

    def __init__(self, device, pool, slots: int = 8, slot_bytes: int = 64 << 20):
        self.device = torch.device(device)
        self.stream = torch.cuda.Stream(self.device)
        self.pool = pool
        self.slot_bytes = slot_bytes
        self.slots = [torch.empty(slot_bytes, dtype=torch.uint8, pin_memory=True) for _ in range(slots)]
        self.free: "queue.Queue[int]" = queue.Queue()
        for k in range(slots):
            self.free.put(k)
        self.events: List[Optional[torch.cuda.Event]] = [None] * slots

    def load(self, path: str, names: List[str], header=None) -> FileLoad:
        """Enqueue the reads + DMAs of ``names`` from the file at ``path``; returns at once."""
        start, meta = header if header is not None else safetensors_header(path)
        for name in names:  # every entry checked before any read is queued
            tag, shape, (b0, b1) = meta[name]
            need = torch.Size(shape).numel() * torch.empty(0, dtype=_ST_DTYPES[tag]).element_size()
            if need != b1 - b0:
                raise ValueError(f"{path}: {name} holds {b1 - b0} bytes, its shape {shape} needs {need}")
        fd = os.open(path, os.O_RDONLY)
        tensors, futures, total = {}, [], 0
        # the blocks allocated below may have been freed by the caller's stream while its kernels
        # still read them: every DMA of this load runs after the caller's stream's work so far
        self.stream.wait_stream(torch.cuda.current_stream(self.device))
        for name in names:
            tag, shape, (b0, b1) = meta[name]
            dst = torch.empty(shape, dtype=_ST_DTYPES[tag], device=self.device)
            dst.record_stream(self.stream)  # not reused by the allocator before its DMAs have run
            tensors[name] = dst
            flat = dst.reshape(-1).view(torch.uint8)
            for off in range(0, b1 - b0, self.slot_bytes):
                n = min(self.slot_bytes, b1 - b0 - off)
                futures.append(self.pool.submit(self._chunk, fd, start + b0 + off, flat[off:off + n]))
            total += b1 - b0
        return FileLoad(fd, tensors, futures, total)

    def _chunk(self, fd: int, off: int, dst: torch.Tensor) -> None:
        k = self.free.get()
        try:
            ev = self.events[k]
            if ev is not None:
                ev.synchronize()  # the slot's previous DMA has read it
            n = dst.numel()
            buf = self.slots[k][:n]
            view = memoryview(buf.numpy())
            got = 0
            while got < n:
                r = os.preadv(fd, [view[got:]], off + got)
                if r <= 0:
                    raise IOError(f"short read at offset {off + got}")
                got += r
            with torch.cuda.stream(self.stream):
                dst.copy_(buf, non_blocking=True)
                ev = torch.cuda.Event()
                ev.record(self.stream)
            self.events[k] = ev
        finally:
            self.free.put(k)

    def wait(self, fl: FileLoad, stream=None) -> Dict[str, torch.Tensor]:
        """Block until every read of ``fl`` is done and its DMAs are enqueued; make ``stream``
        (default: the current one) wait for them; returns the device tensors."""
        try:
            for f in fl.futures:
                f.result()
        finally:
            self.release(fl)
        ev = torch.cuda.Event()
        ev.record(self.stream)
        (stream if stream is not None else torch.cuda.current_stream(self.device)).wait_event(ev)
        return fl.tensors

    @staticmethod
    def release(fl: FileLoad) -> None:
        """Close ``fl``'s file once none of its reads can still run (a failed or abandoned load:
        its other chunks finish or fail first, so no read ever lands on a reused descriptor)."""
        if fl.fd < 0:
            return
        for f in fl.futures:
            f.cancel()
        for f in fl.futures:
            if not f.cancelled():
                f.exception()  # waits; the error, if any, is the caller's to report
        os.close(fl.fd)
        fl.fd = -1
