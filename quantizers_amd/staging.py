"""Host -> device staging through pinned bounce buffers.

A pageable ``tensor.to(device)`` is a synchronous copy through the driver's own small staging
area (the Qwen3-4B model's 8 GB took 7.8 s as ``model.to``).  ``H2DStager`` copies host tensors
in chunks through two pinned buffers: the host memcpy of chunk k+1 overlaps the DMA of chunk k,
which runs on a side stream; the caller's stream waits for the DMAs with one event
(``wait(stream)``) before it uses the device tensors."""
from __future__ import annotations

from typing import List, Optional

import time

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
