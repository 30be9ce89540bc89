"""Multi-GPU image-tile sharding (one process per GPU, torch.distributed).

The reference is single-GPU; each pixel's path depends only on
(pixel_index, random_seed) and the read-only scene (main.cu:40,53), so the
frame shards into independent tiles with the BVH replicated on every GPU.
Tile t (32x32, row-major) belongs to rank t % world (pupil_pt_local_pixels).
Once per frame every rank's compact tile radiance is gathered to rank 0 over
RCCL (backend "nccl") and scattered into the full image — one collective,
~4 MB per rank at 1080p/8 GPUs.  Results are bit-identical to one GPU.
gather_async() runs the snapshot, the collective and the scatter on a side HIP
stream, so frame k's gather overlaps frame k+1's rendering.
"""
from __future__ import annotations

import ctypes as C
import time

import numpy as np

from .abi import check, load_library


def local_pixels(width, height, tile, rank, world) -> np.ndarray:
    lib = load_library()
    n = C.c_uint32(0)
    check(lib.pupil_pt_local_pixels(width, height, tile, rank, world, None, C.byref(n)))
    out = np.zeros(max(1, n.value), np.uint32)
    check(lib.pupil_pt_local_pixels(width, height, tile, rank, world, out.ctypes.data_as(C.POINTER(C.c_uint32)),
                                    C.byref(n)))
    return out[: n.value]


class FrameGather:
    """Gathers every rank's compact (n_local, C) tile buffer into rank 0's full image."""

    def __init__(self, width, height, tile, rank, world, device, channels=4):
        import torch

        self.rank, self.world = rank, world
        self.maps = [torch.from_numpy(local_pixels(width, height, tile, r, world).astype(np.int64)).to(device)
                     for r in range(world)]
        self.counts = [len(m) for m in self.maps]
        self.n_local = self.counts[rank]
        self.send = torch.zeros((max(self.counts), channels), dtype=torch.float32, device=device)
        self.recv = [torch.zeros_like(self.send) for _ in range(world)] if rank == 0 else None
        self.full = (torch.zeros((width * height, channels), dtype=torch.float32, device=device)
                     if rank == 0 else None)
        self._side = None  # gather_async's side stream (created on first use)

    def gather(self, local):
        import torch.distributed as dist

        self.send[: self.n_local].copy_(local)
        dist.gather(self.send, self.recv, dst=0)
        if self.rank == 0:
            for r in range(self.world):
                self.full.index_copy_(0, self.maps[r], self.recv[r][: self.counts[r]])
            return self.full
        return None

    def gather_async(self, local, stream=None):
        """gather() overlapped with the caller's next frame (GPU tensors).

        A side stream waits for `stream`'s work so far, snapshots `local` into the
        send buffer, runs the collective and (rank 0) the scatter into the full
        image; `stream` waits only for the snapshot, so the next frame may start
        at once and overwrite `local`.  Returns a GatherHandle: the full image is
        not usable until ``handle.wait(stream)`` (device-side: `stream` waits for
        the scatter) or ``handle.synchronize()`` (host).  Side-stream work of
        consecutive calls runs in call order, and each call's side work first
        waits for everything enqueued on `stream` before it, so a consumer that
        waited on the handle and then read the image on `stream` is never
        overwritten by a later frame.  CPU tensors / gloo take the synchronous
        path and return an already-complete handle."""
        import torch
        import torch.distributed as dist

        if local.device.type != "cuda":
            t0 = time.perf_counter()
            full = self.gather(local)
            return GatherHandle(full, None, host_ms=(time.perf_counter() - t0) * 1e3)
        if dist.get_backend() != "nccl":  # rehearsal over gloo: stage through host memory, synchronously
            t0 = time.perf_counter()
            host = FrameGather.__new__(FrameGather)
            host.__dict__.update(self.__dict__)
            host.send, host.maps = self.send.cpu(), [m.cpu() for m in self.maps]
            host.recv = [r.cpu() for r in self.recv] if self.recv is not None else None
            host.full = self.full.cpu() if self.full is not None else None
            full = host.gather(local.cpu())
            if self.rank == 0:
                self.full.copy_(full)
            return GatherHandle(self.full if self.rank == 0 else None, None,
                                host_ms=(time.perf_counter() - t0) * 1e3)
        if self._side is None:
            self._side = torch.cuda.Stream(device=local.device)
            self._copied = torch.cuda.Event()
        stream = stream if stream is not None else torch.cuda.current_stream(local.device)
        ready = torch.cuda.Event()
        ready.record(stream)
        done = torch.cuda.Event(enable_timing=True)
        start = torch.cuda.Event(enable_timing=True)
        with torch.cuda.stream(self._side):
            self._side.wait_event(ready)
            self.send[: self.n_local].copy_(local)
            self._copied.record(self._side)
            start.record(self._side)  # the collective + scatter, timed on the side stream
            dist.gather(self.send, self.recv, dst=0)
            if self.rank == 0:
                for r in range(self.world):
                    self.full.index_copy_(0, self.maps[r], self.recv[r][: self.counts[r]])
            done.record(self._side)
        stream.wait_event(self._copied)
        return GatherHandle(self.full if self.rank == 0 else None, done, start=start)

    def wait(self):
        """Block the host until every gather_async() so far has completed."""
        if self._side is not None:
            self._side.synchronize()


class GatherHandle:
    """Completion of one FrameGather.gather_async(): the rank-0 image is valid on a
    stream after wait(stream), on the host after synchronize()."""

    def __init__(self, full, event, start=None, host_ms=None):
        self._full, self._event = full, event
        self._start, self._host_ms = start, host_ms

    def elapsed_ms(self):
        """Time of this gather: side-stream HIP events around the collective and the scatter
        (RCCL), or the host time of the synchronous path (gloo / CPU tensors)."""
        if self._host_ms is not None:
            return self._host_ms
        if self._start is None or self._event is None:
            return None
        self._event.synchronize()
        return self._start.elapsed_time(self._event)

    def wait(self, stream=None):
        """Make `stream` (default: the current stream) wait for the scatter; returns
        the full image (rank 0) or None."""
        if self._event is not None:
            import torch

            (stream if stream is not None else torch.cuda.current_stream()).wait_event(self._event)
        return self._full

    def synchronize(self):
        if self._event is not None:
            self._event.synchronize()
        return self._full

    def done(self) -> bool:
        return self._event is None or self._event.query()
