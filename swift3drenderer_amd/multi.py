"""Multi-GPU frame assembly: interleaved row bands + one gather (RCCL over xGMI on MI355X).

SURVEY.md §8e: every rank holds the whole (small) scene, runs the geometry stage redundantly and
rasterizes only its rows -- frame row y belongs to rank (y // band) % world -- into a compact local
buffer (the library's ``s3r_render_bands``).  One ``gather`` brings the bands to rank 0, which
scatters them back into frame order.  With ``torch.distributed`` on the ``nccl`` backend the gather
is RCCL; the ``gloo`` backend runs the same code on CPU tensors (tests).
"""
from __future__ import annotations

import numpy as np
import torch
import torch.distributed as dist


def band_row_ids(height: int, band: int, nparts: int, part: int) -> np.ndarray:
    """Frame rows owned by `part`, in local storage order (increasing y)."""
    y = np.arange(height)
    return y[(y // band) % nparts == part]


def band_rows(height: int, band: int, nparts: int, part: int) -> int:
    return int(((np.arange(height) // band) % nparts == part).sum())


class BandGather:
    """Per-run buffers for gathering a W x H frame split into `world` interleaved parts."""

    def __init__(self, width: int, height: int, band: int, world: int, rank: int, device):
        self.W, self.H, self.B, self.N, self.rank = width, height, band, world, rank
        self.rows = band_rows(height, band, world, rank)
        self.max_rows = max(band_rows(height, band, world, p) for p in range(world))
        self.send = torch.zeros((self.max_rows, width), dtype=torch.int32, device=device)
        self.recv = None
        self.frame = None
        if rank == 0:
            # one contiguous receive buffer (part p's rows at [p * max_rows, ...)) and, per frame row,
            # its row in that buffer: the de-interleave is then ONE row gather (index_select)
            self.recv_all = torch.empty((world * self.max_rows, width), dtype=torch.int32, device=device)
            self.recv = [self.recv_all[p * self.max_rows:(p + 1) * self.max_rows] for p in range(world)]
            self.frame = torch.empty((height, width), dtype=torch.int32, device=device)
            src = np.empty(height, dtype=np.int64)
            for p in range(world):
                ids = band_row_ids(height, band, world, p)
                src[ids] = p * self.max_rows + np.arange(len(ids))
            self.src_rows = torch.as_tensor(src, device=device)

    def gather(self, group=None):
        """Collective: every rank's `send` (rows [0, rows) valid) -> rank 0's `frame`."""
        dist.gather(self.send, self.recv, dst=0, group=group)
        if self.rank == 0:
            self.deinterleave()
        return self.frame

    def deinterleave(self):
        """Rank 0: the gathered parts in `recv_all` -> `frame` in row order.  On the GPU this is the
        library's one-launch kernel (include/render.h s3r_deinterleave_bands) on the current stream;
        the gloo path (CPU tensors, tests) uses a row gather."""
        if self.recv_all.is_cuda:
            from .renderer import load_library
            lib = load_library()
            st = torch.cuda.current_stream(self.recv_all.device).cuda_stream
            rc = lib.s3r_deinterleave_bands(self.recv_all.data_ptr(), self.max_rows, self.W, self.H, self.B, self.N,
                                            self.frame.data_ptr(), st)
            if rc != 0:
                raise RuntimeError('s3r_deinterleave_bands rejected the split')
        else:
            torch.index_select(self.recv_all, 0, self.src_rows, out=self.frame)
        return self.frame


class HostFrame:
    """One H x W uint32 host frame shared by all ranks of a node (a file in /dev/shm, mapped by every
    process): the destination of s3r_bands_to_host, each rank copying its own bands over its own
    GPU's PCIe link (the direct-D2H alternative to the gather).  Collective: every
    rank constructs and closes it."""

    def __init__(self, width: int, height: int, rank: int, group=None):
        import os
        import uuid
        self.rank = rank
        shared = dist.is_available() and dist.is_initialized()
        if rank != 0 and not shared:
            raise RuntimeError('HostFrame: rank != 0 needs an initialised torch.distributed process group '
                               '(rank 0 creates the shared frame and broadcasts its name)')
        name = [f'/dev/shm/s3r_frame_{os.getpid()}_{uuid.uuid4().hex[:12]}' if rank == 0 else None]
        if dist.is_available() and dist.is_initialized():
            dist.broadcast_object_list(name, src=0, group=group)
        self.path = name[0]
        if rank == 0:
            with open(self.path, 'wb') as f:
                f.truncate(width * height * 4)
        if dist.is_available() and dist.is_initialized():
            dist.barrier(group=group)
        self.frame = np.memmap(self.path, dtype=np.uint32, mode='r+', shape=(height, width))

    def close(self, group=None):
        self.frame._mmap.close()
        if dist.is_available() and dist.is_initialized():
            dist.barrier(group=group)
        if self.rank == 0:
            import os
            try:
                os.unlink(self.path)
            except FileNotFoundError:
                pass


def assemble(parts, height: int, band: int) -> np.ndarray:
    """Host-side reassembly of per-part compact buffers (tests and single-process use)."""
    n = len(parts)
    w = parts[0].shape[1]
    out = np.empty((height, w), dtype=parts[0].dtype)
    for p, buf in enumerate(parts):
        ids = band_row_ids(height, band, n, p)
        out[ids] = buf[: len(ids)]
    return out
