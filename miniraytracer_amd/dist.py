"""Multi-GPU framebuffer assembly: tile shards -> rank 0 with ONE collective.

The reference splits the image into work_queue tiles (work_queue.cpp:64-128) that its threads
pull from one atomic counter.  Here tile k (in the same inverted-Hilbert order) belongs to rank
k % world; each rank renders its tiles into a compact [n_local, 4] buffer in HBM, and one
gather over RCCL (xGMI) brings the equal-size (padded) shards to rank 0, which scatters them into
the W*H framebuffer (row 0 = bottom, G_linearBackBuffer layout, main.cpp:58).  Ray counts are
summed with one all_reduce.  Works with any torch.distributed backend (nccl on GPUs, gloo on CPU
for tests).
"""
import numpy as np
import torch
import torch.distributed as dist

from . import local_pixels, render_desc


class TileGather:
    def __init__(self, width, height, samples, depth, world, rank, device, tile_size=32):
        self.world, self.rank, self.device = world, rank, device
        self.width, self.height = width, height
        self.px = [local_pixels(render_desc(width, height, samples, depth=depth, tile_size=tile_size, rank=r, world=world))
                   for r in range(world)]
        self.counts = [len(p) for p in self.px]
        self.n_max = max(self.counts)
        self.n_local = self.counts[rank]
        self.pad = torch.zeros((self.n_max, 4), dtype=torch.float32, device=device)
        if rank == 0:
            self.bufs = [torch.zeros((self.n_max, 4), dtype=torch.float32, device=device) for _ in range(world)]
            self.idx = [torch.as_tensor(p.astype(np.int64), device=device) for p in self.px]
            self.full = torch.zeros((width * height, 4), dtype=torch.float32, device=device)

    def gather(self, local):
        """local: [n_local, 4] float32 on `device`.  Returns the [H, W, 4] framebuffer on rank 0."""
        return self.finish(self.start(local))

    def start(self, local):
        """Enqueue the gather of `local` (its contents are copied before this returns on the
        device stream, so the caller may render into it again).  Returns a handle for finish()."""
        self.pad[: self.n_local].copy_(local)
        return dist.gather(self.pad, self.bufs if self.rank == 0 else None, dst=0, async_op=True)

    def finish(self, handle):
        """Wait for a start()ed gather and, on rank 0, scatter the shards into the framebuffer."""
        handle.wait()
        if self.rank != 0:
            return None
        for r in range(self.world):
            self.full.index_copy_(0, self.idx[r], self.bufs[r][: self.counts[r]])
        return self.full.view(self.height, self.width, 4)
