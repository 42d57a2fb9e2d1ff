"""Multi-GPU framebuffer assembly: tile shards -> rank 0 with ONE collective.

The reference splits the image into work_queue tiles (work_queue.cpp:64-128) that its threads
pull from one atomic counter.  Here the tiles (in the same inverted-Hilbert order) are dealt to the
ranks in rounds of `world`, each round in its own pseudo-random rank order (local_pixels /
mrt_local_pixels: a fixed deal, so no rank always takes the same position of the curve's small
blocks); each rank renders its tiles into a compact [n_local, 4] buffer in HBM, and one
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
    """One rank's end of the framebuffer gather.  Shards are gathered at their padded size
    (n_max rows): a render writes its n_local rows straight into a padded buffer (bench.py
    allocates its render outputs that way), so no pad copy is made; rank 0 receives all shards
    into ONE [world, n_max, 4] tensor and scatters them into the framebuffer with ONE index_copy_
    (padding rows land on a spare row past the image)."""

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
            self.recv = torch.zeros((world, self.n_max, 4), dtype=torch.float32, device=device)
            self.bufs = list(self.recv.unbind(0))
            spare = width * height  # padding rows of every shard go here
            idx = np.full((world, self.n_max), spare, dtype=np.int64)
            for r, p in enumerate(self.px):
                idx[r, : len(p)] = p
            self.idx = torch.as_tensor(idx.reshape(-1), device=device)
            self.full_ext = torch.zeros((width * height + 1, 4), dtype=torch.float32, device=device)
            self.full = self.full_ext[: width * height]

    def gather(self, local):
        """local: [n_local or n_max, 4] float32 on `device`.  Returns the [H, W, 4] framebuffer on rank 0."""
        return self.finish(self.start(local))

    def start(self, local):
        """Enqueue the gather of `local` (a padded [n_max, 4] buffer is sent as it is; a compact
        [n_local, 4] one is first copied into the padded staging buffer).  The caller must not
        write into a buffer it passed before finish() of that gather.  Returns a handle."""
        src = local
        if local.shape[0] != self.n_max:
            self.pad[: self.n_local].copy_(local)
            src = self.pad
        return dist.gather(src, self.bufs if self.rank == 0 else None, dst=0, async_op=True)

    def finish(self, handle):
        """Wait for a start()ed gather and, on rank 0, scatter the shards into the framebuffer."""
        handle.wait()
        if self.rank != 0:
            return None
        self.scatter()
        return self.full.view(self.height, self.width, 4)

    def scatter(self):
        """Rank 0: the received shards -> framebuffer rows (one index_copy_)."""
        self.full_ext.index_copy_(0, self.idx, self.recv.view(-1, 4))
