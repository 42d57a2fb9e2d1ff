"""World-size-2 gloo test of the multi-GPU path on CPU: tile ownership (tile k -> rank k % world),
padded gather to rank 0 and scatter into the framebuffer reproduce the single-process image bit
for bit.  The per-rank pixels are rendered by the C restatement (CPU stand-in for the GPU), so
this covers the distribution logic of bench.py / miniraytracer_amd.dist without a GPU."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from conftest import ROOT

W, H, SPP = 50, 30, 4


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, q):
    import sys
    sys.path.insert(0, ROOT)
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    import miniraytracer_amd as m
    import oracle
    from miniraytracer_amd.dist import TileGather
    sc = m.select_scene(5, W / H)
    img, rays, _, _ = oracle.render(sc, oracle.desc(W, H, SPP, threads=2))
    tg = TileGather(W, H, SPP, 32, world, rank, torch.device("cpu"), tile_size=16)
    local = torch.from_numpy(img.reshape(-1, 4)[tg.px[rank]].copy())
    full = tg.gather(local)
    full = full.clone() if full is not None else None
    # overlapped form used by bench.py: start() copies the shard, finish() scatters on rank 0
    h = tg.start(local * 0 + local)
    full2 = tg.finish(h)
    if rank == 0:
        assert torch.equal(full, full2)
    total = torch.tensor([len(tg.px[rank])], dtype=torch.int64)
    dist.all_reduce(total)
    if rank == 0:
        q.put((full.numpy().copy(), img, int(total.item())))
    dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3])
def test_gloo_tile_gather_reassembles_image(world):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    full, ref, total = q.get(timeout=300)
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0
    assert total == W * H
    assert np.array_equal(full.view(np.uint32), ref.view(np.uint32))
