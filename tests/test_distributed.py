"""World-size-2/3 gloo test of the multi-GPU path on CPU: tile ownership (the permuted deal of tiles to ranks),
each rank rendering ONLY its own tiles through the product's render path (the CPU backend behind the
same C-ABI: mrt_render with rank / world in the desc, the hot-path code compiled for the host),
padded gather to rank 0 and scatter into the framebuffer.  The assembled image must equal a
one-rank render and the reference fixture (tests/golden/stream_5.npz) bit for bit, and the ray
totals summed over ranks the reference's G_rayCounter.  Covers the distribution logic of bench.py /
miniraytracer_amd.dist without a GPU; no oracle involved."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from conftest import ROOT, golden_stream

G = golden_stream("stream_5.npz")
W, H, SPP, DEPTH = G["w"], G["h"], G["spp"], G["depth"]
TILE = 8


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
    from miniraytracer_amd.dist import TileGather
    sc = m.select_scene(5, W / H)
    r = m.Renderer(sc, "cpu")
    d = m.render_desc(W, H, SPP, depth=DEPTH, tile_size=TILE, rank=rank, world=world, threads=2)
    img, rays = r.render(d)  # this rank's tiles only
    px = m.local_pixels(d)
    tg = TileGather(W, H, SPP, DEPTH, world, rank, torch.device("cpu"), tile_size=TILE)
    assert np.array_equal(px, tg.px[rank])
    local = torch.from_numpy(img.reshape(-1, 4)[px].copy())
    full = tg.gather(local)
    full = full.clone() if full is not None else None
    # overlapped form used by bench.py: start() copies the shard, finish() scatters on rank 0
    h = tg.start(local * 0 + local)
    full2 = tg.finish(h)
    # a render output allocated at the padded shard size is sent as it is (bench.py)
    padded = torch.zeros((tg.n_max, 4), dtype=torch.float32)
    padded[: tg.n_local] = local
    full3 = tg.gather(padded)
    if rank == 0:
        assert torch.equal(full, full2) and torch.equal(full, full3)
    total = torch.tensor([rays], dtype=torch.int64)
    dist.all_reduce(total)  # the ray count's one all_reduce
    if rank == 0:
        one, one_rays = r.render(m.render_desc(W, H, SPP, depth=DEPTH, tile_size=TILE, threads=2))
        q.put((full.numpy().copy(), one, one_rays, int(total.item())))
    dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3])
def test_gloo_tile_gather_reassembles_image(world):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    full, one, one_rays, total = q.get(timeout=300)
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0
    assert total == one_rays == G["rays"]
    assert np.array_equal(full.view(np.uint32), one.view(np.uint32))
    assert np.array_equal(full[..., :3].view(np.uint32), G["image"].view(np.uint32))
