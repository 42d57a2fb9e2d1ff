"""Sample runs (tolerance contract, mode 0): the path kernel sums each pixel's samples in runs of
run_k consecutive samples inside the wave's LDS and stores one affine partial per run (col ->
2^k col + b, the NaN doubling of draw(), main.cpp:161-167); mrt_fold_runs_kernel applies them in
run order.  The per-path radiance is the same as the per-path mode's (same paths, same streams),
so the run image must equal, bit for bit, a numpy restatement of that grouping over the per-path
radiance of an MRT_RF_PATH_DEBUG render (which keeps per-path radiance + the sequential fold)."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def gpu(mrt):
    import torch
    assert torch.cuda.is_available()
    torch.cuda.init()
    return mrt


def run_grouped_image(prgb, ns, chunk, k, max_lum=1000.0):
    """prgb [pixel][s][3] f32 -> the run-mode image: per launch chunk [s0, s1), runs of k samples
    from s0, each folded sequentially from zero (non-finite sample: b doubles, the incoming colour's
    coefficient doubles), applied in order; then draw()'s final divide + luminance clamp
    (main.cpp:168-173)."""
    f = np.float32
    col = np.zeros((prgb.shape[0], 3), dtype=f)
    for s0 in range(0, ns, chunk):
        s1 = min(ns, s0 + chunk)
        for r0 in range(s0, s1, k):
            b = np.zeros_like(col)
            kd = np.zeros(col.shape[0], dtype=np.int64)
            for s in range(r0, min(r0 + k, s1)):
                L = prgb[:, s]
                fin = np.isfinite(L).all(axis=1)
                b = np.where(fin[:, None], b + L, b + b)
                kd += ~fin
            for i in np.nonzero(kd)[0]:
                for _ in range(kd[i]):
                    col[i] = col[i] + col[i]
            col = col + b
    c = col / f(ns)
    lum = (c[:, 0] * f(0.212655) + c[:, 1] * f(0.715158)) + c[:, 2] * f(0.072187)
    big = lum > f(max_lum)
    c[big] = c[big] * (f(max_lum) / lum[big])[:, None]
    return c


def per_path(mrt, r, d):
    ns = d.sqrt_samples ** 2
    px = mrt.local_pixels(d)
    prgb, _ = r.paths(len(px) * ns)
    out = np.zeros((d.width * d.height, ns, 3), dtype=np.float32)
    out[px] = prgb.reshape(ns, len(px), 3).transpose(1, 0, 2)
    return out, px


@pytest.mark.parametrize("sid,w,h,spp,chunk", [(5, 48, 40, 64, 0), (5, 40, 32, 25, 0), (5, 48, 40, 64, 24),
                                               (5, 33, 17, 100, 7), (6, 40, 40, 36, 0)])
def test_run_image_equals_grouped_per_path_fold(gpu, sid, w, h, spp, chunk):
    sc = gpu.select_scene(sid, w / h)
    r = gpu.Renderer(sc, 0)
    k = r.kernel_info()["run_k"]
    if sid == 5:
        assert k > 0, "the C2 kernel runs sample runs"
    if k == 0:
        pytest.skip("kernel without a path-start queue: per-path mode only")
    ns = int(round(spp ** 0.5)) ** 2
    dbg = gpu.render_desc(w, h, spp, numerics="fast", flags=gpu._lib.RF_PATH_DEBUG)
    img_p, rays_p = r.render(dbg)
    prgb, px = per_path(gpu, r, dbg)
    d = gpu.render_desc(w, h, spp, numerics="fast", chunk_samples=chunk)
    img, rays = r.render(d)
    assert rays == rays_p  # the same paths
    want = run_grouped_image(prgb.reshape(w * h, ns, 3), ns, chunk or ns, k)
    got = img[..., :3].reshape(-1, 3)
    assert np.array_equal(got.view(np.uint32), want.view(np.uint32))
    # and the per-path mode's sequential fold differs only by the regrouping
    assert np.abs(got - img_p[..., :3].reshape(-1, 3)).max() <= 1e-5 * max(1.0, float(np.abs(got).max()))
    r.close()


def test_run_renders_are_deterministic(gpu):
    """Runs trace their samples one after another, so which lanes run them does not change the sum."""
    sc = gpu.select_scene(5, 1.0)
    r = gpu.Renderer(sc, 0)
    d = gpu.render_desc(128, 128, 256, numerics="fast")
    a, ra = r.render(d)
    b, rb = r.render(d)
    assert ra == rb
    assert np.array_equal(a.view(np.uint32), b.view(np.uint32))
    r.close()


def test_run_shards_reassemble(gpu):
    """Two ranks' run-mode shards put together equal the one-rank run-mode image bit for bit."""
    w, h, spp = 64, 48, 64
    sc = gpu.select_scene(5, w / h)
    r = gpu.Renderer(sc, 0)
    full, rays = r.render(gpu.render_desc(w, h, spp, numerics="fast"))
    img = np.zeros_like(full)
    tot = 0
    for rank in range(2):
        part, pr = r.render(gpu.render_desc(w, h, spp, numerics="fast", rank=rank, world=2, tile_size=8))
        px = gpu.local_pixels(gpu.render_desc(w, h, spp, rank=rank, world=2, tile_size=8))
        img.reshape(-1, 4)[px] = part.reshape(-1, 4)[px]
        tot += pr
    assert tot == rays
    assert np.array_equal(img[..., :3].view(np.uint32), full[..., :3].view(np.uint32))
    r.close()
