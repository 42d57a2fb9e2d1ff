"""Comparison of a rendered image with a committed shipped-reference fixture (tests/golden/shipped_*.npz).

Used by tests/test_gpu_parity.py and by bench.py (the bench line's `parity` object, computed after the
timed region).  Data only: the fixtures hold what the reference as shipped rendered on the same
per-path streams (tools/make_golden.py); nothing here runs or loads the reference.

Two fixture shapes:
  shipped_stream_5.npz   the whole C2 image (500x500, 1024 spp): per-pixel RMSE over every pixel
  shipped_full_<id>.npz  C3 / C4 / C5 at full resolution: a 32x32 grid of block means, channel means,
                         a band of rows and a seeded pixel sample; per-pixel RMSE over band + sample
  shipped_ownspp_<id>.npz  C3 / C4 / C5 at their own spp, a pixel list only (compare_pixels)
  shipped_ownspp_full_9.npz  C3 at its own spp (4096), the whole 800x800 image
"""
import os

import numpy as np

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def fixture_for(scene, width, height, spp, depth=32):
    """Path of the shipped-reference fixture rendered at exactly this config, or None."""
    for name in (f"shipped_stream_{scene}.npz", f"shipped_full_{scene}.npz"):
        p = os.path.join(GOLDEN, name)
        if os.path.exists(p):
            meta = [int(x) for x in np.load(p)["meta"]]
            if meta == [scene, width, height, spp, depth]:
                return p
    return None


def _rmse(a, b):
    return float(np.sqrt(((np.asarray(a, np.float64) - np.asarray(b, np.float64)) ** 2).mean()))


def compare(img, rays, path):
    """img: (H, W, >=3) float32, row 0 = bottom; rays: the render's ray total.  Returns a dict of
    per-pixel RMSE (whole image or band + sample), block-mean RMSE, max |channel-mean delta|, ray
    ratio and what the per-pixel figure was computed over."""
    g = np.load(path)
    im = np.asarray(img[..., :3], dtype=np.float32)
    h, w = im.shape[:2]
    out = {"fixture": os.path.basename(path), "spp": int(g["meta"][3]), "ray_ratio": float(rays / float(g["rays"][0]))}
    if "image" in g.files:  # the whole image
        ref = g["image"]
        out["rmse"] = _rmse(im, ref)
        out["over"] = f"all {w * h} pixels"
        b = 25
        bm = im.reshape(h // b, b, w // b, b, 3).mean(axis=(1, 3), dtype=np.float64)
        rbm = g["block_mean"] if "block_mean" in g.files else ref.reshape(h // b, b, w // b, b, 3).mean(axis=(1, 3), dtype=np.float64)
        out["block_rmse"] = _rmse(bm, rbm)
        out["block"] = f"{b}x{b} px"
        # where the squared error sits: the share of the ten largest pixels
        e2 = ((im.astype(np.float64) - ref) ** 2).sum(axis=-1).ravel()
        top = np.argsort(e2)[::-1][:10]
        out["top10_share"] = float(e2[top].sum() / max(e2.sum(), 1e-300))
        out["top10"] = [[int(i % w), int(i // w), float(np.sqrt(e2[i] / 3))] for i in top]
    else:  # band + sample
        r0, r1 = (int(x) for x in g["band_rows"])
        flat = im.reshape(-1, 3)
        d = np.concatenate([(im[r0:r1] - g["band"]).reshape(-1, 3), flat[g["sample_idx"]] - g["sample"]]).astype(np.float64)
        out["rmse"] = float(np.sqrt((d ** 2).mean()))
        out["over"] = f"rows {r0}-{r1 - 1} + {len(g['sample_idx'])} seeded pixels"
        gg = g["block_mean"].shape[0]
        bh, bw = h // gg, w // gg
        bm = im[:bh * gg, :bw * gg].reshape(gg, bh, gg, bw, 3).mean(axis=(1, 3), dtype=np.float64)
        out["block_rmse"] = _rmse(bm, g["block_mean"])
        out["block"] = f"{bh}x{bw} px"
    gmean = g["mean"] if "mean" in g.files else g["image"].reshape(-1, 3).mean(axis=0, dtype=np.float64)
    out["mean_delta"] = float(np.abs(im.reshape(-1, 3).mean(axis=0, dtype=np.float64) - gmean).max())
    return out


def compare_pixels(img, rays, g):
    """A pixel-list render (mrt_render_desc.pixels = g["pixels"]) against shipped_ownspp_<id>.npz:
    per-pixel RMSE over the list, max |channel-mean delta| of the list, ray ratio of the list."""
    vals = np.asarray(img, np.float32).reshape(-1, img.shape[-1])[g["pixels"], :3]
    d = vals.astype(np.float64) - g["values"]
    return {"fixture": f"shipped_ownspp_{int(g['meta'][0])}", "spp": int(g["meta"][3]), "pixels": int(g["pixels"].size),
            "rmse": float(np.sqrt((d ** 2).mean())), "mean_delta": float(np.abs(d.mean(axis=0)).max()),
            "ray_ratio": float(rays / float(g["rays"][0]))}
