#!/usr/bin/env python3
"""Experiment: how far the tolerance contract strays from the exact contract (= the reference as
shipped) path by path.  Both contracts render the same per-path streams with
MRT_RF_PATH_DEBUG; per config: the fraction of paths whose ray count differs or whose radiance
differs by more than 1e-3 relative (diverged paths), and the per-path mean squared radiance
difference D2 -- the per-pixel RMSE at N spp is then about sqrt(D2 / 3 / N) (independent paths;
per channel), without the lottery of which pixels a firefly lands in.  One JSON line per config.
  python tools/divergence.py          (MRT_EXPERIMENT_LIB selects an A/B build of the fast contract)"""
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import miniraytracer_amd as m  # noqa: E402

tag = os.path.basename(os.environ.get("MRT_EXPERIMENT_LIB", "intree")).replace(".so", "").replace("libmrt_", "")
# (name, scene, width, height, spp of this probe, the config's own spp)
CASES = [("C2", 5, 250, 250, 256, 1024), ("C3", 9, 200, 200, 256, 4096), ("C4", 8, 256, 256, 64, 2025), ("C5", 7, 256, 256, 64, 8100)]
for name, sid, w, h, spp, own in CASES:
    r = m.Renderer(m.select_scene(sid, 1.0), 0)
    out = {}
    for num in ("exact", "fast"):
        d = m.render_desc(w, h, spp, numerics=num, flags=m._lib.RF_PATH_DEBUG)
        _, rays = r.render(d)
        ns = d.sqrt_samples ** 2
        out[num] = r.paths(len(m.local_pixels(d)) * ns) + (rays,)
    (a, ar, at), (b, br, bt) = out["exact"], out["fast"]
    a = a.reshape(-1, 3).astype(np.float64)
    b = b.reshape(-1, 3).astype(np.float64)
    ok = np.isfinite(a).all(1) & np.isfinite(b).all(1)
    dd = np.abs(a - b).max(1)
    rel = dd / np.maximum(np.abs(a).max(1), 1e-3)
    div = (ar != br) | (rel > 1e-3) | ~ok
    d2 = float((((a - b) ** 2).sum(1))[ok].mean())
    print(json.dumps({"tag": tag, "config": name, "paths": int(a.shape[0]), "diverged_pct": round(100 * float(div.mean()), 5),
                      "rays_differ_pct": round(100 * float((ar != br).mean()), 5), "ray_ratio": round(bt / at, 6),
                      "D2": d2, "est_rmse_own_spp": round(float(np.sqrt(d2 / 3 / own)), 7)}), flush=True)
    r.close()
