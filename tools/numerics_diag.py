#!/usr/bin/env python3
"""Experiment: per-path comparison of the two numerics contracts on one scene (PATH_DEBUG renders):
writes gpurun_out/numdiag_<lib>.npz with per-path ray counts and radiance of both contracts."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import miniraytracer_amd as m  # noqa: E402

sid, w, h, spp = (int(x) for x in (sys.argv[1:5] if len(sys.argv) > 4 else (5, 96, 96, 256)))
tag = os.path.basename(os.environ.get("MRT_EXPERIMENT_LIB", "intree"))
r = m.Renderer(m.select_scene(sid, w / h), 0)
res = {}
for num in ("exact", "fast"):
    d = m.render_desc(w, h, spp, numerics=num, flags=m._lib.RF_PATH_DEBUG)
    img, rays = r.render(d)
    ns = d.sqrt_samples ** 2
    px = m.local_pixels(d)
    prgb, prays = r.paths(len(px) * ns)
    full_rgb = np.zeros((w * h, ns, 3), dtype=np.float32)
    full_rays = np.zeros((w * h, ns), dtype=np.uint32)
    full_rgb[px] = prgb.reshape(ns, len(px), 3).transpose(1, 0, 2)
    full_rays[px] = prays.reshape(ns, len(px)).T
    res[num + "_rgb"], res[num + "_rays"], res[num + "_img"] = full_rgb, full_rays, img
os.makedirs(os.path.join(ROOT, "gpurun_out"), exist_ok=True)
np.savez_compressed(os.path.join(ROOT, "gpurun_out", f"numdiag_{tag}_{sid}.npz"), **res)
dr = res["fast_rays"].astype(np.int64) - res["exact_rays"]
print(tag, "paths differing", int((dr != 0).sum()), "of", dr.size, "ray diff", int(dr.sum()))
