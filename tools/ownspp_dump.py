#!/usr/bin/env python3
"""Experiment / record: render the pixel lists of tests/golden/shipped_ownspp_<id>.npz (the BASELINE
configs C3 / C4 / C5 at their own spp) under both numerics contracts and write the GPU values to
gpurun_out/ownspp_<tag>.npz (with the fixture values beside them) plus a summary line per render.
  python tools/ownspp_dump.py [scene ids]      (MRT_EXPERIMENT_LIB selects an A/B build)"""
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
import miniraytracer_amd as m  # noqa: E402
from fixture_cmp import compare_pixels  # noqa: E402

tag = os.path.basename(os.environ.get("MRT_EXPERIMENT_LIB", "intree")).replace(".so", "")
sids = [int(a) for a in sys.argv[1:]] or [9, 8, 7]
numerics = os.environ.get("MRT_OWNSPP_NUMERICS", "exact,fast").split(",")
out = {}
for sid in sids:
    g = np.load(os.path.join(ROOT, "tests", "golden", f"shipped_ownspp_{sid}.npz"))
    _, w, h, spp, depth = (int(x) for x in g["meta"])
    r = m.Renderer(m.select_scene(sid, w / h), 0)
    out[f"s{sid}_ref"] = g["values"]
    out[f"s{sid}_pixels"] = g["pixels"]
    for num in numerics:
        t0 = time.perf_counter()
        img, rays = r.render(m.render_desc(w, h, spp, depth=depth, numerics=num, pixels=g["pixels"]))
        dt = time.perf_counter() - t0
        out[f"s{sid}_{num}"] = img.reshape(-1, 4)[g["pixels"], :3].copy()
        c = compare_pixels(img, rays, g)
        print(json.dumps({"tag": tag, "numerics": num, "seconds": round(dt, 3), **c}), flush=True)
    r.close()
os.makedirs(os.path.join(ROOT, "gpurun_out"), exist_ok=True)
np.savez_compressed(os.path.join(ROOT, "gpurun_out", f"ownspp_{tag}.npz"), **out)
