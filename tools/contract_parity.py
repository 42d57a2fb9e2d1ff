#!/usr/bin/env python3
"""Experiment: one numerics-contract build (MRT_EXPERIMENT_LIB, tools/build_variant.sh; default the
in-tree library) against the reference as shipped at every BASELINE config's own spp -- C2 whole
image (shipped_stream_5.npz), C3 / C4 / C5 pixel lists (shipped_ownspp_<id>.npz) -- with the path
kernel's time (median of 3 renders) of C2 at full size and the paths the fast kernel handed over
to the exact arithmetic per render.  One JSON line per (config, numerics).
  python tools/contract_parity.py [fast|exact ...]"""
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
import miniraytracer_amd as m  # noqa: E402
from fixture_cmp import compare, compare_pixels  # noqa: E402

tag = os.path.basename(os.environ.get("MRT_EXPERIMENT_LIB", "intree")).replace(".so", "").replace("libmrt_", "")
G = os.path.join(ROOT, "tests", "golden")
for num in sys.argv[1:] or ["fast"]:
    r = m.Renderer(m.select_scene(5, 1.0), 0)
    d = m.render_desc(500, 500, 1024, numerics=num)
    ms = []
    for _ in range(3):
        img, rays = r.render(d)
        t, n = r.kernel_ms()
        ms.append(t / n)
    c = compare(img, rays, os.path.join(G, "shipped_stream_5.npz"))
    print(json.dumps({"tag": tag, "numerics": num, "config": "C2", "kernel_ms": round(float(np.median(ms)), 3),
                      "grays": round(rays / np.median(ms) / 1e6, 2), "handed_over": r.kernel_info()["handed_over"] // 3, **c}), flush=True)
    r.close()
    # C3 over the whole image at its own spp (shipped_ownspp_full_9.npz); images kept for analysis
    g = os.path.join(G, "shipped_ownspp_full_9.npz")
    _, w, h, spp, depth = (int(x) for x in np.load(g)["meta"])
    r = m.Renderer(m.select_scene(9, w / h), 0)
    img, rays = r.render(m.render_desc(w, h, spp, depth=depth, numerics=num))
    t, n = r.kernel_ms()
    c = compare(img, rays, g)
    if os.environ.get("MRT_PARITY_SAVE"):
        np.save(os.path.join(os.environ["MRT_PARITY_SAVE"], f"c3full_{tag}_{num}.npy"), img[..., :3])
    print(json.dumps({"tag": tag, "numerics": num, "config": "C3 whole image", "kernel_ms": round(t, 3),
                      "grays": round(rays / t / 1e6, 2), "handed_over": r.kernel_info()["handed_over"], **c}), flush=True)
    r.close()
    for sid in (9, 8, 7):
        g = np.load(os.path.join(G, f"shipped_ownspp_{sid}.npz"))
        _, w, h, spp, depth = (int(x) for x in g["meta"])
        r = m.Renderer(m.select_scene(sid, w / h), 0)
        img, rays = r.render(m.render_desc(w, h, spp, depth=depth, numerics=num, pixels=g["pixels"]))
        t, n = r.kernel_ms()
        c = compare_pixels(img, rays, g)
        print(json.dumps({"tag": tag, "numerics": num, "config": {9: "C3", 8: "C4", 7: "C5"}[sid], "kernel_ms": round(t, 3),
                          "grays": round(rays / t / 1e6, 2), "handed_over": r.kernel_info()["handed_over"], **c}), flush=True)
        r.close()
