#!/usr/bin/env python3
"""Experiment: the samples of a few pixels (array coordinates x,y of the image r.render returns)
whose path radiance is non-finite under each numerics contract (MRT_RF_PATH_DEBUG renders of a pixel
list, GPU), each with the other contract's radiance for the same sample and both paths' ray counts:
which of the reference's non-finite samples (main.cpp:162-164 doubles the running colour for them)
the fast arithmetic misses or adds.
    python tools/nonfinite_pixels.py sid w h spp x,y [x,y ...]   -> one JSON line per pixel"""
import json
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import miniraytracer_amd as mrt  # noqa: E402

sid, w, h, spp = (int(x) for x in sys.argv[1:5])
xy = [tuple(int(v) for v in a.split(",")) for a in sys.argv[5:]]
pix = np.array([y * w + x for x, y in xy], np.uint32)
r = mrt.Renderer(mrt.select_scene(sid, w / h), 0)
res = {}
for num in ("exact", "fast"):
    d = mrt.render_desc(w, h, spp, numerics=num, flags=mrt._lib.RF_PATH_DEBUG, pixels=pix)
    r.render(d)
    ns = d.sqrt_samples ** 2
    rgb, rays = r.paths(len(pix) * ns)
    res[num] = (rgb.reshape(ns, len(pix), 3), rays.reshape(ns, len(pix)))
for k, (x, y) in enumerate(xy):
    out = {"scene": sid, "x": x, "y": y}
    for a, b in (("exact", "fast"), ("fast", "exact")):
        ra, na = res[a][0][:, k], res[a][1][:, k]
        rb, nb = res[b][0][:, k], res[b][1][:, k]
        bad = np.nonzero(~np.isfinite(ra).all(axis=1))[0]
        out[a] = [{"s": int(s), "rays": int(na[s]), "other": [float(v) for v in rb[s]], "other_rays": int(nb[s])} for s in bad]
    print(json.dumps(out), flush=True)
r.close()
