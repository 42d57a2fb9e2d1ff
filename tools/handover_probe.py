#!/usr/bin/env python3
"""Experiment: single-pixel renders of the tolerance contract (the fast kernel's hand-over of
rounding-critical paths on) -- how many of the pixel's paths were handed over
(mrt_kernel_info.handed_over) and the pixel against the exact contract and, when given, a
whole-image fixture of the reference as shipped.
    python tools/handover_probe.py sid w h spp [fixture.npz] x,y [x,y ...]  -> one JSON line per pixel"""
import json
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import miniraytracer_amd as mrt  # noqa: E402

sid, w, h, spp = (int(x) for x in sys.argv[1:5])
rest = sys.argv[5:]
ref = None
if rest and rest[0].endswith(".npz"):
    ref = np.load(rest[0])["image"][..., :3].reshape(h, w, 3)
    rest = rest[1:]
r = mrt.Renderer(mrt.select_scene(sid, w / h), 0)
for a in rest:
    x, y = (int(v) for v in a.split(","))
    px = np.array([y * w + x], np.uint32)
    out = {"scene": sid, "x": x, "y": y}
    for num in ("fast", "exact"):
        before = r.kernel_info()["handed_over"]
        img, _ = r.render(mrt.render_desc(w, h, spp, numerics=num, pixels=px))
        out[num] = [float(v) for v in img[y, x, :3]]
        out[num + "_handed_over"] = r.kernel_info()["handed_over"] - before
    if ref is not None:
        out["ref"] = [float(v) for v in ref[y, x]]
    print(json.dumps(out), flush=True)
r.close()
