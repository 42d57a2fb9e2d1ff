#!/usr/bin/env python3
"""Experiment: WHICH paths end non-finite (main.cpp:162-164 doubles the running colour for them)
under each numerics contract -- per-path radiance of MRT_RF_PATH_DEBUG renders (GPU), listed as
(x, y, sample, rays, r, g, b) -- and how many of the two contracts' lists coincide.  The exact
contract's list is the reference's own (its paths are the reference's bit for bit).
    python tools/nonfinite_paths.py sid:w:h:spp [...]   -> one JSON line per config
"""
import json
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import miniraytracer_amd as mrt  # noqa: E402

for spec in sys.argv[1:]:
    sid, w, h, spp = (int(x) for x in spec.split(":"))
    r = mrt.Renderer(mrt.select_scene(sid, w / h), 0)
    out = {"scene": sid, "w": w, "h": h, "spp": spp}
    keys = {}
    for num in ("exact", "fast"):
        d = mrt.render_desc(w, h, spp, numerics=num, flags=mrt._lib.RF_PATH_DEBUG)
        r.render(d)
        ns = d.sqrt_samples ** 2
        px = mrt.local_pixels(d)
        rgb, rays = r.paths(len(px) * ns)
        bad = np.nonzero(~np.isfinite(rgb).all(axis=1))[0]
        sl, lp = np.divmod(bad, len(px))  # [s][local pixel]
        pix = px[lp]
        keys[num] = set(zip(pix.tolist(), sl.tolist()))
        out[num] = [[int(p % w), int(p // w), int(s), int(rays[i]), *[float(v) for v in rgb[i]]] for p, s, i in zip(pix, sl, bad)]
        del rgb, rays
    out["both"] = len(keys["exact"] & keys["fast"])
    print(json.dumps(out), flush=True)
    r.close()
