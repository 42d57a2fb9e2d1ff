#!/usr/bin/env python3
"""Count the non-finite per-path samples (main.cpp:162-164: `sample = color` when a component is
inf or NaN) of the tolerance-contract kernels on the BASELINE configs, from the per-path radiance
of MRT_RF_PATH_DEBUG renders (GPU).  Prints one JSON line per config.

    python tools/nonfinite_probe.py [--spp N] [--scenes 5,9,8,7]
"""
import argparse
import json
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import miniraytracer_amd as mrt  # noqa: E402

SIZES = {5: (500, 500), 9: (800, 800), 8: (1024, 1024), 7: (2048, 2048)}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--spp", type=int, default=256)
    ap.add_argument("--scenes", default="5,9,8,7")
    ap.add_argument("--numerics", default="fast")
    a = ap.parse_args()
    for sid in [int(x) for x in a.scenes.split(",")]:
        w, h = SIZES[sid]
        sc = mrt.select_scene(sid, w / h)
        r = mrt.Renderer(sc, 0)
        d = mrt.render_desc(w, h, a.spp, numerics=a.numerics, flags=mrt._lib.RF_PATH_DEBUG)
        _, rays = r.render(d)
        n = w * h * (int(a.spp ** 0.5) ** 2)
        rgb, _ = r.paths(n)
        bad = ~np.isfinite(rgb).all(axis=1)
        big = (np.abs(np.where(np.isfinite(rgb), rgb, 0)) > 2.0 ** 27).any(axis=1)
        print(json.dumps({"scene": sid, "w": w, "h": h, "spp": a.spp, "numerics": a.numerics, "paths": n, "rays": rays,
                          "nonfinite": int(bad.sum()), "above_2^27": int(big.sum()),
                          "max_finite": float(np.max(np.where(np.isfinite(rgb), rgb, 0)))}), flush=True)
        del rgb, bad, big
        r.close()


if __name__ == "__main__":
    main()
