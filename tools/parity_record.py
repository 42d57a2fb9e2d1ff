#!/usr/bin/env python3
"""Parity of the full BASELINE workloads on the GPU against the reference AS SHIPPED on the same
per-path streams, under both numerics contracts -> one JSON record (profiles/r03_parity.json).

Fixtures (tests/golden, tools/make_golden.py): C2 shipped_stream_5.npz (whole 500x500 image,
1024 spp); C3 / C4 / C5 shipped_full_<id>.npz (full resolution, 1024 spp: block means, channel means,
a band of rows, a seeded pixel sample) and shipped_ownspp_<id>.npz (the configs' own spp, a pixel
list).  The same comparisons as tests/fixture_cmp.py, which the GPU tests assert on.

Usage (GPU box): python tools/parity_record.py [--out gpurun_out/parity.json] [--scenes 5,9,8,7]
"""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--out", default=os.path.join(ROOT, "gpurun_out", "parity.json"))
    ap.add_argument("--scenes", default="5,9,8,7")
    ap.add_argument("--numerics", default="exact,fast")
    a = ap.parse_args()
    import miniraytracer_amd as m
    from fixture_cmp import GOLDEN, compare, compare_pixels
    rec = {"what": "GPU render vs the reference as shipped, same per-path streams", "configs": []}
    for sid in (int(x) for x in a.scenes.split(",")):
        path = os.path.join(GOLDEN, f"shipped_stream_{sid}.npz" if sid == 5 else f"shipped_full_{sid}.npz")
        g = np.load(path)
        _, w, h, spp, depth = (int(x) for x in g["meta"])
        r = m.Renderer(m.select_scene(sid, w / h), device=0)
        for numerics in a.numerics.split(","):
            t0 = time.perf_counter()
            img, rays = r.render(m.render_desc(w, h, spp, depth=depth, numerics=numerics))
            dt = time.perf_counter() - t0
            c = compare(img, rays, path)
            c.update(scene=sid, width=w, height=h, numerics=numerics, rays=int(rays), render_s=round(dt, 3),
                     kernel_features=r.kernel_info()["kernel_features"])
            rec["configs"].append(c)
            print(json.dumps(c), flush=True)
        own = os.path.join(GOLDEN, f"shipped_ownspp_{sid}.npz")
        if os.path.exists(own):
            g = np.load(own)
            _, w, h, spp, depth = (int(x) for x in g["meta"])
            for numerics in a.numerics.split(","):
                img, rays = r.render(m.render_desc(w, h, spp, depth=depth, numerics=numerics, pixels=g["pixels"]))
                c = compare_pixels(img, rays, g)
                c.update(scene=sid, width=w, height=h, numerics=numerics, rays=int(rays), own_spp=True)
                rec["configs"].append(c)
                print(json.dumps(c), flush=True)
        r.close()
    os.makedirs(os.path.dirname(a.out), exist_ok=True)
    json.dump(rec, open(a.out, "w"), indent=1)


if __name__ == "__main__":
    main()
