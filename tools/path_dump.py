#!/usr/bin/env python3
"""Experiment: per-path radiance and ray counts of GPU renders (MRT_RF_PATH_DEBUG), in the harness's
stream layout (path k = pixel * ns + s), for comparison with the reference builds' --h-paths dumps
(numerics diagnosis).  Writes gpurun_out/paths_<tag>_<sid>_<numerics>.npz.
  python tools/path_dump.py sid:w:h:spp [...]     (MRT_EXPERIMENT_LIB selects an A/B build;
                                                    MRT_DUMP_NUMERICS=exact,fast by default)"""
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import miniraytracer_amd as m  # noqa: E402

tag = os.path.basename(os.environ.get("MRT_EXPERIMENT_LIB", "intree")).replace(".so", "").replace("libmrt_", "")
os.makedirs(os.path.join(ROOT, "gpurun_out"), exist_ok=True)
for spec in sys.argv[1:]:
    sid, w, h, spp = (int(x) for x in spec.split(":"))
    r = m.Renderer(m.select_scene(sid, w / h), 0)
    for num in os.environ.get("MRT_DUMP_NUMERICS", "exact,fast").split(","):
        d = m.render_desc(w, h, spp, numerics=num, flags=m._lib.RF_PATH_DEBUG)
        _, rays = r.render(d)
        ns = d.sqrt_samples ** 2
        px = m.local_pixels(d)
        prgb, prays = r.paths(len(px) * ns)
        rgb = np.zeros((w * h, ns, 3), dtype=np.float32)
        pr = np.zeros((w * h, ns), dtype=np.uint32)
        rgb[px] = prgb.reshape(ns, len(px), 3).transpose(1, 0, 2)
        pr[px] = prays.reshape(ns, len(px)).T
        cmp_dir = os.environ.get("MRT_DUMP_CMP")  # compare with the reference builds' dumps there
        if cmp_dir:
            for b in ("mrt_ref", "mrt_ref_exact"):
                base = os.path.join(cmp_dir, f"s_{b}_{sid}")
                if not os.path.exists(base + ".rgb.npy"):
                    continue
                ref = np.load(base + ".rgb.npy").astype(np.float64)
                rr = np.load(base + ".rays.npy")
                x = rgb.reshape(-1, 3).astype(np.float64)
                dd = np.abs(x - ref).max(1)
                rel = dd / np.maximum(np.abs(ref).max(1), 1e-6)
                print(json.dumps({"tag": tag, "scene": sid, "numerics": num, "vs": b, "paths": int(dd.size),
                                  "rays_differ_pct": round(100 * float((pr.reshape(-1) != rr).mean()), 5),
                                  "diverged_pct": round(100 * float((rel > 1e-3).mean()), 5),
                                  "bits_differ_pct": round(100 * float((dd > 0).mean()), 3),
                                  "ray_ratio": round(float(pr.sum()) / float(rr.sum()), 7)}), flush=True)
        else:
            np.savez_compressed(os.path.join(ROOT, "gpurun_out", f"paths_{tag}_{sid}_{num}.npz"), rgb=rgb.reshape(-1, 3),
                                rays=pr.reshape(-1))
        print(tag, sid, num, "rays", rays, flush=True)
    r.close()
