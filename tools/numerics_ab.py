#!/usr/bin/env python3
"""Experiment: tolerance-contract variants (exp/libmrt_<tag>.so, tools/build_variant.sh) against the
reference as shipped on the shipped_stream fixtures: ray-count ratio and per-pixel RMSE, plus the
C2 kernel time.  One subprocess per library (ctypes loads one libmrt per process).
  python tools/numerics_ab.py tag1 tag2 ...      (tag 'intree' = miniraytracer_amd/libmrt.so)"""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

CHILD = r'''
import json, os, sys, time
import numpy as np
sys.path.insert(0, ROOT)
import miniraytracer_amd as m
out = {}
for sid in (5, 8, 7):
    g = np.load(os.path.join(ROOT, "tests", "golden", f"shipped_stream_{sid}_small.npz"))
    _, w, h, spp, depth = (int(x) for x in g["meta"])
    r = m.Renderer(m.select_scene(sid, w / h), 0)
    img, rays = r.render(m.render_desc(w, h, spp, depth=depth, numerics="fast"))
    d = img[..., :3].astype(np.float64) - g["image"]
    out[f"s{sid}_rays_ratio"] = round(rays / float(g["rays"][0]) - 1, 6)
    out[f"s{sid}_rmse"] = round(float(np.sqrt((d ** 2).mean())), 6)
    out[f"s{sid}_dmean"] = round(float(d.mean()), 7)
g = np.load(os.path.join(ROOT, "tests", "golden", "shipped_stream_5.npz"))
r = m.Renderer(m.select_scene(5, 1.0), 0)
d = m.render_desc(500, 500, 1024, numerics="fast")
img, rays = r.render(d)
out["c2_rays_ratio"] = round(rays / float(g["rays"][0]) - 1, 6)
out["c2_rmse"] = round(float(np.sqrt(((img[..., :3].astype(np.float64) - g["image"]) ** 2).mean())), 7)
ms = []
for _ in range(3):
    r.render(d)
    t, n = r.kernel_ms()
    ms.append(t / n)
out["c2_kernel_ms"] = round(float(np.median(ms)), 3)
out["vgprs"] = r.kernel_info()["vgprs"]
print(json.dumps(out))
'''


def main():
    for tag in sys.argv[1:]:
        env = dict(os.environ)
        if tag != "intree":
            env["MRT_EXPERIMENT_LIB"] = os.path.join(ROOT, "exp", f"libmrt_{tag}.so")
        p = subprocess.run([sys.executable, "-c", "ROOT=%r\n" % ROOT + CHILD], env=env, capture_output=True, text=True,
                           timeout=600)
        line = p.stdout.strip().splitlines()[-1] if p.stdout.strip() else p.stderr[-500:]
        print(json.dumps({"tag": tag, **(json.loads(line) if line.startswith("{") else {"error": line})}), flush=True)


if __name__ == "__main__":
    main()
