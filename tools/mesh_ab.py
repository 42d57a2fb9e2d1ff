#!/usr/bin/env python3
"""Experiment: C3/C4/C5-shaped renders (fewer spp) per library variant (exp/libmrt_<tag>.so via
MRT_EXPERIMENT_LIB; 'intree' = the in-tree build): path-kernel ms per launch, both numerics slots.
  python tools/mesh_ab.py tag1 tag2 ..."""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CASES = os.environ.get("MESH_CASES", "9:800:800:1024 8:1024:1024:256 7:2048:2048:64")
CHILD = r'''
import json, os, sys
import numpy as np
sys.path.insert(0, ROOT)
import miniraytracer_amd as m
out = {}
for c in CASES.split():
    sid, w, h, spp = (int(x) for x in c.split(":"))
    r = m.Renderer(m.select_scene(sid, w / h), 0)
    for num in ("exact", "fast"):
        d = m.render_desc(w, h, spp, numerics=num)
        img, rays = r.render(d)
        ms = []
        for _ in range(2):
            r.render(d)
            t, n = r.kernel_ms()
            ms.append(t / n)
        out[f"s{sid}_{num}_ms"] = round(float(min(ms)), 2)
        out[f"s{sid}_{num}_grays"] = round(rays / min(ms) / 1e6, 3)
        out[f"s{sid}_{num}_rays"] = int(rays)
        out[f"s{sid}_{num}_sum"] = float(img[..., :3].astype(np.float64).sum())
    ki = r.kernel_info()
    out[f"s{sid}_vgprs"] = ki["vgprs"]
    out[f"s{sid}_tree"] = f"wg{ki['wg']}:t{ki['tree_nodes']}:lds{ki['lds_bytes']}:g{ki['grid']}"
print(json.dumps(out))
'''


def main():
    for tag in sys.argv[1:]:
        env = dict(os.environ)
        if tag != "intree":
            env["MRT_EXPERIMENT_LIB"] = os.path.join(ROOT, "exp", f"libmrt_{tag}.so")
        p = subprocess.run([sys.executable, "-c", f"ROOT={ROOT!r}\nCASES={CASES!r}\n" + CHILD], env=env,
                           capture_output=True, text=True, timeout=900)
        line = p.stdout.strip().splitlines()[-1] if p.stdout.strip() else p.stderr[-800:]
        print(json.dumps({"tag": tag, **(json.loads(line) if line.startswith("{") else {"error": line})}), flush=True)


if __name__ == "__main__":
    main()
