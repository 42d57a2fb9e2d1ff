"""Experiment: branch occupancy of the path kernel (needs an exp build with -DMRT_BSTATS, loaded via
MRT_EXPERIMENT_LIB).  Per counting point: wave executions, lanes counted, lanes per execution."""
import ctypes as C
import os
import sys
import numpy as np
sys.path.insert(0, ".")
import miniraytracer_amd as m
from miniraytracer_amd._lib import lib
scene, w, h, spp = (int(a) for a in (sys.argv[1:] + ["5", "500", "500", "64"])[:4])
sc = m.select_scene(scene, w / h)
r = m.Renderer(sc, 0)
d = m.render_desc(w, h, spp, numerics=os.environ.get("NUMERICS", "fast"))
out = (C.c_ulonglong * 64)()
lib().mrt_debug_bstats(out, 1)
img, rays = r.render(d)
lib().mrt_debug_bstats(out, 1)
v = np.array(list(out), dtype=np.float64).reshape(32, 2)
names = {0: "shade entry", 1: "miss", 2: "light", 3: "depth end", 4: "metal", 5: "dielectric", 6: "diffuse",
         7: "diffuse: light-sampled (cond)", 8: "instance reached (cond in)", 9: "instance body (cond in)",
         10: "new path", 11: "box6 reached (cond in)", 12: "make_ray (cond finish_scatter)", 14: "shade entry (cond hit)",
         15: "make_ray reached (cond active)"}
print(f"scene {scene} {w}x{h}x{spp}: rays {rays}")
for i, (ex, ln) in enumerate(v):
    if ex:
        print(f"  {i:2d} {names.get(i, '?'):34s} exec {ex:12.0f}  lanes {ln:14.0f}  lanes/exec {ln / ex:6.2f}  per ray: exec {ex / rays:.4f} lanes {ln / rays:.4f}")
