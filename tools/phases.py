"""Experiment: per-phase wave time of the path kernel (needs a -DMRT_PHASES build at
miniraytracer_amd/libmrt.so).  Prints the share of s_memtime cycles per phase."""
import ctypes as C
import sys
import numpy as np
sys.path.insert(0, ".")
import miniraytracer_amd as m
from miniraytracer_amd._lib import lib
scene, w, h, spp = (int(a) for a in (sys.argv[1:] + ["5", "500", "500", "256"])[:4])
sc = m.select_scene(scene, w / h)
r = m.Renderer(sc, 0)
d = m.render_desc(w, h, spp, numerics=__import__("os").environ.get("NUMERICS", "exact"))
r.render(d)
NPH = int(__import__("os").environ.get("NPH", "12"))
out = (C.c_ulonglong * NPH)()
lib().mrt_debug_phases(out, 1)
img, rays = r.render(d)
lib().mrt_debug_phases(out, 1)
v = np.array(list(out), dtype=np.float64)
names = ["loop+pool", "hit:record", "shade:pdf+lev", "write+bottom", "new path", "fold", "shade:mat+dir", "-", "make_ray|hit:list/inst", "hit:prim", "hit:volume", "hit:bvh"][:NPH]
print(f"scene {scene} {w}x{h}x{spp}: rays {rays}")
for n, x in zip(names, v):
    print(f"  {n:12s} {100 * x / v.sum():6.2f}%")
