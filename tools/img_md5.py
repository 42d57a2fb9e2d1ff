#!/usr/bin/env python3
"""Experiment: md5 of a fast-contract image and its ray total (bit-identity checks of A/B builds:
MRT_EXPERIMENT_LIB).  python tools/img_md5.py sid w h spp"""
import hashlib
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import miniraytracer_amd as m  # noqa: E402

sid, w, h, spp = (int(x) for x in sys.argv[1:5])
img, rays = m.Renderer(m.select_scene(sid, w / h), 0).render(m.render_desc(w, h, spp, numerics=os.environ.get("MRT_NUMERICS", "fast")))
print(os.path.basename(os.environ.get("MRT_EXPERIMENT_LIB", "intree")), sid, rays, hashlib.md5(img.tobytes()).hexdigest(), flush=True)
