import gzip
import json
import os
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
GOLDEN = os.path.join(ROOT, "tests", "golden")
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs the HIP render path)")


SCENE_SIZES = {0: (200, 100), 1: (200, 100), 2: (200, 100), 3: (200, 100), 4: (200, 100), 5: (500, 500),
               6: (500, 500), 7: (2048, 2048), 8: (1024, 1024), 9: (800, 800)}


def golden_stream(name):
    g = np.load(os.path.join(GOLDEN, name))
    sid, w, h, spp, depth, mode, rays = (int(x) for x in g["meta"])
    return dict(sid=sid, w=w, h=h, spp=spp, depth=depth, mode=mode, rays=rays, image=g["image"],
                path_rgb=g["path_rgb"], path_rays=g["path_rays"])


def golden_scene(sid):
    with gzip.open(os.path.join(GOLDEN, f"scene_{sid}.json.gz"), "rt") as f:
        return json.load(f)


def canon_scene(o):
    """Blob dump schema -> fixture schema (see tools/make_golden.py)."""
    if isinstance(o, dict):
        if o.get("k") == "pod_bvh":
            o = dict(o)
            o["nodes"] = [[b, l, order] if c == 0 else [b, off, c] for b, l, off, c, order in o["nodes"]]
        return {k: canon_scene(v) for k, v in o.items() if k not in ("perlin_ranvec", "perlin_perm")}
    if isinstance(o, list):
        return [canon_scene(x) for x in o]
    return o


@pytest.fixture(scope="session")
def mrt():
    import miniraytracer_amd
    return miniraytracer_amd


@pytest.fixture(scope="session")
def orc():
    import oracle
    return oracle
