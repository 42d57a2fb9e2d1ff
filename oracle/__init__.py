"""oracle -- TEST INFRASTRUCTURE ONLY.

Parity checkers for the MI355X render path.  Importable only by tests/, __graft_entry__.smoke()
and bench.py's cpu_baseline leg; never by the product package (miniraytracer_amd).

* ``liboracle.so`` (oracle/mrt_oracle.c): plain-C restatement of the reference render path,
  consuming the same flattened scene (mrt_scene_view) the GPU consumes.
* ``_ref/mrt_ref`` / ``_ref/mrt_ref_exact``: the reference's own code built by
  oracle/ref/build_ref.sh from /root/reference (only where that tree exists; the binaries travel
  to the GPU box as build outputs).
"""
import ctypes as C
import json
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(HERE, "liboracle.so")
REF_DIR = os.path.join(HERE, "_ref")


class OracleDesc(C.Structure):
    _fields_ = [("width", C.c_uint32), ("height", C.c_uint32), ("sqrt_samples", C.c_uint32),
                ("max_bounces", C.c_uint32), ("max_luminance", C.c_float), ("mode", C.c_uint32),
                ("seed", C.c_uint64), ("threads", C.c_uint32), ("y0", C.c_uint32), ("y1", C.c_uint32)]


_lib = None


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise RuntimeError(f"{LIB_PATH} not built (make oracle/liboracle.so)")
        L = C.CDLL(LIB_PATH)
        L.oracle_render.argtypes = [C.c_void_p, C.POINTER(OracleDesc), C.c_void_p, C.c_void_p, C.c_void_p]
        L.oracle_render.restype = C.c_uint64
        L.oracle_path.argtypes = [C.c_void_p, C.POINTER(OracleDesc), C.c_uint32, C.c_uint32, C.c_uint32, C.c_void_p]
        L.oracle_path.restype = C.c_uint32
        L.oracle_hit.argtypes = [C.c_void_p, C.c_void_p, C.c_void_p, C.c_float, C.c_int, C.c_uint64, C.c_void_p]
        L.oracle_hit.restype = C.c_int
        L.oracle_render_ref_order.argtypes = [C.c_void_p, C.POINTER(OracleDesc), C.c_uint32, C.c_uint64, C.c_uint64, C.c_void_p]
        L.oracle_render_ref_order.restype = C.c_uint64
        L.oracle_pcg_stream.argtypes = [C.c_uint64, C.c_uint64, C.c_uint32, C.c_void_p]
        L.oracle_samplers.argtypes = [C.c_uint64, C.c_uint64, C.c_uint32, C.c_uint32, C.c_void_p]
        _lib = L
    return _lib


def desc(width, height, samples, depth=32, max_luminance=1000.0, mode=0, seed=11350390909718046443, threads=1,
         y0=0, y1=0):
    sq = int(np.sqrt(np.float32(samples)))
    return OracleDesc(width, height, sq, depth, max_luminance, mode, seed, threads, y0, y1)


def render(scene, d, paths=False):
    """Render with the C restatement. scene: miniraytracer_amd.Scene (its mrt_scene_view)."""
    img = np.zeros((d.height, d.width, 4), dtype=np.float32)
    ns = d.sqrt_samples ** 2
    prgb = np.zeros((d.height * d.width * ns, 3), dtype=np.float32) if paths else None
    prays = np.zeros(d.height * d.width * ns, dtype=np.uint32) if paths else None
    rays = lib().oracle_render(C.byref(scene.view), C.byref(d), img.ctypes.data,
                               prgb.ctypes.data if paths else None, prays.ctypes.data if paths else None)
    return img, rays, prgb, prays


def render_ref_order(scene, d, tile_size=32):
    """The reference's own deterministic mode (-threads 1): one worker stream seeded as main() seeds
    worker 0 (main.cpp:357-361), work_queue tile order, draw() (mode 0) / draw2() (mode 1).
    Returns (image [H, W, 4], rays)."""
    img = np.zeros((d.height, d.width, 4), dtype=np.float32)
    st, sq = scene.worker_seeds(1)[0]
    rays = lib().oracle_render_ref_order(C.byref(scene.view), C.byref(d), tile_size, st, sq, img.ctypes.data)
    return img, rays


def hit(scene, o, d, time, inside, seed=0):
    o = np.ascontiguousarray(o, dtype=np.float32)
    d = np.ascontiguousarray(d, dtype=np.float32)
    out = np.zeros(7, dtype=np.float32)
    h = lib().oracle_hit(C.byref(scene.view), o.ctypes.data, d.ctypes.data, float(time), int(inside), int(seed), out.ctypes.data)
    return bool(h), out


def pcg_stream(st, sq, n):
    out = np.zeros(n, dtype=np.uint32)
    lib().oracle_pcg_stream(st, sq, n, out.ctypes.data)
    return out


def samplers(st, sq, n, which):
    out = np.zeros((n, 3), dtype=np.float32)
    lib().oracle_samplers(st, sq, n, which, out.ctypes.data)
    return out


# ---- the reference binary (oracle/_ref) ----
def ref_binary(exact=True, name=None):
    p = os.path.join(REF_DIR, name or ("mrt_ref_exact" if exact else "mrt_ref"))
    return p if os.path.exists(p) else None


def run_ref(args, exact=True, cwd=None, timeout=3600, name=None):
    """Run the reference oracle binary (or the build `name` in oracle/_ref); returns the parsed JSON
    of its last stdout line."""
    b = ref_binary(exact, name)
    if b is None:
        raise FileNotFoundError("oracle/_ref not built")
    out = subprocess.run([b] + [str(a) for a in args], capture_output=True, text=True, cwd=cwd, timeout=timeout,
                         check=True).stdout
    return json.loads(out.strip().splitlines()[-1])
