"""The two-level pod_bvh walk (Mesh4, miniraytracer_amd/csrc/mrt_trace.h, MRT_MESH4 kernels) against
the binary walk it replaces, on the host: both resumable steps (mesh_step) compiled for the CPU and
run to completion over random rays per mesh (mrt_debug_mesh4_walks, mrt_cpu.hip), one ray in four
not nice (a zero direction component, so the parents' boxes are tested too).  Bar: the same result,
t, triangle and barycentrics bit for bit on every ray -- the walk visits the reference's leaves in
pod_bvh::hit's order (triangle.h:171-221) -- and a stack never deeper than the bound the host
sizes LDS by."""
import ctypes as C

import numpy as np
import pytest


@pytest.mark.parametrize("sid", [8, 9])
def test_two_level_mesh_walk_equals_binary_walk(mrt, sid):
    sc = mrt.select_scene(sid, 1.0)
    fn = mrt.lib().mrt_debug_mesh4_walks
    fn.argtypes = [C.c_void_p, C.c_uint32, C.c_uint64, C.c_void_p]
    fn.restype = C.c_int
    out = np.zeros(5, dtype=np.uint64)
    assert fn(C.byref(sc.view), 20000, 12345, out.ctypes.data) == 0
    entered, hits, bad, deep, bound = (int(x) for x in out)
    assert entered > 5000 and hits > 1000, out
    assert bad == 0, out
    assert 0 < deep <= bound, out
    sc.close()
