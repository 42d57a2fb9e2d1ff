"""Experiment: wave timeline of one path-kernel launch (needs an experiment build with -DMRT_WTIMES,
loaded through MRT_EXPERIMENT_LIB).  Per wave: start, pool exhausted, end (s_memrealtime, 100 MHz).
Prints, in microseconds from the first wave's start: the spread of wave starts (dispatch ramp),
when the waves found the work handed out, and when they ended (the tail).
  python tools/wtimes.py [scene W H spp ...]   (several spp values: one launch each)"""
import ctypes as C
import os
import sys
import numpy as np
sys.path.insert(0, ".")
import miniraytracer_amd as m
from miniraytracer_amd._lib import lib

args = [int(a) for a in sys.argv[1:]] or [5, 500, 500, 16, 128, 1024]
scene, w, h, spps = args[0], args[1], args[2], args[3:]
sc = m.select_scene(scene, w / h)
r = m.Renderer(sc, 0)
NW = 16384
buf = (C.c_ulonglong * (7 * NW))()
for spp in spps:
    d = m.render_desc(w, h, spp, depth=int(os.environ.get("DEPTH", "32")), numerics=os.environ.get("NUMERICS", "fast"))
    r.render(d)
    C.memset(buf, 0, C.sizeof(buf))
    img, rays = r.render(d)
    if lib().mrt_debug_wtimes(buf, NW):
        raise SystemExit("mrt_debug_wtimes failed")
    a = np.frombuffer(buf, dtype=np.uint64).reshape(NW, 7).astype(np.int64)
    a = a[a[:, 0] != 0]
    t0 = a[:, 0].min()
    st, ex, en = (a[:, 0] - t0) / 100.0, (a[:, 1] - t0) / 100.0, (a[:, 2] - t0) / 100.0
    ex = np.where(a[:, 1] != 0, ex, np.nan)
    q = lambda x: " ".join(f"{np.nanpercentile(x, p):8.1f}" for p in (0, 10, 50, 90, 99, 100))
    print(f"scene {scene} {w}x{h}x{spp}: rays {rays}, waves {len(a)}  (percentiles 0/10/50/90/99/100, us)")
    print(f"  start      {q(st)}")
    print(f"  exhausted  {q(ex)}")
    print(f"  end        {q(en)}")
    print(f"  end-exh    {q(en - ex)}")
    ff = np.where((a[:, 3] >> 20) != 0, st + (a[:, 3] >> 20) / 100.0, np.nan)
    print(f"  first fail {q(ff)}")
    print(f"  exh-fail   {q(ex - ff)}")
    nok, nfail = a[:, 6] & 0xFFFFFFFF, a[:, 6] >> 32
    print(f"  claim atomics per wave: ok {nok.mean():.1f}, failed {nfail.mean():.1f}; mean latency ok "
          f"{a[:, 4].sum() / max(nok.sum(), 1) / 100:.2f} us, failed {a[:, 5].sum() / max(nfail.sum(), 1) / 100:.2f} us")
    print(f"  time in failed atomics per wave {q(a[:, 5] / 100.0)}")
    print(f"  time in ok atomics per wave     {q(a[:, 4] / 100.0)}")
    xcd = (a[:, 3] & 0xFFFFF) % 8
    print("  per XCD (by workgroup % 8) last end: " + " ".join(f"{en[xcd == k].max():.1f}" for k in range(8)))
    print("  per XCD median exhausted:            " + " ".join(f"{np.nanmedian(ex[xcd == k]):.1f}" for k in range(8)))
