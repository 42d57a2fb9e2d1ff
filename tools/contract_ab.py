#!/usr/bin/env python3
"""Numerics-contract A/B (DESIGN.md "Numerics contracts"): for C2-C5, the exact contract (bit-for-bit
the reference built exact) against the tolerance contract (FMA contraction, hardware rcp/sqrt/rsq,
f32 transcendentals, forward fold), each priced by
  * Grays/s of the path kernel (HIP events, tools/mesh_ab.py protocol; C5 at 256 spp of 8100: the
    per-ray rate does not depend on spp),
  * VALU wave-instructions and active-lane instructions per ray (rocprofv3 SQ counters of the same
    workloads, profiles/<tag>_pmc.json from tools/profile.sh / tools/prof_configs.sh),
  * per-pixel RMSE and ray-count ratio against the reference AS SHIPPED on the same per-path streams
    (tests/golden: C2 shipped_stream_5.npz, the whole image; C3-C5 shipped_full_<id>.npz, full
    resolution at 1024 spp, per-pixel RMSE over a band of rows + a seeded pixel sample,
    tests/fixture_cmp.py).

  python tools/contract_ab.py --measure                   (GPU box) -> gpurun_out/contract_ab_measure.json
  python tools/contract_ab.py --summarize TAG [PMC ...]   -> profiles/TAG_contract_ab.json (+ table)"""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CASES = {"C2": (5, 500, 500, 1024), "C3": (9, 800, 800, 1024), "C4": (8, 1024, 1024, 256), "C5": (7, 2048, 2048, 256)}
FIXTURE = {"C2": "shipped_stream_5.npz", "C3": "shipped_full_9.npz", "C4": "shipped_full_8.npz", "C5": "shipped_full_7.npz"}


def measure():
    import numpy as np
    sys.path.insert(0, ROOT)
    import miniraytracer_amd as m
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    from fixture_cmp import compare
    out = {}
    for name, (sid, w, h, spp) in CASES.items():
        r = m.Renderer(m.select_scene(sid, w / h), 0)
        g = np.load(os.path.join(ROOT, "tests", "golden", FIXTURE[name]))
        meta = [int(x) for x in g["meta"]]
        fw, fh, fspp, fdepth = meta[1], meta[2], meta[3], meta[4]
        rf = m.Renderer(m.select_scene(sid, fw / fh), 0) if (fw, fh) != (w, h) else r
        for num in ("exact", "fast"):
            d = m.render_desc(w, h, spp, numerics=num)
            _, rays = r.render(d)
            ms = []
            for _ in range(2):
                r.render(d)
                t, n = r.kernel_ms()
                ms.append(t)
            img, frays = rf.render(m.render_desc(fw, fh, fspp, depth=fdepth, numerics=num))
            c = compare(img, frays, os.path.join(ROOT, "tests", "golden", FIXTURE[name]))
            out[f"{name}_{num}"] = {"grays": round(rays / min(ms) / 1e6, 3), "kernel_ms": round(min(ms), 3), "rays": int(rays),
                                    "rmse": c["rmse"], "ray_ratio": c["ray_ratio"] - 1, "block_rmse": c["block_rmse"],
                                    "fixture": f"{FIXTURE[name]} ({fw}x{fh}, {fspp} spp; {c['over']})"}
            print(name, num, out[f"{name}_{num}"], flush=True)
    os.makedirs(os.path.join(ROOT, "gpurun_out"), exist_ok=True)
    json.dump(out, open(os.path.join(ROOT, "gpurun_out", "contract_ab_measure.json"), "w"), indent=1)


def summarize(tag, pmcs):
    meas = json.load(open(os.path.join(ROOT, "gpurun_out", "contract_ab_measure.json")))
    cfg_of = {(5, 500, 500): "C2", (9, 800, 800): "C3", (8, 1024, 1024): "C4", (7, 2048, 2048): "C5"}
    inst = {}
    for p in pmcs:
        d = json.load(open(p))
        wc = d["workload_config"]
        name = cfg_of.get(tuple(wc[:3]))
        for k, e in d["kernels"].items():
            num = "fast" if k.endswith("_fast") else "exact"
            sq = e.get("sq") or {}
            rays = e.get("rays_per_launch")
            if name and sq and rays:
                inst[f"{name}_{num}"] = {"valu_wave_inst_per_ray": sq["SQ_INSTS_VALU"] / rays,
                                         "valu_lane_inst_per_ray": sq["SQ_THREAD_CYCLES_VALU"] / rays,  # active lanes summed over VALU instructions
                                         "valu_lane_util": e.get("valu_lane_util"), "pmc": os.path.relpath(p, ROOT)}
    res = {}
    print(f"{'config':6s} {'contract':8s} {'Grays/s':>8s} {'wave-inst/ray':>13s} {'lane-inst/ray':>13s} {'RMSE vs shipped':>15s} {'rays vs shipped':>15s}")
    for key in sorted(meas):
        r = dict(meas[key], **inst.get(key, {}))
        res[key] = r
        name, num = key.split("_")
        print(f"{name:6s} {num:8s} {r['grays']:8.2f} {r.get('valu_wave_inst_per_ray', float('nan')):13.1f} "
              f"{r.get('valu_lane_inst_per_ray', float('nan')):13.0f} {r['rmse']:15.2e} {r['ray_ratio']:+15.2e}")
    json.dump(res, open(os.path.join(ROOT, "profiles", f"{tag}_contract_ab.json"), "w"), indent=1)


if __name__ == "__main__":
    ap = argparse.ArgumentParser()
    ap.add_argument("--measure", action="store_true")
    ap.add_argument("--summarize", metavar="TAG")
    ap.add_argument("pmc", nargs="*")
    a = ap.parse_args()
    if a.measure:
        measure()
    if a.summarize:
        summarize(a.summarize, a.pmc)
