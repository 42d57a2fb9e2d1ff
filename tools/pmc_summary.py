#!/usr/bin/env python3
"""Summarise a tools/profile.sh run (gpurun_out/prof) into profiles/:

  profiles/<tag>_kernel_stats.csv   rocprofv3 --kernel-trace --stats summary (copied)
  profiles/<tag>_pmc.json           per-launch counters of every mrt_path_kernel build (exact /
                                    fast) + derived metrics, per-dispatch wave check
  profiles/pmc_s<scene>_<W>x<H>.json  what bench.py reads for its roofline (per-ray VALU
                                    wave-instructions and HBM bytes, lane utilisation, issue busy),
                                    keyed by the workload config of the profiled bench run

HBM bytes follow MI355X_MICROARCH.md "HBM": FETCH_SIZE / WRITE_SIZE are in KiB and come from
separate passes; on gfx950 FETCH_SIZE reports half the bytes of wide coalesced reads, so it is
doubled before adding WRITE_SIZE.  VALU busy = 2 cycles per wave64 VALU instruction (SIMD-32) over
the SIMD cycles of the dispatch, the clock taken from GRBM_GUI_ACTIVE (summed over the 8 XCDs,
MI355X_MICROARCH.md "DVFS give-back"): an issue-slot estimate (transcendental / f64 instructions
occupy more than 2 cycles, so it is a lower bound).  Lane utilisation = SQ_THREAD_CYCLES_VALU /
(64 SQ_ACTIVE_INST_VALU).

The workload config is read from the profiled bench run's own JSON line (trace.log), so a
profile is labelled with what actually ran.

Usage: pmc_summary.py <tag> [--prof DIR] [--no-bench-file]
"""
import argparse
import collections
import csv
import json
import os
import shutil

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
N_SIMD = 1024  # 256 CUs x 4 SIMDs


def kernel_key(name):
    """one key per numerics contract: the tolerance contract's builds (mrt_path_kernel_fast, _fastz,
    _pex: mrt_launch.h kFtzVariant / kPathExact) under mrt_path_kernel_fast, the exact build under
    mrt_path_kernel"""
    base = name.split("(")[0]
    if "mrt_path_kernel_fast" in base or "mrt_path_kernel_pex" in base:
        return "mrt_path_kernel_fast"
    return "mrt_path_kernel" if "mrt_path_kernel" in base else base


def per_dispatch(path):
    """{dispatch id: (kernel key, {counter: value}, meta)} of one counter-collection CSV."""
    out = {}
    for r in csv.DictReader(open(path)):
        d = out.setdefault(r["Dispatch_Id"], [kernel_key(r["Kernel_Name"]), collections.defaultdict(float), {}])
        d[1][r["Counter_Name"]] += float(r["Counter_Value"])
        d[2] = {k: r.get(k) for k in ("Grid_Size", "Workgroup_Size", "LDS_Block_Size", "Scratch_Size", "VGPR_Count",
                                      "SGPR_Count", "Accum_VGPR_Count")}
    return out


def mean_by_kernel(disp):
    agg, n, meta = collections.defaultdict(lambda: collections.defaultdict(float)), collections.Counter(), {}
    for k, c, m in disp.values():
        n[k] += 1
        meta[k] = m
        for name, v in c.items():
            agg[k][name] += v
    return {k: {name: v / n[k] for name, v in agg[k].items()} for k in agg}, n, meta


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("tag")
    ap.add_argument("--prof", default=os.path.join(ROOT, "gpurun_out", "prof"))
    ap.add_argument("--no-bench-file", action="store_true")
    a = ap.parse_args()
    out = os.path.join(ROOT, "profiles")
    os.makedirs(out, exist_ok=True)
    stats = os.path.join(a.prof, "trace", "run_kernel_stats.csv")
    shutil.copy(stats, os.path.join(out, f"{a.tag}_kernel_stats.csv"))
    avg_ns = {}
    for r in csv.DictReader(open(stats)):
        avg_ns.setdefault(kernel_key(r["Name"]), float(r["AverageNs"]))
    fetch, n_f, meta = mean_by_kernel(per_dispatch(os.path.join(a.prof, "fetch", "run_counter_collection.csv")))
    write, _, _ = mean_by_kernel(per_dispatch(os.path.join(a.prof, "write", "run_counter_collection.csv")))
    sqp = os.path.join(a.prof, "sq", "run_counter_collection.csv")
    sqd = per_dispatch(sqp) if os.path.exists(sqp) else {}
    sq, _, _ = mean_by_kernel(sqd)
    # workload and rays of one launch: the bench line of the trace pass (one launch per step at
    # these sizes, --pipeline 1)
    rays_per_launch, cfg = None, None
    tl = os.path.join(a.prof, "trace.log")
    for line in open(tl):
        if line.startswith("{") and '"rays_per_step"' in line:
            c = json.loads(line)["config"]
            rays_per_launch = c["rays_per_step"]
            cfg = [c["scene"], c["width"], c["height"], c["spp"], c["depth"]]
    if cfg is None:
        raise SystemExit(f"{tl}: no bench line (the trace pass failed?)")
    res = {"workload_config": cfg, "kernels": {}, "sq_wave_check": []}
    for did, (k, c, m) in sorted(sqd.items(), key=lambda t: int(t[0])):
        try:
            grid_waves = int(m["Grid_Size"]) // 64
        except (TypeError, ValueError):
            grid_waves = None
        res["sq_wave_check"].append({"dispatch": int(did), "kernel": k, "SQ_WAVES": c.get("SQ_WAVES"), "grid_waves": grid_waves})
    for k in fetch:
        if not k.startswith("mrt_path_kernel"):
            continue
        e = {"launches": n_f[k], "dispatch": meta[k], "rays_per_launch": rays_per_launch, "FETCH_SIZE_KiB": fetch[k].get("FETCH_SIZE"),
             "WRITE_SIZE_KiB": write.get(k, {}).get("WRITE_SIZE")}
        e["hbm_bytes_per_launch"] = 2 * e["FETCH_SIZE_KiB"] * 1024 + (e["WRITE_SIZE_KiB"] or 0) * 1024
        if rays_per_launch:
            e["hbm_bytes_per_ray"] = e["hbm_bytes_per_launch"] / rays_per_launch
            e["write_bytes_per_ray"] = (e["WRITE_SIZE_KiB"] or 0) * 1024 / rays_per_launch
        if k in avg_ns:
            e["avg_kernel_ns"] = avg_ns[k]
            e["hbm_GBps"] = e["hbm_bytes_per_launch"] / avg_ns[k]
            e["hbm_frac"] = e["hbm_GBps"] / 8000.0
        s = sq.get(k)
        if s:
            e["sq"] = s
            if rays_per_launch:
                e["valu_insts_per_ray"] = s["SQ_INSTS_VALU"] / rays_per_launch
            if s.get("SQ_ACTIVE_INST_VALU"):
                e["valu_lane_util"] = s["SQ_THREAD_CYCLES_VALU"] / (64.0 * s["SQ_ACTIVE_INST_VALU"])
            if s.get("SQ_WAVE_CYCLES"):
                e["wait_any_fraction"] = s["SQ_WAIT_ANY"] / s["SQ_WAVE_CYCLES"]
            if s.get("GRBM_GUI_ACTIVE"):
                cycles = s["GRBM_GUI_ACTIVE"] / 8.0
                e["gpu_cycles"] = cycles
                e["valu_busy"] = 2.0 * s["SQ_INSTS_VALU"] / (N_SIMD * cycles)
                if k in avg_ns:
                    e["effective_clock_GHz"] = cycles / avg_ns[k]
        res["kernels"][k] = e
    json.dump(res, open(os.path.join(out, f"{a.tag}_pmc.json"), "w"), indent=1)
    if not a.no_bench_file:
        by = {}
        for k, e in res["kernels"].items():
            if "mrt_wf_" in k:
                continue
            num = "fast" if k.endswith("_fast") else "exact"
            by[num] = {x: e.get(x) for x in ("valu_insts_per_ray", "hbm_bytes_per_ray", "write_bytes_per_ray", "valu_busy",
                                             "valu_lane_util", "avg_kernel_ns", "rays_per_launch")}
        name = f"pmc_s{cfg[0]}_{cfg[1]}x{cfg[2]}.json"
        json.dump({"config": cfg, "by_numerics": by, "source": f"profiles/{a.tag}_pmc.json"},
                  open(os.path.join(out, name), "w"), indent=1)
    print(json.dumps(res, indent=1)[:6000])


if __name__ == "__main__":
    main()
