#!/usr/bin/env python3
"""Summarise a tools/profile.sh run (gpurun_out/prof) into profiles/:

  profiles/<tag>_kernel_stats.csv   rocprofv3 --kernel-trace --stats summary (copied)
  profiles/<tag>_pmc.json           per-launch counters of mrt_path_kernel + derived metrics
  profiles/pmc_cornell_c2.json      HBM bytes per launch read by bench.py (roofline.traffic)

HBM bytes follow MI355X_MICROARCH.md "HBM": FETCH_SIZE / WRITE_SIZE are in KiB and come from
separate passes; on gfx950 FETCH_SIZE reports half the bytes of wide coalesced reads, so it is
doubled before adding WRITE_SIZE.
"""
import csv
import collections
import json
import os
import shutil
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def per_launch(path, kernel="mrt_path_kernel"):
    rows = list(csv.DictReader(open(path)))
    agg, ids, meta = collections.defaultdict(float), set(), {}
    for r in rows:
        if kernel in r["Kernel_Name"]:
            agg[r["Counter_Name"]] += float(r["Counter_Value"])
            ids.add(r["Dispatch_Id"])
            meta = {k: r[k] for k in ("Grid_Size", "Workgroup_Size", "LDS_Block_Size", "Scratch_Size", "VGPR_Count", "SGPR_Count")}
    n = max(len(ids), 1)
    return {k: v / n for k, v in agg.items()}, n, meta


def main():
    tag = sys.argv[1] if len(sys.argv) > 1 else "r01"
    prof = os.path.join(ROOT, "gpurun_out", "prof")
    out = os.path.join(ROOT, "profiles")
    os.makedirs(out, exist_ok=True)
    shutil.copy(os.path.join(prof, "trace", "run_kernel_stats.csv"), os.path.join(out, f"{tag}_kernel_stats.csv"))
    fetch, n, meta = per_launch(os.path.join(prof, "fetch", "run_counter_collection.csv"))
    write, _, _ = per_launch(os.path.join(prof, "write", "run_counter_collection.csv"))
    res = {"kernel": "mrt_path_kernel", "launches": n, "dispatch": meta,
           "FETCH_SIZE_KiB": fetch.get("FETCH_SIZE"), "WRITE_SIZE_KiB": write.get("WRITE_SIZE")}
    hbm = 2 * fetch["FETCH_SIZE"] * 1024 + write["WRITE_SIZE"] * 1024
    res["hbm_bytes_per_launch"] = hbm
    sqp = os.path.join(prof, "sq", "run_counter_collection.csv")
    if os.path.exists(sqp):
        sq, _, _ = per_launch(sqp)
        res["sq"] = sq
        if sq.get("SQ_ACTIVE_INST_VALU"):
            res["valu_lane_utilization"] = sq["SQ_THREAD_CYCLES_VALU"] / (64.0 * sq["SQ_ACTIVE_INST_VALU"])
        if sq.get("SQ_WAVE_CYCLES"):
            res["wait_any_fraction"] = sq["SQ_WAIT_ANY"] / sq["SQ_WAVE_CYCLES"]
    for r in csv.DictReader(open(os.path.join(prof, "trace", "run_kernel_stats.csv"))):
        if "mrt_path_kernel" in r["Name"]:
            res["avg_kernel_ns"] = float(r["AverageNs"])
            res["hbm_GBps"] = hbm / float(r["AverageNs"])
    json.dump(res, open(os.path.join(out, f"{tag}_pmc.json"), "w"), indent=1)
    cfg = [int(x) for x in os.environ.get("PMC_CONFIG", "5 500 500 1024 32").split()]
    json.dump({"config": cfg, "hbm_bytes_per_launch": hbm, "source": f"profiles/{tag}_pmc.json"},
              open(os.path.join(out, "pmc_cornell_c2.json"), "w"))
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
