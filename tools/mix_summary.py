"""Summarise tools/pmc_mix.sh output: per-launch instruction counts of mrt_path_kernel."""
import collections, csv, glob, sys
agg = collections.defaultdict(float)
ids = collections.defaultdict(set)
for f in glob.glob("gpurun_out/mix/p*/**/run_counter_collection.csv", recursive=True) + glob.glob("gpurun_out/mix/p*/run_counter_collection.csv"):
    for r in csv.DictReader(open(f)):
        if "mrt_path_kernel" in r["Kernel_Name"]:
            agg[r["Counter_Name"]] += float(r["Counter_Value"])
            ids[r["Counter_Name"]].add((f, r["Dispatch_Id"]))
valu = agg["SQ_INSTS_VALU"] / max(len(ids["SQ_INSTS_VALU"]), 1)
for k in sorted(agg):
    v = agg[k] / max(len(ids[k]), 1)
    print(f"{k:28s} {v:16.4g}  {100 * v / valu:6.1f}% of VALU")
