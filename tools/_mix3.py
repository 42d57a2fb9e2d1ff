import csv, collections, glob, sys, json
for w in sys.argv[1:]:
    agg = collections.defaultdict(float); ids = set()
    for f in glob.glob(f"gpurun_out/mix3/{w}/**/run_counter_collection.csv", recursive=True) + glob.glob(f"gpurun_out/mix3/{w}/run_counter_collection.csv"):
        for r in csv.DictReader(open(f)):
            if "mrt_path_kernel" in r["Kernel_Name"]:
                agg[r["Counter_Name"]] += float(r["Counter_Value"]); ids.add(r["Dispatch_Id"])
    n = len(ids)
    line = [l for l in open(f"gpurun_out/mix3/{w}.log") if l.startswith('{"metric"')][-1]
    rays = json.loads(line)["config"]["rays_per_step"]
    v = {k: x / n for k, x in agg.items()}
    print(w, "launches", n, "VALU/ray(wave-instr*64)", 64 * v["SQ_INSTS_VALU"] / rays, "lane util", v["SQ_THREAD_CYCLES_VALU"] / (64 * v["SQ_ACTIVE_INST_VALU"]),
          "SALU/VALU", v["SQ_INSTS_SALU"] / v["SQ_INSTS_VALU"], "wait_inst/wave", v["SQ_WAIT_INST_ANY"] / v["SQ_WAVE_CYCLES"])
