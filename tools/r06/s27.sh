#!/bin/bash
# round 6 session 27: the walks' box tests without VALU overhead -- the child-order selects of lane
# booleans as mask logic (sel_b), the box test's slow-path check a wave flag computed once per walk
# (aabb_hit_b), its two outcomes merged as bounds before one comparison: the GPU suite on this tree,
# A/B against the tree before (exp/libmrt_base.so) on C4, C5, C3, C2, random spheres (fast and exact),
# and against the same with 32-bit node offsets (o32: MRT_WIDE_OFF32), then SQ_INSTS_VALU per ray of the
# C4 path-exact kernel for the three
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out/r06
set -o pipefail
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/ -x -v -m gpu --timeout 240 --timeout-method thread > gpurun_out/r06/s27_suite.log 2>&1
rc=$?; tail -3 gpurun_out/r06/s27_suite.log
[ $rc -eq 0 ] || exit $rc
MRT_EXPERIMENT_LIB=exp/libmrt_o32.so timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -x -v -m gpu --timeout 200 --timeout-method thread \
    -k "stream or shape_specialised or linear_program or own_spp or equals_cpu or path_exact or contract or wide" > gpurun_out/r06/s27_o32_tests.log 2>&1 \
    || { tail -30 gpurun_out/r06/s27_o32_tests.log; exit 3; }
tail -2 gpurun_out/r06/s27_o32_tests.log
LIBS="base o32" CFGS="8,1024,1024,256 7,2048,2048,64 9,800,800,256 5,500,500,1024 0,1200,800,64" ROUNDS=2 bash tools/ab.sh || exit 3
LIBS="base o32" CFGS="0,600,400,32 8,256,256,64" ROUNDS=1 BENCH_ARGS="--numerics exact" bash tools/ab.sh || exit 3
for t in intree base o32; do
  lib=""; [ $t != intree ] && lib=exp/libmrt_$t.so
  MRT_EXPERIMENT_LIB=$lib timeout -s KILL 300 rocprofv3 --pmc SQ_INSTS_VALU SQ_WAVES -d gpurun_out/r06/s27_sq_$t -o run --output-format csv -- \
      python3 bench.py --steps 1 --warmup 0 --kernel-reps 1 --pipeline 1 --no-cpu-baseline --no-other-walk --no-parity --no-compare-numerics \
      --scene 8 --width 1024 --height 1024 --samples 256 > gpurun_out/r06/s27_sq_$t.log 2>&1 || exit 3
  python - gpurun_out/r06/s27_sq_$t gpurun_out/r06/s27_sq_$t.log $t <<'PY'
import csv, glob, json, sys, collections
f = glob.glob(sys.argv[1] + "/**/run_counter_collection.csv", recursive=True)[0]
d = collections.defaultdict(lambda: collections.defaultdict(float)); names = {}
for r in csv.DictReader(open(f)):
    d[r["Dispatch_Id"]][r["Counter_Name"]] += float(r["Counter_Value"]); names[r["Dispatch_Id"]] = r["Kernel_Name"]
j = json.loads([l for l in open(sys.argv[2]) if l.startswith("{")][-1])
rays = j["config"]["rays_per_step"]
for k, v in d.items():
    if "pex" in names[k]:
        print(f"{sys.argv[3]}: {names[k][:60]} dispatch {k}: SQ_INSTS_VALU {v['SQ_INSTS_VALU']:.4e}, per ray {v['SQ_INSTS_VALU'] / rays:.2f} (rays {rays})")
PY
done
