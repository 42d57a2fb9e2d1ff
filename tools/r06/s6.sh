#!/bin/bash
# round 6 session 6: the bvh_node leaf / volume records made after the walk (mrt_lin.h MRT_LIN_DEFER):
# the GPU suite, then A/B against the same tree built with MRT_LIN_DEFER=0 (exp/libmrt_nodefer.so) on
# book2 (C5 shape), random spheres, C2 and C2 through the interpreter, then the C5 PMC passes
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out/r06
set -o pipefail
timeout -k 10 600 python -u -m pytest tests/ -x -v -m gpu --timeout 240 --timeout-method thread > gpurun_out/r06/s6_suite.log 2>&1
rc=$?; tail -3 gpurun_out/r06/s6_suite.log
[ $rc -eq 0 ] || exit $rc
LIBS="nodefer" CFGS="7,2048,2048,64 0,1200,800,64 5,500,500,1024" ROUNDS=2 bash tools/ab.sh || exit 3
for r in 1 2; do
  for tag in intree nodefer; do
    lib=""; [ $tag != intree ] && lib=exp/libmrt_$tag.so
    MRT_NO_SIG=1 MRT_EXPERIMENT_LIB=$lib timeout -k 10 300 python bench.py --no-cpu-baseline --no-compare-numerics --no-other-walk \
        --no-parity --steps 10 --warmup 2 > gpurun_out/r06/s6_interp_${tag}_$r.log 2>&1 || exit 3
    python tools/show_bench.py gpurun_out/r06/s6_interp_${tag}_$r.log "interp $tag $r"
  done
done
PROF_CFGS="c5:7:2048:2048:64" bash tools/prof_configs.sh || exit 3
