#!/bin/bash
# A/B of path-kernel builds on the bvh_node / mesh workloads: for each library (default: the
# in-tree build; more as exp/libmrt_<tag>.so via LIBS="tag1 tag2"), one bench run per workload
# (fast contract, kernel time by HIP events) -> gpurun_out/ab_<tag>_<scene>.log + a summary line.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
CFGS=${CFGS:-"7,2048,2048,64 0,1200,800,64 1,1200,800,64 8,1024,1024,256 9,800,800,256"}
for tag in intree ${LIBS:-}; do
  for cfg in $CFGS; do
    IFS=, read sid W H S <<< "$cfg"
    lib=""; [ "$tag" != intree ] && lib="exp/libmrt_$tag.so"
    MRT_EXPERIMENT_LIB=$lib timeout -k 10 300 python bench.py --no-cpu-baseline --no-compare-numerics --no-other-walk --steps 3 --warmup 1 \
        --scene $sid --width $W --height $H --samples $S > gpurun_out/ab_${tag}_$sid.log 2>&1 || exit 3
    python tools/show_bench.py gpurun_out/ab_${tag}_$sid.log "$tag scene $sid"
  done
done
