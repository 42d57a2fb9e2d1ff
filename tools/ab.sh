#!/bin/bash
# Interleaved A/B of path-kernel builds: for each round, each library (the in-tree build, then
# exp/libmrt_<tag>.so for LIBS="tag1 tag2 ...", or the in-tree build under VAR=value for a tag of
# that form), one bench run per workload (fast contract, no CPU
# baseline) -> gpurun_out/ab_<tag>_<scene>_<round>.log; a summary line per run (ms per step, path
# kernel ms by HIP events).  ROUNDS alternations (default 2) so box drift hits every build alike.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
CFGS=${CFGS:-"5,500,500,1024"}
STEPS=${STEPS:-10}
for r in $(seq 1 "${ROUNDS:-2}"); do
  for tag in intree ${LIBS:-}; do
    for cfg in $CFGS; do
      IFS=, read sid W H S <<< "$cfg"
      # a tag VAR=value runs the in-tree library with that environment variable set
      lib=""; envv="MRT_AB_TAG=$tag"
      case "$tag" in intree) ;; *=*) envv=$tag ;; *) lib="exp/libmrt_$tag.so" ;; esac
      log=gpurun_out/ab_${tag//=/-}_${sid}_$r.log
      env "$envv" MRT_EXPERIMENT_LIB=$lib timeout -k 10 300 python bench.py --no-cpu-baseline --no-compare-numerics --no-other-walk \
          --no-parity --steps "$STEPS" --warmup 2 --scene "$sid" --width "$W" --height "$H" --samples "$S" ${BENCH_ARGS:-} > "$log" 2>&1 || exit 3
      python tools/show_bench.py "$log" "$tag scene $sid round $r"
    done
  done
done
