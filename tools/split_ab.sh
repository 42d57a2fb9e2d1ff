#!/bin/bash
# A/B of the split form (MRT_SPLIT, mrt_wavefront.h) against the persistent path kernel on the
# volume scenes: bench runs (fast contract = the path-exact build for these scenes) of the in-tree
# library with MRT_SPLIT=0 / 1 and of exp/libmrt_<tag>.so (LIBS="w4 w6 ...": other hit-kernel
# shapes) with MRT_SPLIT=1, ROUNDS alternations -> gpurun_out/split_<tag>_<scene>_<round>.log
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
CFGS=${CFGS:-"7,2048,2048,64"}
STEPS=${STEPS:-5}
for r in $(seq 1 "${ROUNDS:-2}"); do
  for tag in ${TAGS:-base intree} ${LIBS:-}; do
    for cfg in $CFGS; do
      IFS=, read sid W H S <<< "$cfg"
      lib=""; sp=1
      # (<lib>:0 -- that library's persistent path kernel, MRT_SPLIT=0)
      case "$tag" in base) sp=0 ;; intree) ;; *:0) lib="exp/libmrt_${tag%:0}.so"; sp=0 ;; *) lib="exp/libmrt_$tag.so" ;; esac
      log=gpurun_out/split_${tag/:/-}${SFX:-}_${sid}_$r.log
      MRT_SPLIT=$sp MRT_EXPERIMENT_LIB=$lib timeout -k 10 300 python bench.py --no-cpu-baseline --no-compare-numerics --no-other-walk \
          --no-parity --steps "$STEPS" --warmup 1 --scene "$sid" --width "$W" --height "$H" --samples "$S" ${BENCH_ARGS:-} > "$log" 2>&1 || exit 3
      python tools/show_bench.py "$log" "$tag${SFX:-} split=$sp scene $sid round $r"
    done
  done
done
