#!/bin/bash
# experiment: fold kernel (lean = MRT_RF_FOLD_BEHIND beside the next path kernel, full = after it)
# x render contexts pipelined on streams (bench.py --pipeline)
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
for c in ${CASES:-"lean 2" "full 2" "lean 3" "full 3" "lean 4"}; do
  set -- $c
  timeout -k 10 200 python bench.py --no-cpu-baseline --no-compare-numerics --steps ${STEPS:-12} --fold $1 --pipeline $2 > gpurun_out/fab_$1_$2.log 2>&1 || exit 3
  python tools/_show.py gpurun_out/fab_$1_$2.log "$1 pipeline=$2"
done
