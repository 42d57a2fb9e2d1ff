#!/bin/bash
# experiment: resumable mesh walk -- lanes with other work needed before the walk loop yields
# (MRT_WALK_OTHER: 16 in-tree; exp builds 8 / 24 / 32), C3 teapot and C4 bunny at 256 spp
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
for cfg in "9 800 800 256" "8 1024 1024 256"; do
  set -- $cfg
  for w in intree wo8 wo24 wo32 intree; do
    lib=""; [ "$w" != intree ] && lib=$PWD/exp/libmrt_$w.so
    MRT_EXPERIMENT_LIB=$lib timeout -k 10 200 python bench.py --no-cpu-baseline --no-compare-numerics --steps 3 --warmup 1 --kernel-reps 1 \
      --scene $1 --width $2 --height $3 --samples $4 > gpurun_out/wo_$1_$w.log 2>&1 || exit 3
    python tools/_show.py gpurun_out/wo_$1_$w.log "scene $1 $w"
  done
done
