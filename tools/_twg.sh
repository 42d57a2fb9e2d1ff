#!/bin/bash
# experiment: workgroup size of the bvh_node (treelet) kernels: one 16-wave group per CU (in-tree)
# vs 8- / 4-wave groups (each with its own treelet copy); C5 book2 at 2048^2 x 64 spp, scene 0
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
for cfg in "7 2048 2048 64" "0 1200 800 64"; do
  set -- $cfg
  for w in intree twg512 twg256; do
    lib=""; [ "$w" != intree ] && lib=$PWD/exp/libmrt_$w.so
    MRT_EXPERIMENT_LIB=$lib timeout -k 10 200 python bench.py --no-cpu-baseline --no-compare-numerics --steps 2 --warmup 1 --kernel-reps 1 --pipeline 1 \
      --scene $1 --width $2 --height $3 --samples $4 > gpurun_out/twg_$1_$w.log 2>&1 || exit 3
    python tools/_show.py gpurun_out/twg_$1_$w.log "scene $1 $w"
  done
done
