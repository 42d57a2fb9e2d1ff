#!/bin/bash
# experiment: lean fold workgroup size (256 in-tree; exp builds 64 / 128), default bench (3 contexts)
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
for w in intree lw64 lw128 intree lw64; do
  lib=""; [ "$w" != intree ] && lib=$PWD/exp/libmrt_$w.so
  MRT_EXPERIMENT_LIB=$lib timeout -k 10 200 python bench.py --no-cpu-baseline --no-compare-numerics --steps 16 > gpurun_out/lw_$w.log 2>&1 || exit 3
  python tools/_show.py gpurun_out/lw_$w.log "$w"
done
