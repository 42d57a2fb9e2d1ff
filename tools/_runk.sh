#!/bin/bash
# experiment: sample-run length sweep (MRT_RUN_K; 0 = per-path radiance + fold) on C2
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
for k in ${KS:-0 16 4 8 32 64}; do
  MRT_EXPERIMENT_LIB=$PWD/exp/libmrt_x.so MRT_RUN_K=$k timeout -k 10 200 python bench.py --no-cpu-baseline --no-compare-numerics \
    --steps 10 --warmup 1 --kernel-reps 1 ${BARGS:-} > gpurun_out/rk_$k.log 2>&1 || exit 3
  python tools/_show.py gpurun_out/rk_$k.log "K=$k"
done
