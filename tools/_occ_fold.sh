#!/bin/bash
# experiment: does the fold of step i overlap step i+1's path kernel when the path kernel leaves
# room on each CU (MRT_BLOCKS_PER_CU) and a step is split into launches (--chunk-samples)?
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
run() {  # tag nb chunk
  MRT_EXPERIMENT_LIB=$PWD/exp/libmrt_x.so MRT_BLOCKS_PER_CU=$2 timeout -k 10 200 python bench.py --no-cpu-baseline --no-compare-numerics \
    --steps 10 --warmup 1 --kernel-reps 1 --chunk-samples $3 > gpurun_out/of_$1.log 2>&1 || exit 3
  python tools/_show.py gpurun_out/of_$1.log "$1 nb=$2 chunk=$3"
}
run base 28 0 && run c512 28 512 && run n24 24 0 && run n24c512 24 512 && run n24c256 24 256 && run n20c512 20 512 && run n26c512 26 512
