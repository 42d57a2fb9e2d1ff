#!/bin/bash
# experiment: per-step time with the path kernel at 6 waves/SIMD (MRT_BLOCKS_PER_CU=24, room for a
# fold beside it) x fold kernel x pipeline depth; kernel trace of one case
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
for c in "24 full 2" "24 full 3" "24 lean 3" "28 lean 3"; do
  set -- $c
  MRT_EXPERIMENT_LIB=$PWD/exp/libmrt_occ.so MRT_BLOCKS_PER_CU=$1 timeout -k 10 200 python bench.py --no-cpu-baseline --no-compare-numerics --steps 12 --fold $2 --pipeline $3 > gpurun_out/ot_$1_$2_$3.log 2>&1 || exit 3
  python tools/_show.py gpurun_out/ot_$1_$2_$3.log "nb=$1 $2 pipeline=$3"
done
