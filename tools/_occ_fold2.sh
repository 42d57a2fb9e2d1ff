#!/bin/bash
# experiment: path-kernel grid one or two waves per CU short of full (MRT_BLOCKS_PER_CU 27 / 26) so
# one SIMD per CU has room for a fold wave beside it, x fold kernel, three contexts
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
for c in "27 full 3" "27 lean 3" "26 full 3" "28 lean 3" "27 full 2"; do
  set -- $c
  MRT_EXPERIMENT_LIB=$PWD/exp/libmrt_occ.so MRT_BLOCKS_PER_CU=$1 timeout -k 10 200 python bench.py --no-cpu-baseline --no-compare-numerics --steps 12 --fold $2 --pipeline $3 > gpurun_out/o2_$1_$2_$3.log 2>&1 || exit 3
  python tools/_show.py gpurun_out/o2_$1_$2_$3.log "nb=$1 $2 pipeline=$3"
done
