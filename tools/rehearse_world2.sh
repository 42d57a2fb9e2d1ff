#!/bin/bash
# Two ranks of the multi-GPU bench on ONE GPU (MRT_SAME_GPU=1): the launcher, the rank processes and
# the tile gather, over RCCL (nccl) and then gloo.  A step that times out, aborts or crashes ends the
# script (no further GPU step); an ordinary failure (e.g. RCCL refusing two ranks on one device) is
# recorded and the next backend runs.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for be in nccl gloo; do
  MRT_SAME_GPU=1 MRT_DIST_BACKEND=$be timeout -k 10 150 python bench.py --gpus 2 --steps 3 --warmup 1 --no-cpu-baseline \
      --no-other-walk --no-compare-numerics --verify > gpurun_out/world2_$be.log 2>&1
  rc=$?
  echo "$be rc=$rc" | tee -a gpurun_out/world2_rc.txt
  case $rc in 0|1|2|3) ;; *) exit $rc ;; esac
done
