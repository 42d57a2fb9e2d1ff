#!/bin/bash
# round 6 session 34: session 2 again on the final tree (r06_f5) -- every N = 8 share
# of C4 (bunny 1024^2 x 2048 spp) and C5 (book2 2048^2 x 8192 spp) against the N = 1 render, and two
# ranks of C4 on one GPU over gloo with --verify (reduced spp)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out/r06
set -o pipefail
MRT_SAME_GPU=1 MRT_DIST_BACKEND=gloo timeout -k 10 300 python bench.py --gpus 2 --scene 8 --width 1024 --height 1024 --samples 64 \
    --steps 2 --warmup 1 --verify --no-cpu-baseline --no-compare-numerics --no-other-walk --no-parity > gpurun_out/r06/s34_world2_c4.log 2>&1 || exit 3
echo "== C4 (scene 8, 1024x1024, 2048 spp)"
CFGS="1,0 8,0 8,1 8,2 8,3 8,4 8,5 8,6 8,7" STEPS=6 WARMUP=2 SCALE_ARGS="--scene 8 --width 1024 --height 1024 --samples 2048" \
    bash tools/scale_rehearsal.sh || exit 3
mkdir -p gpurun_out/r06/s34_c4 && mv gpurun_out/scale_*.log gpurun_out/r06/s34_c4/
echo "== C5 (scene 7, 2048x2048, 8192 spp)"
CFGS="1,0 8,0 8,1 8,2 8,3 8,4 8,5 8,6 8,7" STEPS=2 WARMUP=1 RUN_TIMEOUT=400 SCALE_ARGS="--scene 7 --width 2048 --height 2048 --samples 8192" \
    bash tools/scale_rehearsal.sh || exit 3
mkdir -p gpurun_out/r06/s34_c5 && mv gpurun_out/scale_*.log gpurun_out/r06/s34_c5/
