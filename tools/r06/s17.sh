#!/bin/bash
# round 6 session 17: path starts batched (MRT_START_MIN 8 / 16: exp/libmrt_sm8.so, sm16) in the
# resumable mesh loop and the plain loop, A/B on C4, C3, C5, random spheres
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out/r06
LIBS="sm8 sm16" CFGS="8,1024,1024,256 9,800,800,256 7,2048,2048,64 0,1200,800,64" ROUNDS=2 bash tools/ab.sh || exit 3
