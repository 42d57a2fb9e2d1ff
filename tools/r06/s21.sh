#!/bin/bash
# round 6 session 21: the path-exact bunny kernel at 7 waves per SIMD (72 VGPRs, 1 spilled, exp/libmrt_m7.so)
# against 8 (64, 13 spilled) now that majority leaf postponing holds another register; C4
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out/r06
LIBS="m7" CFGS="8,1024,1024,256" ROUNDS=3 bash tools/ab.sh || exit 3
