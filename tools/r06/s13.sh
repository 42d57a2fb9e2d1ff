#!/bin/bash
# round 6 session 13: the GPU suite with two mesh-walk steps per yield check in tree; book2's
# path-exact kernel now spill-free at 6 waves per SIMD tried at 7 (2 x 14-wave groups, 72 VGPRs, 13
# spilled: exp/libmrt_p7.so) and 8 (2 x 16, 64 VGPRs, 27 spilled: p8), C5 shape and Cornell smoke
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out/r06
set -o pipefail
timeout -k 10 600 python -u -m pytest tests/ -x -v -m gpu --timeout 240 --timeout-method thread > gpurun_out/r06/s13_suite.log 2>&1
rc=$?; tail -3 gpurun_out/r06/s13_suite.log
[ $rc -eq 0 ] || exit $rc
LIBS="p7 p8" CFGS="7,2048,2048,64 6,500,500,256" ROUNDS=2 bash tools/ab.sh || exit 3
