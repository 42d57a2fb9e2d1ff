#!/bin/bash
# round 6 session 14: the walks specialised on the wave's "some ray not nice" answer (decided once
# per walk; the common walk without a slow-path branch per box test): the GPU suite, then A/B
# against the previous commit's build (exp/libmrt_base.so) on C5, C4, C3, random spheres, C2
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out/r06
set -o pipefail
timeout -k 10 600 python -u -m pytest tests/ -x -v -m gpu --timeout 240 --timeout-method thread > gpurun_out/r06/s14_suite.log 2>&1
rc=$?; tail -3 gpurun_out/r06/s14_suite.log
[ $rc -eq 0 ] || exit $rc
LIBS="base" CFGS="7,2048,2048,64 8,1024,1024,256 9,800,800,256 0,1200,800,64 5,500,500,1024" ROUNDS=3 bash tools/ab.sh || exit 3
