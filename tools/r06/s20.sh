#!/bin/bash
# round 6 session 20: majority leaf postponing in the path-exact build in tree: the GPU suite, then the
# path-exact bunny's yield threshold (MRT_WALK_MIN 24 / 40 / 48 against the build's 32) on C4
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out/r06
set -o pipefail
timeout -k 10 600 python -u -m pytest tests/ -x -v -m gpu --timeout 240 --timeout-method thread > gpurun_out/r06/s20_suite.log 2>&1
rc=$?; tail -3 gpurun_out/r06/s20_suite.log
[ $rc -eq 0 ] || exit $rc
LIBS="MRT_WALK_MIN=24 MRT_WALK_MIN=40 MRT_WALK_MIN=48" CFGS="8,1024,1024,256" ROUNDS=2 bash tools/ab.sh || exit 3
