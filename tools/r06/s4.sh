#!/bin/bash
# round 6 session 4: the GPU suite on the current tree (instance ray recomputed after the walk,
# bench's multi-rank path over the C-ABI gather), then session 2 (the C4 / C5 8-share rehearsal)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out/r06
set -o pipefail
timeout -k 10 600 python -u -m pytest tests/ -x -v -m gpu --timeout 240 --timeout-method thread > gpurun_out/r06/s4_suite.log 2>&1
rc=$?; tail -3 gpurun_out/r06/s4_suite.log
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
bash tools/r06/s2.sh
