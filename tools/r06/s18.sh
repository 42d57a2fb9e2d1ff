#!/bin/bash
# round 6 session 18: batched path starts in tree (resumable loop: 16 fast / 8 path-exact), the GPU
# suite, then A/B against the neighbours (hi: 24 / 12, lo: 12 / 5) on C3 and C4
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out/r06
set -o pipefail
timeout -k 10 600 python -u -m pytest tests/ -x -v -m gpu --timeout 240 --timeout-method thread > gpurun_out/r06/s18_suite.log 2>&1
rc=$?; tail -3 gpurun_out/r06/s18_suite.log
[ $rc -eq 0 ] || exit $rc
LIBS="hi lo" CFGS="8,1024,1024,256 9,800,800,256" ROUNDS=3 bash tools/ab.sh || exit 3
