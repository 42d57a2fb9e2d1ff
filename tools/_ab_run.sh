#!/bin/bash
# experiment call: GPU parity tests of the in-tree build, then mesh_ab over the given variant tags
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
if [ "${SKIP_TESTS:-0}" != 1 ]; then
  timeout -k 10 600 python -u -m pytest tests/ -x -q -m gpu --timeout 300 --timeout-method thread > gpurun_out/ab_tests.log 2>&1
  rc=$?; tail -3 gpurun_out/ab_tests.log; [ $rc -ne 0 ] && exit $rc
fi
timeout -k 10 900 python -u tools/mesh_ab.py "$@" 2>&1 | tee gpurun_out/ab.log
