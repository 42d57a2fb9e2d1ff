#!/bin/bash
# round 6 session 1: the new ABI-6 tests (async shapes, RCCL gather via the C-ABI, CLI -gather rccl),
# then the whole GPU suite, the smoke and the default bench
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out/r06
set -o pipefail
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -v -m gpu --timeout 120 --timeout-method thread \
    -k "different_shapes or rccl or async_fold or c3_whole" > gpurun_out/r06/s1_new.log 2>&1 || exit $?
SKIP_PROF=1 bash tools/gpu_session.sh
