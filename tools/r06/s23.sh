#!/bin/bash
# round 6 session 23: leaf postponing in the bvh_node walk in tree for the kernels without volumes
# (MRT_BVHW_SPEC 3): the GPU suite, then A/B against the while-while walk everywhere (sp0) on the
# sky-lit bvh_node scenes 0-4 (fast) and scene 0 / 2 under the exact contract
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out/r06
set -o pipefail
timeout -k 10 600 python -u -m pytest tests/ -x -v -m gpu --timeout 240 --timeout-method thread > gpurun_out/r06/s23_suite.log 2>&1
rc=$?; tail -3 gpurun_out/r06/s23_suite.log
[ $rc -eq 0 ] || exit $rc
LIBS="sp0" CFGS="0,1200,800,64 1,1200,800,64 2,800,400,256 3,800,400,256 4,800,400,256" ROUNDS=2 bash tools/ab.sh || exit 3
LIBS="sp0" CFGS="0,600,400,32 2,400,200,64" ROUNDS=2 BENCH_ARGS="--numerics exact" bash tools/ab.sh || exit 3
