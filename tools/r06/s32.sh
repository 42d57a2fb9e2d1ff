#!/bin/bash
# round 6 session 32: the bvh_node walk's empty-stack mark (mrt_trace.h MRT_BVHW_SENT: the stack's
# bottom holds kBvhwEmpty, so no lane returns from inside the walk's inner loop) -- the GPU suite on
# this tree, then A/B against the same sources without it (nosent, all four builds) and the tree's
# flags through tools/build_variant.sh (ctl): book2 (C5's kernel), scenes 0 and 2, fast and exact
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out/r06
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/ -x -q -m gpu --timeout 240 --timeout-method thread > gpurun_out/r06/s32_suite.log 2>&1
rc=$?; tail -2 gpurun_out/r06/s32_suite.log
[ $rc -eq 0 ] || exit $rc
LIBS="nosent ctl" CFGS="7,2048,2048,64 0,1200,800,64 2,1200,800,64" ROUNDS=2 bash tools/ab.sh || exit 3
LIBS="nosent" CFGS="7,1024,1024,16 0,600,400,32" ROUNDS=1 BENCH_ARGS="--numerics exact" bash tools/ab.sh || exit 3
