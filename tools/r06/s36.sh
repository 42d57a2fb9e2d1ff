#!/bin/bash
# round 6 session 36: the bvh_node walk's push without a branch (MRT_BVHW_PUSH_ALWAYS, variant library pusha: the far
# child stored by every lane above its stack's top, the pointer advanced by the push condition) -- the GPU tests of
# the bvh_node scenes through it, then A/B against the tree: book2 (C5's kernel) and scenes 0 / 2, fast and exact
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out/r06
export TMPDIR=/tmp
MRT_EXPERIMENT_LIB=exp/libmrt_pusha.so timeout -k 10 600 python -u -m pytest tests/ -x -q -m gpu --timeout 240 --timeout-method thread > gpurun_out/r06/s36_suite.log 2>&1
rc=$?; tail -2 gpurun_out/r06/s36_suite.log
[ $rc -eq 0 ] || exit $rc
LIBS="pusha" CFGS="7,2048,2048,64 0,1200,800,64 2,1200,800,64" ROUNDS=2 bash tools/ab.sh || exit 3
LIBS="pusha" CFGS="7,1024,1024,16 0,600,400,32" ROUNDS=1 BENCH_ARGS="--numerics exact" bash tools/ab.sh || exit 3
