#!/bin/bash
# round 6 session 35: session 33 again with MRT_MESH_SENT defined above mesh_step (s33 had defined it below: mesh_step
# kept its empty-stack test while the walk started with the mark on the stack -- the parity failure), as a variant
# library (msent: all four builds with it; the tree builds it off): the GPU tests through it, then A/B against the
# tree on the teapot (C3) and the bunny (C4), fast and exact
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out/r06
export TMPDIR=/tmp
MRT_EXPERIMENT_LIB=exp/libmrt_msent.so timeout -k 10 600 python -u -m pytest tests/ -x -q -m gpu --timeout 240 --timeout-method thread > gpurun_out/r06/s35_suite.log 2>&1
rc=$?; tail -2 gpurun_out/r06/s35_suite.log
[ $rc -eq 0 ] || exit $rc
LIBS="msent" CFGS="9,800,800,256 8,1024,1024,256" ROUNDS=2 bash tools/ab.sh || exit 3
LIBS="msent" CFGS="9,400,400,64 8,512,512,64" ROUNDS=1 BENCH_ARGS="--numerics exact" bash tools/ab.sh || exit 3
