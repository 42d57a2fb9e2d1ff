#!/bin/bash
# round 6 session 33: the resumable mesh walk's empty-stack mark (mrt_trace.h MRT_MESH_SENT: the stack's bottom
# holds kMeshEmpty, so a pop needs no empty-stack test) -- the GPU suite on this tree, then A/B against the same
# sources without it (nomsent, all four builds) and the tree's flags through tools/build_variant.sh (ctl): the
# teapot (C3) and the bunny (C4), fast and exact
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out/r06
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/ -x -q -m gpu --timeout 240 --timeout-method thread > gpurun_out/r06/s33_suite.log 2>&1
rc=$?; tail -2 gpurun_out/r06/s33_suite.log
[ $rc -eq 0 ] || exit $rc
LIBS="nomsent ctl" CFGS="9,800,800,256 8,1024,1024,256" ROUNDS=2 bash tools/ab.sh || exit 3
LIBS="nomsent" CFGS="9,400,400,64 8,512,512,64" ROUNDS=1 BENCH_ARGS="--numerics exact" bash tools/ab.sh || exit 3
