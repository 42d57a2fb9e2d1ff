#!/bin/bash
# round 6 session 19: leaf postponing (MRT_MESH_SPEC) with the step type chosen by majority
# (specmaj: a leaf step when at least as many lanes can take one as an inner step) and at 8 parked
# runs (spec8), on top of the batched path starts; bit-exactness of scenes 8 / 9 through specmaj,
# then A/B on C4 and C3
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out/r06
set -o pipefail
MRT_EXPERIMENT_LIB=exp/libmrt_specmaj.so timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -x -v -m gpu --timeout 200 --timeout-method thread \
    -k "stream or shape_specialised or linear_program or own_spp or equals_cpu or path_exact or contract" > gpurun_out/r06/s19_tests.log 2>&1 \
    || { tail -30 gpurun_out/r06/s19_tests.log; exit 3; }
tail -2 gpurun_out/r06/s19_tests.log
LIBS="specmaj spec8" CFGS="8,1024,1024,256 9,800,800,256" ROUNDS=2 bash tools/ab.sh || exit 3
