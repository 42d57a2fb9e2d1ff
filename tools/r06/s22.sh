#!/bin/bash
# round 6 session 22: leaf postponing by majority in the bvh_node walk (mrt_trace.h MRT_BVHW_SPEC:
# bs1 = a lane parks its first leaf and walks on, bs2 = the step type chosen by majority without
# parking) against the while-while walk; bit-exactness through bs1, then A/B on book2 (C5 shape),
# random spheres and scene 2
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out/r06
set -o pipefail
MRT_EXPERIMENT_LIB=exp/libmrt_bs1.so timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -x -v -m gpu --timeout 200 --timeout-method thread \
    -k "stream or shape_specialised or linear_program or own_spp or equals_cpu or path_exact or contract or wide" > gpurun_out/r06/s22_tests.log 2>&1 \
    || { tail -30 gpurun_out/r06/s22_tests.log; exit 3; }
tail -2 gpurun_out/r06/s22_tests.log
LIBS="bs1 bs2" CFGS="7,2048,2048,64 0,1200,800,64 2,800,400,256" ROUNDS=2 bash tools/ab.sh || exit 3
