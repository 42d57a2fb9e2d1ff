#!/bin/bash
# round 6 session 15: the treelet's nodes chosen by surface area instead of by depth
# (MRT_TREELET_ORDER=area, mrt_render.hip area_order): GPU tests of the bvh_node scenes with it,
# then A/B on C5 and random spheres (the treelet kernels)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out/r06
set -o pipefail
MRT_TREELET_ORDER=area timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -x -v -m gpu --timeout 200 --timeout-method thread \
    -k "stream or linear_program or own_spp or equals_cpu or path_exact or contract" > gpurun_out/r06/s15_tests.log 2>&1 \
    || { tail -30 gpurun_out/r06/s15_tests.log; exit 3; }
tail -2 gpurun_out/r06/s15_tests.log
LIBS="MRT_TREELET_ORDER=area" CFGS="7,2048,2048,64 0,1200,800,64 2,1200,800,64" ROUNDS=3 bash tools/ab.sh || exit 3
