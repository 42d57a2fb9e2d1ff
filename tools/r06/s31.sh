#!/bin/bash
# round 6 session 31: the resumable mesh walk's tuning re-measured on the final tree (its box tests
# cheaper since section 21): leaf postponing by majority in the FAST build (spec; the teapot, C3),
# three walk steps per yield check (u3; fast and path-exact), the yield threshold (MRT_WALK_MIN
# 24 / 40 / 48), against the tree (intree) and the same flags built by tools/build_variant.sh (ctl)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out/r06
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q -m gpu --timeout 200 --timeout-method thread -k "shape_specialised or (full_resolution and fast) or (own_spp and fast)" > gpurun_out/r06/s31_tests.log 2>&1 || { tail -20 gpurun_out/r06/s31_tests.log; exit 3; }
tail -1 gpurun_out/r06/s31_tests.log
for lib in spec u3; do
  MRT_EXPERIMENT_LIB=exp/libmrt_$lib.so timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q -m gpu --timeout 200 --timeout-method thread -k "shape_specialised or (full_resolution and fast) or (own_spp and fast)" > gpurun_out/r06/s31_tests_$lib.log 2>&1 || { tail -20 gpurun_out/r06/s31_tests_$lib.log; exit 3; }
  echo "$lib: $(tail -1 gpurun_out/r06/s31_tests_$lib.log)"
done
LIBS="ctl spec u3 MRT_WALK_MIN=24 MRT_WALK_MIN=40 MRT_WALK_MIN=48" CFGS="9,800,800,256 8,1024,1024,256" ROUNDS=2 bash tools/ab.sh || exit 3
