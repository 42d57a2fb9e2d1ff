#!/bin/bash
# round 6 session 12: leaf postponing in the resumable mesh walk (mrt_trace.h mesh_step_spec,
# exp/libmrt_spec*.so: a leaf step once 32 / 16 / 48 lanes hold a parked run) and two / three walk
# steps between yield checks (exp/libmrt_wu2.so, wu3): bit-exactness of the room + mesh scenes through
# the spec build (GPU tests on scenes 8 / 9 with MRT_EXPERIMENT_LIB), then A/B on C4 and C3
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out/r06
set -o pipefail
for lib in spec wu2; do
  MRT_EXPERIMENT_LIB=exp/libmrt_$lib.so timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -x -v -m gpu --timeout 200 --timeout-method thread \
      -k "stream or shape_specialised or linear_program or own_spp or equals_cpu or path_exact or contract" > gpurun_out/r06/s12_tests_$lib.log 2>&1 \
      || { tail -30 gpurun_out/r06/s12_tests_$lib.log; exit 3; }
  tail -2 gpurun_out/r06/s12_tests_$lib.log
done
LIBS="spec spec16 spec48 wu2 wu3" CFGS="8,1024,1024,256 9,800,800,256" ROUNDS=2 bash tools/ab.sh || exit 3
# the default bench command under the rocprofv3 kernel trace (the bench line's kernel time against
# the trace's average)
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r06/bench_trace -o run --output-format csv -- python3 bench.py > gpurun_out/r06/s12_bench_trace.log 2>&1 || exit 3
python tools/show_bench.py gpurun_out/r06/s12_bench_trace.log "bench under the kernel trace"
