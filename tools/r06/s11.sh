#!/bin/bash
# round 6 session 11: the async fold's retrace beside the next launch in slots that launch leaves free
# (kRetraceSide): its GPU tests, the suite, then A/B against MRT_RETRACE_SIDE=0 (the retrace on the
# render's stream) and other slot counts, C2 at N = 1 and the N = 8 share 6 at each step shape
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out/r06
set -o pipefail
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -v -m gpu --timeout 120 --timeout-method thread \
    -k "async or retrace" > gpurun_out/r06/s11_new.log 2>&1 || { tail -30 gpurun_out/r06/s11_new.log; exit 3; }
tail -3 gpurun_out/r06/s11_new.log
timeout -k 10 600 python -u -m pytest tests/ -x -v -m gpu --timeout 240 --timeout-method thread > gpurun_out/r06/s11_suite.log 2>&1
rc=$?; tail -3 gpurun_out/r06/s11_suite.log
[ $rc -eq 0 ] || exit $rc
LIBS="MRT_RETRACE_SIDE=0 MRT_RETRACE_SIDE=64" CFGS="5,500,500,1024" STEPS=30 ROUNDS=3 bash tools/ab.sh || exit 3
for shape in "--pipeline 1 --fold async" "--pipeline 2 --fold async"; do
  echo "== N = 8 share 6: $shape"
  BENCH_ARGS="--emulate-world 8 --emulate-rank 6 --emulate-gather $shape" LIBS="MRT_RETRACE_SIDE=0 MRT_RETRACE_SIDE=64" CFGS="5,500,500,1024" \
      STEPS=60 ROUNDS=2 bash tools/ab.sh || exit 3
done
echo "== N = 8 share 6: --pipeline 3 --fold full"
BENCH_ARGS="--emulate-world 8 --emulate-rank 6 --emulate-gather --pipeline 3 --fold full" CFGS="5,500,500,1024" STEPS=60 ROUNDS=2 bash tools/ab.sh || exit 3
