#!/bin/bash
# round-3: GPU suite on the new claim policy; pipeline depth at an 8-rank share; host-side biased-list count A/B
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
step() {
    local name=$1 t=$2; shift 2
    echo "== $name $(date +%T)"
    timeout -k 10 "$t" "$@" > "gpurun_out/$name.log" 2>&1
    local rc=$?
    echo "== $name rc=$rc $(date +%T)"
    cat "gpurun_out/$name.log" | cut -c1-300
    if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "stopping after $name (rc=$rc)"; exit $rc; fi
    return 0
}
step gpu_tests 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread
for rep in 1 2 3; do
  for p in 1 2 3; do
    CFGS="8,1" STEPS=60 SCALE_ARGS="--pipeline $p" step pipe_p${p}_$rep 300 bash tools/scale_rehearsal.sh
  done
done
CFGS="7,2048,2048,64 0,1200,800,64 1,1200,800,64" LIBS="old" step ab_nbleaf 900 bash tools/ab_walk.sh
exit 0
