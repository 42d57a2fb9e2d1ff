#!/bin/bash
# round-3: GPU suite, bvh/mesh A/B against the pre-change build, full rehearsal on the final claim policy and tile deal
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
CFGS="7,2048,2048,64 0,1200,800,64 1,1200,800,64 8,1024,1024,256 9,800,800,256" LIBS="old" step ab_final 900 bash tools/ab_walk.sh
CFGS="1,0 2,0 2,1 4,0 4,1 4,2 4,3 8,0 8,1 8,2 8,3 8,4 8,5 8,6 8,7" STEPS=60 step scale_final 900 bash tools/scale_rehearsal.sh
exit 0
