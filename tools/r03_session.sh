#!/bin/bash
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
step() {
    local name=$1 t=$2; shift 2
    echo "== $name $(date +%T)"
    timeout -k 10 "$t" "$@" > "gpurun_out/$name.log" 2>&1
    local rc=$?
    echo "== $name rc=$rc $(date +%T)"
    tail -4 "gpurun_out/$name.log"
    if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "stopping after $name (rc=$rc)"; exit $rc; fi
    return 0
}
step gpu_tests 900 python -u -m pytest tests/ -x -v -m gpu --timeout 300 --timeout-method thread
step parity 300 python tools/parity_record.py --scenes 5,9,8,7 --out gpurun_out/parity_s2.json
LIBS="lockstep nomtree" step ab 900 bash tools/ab_walk.sh
exit 0
