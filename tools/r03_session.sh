#!/bin/bash
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
step() {
    local name=$1 t=$2; shift 2
    echo "== $name $(date +%T)"
    timeout -k 10 "$t" "$@" > "gpurun_out/$name.log" 2>&1
    local rc=$?
    echo "== $name rc=$rc $(date +%T)"
    tail -1 "gpurun_out/$name.log" | cut -c1-400
    if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "stopping after $name (rc=$rc)"; exit $rc; fi
    return 0
}
step gpu_tests 900 python -u -m pytest tests/ -v -m gpu --timeout 300 --timeout-method thread
step par7 200 python tools/parity_record.py --scenes 7 --out gpurun_out/par7_unitfix.json
B="python bench.py --no-cpu-baseline --no-compare-numerics --no-other-walk --no-parity --steps 20 --warmup 5"
for p in 1 2 3; do for i in 1 2 3 4; do step pipe${p}_$i 120 $B --pipeline $p; done; done
for p in 1 2 3; do step w8pipe$p 120 $B --steps 40 --emulate-world 8 --emulate-gather --pipeline $p; done
CFGS="7,2048,2048,64 0,1200,800,64 1,1200,800,64" LIBS="plainwide" step ab 900 bash tools/ab_walk.sh
exit 0
