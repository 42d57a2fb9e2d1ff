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
step smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
step gpu_tests 900 python -u -m pytest tests/ -x -v -m gpu --timeout 300 --timeout-method thread -k "not full_resolution"
step parity 300 python tools/parity_record.py --scenes 5,9 --out gpurun_out/parity_s1.json
step bench 600 python bench.py --steps 20 --warmup 5
step prof 900 bash tools/profile.sh
exit 0
