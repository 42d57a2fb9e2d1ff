#!/bin/bash
# round-3: bf16 per-path radiance (tolerance contract): GPU suite, parity at every config, bench, 8-rank rehearsal
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
step parity 600 python tools/parity_record.py --numerics fast
step bench 600 python bench.py --no-cpu-baseline --no-other-walk --steps 20 --warmup 5
CFGS="1,0 8,0 8,1 8,2 8,3 8,4 8,5 8,6 8,7" STEPS=60 step scale_bf16 900 bash tools/scale_rehearsal.sh
exit 0
