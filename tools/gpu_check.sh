#!/bin/bash
# One GPU session: smoke -> GPU parity tests -> short bench.  Each GPU step has its own time
# limit; a crash / fault / timeout (exit status other than 0 or 1) stops the session there.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
step() {  # name timeout cmd...
    local name=$1 t=$2; shift 2
    echo "== $name $(date +%T)"
    timeout -k 10 "$t" "$@" > "gpurun_out/$name.log" 2>&1
    local rc=$?
    echo "== $name rc=$rc $(date +%T)"
    tail -5 "gpurun_out/$name.log"
    if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "stopping after $name (rc=$rc)"; exit $rc; fi
    return 0
}
[ "${SKIP_SMOKE:-0}" = 1 ] || step smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
[ "${SKIP_TESTS:-0}" = 1 ] || step gpu_tests 900 python -m pytest tests/ -x -q -m gpu
[ "${SKIP_BENCH:-0}" = 1 ] || step bench 900 python bench.py ${BENCH_ARGS:-}
