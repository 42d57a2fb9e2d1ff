#!/bin/bash
# One GPU call: smoke -> GPU parity tests -> bench -> rocprofv3 passes of the C2 bench.  Every step
# under its own time limit; a crash / fault / timeout (any status other than 0 or 1) stops the call.
# SKIP_SMOKE / SKIP_TESTS / SKIP_BENCH / SKIP_PROF=1 drop steps; TESTS selects pytest targets.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
step() {  # name timeout cmd...
    local name=$1 t=$2; shift 2
    echo "== $name $(date +%T)"
    timeout -k 10 "$t" "$@" > "gpurun_out/$name.log" 2>&1
    local rc=$?
    echo "== $name rc=$rc $(date +%T)"
    tail -4 "gpurun_out/$name.log"
    if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "stopping after $name (rc=$rc)"; exit $rc; fi
    return 0
}
[ "${SKIP_SMOKE:-0}" = 1 ] || step smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
[ "${SKIP_TESTS:-0}" = 1 ] || step gpu_tests 900 python -u -m pytest ${TESTS:-tests/} -x -v -m gpu --timeout 300 --timeout-method thread
[ "${SKIP_BENCH:-0}" = 1 ] || step bench 600 python bench.py ${BENCH_ARGS:-}
[ "${SKIP_PROF:-0}" = 1 ] || step prof 900 bash tools/profile.sh
[ "${PROF_CFG:-0}" = 1 ] && step prof_cfg 1200 bash tools/prof_configs.sh
exit 0
