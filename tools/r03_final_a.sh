#!/bin/bash
# round-3 final tree, part A: GPU suite, smoke, rocprofv3 kernel trace + PMC passes for C2 and for
# C3-C5 at full resolution (tools/profile.sh, tools/prof_configs.sh), contract A/B measurement.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
step() {
    local name=$1 t=$2; shift 2
    echo "== $name $(date +%T)"
    timeout -k 10 "$t" "$@" > "gpurun_out/$name.log" 2>&1
    local rc=$?
    echo "== $name rc=$rc $(date +%T)"
    tail -3 "gpurun_out/$name.log" | cut -c1-300
    if [ $rc -ne 0 ]; then echo "stopping after $name (rc=$rc)"; exit $rc; fi
    return 0
}
step gpu_tests 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread
step smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
step prof_c2 900 bash tools/profile.sh
step prof_cfgs 1500 bash tools/prof_configs.sh
step contract_ab 900 python tools/contract_ab.py --measure
exit 0
