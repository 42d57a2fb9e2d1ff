#!/bin/bash
# round-3 measurement session: tests, parity record, default bench, rocprofv3 profiles of C2-C5,
# contract A/B, full-size configs, scaling rehearsal.  Every GPU step under its own time limit; a
# crash / fault / timeout (any status other than 0 or 1) stops the call.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
step() {
    local name=$1 t=$2; shift 2
    echo "== $name $(date +%T)"
    timeout -k 10 "$t" "$@" > "gpurun_out/$name.log" 2>&1
    local rc=$?
    echo "== $name rc=$rc $(date +%T)"
    tail -2 "gpurun_out/$name.log" | cut -c1-300
    if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "stopping after $name (rc=$rc)"; exit $rc; fi
    return 0
}
[ "${SKIP_TESTS:-0}" = 1 ] || step gpu_tests 900 python -u -m pytest tests/ -v -m gpu --timeout 300 --timeout-method thread
[ "${SKIP_SMOKE:-0}" = 1 ] || step smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
[ "${SKIP_PARITY:-0}" = 1 ] || step parity 600 python tools/parity_record.py --out gpurun_out/parity_final.json
[ "${SKIP_BENCH:-0}" = 1 ] || step bench 600 python bench.py --gpus 1 --steps 20 --warmup 5
[ "${SKIP_PROF:-0}" = 1 ] || step prof 900 bash tools/profile.sh
[ "${SKIP_PROF:-0}" = 1 ] || step prof_cfg 1200 bash tools/prof_configs.sh
[ "${SKIP_AB:-0}" = 1 ] || step contract_ab 900 python tools/contract_ab.py --measure
[ "${SKIP_CFG:-0}" = 1 ] || step configs 1200 bash tools/configs.sh
[ "${SKIP_SCALE:-0}" = 1 ] || CFGS="1,0 2,0 2,1 4,0 4,3 8,0 8,1 8,2 8,3 8,4 8,5 8,6 8,7" step scale 900 bash tools/scale_rehearsal.sh
[ "${SKIP_SCALE:-0}" = 1 ] || CFGS="2,0 4,0" SCALE_ARGS="--pipeline 1" step scale_p1 900 bash tools/scale_rehearsal.sh
[ "${SKIP_SCALE:-0}" = 1 ] || CFGS="2,0 4,0" SCALE_ARGS="--pipeline 3" step scale_p3 900 bash tools/scale_rehearsal.sh
exit 0
