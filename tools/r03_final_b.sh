#!/bin/bash
# round-3 final tree, part B (after the PMC summaries of part A are committed under profiles/):
# parity at every config's resolution, the full-size BASELINE configs, the 8-rank rehearsal and
# the default bench line (with the CPU baseline).
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
step parity 900 python tools/parity_record.py
step configs 1200 bash tools/configs.sh
CFGS="1,0 2,0 2,1 4,0 4,1 4,2 4,3 8,0 8,1 8,2 8,3 8,4 8,5 8,6 8,7" STEPS=60 step scale 900 bash tools/scale_rehearsal.sh
step bench 900 python bench.py
exit 0
