#!/bin/bash
# Round-3 A/B call: the in-tree library against exp/libmrt_$LIB.so on C2 (interleaved), then
# C1 / C3 / C4 / C5 shapes, then the GPU suite against the variant.  Every step under its own limit;
# any failure ends the call.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
LIB=${LIB:-v2}
step() {
    local name=$1 t=$2; shift 2
    echo "== $name $(date +%T)"
    timeout -k 10 "$t" "$@" > "gpurun_out/$name.log" 2>&1
    local rc=$?
    echo "== $name rc=$rc $(date +%T)"
    grep -E "scene|passed|failed|error" "gpurun_out/$name.log" | tail -12 | cut -c1-300
    if [ $rc -ne 0 ]; then echo "stopping after $name (rc=$rc)"; exit $rc; fi
    return 0
}
LIBS=$LIB ROUNDS=3 step ab_c2 600 bash tools/ab.sh
LIBS=$LIB ROUNDS=1 STEPS=3 CFGS="0,1200,800,64 9,800,800,256 8,1024,1024,256 7,2048,2048,64" step ab_cfg 900 bash tools/ab.sh
[ "${SKIP_TESTS:-0}" = 1 ] || MRT_EXPERIMENT_LIB=exp/libmrt_$LIB.so step gpu_tests_$LIB 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread
exit 0
