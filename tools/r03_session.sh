#!/bin/bash
# round-3: Bvh4 walk (two bvh_node levels per visit) against the binary walk; GPU suite
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
for rep in 1 2; do
  CFGS="7,2048,2048,64 0,1200,800,64 1,1200,800,64 5,500,500,1024" LIBS="bin" step ab_bvh4_$rep 900 bash tools/ab_walk.sh
done
exit 0
