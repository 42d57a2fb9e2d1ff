#!/bin/bash
# round-3: per-wave mesh treelet again, now read with LDS instructions
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
for rep in 1 2; do
  CFGS="8,1024,1024,256 9,800,800,256" LIBS="mtree" step ab_mtree_$rep 900 bash tools/ab_walk.sh
done
exit 0
