#!/bin/bash
# round 6 session 9: the GPU suite on the tree with the per-lane ray count in LDS (MRT_LDS_RAYS) and
# the exact interpreter at 5 waves; A/B of that count against a register (exp/libmrt_norays.so) and of
# the branch-free walk stacks (MRT_MESH_BF / MRT_BVHW_BF, exp/libmrt_bf.so) on C2, C5, C4, C3, random
# spheres; the exact interpreter in tree
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out/r06
set -o pipefail
timeout -k 10 600 python -u -m pytest tests/ -x -v -m gpu --timeout 240 --timeout-method thread > gpurun_out/r06/s9_suite.log 2>&1
rc=$?; tail -3 gpurun_out/r06/s9_suite.log
[ $rc -eq 0 ] || exit $rc
LIBS="norays bf" CFGS="5,500,500,1024 7,2048,2048,64 8,1024,1024,256 9,800,800,256 0,1200,800,64" ROUNDS=2 bash tools/ab.sh || exit 3
for r in 1 2; do
  MRT_NO_SIG=1 timeout -k 10 300 python bench.py --numerics exact --no-cpu-baseline --no-compare-numerics \
      --no-other-walk --no-parity --steps 6 --warmup 1 > gpurun_out/r06/s9_exint_$r.log 2>&1 || exit 3
  python tools/show_bench.py gpurun_out/r06/s9_exint_$r.log "exact interp (5 waves) $r"
done
