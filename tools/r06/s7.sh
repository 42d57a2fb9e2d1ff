#!/bin/bash
# round 6 session 7: the retrace of an async-fold launch on the fold stream (its own list per radiance
# parity): the GPU suite, the default bench, then C2 shares under each step shape
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out/r06
set -o pipefail
# (the GPU suite of this tree: session 6, same call)
timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/r06/s7_bench.log 2>&1 || exit 3
python tools/show_bench.py gpurun_out/r06/s7_bench.log "bench"
VARIANTS="1,0,n1,;8,6,n8r6_p3full,--pipeline 3 --fold full;8,6,n8r6_p1async,--pipeline 1 --fold async;8,6,n8r6_p2async,--pipeline 2 --fold async;8,6,n8r6_p3async,--pipeline 3 --fold async" \
    ROUNDS=2 bash tools/scale_variants.sh || exit 3
