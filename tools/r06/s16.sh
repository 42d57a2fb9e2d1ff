#!/bin/bash
# round 6 session 16: the work_queue tile size of the rank deal (bench --tile-size, the reference's
# -tilesize): 4-px tiles against 8 -- every N = 8 share of C2 and the N = 1 step at each
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out/r06
V="1,0,n1_t8,--tile-size 8;1,0,n1_t4,--tile-size 4"
for r in 0 1 2 3 4 5 6 7; do V="$V;8,$r,n8r${r}_t8,--tile-size 8;8,$r,n8r${r}_t4,--tile-size 4"; done
VARIANTS="$V" ROUNDS=1 STEPS=60 bash tools/scale_variants.sh || exit 3
