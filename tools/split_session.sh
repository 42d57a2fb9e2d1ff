#!/bin/bash
# GPU session of the split-form A/B (round 4): the path-exact kernels' workgroup shapes for the
# persistent kernel (<lib>:0) and the split form, book2 at C5's resolution (64 spp) and scene 6.
set -e
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
LIBS="p5g256:0 p5g256 p5g512:0 p5g512 p4:0 p4 w6" ROUNDS=2 tools/split_ab.sh > gpurun_out/s5_split_ab.txt 2>&1
CFGS="6,600,600,64" LIBS="p5g256:0 p5g256" ROUNDS=1 tools/split_ab.sh >> gpurun_out/s5_split_ab.txt 2>&1
