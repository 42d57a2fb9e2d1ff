#!/bin/bash
# round 6 session 26: the wave's issue priority raised while it walks the scene (s_setprio 1 / 3 around
# the walk, MRT_PRIO_WALK: wp1 / wp3) against none, on C2, C5 shape, C4 shape, C3 shape
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out/r06
LIBS="wp1 wp3" CFGS="5,500,500,1024 7,2048,2048,64 8,1024,1024,256 9,800,800,256" ROUNDS=2 bash tools/ab.sh || exit 3
