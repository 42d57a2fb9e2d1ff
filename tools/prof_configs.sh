#!/bin/bash
# rocprofv3 passes (tools/profile.sh) for the BASELINE workloads beyond C2, each into its own
# gpurun_out/prof_<name>: C3 teapot, C4 bunny, C5 book2 at their full resolution with fewer spp (the
# path kernel's per-ray behaviour does not depend on spp; one launch per render at these sizes).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
set -e
CFGS=${PROF_CFGS:-"c3:9:800:800:256 c4:8:1024:1024:256 c5:7:2048:2048:64"}
for cfg in $CFGS; do
  IFS=: read name sid W H S <<< "$cfg"
  PROF_OUT=gpurun_out/prof_$name PROF_ARGS="--steps 1 --warmup 0 --kernel-reps 1 --pipeline 1 --no-cpu-baseline --no-other-walk --no-parity --scene $sid --width $W --height $H --samples $S" \
    bash tools/profile.sh
  echo "== $name done $(date +%T)"
done
