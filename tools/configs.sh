#!/bin/bash
# BASELINE.json configs C2-C5 at their full sizes on one GPU (one timed render each; C4/C5 are
# 8-GPU configs in BASELINE.json, run here on one GPU for the per-GPU rate).  Each run under
# its own time limit; a failure stops the script.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
CFGS=${CFGS:-"5,500,500,1024 9,800,800,4096 8,1024,1024,2048 7,2048,2048,8192"}
for cfg in $CFGS; do
  IFS=, read sid W H S <<< "$cfg"
  echo "== scene $sid ${W}x${H} ${S}spp $(date +%T)"
  timeout -k 10 400 python bench.py --no-cpu-baseline --steps 1 --warmup 0 --kernel-reps 1 \
      --scene $sid --width $W --height $H --samples $S > gpurun_out/cfg_$sid.log 2>&1 || exit 3
  python tools/show_bench.py gpurun_out/cfg_$sid.log "scene $sid"
done
