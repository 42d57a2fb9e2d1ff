#!/bin/bash
# check: run-to-run spread of the default bench on one box (and the full fold beside it)
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
for i in 1 2 3; do
  timeout -k 10 200 python bench.py --no-cpu-baseline --steps 20 > gpurun_out/rep_$i.log 2>&1 || exit 3
  python tools/_show.py gpurun_out/rep_$i.log "default run $i"
done
timeout -k 10 200 python bench.py --no-cpu-baseline --steps 20 --fold full > gpurun_out/rep_full.log 2>&1 || exit 3
python tools/_show.py gpurun_out/rep_full.log "full fold"
timeout -k 10 200 python bench.py --no-cpu-baseline --steps 20 --fold full --pipeline 2 > gpurun_out/rep_full2.log 2>&1 || exit 3
python tools/_show.py gpurun_out/rep_full2.log "full fold pipeline 2"
