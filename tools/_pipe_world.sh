#!/bin/bash
# experiment: pipeline depth per rank share (bench --emulate-world N, automatic fold)
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
for n in 4 8; do for p in 1 2 3 4; do
  timeout -k 10 200 python bench.py --no-cpu-baseline --no-compare-numerics --steps 40 --emulate-world $n --pipeline $p > gpurun_out/pw_${n}_$p.log 2>&1 || exit 3
  python tools/_show.py gpurun_out/pw_${n}_$p.log "world=$n pipeline=$p"
done; done
