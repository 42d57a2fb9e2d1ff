#!/bin/bash
# experiment: lean vs full fold on one rank's tile share (bench --emulate-world N), three contexts
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
for n in 1 2 4 8; do for f in lean full; do
  timeout -k 10 200 python bench.py --no-cpu-baseline --no-compare-numerics --steps 30 --emulate-world $n --fold $f > gpurun_out/fw_${n}_$f.log 2>&1 || exit 3
  python tools/_show.py gpurun_out/fw_${n}_$f.log "world=$n $f"
done; done
