#!/bin/bash
# Round-4 probe batch I: the 8-rank rehearsal repeated (every rank's share, three passes, 60 and
# 240 timed steps) to see whether the slow rank is a property of a share or a random stall.
mkdir -p gpurun_out
for pass in 1 2 3; do
  for S in 60 240; do
    CFGS="8,0 8,1 8,2 8,3 8,4 8,5 8,6 8,7" STEPS=$S timeout -k 10 400 bash tools/scale_rehearsal.sh > gpurun_out/r04_reh_${pass}_$S.log 2>&1 || exit 1
    echo "pass $pass steps $S: $(grep -o '[0-9.]* ms/step' gpurun_out/r04_reh_${pass}_$S.log | cut -d' ' -f1 | tr '\n' ' ')"
  done
done
