#!/bin/bash
# Round-4 probe batch H: occupancy of the path-exact book2 kernel (C5's scene, fast contract):
# in-tree 4 waves/SIMD in 1 x 16-wave groups; p5a 5 waves in 4-wave groups; p5b 5 waves in
# 2 x 10; p6 6 waves in 2 x 12 (spills).
mkdir -p gpurun_out
LIBS="p5a p5b p6" CFGS="7,2048,2048,64" STEPS=3 ROUNDS=2 timeout -k 10 400 bash tools/ab.sh > gpurun_out/r04_ab_pex.log 2>&1 || exit 1
cat gpurun_out/r04_ab_pex.log
