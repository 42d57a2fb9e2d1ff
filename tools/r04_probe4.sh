#!/bin/bash
# Round-4 probe batch D: the interpreter's one-step box instances (MRT_F_BOXINST) on C2 through
# the interpreter (MRT_NO_SIG=1): in-tree (6 waves/SIMD), lg5 (5 waves), nbx / nbx5 (the step not
# compiled in, 6 / 5 waves).
mkdir -p gpurun_out
MRT_NO_SIG=1 LIBS="lg5 nbx nbx5" CFGS="5,500,500,1024" STEPS=10 ROUNDS=2 timeout -k 10 400 bash tools/ab.sh > gpurun_out/r04_ab_boxinst2.log 2>&1 || exit 1
cat gpurun_out/r04_ab_boxinst2.log
