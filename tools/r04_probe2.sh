#!/bin/bash
# Round-4 probe batch B: contract divergence and A/B of the fast-contract contraction builds
# (exp/libmrt_{foff,foffd,fon}.so), the launch timeline (exp/libmrt_wt.so).
mkdir -p gpurun_out
for L in intree foff foffd fon; do
  if [ $L = intree ]; then unset MRT_EXPERIMENT_LIB; else export MRT_EXPERIMENT_LIB=exp/libmrt_$L.so; fi
  timeout -k 10 150 python -u tools/divergence.py >> gpurun_out/r04_div2.log 2>&1 || exit 1
done
unset MRT_EXPERIMENT_LIB
cat gpurun_out/r04_div2.log
LIBS="foff foffd fon" CFGS="5,500,500,1024 7,2048,2048,64" STEPS=5 ROUNDS=2 timeout -k 10 400 bash tools/ab.sh > gpurun_out/r04_ab.log 2>&1 || exit 1
tail -20 gpurun_out/r04_ab.log
MRT_EXPERIMENT_LIB=exp/libmrt_wt.so timeout -k 10 120 python tools/wtimes.py 5 500 500 16 64 1024 > gpurun_out/r04_wtimes.log 2>&1 || exit 1
cat gpurun_out/r04_wtimes.log
