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
# radiance write amplification vs claim size (C2, fast contract): HBM counters per build
for L in intree bat128 bat64; do
  if [ $L = intree ]; then unset MRT_EXPERIMENT_LIB; else export MRT_EXPERIMENT_LIB=exp/libmrt_$L.so; fi
  PROF_OUT=gpurun_out/prof_$L timeout -k 10 600 bash tools/profile.sh > gpurun_out/prof_$L.log 2>&1 || exit 1
  python tools/pmc_summary.py r04_claim_$L --prof gpurun_out/prof_$L --no-bench-file > gpurun_out/pmc_$L.txt 2>&1; tail -5 gpurun_out/pmc_$L.txt; cp profiles/r04_claim_${L}_pmc.json gpurun_out/ 2>/dev/null || true
done
unset MRT_EXPERIMENT_LIB
