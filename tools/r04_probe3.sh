#!/bin/bash
# Round-4 probe batch C: GPU parity suite on the slab-op gating, then A/B of the bvh_node +
# volume variant (exp/libmrt_nob2.so: without it) and of 1 x 16-wave groups (exp/libmrt_t16.so).
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -q --timeout 300 --timeout-method thread > gpurun_out/r04_t4.log 2>&1
rc=$?; tail -6 gpurun_out/r04_t4.log; [ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
LIBS="nob2 t16" CFGS="7,2048,2048,64 0,1200,800,64" STEPS=3 ROUNDS=2 timeout -k 10 500 bash tools/ab.sh > gpurun_out/r04_ab_c5.log 2>&1 || exit 1
cat gpurun_out/r04_ab_c5.log
