#!/bin/bash
# Round-4 probe batch A: GPU parity suite, the two-level mesh walk (exp/libmrt_m4.so) parity and
# A/B, interpreter rewrite on/off.  Every GPU step has its own time limit; the batch stops at the
# first failing step.
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -q --timeout 300 --timeout-method thread > gpurun_out/r04_t3.log 2>&1
rc=$?; tail -8 gpurun_out/r04_t3.log; [ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
MRT_EXPERIMENT_LIB=exp/libmrt_m4.so timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -q -k "8 or 9" --timeout 300 --timeout-method thread > gpurun_out/r04_m4_parity.log 2>&1
rc=$?; tail -4 gpurun_out/r04_m4_parity.log; [ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
LIBS="m4 w6m" CFGS="9,800,800,256 8,1024,1024,256" STEPS=3 ROUNDS=2 timeout -k 10 400 bash tools/ab.sh > gpurun_out/r04_ab_m4.log 2>&1 || exit 1
cat gpurun_out/r04_ab_m4.log
MRT_EXPERIMENT_LIB=exp/libmrt_b2v.so timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -q -k "7" --timeout 300 --timeout-method thread > gpurun_out/r04_b2v_parity.log 2>&1
rc=$?; tail -4 gpurun_out/r04_b2v_parity.log; [ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
LIBS="b2v b2v16" CFGS="7,2048,2048,64" STEPS=3 ROUNDS=2 timeout -k 10 300 bash tools/ab.sh > gpurun_out/r04_ab_b2v.log 2>&1 || exit 1
cat gpurun_out/r04_ab_b2v.log
for V in 0 1; do
  MRT_NO_SIG=1 MRT_NO_REWRITE=$V timeout -k 10 200 python bench.py --no-cpu-baseline --no-compare-numerics --no-other-walk --no-parity --steps 10 > gpurun_out/r04_interp_$V.log 2>&1 || exit 1
  python tools/show_bench.py gpurun_out/r04_interp_$V.log "interpreter rewrite-off=$V"
done
