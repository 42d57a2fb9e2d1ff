#!/bin/bash
# Round-4 probe batch J: exact division without the IEEE sequence (div_x) -- GPU suite (bit-exact
# fixtures) and A/B against the tree before it (exp/libmrt_head.so): C4 / C5 tolerance contract
# (path-exact kernels), C2 exact contract.
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -q -x --timeout 300 --timeout-method thread > gpurun_out/r04_t7.log 2>&1
rc=$?; tail -4 gpurun_out/r04_t7.log; [ $rc -eq 0 ] || exit $rc
LIBS="head" CFGS="8,1024,1024,256 7,2048,2048,64" STEPS=3 ROUNDS=2 timeout -k 10 400 bash tools/ab.sh > gpurun_out/r04_ab_dx.log 2>&1 || exit 1
cat gpurun_out/r04_ab_dx.log
BENCH_ARGS="--numerics exact" LIBS="head" CFGS="5,500,500,1024 9,800,800,256" STEPS=5 ROUNDS=2 timeout -k 10 400 bash tools/ab.sh > gpurun_out/r04_ab_dx2.log 2>&1 || exit 1
cat gpurun_out/r04_ab_dx2.log
# the interpreter's rect records from registers: the same bits as through the node load (norr)
for L in intree norr; do
  if [ $L = intree ]; then unset MRT_EXPERIMENT_LIB; else export MRT_EXPERIMENT_LIB=exp/libmrt_$L.so; fi
  for sid in 5 9; do MRT_NO_SIG=1 timeout -k 10 120 python tools/img_md5.py $sid 96 96 64 || exit 1; done
done
unset MRT_EXPERIMENT_LIB
MRT_NO_SIG=1 LIBS="head norr" CFGS="5,500,500,1024" STEPS=10 ROUNDS=2 timeout -k 10 300 bash tools/ab.sh > gpurun_out/r04_ab_park.log 2>&1 || exit 1
cat gpurun_out/r04_ab_park.log
# scene 6 (Cornell smoke: volumes in instances, the generic machine; path-exact under the tolerance contract)
timeout -k 10 300 python bench.py --no-cpu-baseline --no-other-walk --steps 3 --warmup 1 --scene 6 --width 600 --height 600 --samples 256 > gpurun_out/r04_scene6.log 2>&1 || exit 1
python tools/show_bench.py gpurun_out/r04_scene6.log "scene 6 600x600x256"
# the 8-rank share (rank 6, the slowest share in the rehearsals) at 3 / 4 / 6 pipelined contexts
for NP in 3 4 6; do
  timeout -k 10 200 python bench.py --no-cpu-baseline --no-compare-numerics --no-other-walk --no-parity --steps 120 --warmup 4 \
      --emulate-world 8 --emulate-rank 6 --emulate-gather --pipeline $NP > gpurun_out/r04_pipe_$NP.log 2>&1 || exit 1
  python tools/show_bench.py gpurun_out/r04_pipe_$NP.log "8-rank share 6, $NP contexts"
done
