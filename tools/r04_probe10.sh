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
# scene 6 (Cornell smoke: volumes in instances, the generic machine; path-exact under the tolerance contract)
timeout -k 10 300 python bench.py --no-cpu-baseline --no-other-walk --steps 3 --warmup 1 --scene 6 --width 600 --height 600 --samples 256 > gpurun_out/r04_scene6.log 2>&1 || exit 1
python tools/show_bench.py gpurun_out/r04_scene6.log "scene 6 600x600x256"
