#!/bin/bash
# Round-4 probe batch G: the path-exact tolerance variants (kPathExact): GPU suite, own-spp parity
# and speed of both contracts, C2 bench.
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -q --timeout 300 --timeout-method thread > gpurun_out/r04_t6.log 2>&1
rc=$?; tail -6 gpurun_out/r04_t6.log; [ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 300 python -u tools/contract_parity.py fast exact > gpurun_out/r04_cp3.log 2>&1 || exit 1
cut -c1-200 gpurun_out/r04_cp3.log
timeout -k 10 200 python bench.py --no-cpu-baseline --steps 10 > gpurun_out/r04_bench_a.log 2>&1 || exit 1
python tools/show_bench.py gpurun_out/r04_bench_a.log "bench C2"
