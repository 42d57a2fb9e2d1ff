#!/bin/bash
# round-2 final-tree measurement call: GPU suite, default bench, rocprofv3 stats of the default bench
# command, profile.sh passes for C2 and C3-C5, full-size config renders (each step time-limited)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/gt.log 2>&1 || { tail -5 gpurun_out/gt.log; exit 1; }
tail -1 gpurun_out/gt.log
timeout -k 10 300 python bench.py > gpurun_out/bench.log 2>&1 || exit 2
tail -1 gpurun_out/bench.log | cut -c1-200
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/benchprof -o run --output-format csv -- python3 bench.py --no-cpu-baseline > gpurun_out/benchprof.log 2>&1 || exit 3
echo "bench prof done $(date +%T)"
timeout -k 10 400 bash tools/profile.sh > gpurun_out/prof.log 2>&1 || exit 4
echo "prof done $(date +%T)"
timeout -k 10 600 bash tools/prof_configs.sh > gpurun_out/profcfg.log 2>&1 || exit 5
echo "prof_configs done $(date +%T)"
timeout -k 10 300 bash tools/configs.sh > gpurun_out/configs.log 2>&1 || exit 6
echo "configs done $(date +%T)"
