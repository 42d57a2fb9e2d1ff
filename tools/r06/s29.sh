#!/bin/bash
# round 6 session 29: s28 with the listening retrace on its own stream (on the fold stream it waited behind the previous
# launch's fold, which its 16 free slots had slowed to the length of the path kernel: s28 measured -6%)
# -- the GPU suite on this tree, then A/B against MRT_LISTEN=0 (the retrace after the path kernel):
# C2 and C3 steps, C2 N = 1 / N = 8 shares, and the kernel trace of the default bench
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out/r06
set -o pipefail
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/ -x -v -m gpu --timeout 240 --timeout-method thread > gpurun_out/r06/s29_suite.log 2>&1
rc=$?; tail -3 gpurun_out/r06/s29_suite.log
[ $rc -eq 0 ] || exit $rc
LIBS="MRT_LISTEN=8 MRT_LISTEN=0" CFGS="5,500,500,1024 9,800,800,256" ROUNDS=2 bash tools/ab.sh || exit 3
for v in 16 8 0; do
  for cfg in "1,0" "8,0" "8,6"; do
    IFS=, read n r <<< "$cfg"
    MRT_LISTEN=$v timeout -k 10 300 python bench.py --no-cpu-baseline --no-compare-numerics --no-other-walk --no-parity --steps 40 --warmup 4 \
        --emulate-world $n --emulate-rank $r --emulate-gather --step-times > gpurun_out/r06/s29_scale_${v}_${n}_$r.log 2>&1 || exit 3
    python tools/show_bench.py gpurun_out/r06/s29_scale_${v}_${n}_$r.log "listen=$v N=$n rank $r"
  done
done
timeout -s KILL 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r06/s29_kt -o run --output-format csv -- \
    python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-other-walk --no-compare-numerics > gpurun_out/r06/s29_kt.log 2>&1 || exit 3
f=$(find gpurun_out/r06/s29_kt -name "run_kernel_stats.csv" | head -1); cat "$f" | cut -c1-160 | head -12
