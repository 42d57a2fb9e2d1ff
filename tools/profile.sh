#!/bin/bash
# rocprofv3 passes for the C2 bench (run on the GPU box from the repo root):
#   1. kernel trace + stats            -> gpurun_out/prof/trace
#   2. FETCH_SIZE / WRITE_SIZE         -> separate PMC passes (gfx950 TCC slot limits)
#   3. SQ counters (VALU activity, waits)
# Each pass under its own time limit; any failure stops the script.
set -e
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/prof
mkdir -p $OUT
ARGS=${PROF_ARGS:-"--steps 1 --warmup 0 --no-cpu-baseline"}
rocprofv3 -L > $OUT/counters.txt 2>&1 || true
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/trace -o run --output-format csv -- python3 bench.py $ARGS > $OUT/trace.log 2>&1
echo trace done
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE -d $OUT/fetch -o run --output-format csv -- python3 bench.py $ARGS > $OUT/fetch.log 2>&1
echo fetch done
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE -d $OUT/write -o run --output-format csv -- python3 bench.py $ARGS > $OUT/write.log 2>&1
echo write done
if [ -n "${PROF_SQ:-}" ]; then
  timeout -k 10 300 rocprofv3 --pmc $PROF_SQ -d $OUT/sq -o run --output-format csv -- python3 bench.py $ARGS > $OUT/sq.log 2>&1
  echo sq done
fi
find $OUT -name "*.csv" | head -50
