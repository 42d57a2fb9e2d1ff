#!/bin/bash
# rocprofv3 passes for one bench workload (run on the GPU box from the repo root), each pass a run
# of its own under its own time limit; any failure stops the script:
#   1. kernel trace + stats                               -> gpurun_out/prof/trace
#   2. FETCH_SIZE, 3. WRITE_SIZE (separate: TCC slots)    -> gpurun_out/prof/{fetch,write}
#   4. SQ counters (VALU issue / lanes / waits) + GRBM_GUI_ACTIVE (clock) -> gpurun_out/prof/sq
# The bench runs with --pipeline 1 so no two kernels of the workload overlap in a counter window.
# PROF_ARGS selects the workload (default: C2, both numerics contracts in one process).
set -e
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=${PROF_OUT:-gpurun_out/prof}
mkdir -p $OUT
ARGS=${PROF_ARGS:-"--steps 1 --warmup 0 --kernel-reps 1 --pipeline 1 --no-cpu-baseline --no-other-walk --no-parity"}
SQ=${PROF_SQ:-"SQ_WAVES,SQ_INSTS_VALU,SQ_ACTIVE_INST_VALU,SQ_THREAD_CYCLES_VALU,SQ_WAVE_CYCLES,SQ_WAIT_ANY,SQ_WAIT_INST_ANY,SQ_BUSY_CYCLES,GRBM_GUI_ACTIVE"}
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/trace -o run --output-format csv -- python3 bench.py $ARGS > $OUT/trace.log 2>&1
echo "trace done $(date +%T)"
timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE -d $OUT/fetch -o run --output-format csv -- python3 bench.py $ARGS > $OUT/fetch.log 2>&1
echo "fetch done $(date +%T)"
timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE -d $OUT/write -o run --output-format csv -- python3 bench.py $ARGS > $OUT/write.log 2>&1
echo "write done $(date +%T)"
timeout -s KILL 300 rocprofv3 --pmc $SQ -d $OUT/sq -o run --output-format csv -- python3 bench.py $ARGS > $OUT/sq.log 2>&1
echo "sq done $(date +%T)"
