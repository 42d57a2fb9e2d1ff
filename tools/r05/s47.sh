# round-5: the async fold over chunked renders (each launch's fold beside the next launch's kernel):
# its GPU tests, the full GPU suite, then C3 / C4 / C5 at full size, one render each, fold full vs
# async (bench --fold), interleaved per config
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
O=gpurun_out/r05
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k async_fold > $O/s47_test.log 2>&1 || exit 3
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/s47_suite.log 2>&1 || exit 4
for cfg in "9,800,800,4096" "8,1024,1024,2048" "7,2048,2048,8192"; do
  IFS=, read sid W H S <<< "$cfg"
  for f in full async; do
    log=$O/s47_${sid}_$f.log
    timeout -k 10 400 python bench.py --no-cpu-baseline --no-compare-numerics --no-other-walk --steps 1 --warmup 0 --kernel-reps 1 \
        --scene $sid --width $W --height $H --samples $S --fold $f > $log 2>&1 || exit 5
    python tools/show_bench.py $log "scene $sid $f"
    grep -o '"rmse": [0-9.e-]*' $log | head -1
  done
done
