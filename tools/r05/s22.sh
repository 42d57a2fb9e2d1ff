# round-5: the retrace on the program as compiled (the interpreter's rewritten program has fast-only
# ops); GPU suite; bench line (other_walk parity)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
O=gpurun_out/r05
mkdir -p $O
timeout -k 10 500 python3 -u -m pytest tests -m gpu -q -x --timeout 200 --timeout-method thread -k "retraced or interpreter or smoke" -s > $O/gpu_tests_22a.log 2>&1 || exit 1
timeout -k 10 500 python3 -u -m pytest tests -m gpu -q -x --timeout 200 --timeout-method thread > $O/gpu_tests_22.log 2>&1 || exit 1
timeout -k 10 400 python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline > $O/bench_22.log 2>&1
