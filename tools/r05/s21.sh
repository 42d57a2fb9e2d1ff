# round-5 final tree, part 1: GPU suite, smoke, the default bench line (with the CPU baseline), and
# the BASELINE configs C2-C5 at full size
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
O=gpurun_out/r05
mkdir -p $O
timeout -k 10 500 python3 -u -m pytest tests -m gpu -q -x --timeout 200 --timeout-method thread > $O/gpu_tests_21.log 2>&1 || exit 1
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > $O/smoke_21.log 2>&1 || exit 1
timeout -k 10 400 python3 bench.py --steps 20 --warmup 5 > $O/bench_21.log 2>&1 || exit 1
timeout -k 10 900 bash tools/configs.sh > $O/configs_21.txt 2>&1
