# round-5: the async fold as bench.py's default at one context: its GPU test, the full GPU suite,
# two ranks on one GPU over gloo with the async fold (gather on its own stream after join) and
# --verify, and the default bench line
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
O=gpurun_out/r05
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k async_fold > $O/s43_test.log 2>&1 || exit 3
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/s43_suite.log 2>&1 || exit 4
MRT_SAME_GPU=1 MRT_DIST_BACKEND=gloo timeout -k 10 200 python bench.py --gpus 2 --steps 3 --warmup 1 --no-cpu-baseline \
    --no-other-walk --no-compare-numerics --verify > $O/s43_world2_gloo.log 2>&1 || exit 5
timeout -k 10 400 python bench.py > $O/s43_bench.log 2>&1 || exit 6
