# round-5 final tree (bench default 20 steps): the default bench line, and the rocprofv3 kernel trace of the same
# default command
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
O=gpurun_out/r05
mkdir -p $O

timeout -k 10 400 python bench.py > $O/s49_bench.log 2>&1 || exit 4
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/s49_trace -o run --output-format csv -- python3 bench.py > $O/s49_trace.log 2>&1 || exit 5
