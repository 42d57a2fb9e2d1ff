# round-5: the last chunk's retrace beside the fold + a fixup of its pixels (in tree) vs the retrace
# before the fold (MRT_RETRACE_OVERLAP=0): GPU tests (incl. bit-identity of the two), A/B on C2 through
# both walks and C3; kernel trace of a C2 bench
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
O=gpurun_out/r05
mkdir -p $O
timeout -k 10 500 python3 -u -m pytest tests -m gpu -q -x --timeout 200 --timeout-method thread > $O/gpu_tests_32.log 2>&1 || exit 1
ROUNDS=3 STEPS=20 LIBS="MRT_RETRACE_OVERLAP=0" CFGS="5,500,500,1024 9,800,800,256" timeout -k 10 600 bash tools/ab.sh > $O/ab_s32.txt 2>&1 || exit 1
MRT_NO_SIG=1 ROUNDS=2 STEPS=10 LIBS="MRT_RETRACE_OVERLAP=0" CFGS="5,500,500,1024" timeout -k 10 300 bash tools/ab.sh > $O/ab_s32b.txt 2>&1 || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/kt_ov -o run --output-format csv -- python3 bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-other-walk --no-parity --no-compare-numerics > $O/kt_ov.log 2>&1
