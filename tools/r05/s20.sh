# round-5: the interpreter parks the query ray only for programs that need it (in tree; nopark =
# always, as before) and fetches the instance's words before the record's node (nopref = after);
# C2 through the interpreter; GPU tests
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
O=gpurun_out/r05
mkdir -p $O
timeout -k 10 500 python3 -u -m pytest tests -m gpu -q -x --timeout 200 --timeout-method thread > $O/gpu_tests_20.log 2>&1 || exit 1
MRT_NO_SIG=1 ROUNDS=3 STEPS=10 LIBS="nopark nopref" CFGS="5,500,500,1024" timeout -k 10 600 bash tools/ab.sh > $O/ab_s20.txt 2>&1
