# round-5: the fast program rewrite drops the root object_list's LIST / LIST_END pair (in tree) vs
# keeps it (noroot); GPU tests; C2 through the interpreter
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
O=gpurun_out/r05
mkdir -p $O
timeout -k 10 500 python3 -u -m pytest tests -m gpu -q -x --timeout 200 --timeout-method thread > $O/gpu_tests_27.log 2>&1 || exit 1
MRT_NO_SIG=1 ROUNDS=3 STEPS=10 LIBS="noroot" CFGS="5,500,500,1024" timeout -k 10 600 bash tools/ab.sh > $O/ab_s27.txt 2>&1
