# round-5: the interpreter's dispatch chain with the room op, the one-step box instance and box.h
# lists right after primitives (in tree) vs the former order (noro); C2 through the interpreter; tests
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
O=gpurun_out/r05
mkdir -p $O
timeout -k 10 500 python3 -u -m pytest tests -m gpu -q -x --timeout 200 --timeout-method thread > $O/gpu_tests_33.log 2>&1 || exit 1
MRT_NO_SIG=1 ROUNDS=3 STEPS=10 LIBS="noro" CFGS="5,500,500,1024" timeout -k 10 600 bash tools/ab.sh > $O/ab_s33.txt 2>&1
