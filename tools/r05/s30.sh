# round-5: interpreter: face nodes selected from the ops' uniform words (in tree) vs a per-lane load
# (nosel); the walk ending at the op flagged MRT_F_LAST (in tree) vs at the END op (nolast); tests
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
O=gpurun_out/r05
mkdir -p $O
timeout -k 10 500 python3 -u -m pytest tests -m gpu -q -x --timeout 200 --timeout-method thread > $O/gpu_tests_30.log 2>&1 || exit 1
MRT_NO_SIG=1 ROUNDS=3 STEPS=10 LIBS="nosel nolast" CFGS="5,500,500,1024" timeout -k 10 600 bash tools/ab.sh > $O/ab_s30.txt 2>&1
