# round-5: the interpreter's ops fetched whole into SGPRs (in tree) vs in place (nofetch), and the
# one-step box instance without its instance box test (noaabb); C2 through the interpreter; tests
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
O=gpurun_out/r05
mkdir -p $O
timeout -k 10 500 python3 -u -m pytest tests -m gpu -q -x --timeout 200 --timeout-method thread > $O/gpu_tests_13.log 2>&1 || exit 1
MRT_NO_SIG=1 ROUNDS=3 STEPS=10 LIBS="nofetch noaabb" CFGS="5,500,500,1024" timeout -k 10 600 bash tools/ab.sh > $O/ab_s13.txt 2>&1
