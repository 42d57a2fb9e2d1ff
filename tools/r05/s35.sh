# round-5: the resumable mesh loop's radiance store held for the next iteration (in tree) vs issued
# at the path's end (nohs); C3 and C4; GPU tests
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
O=gpurun_out/r05
mkdir -p $O
timeout -k 10 500 python3 -u -m pytest tests -m gpu -q -x --timeout 200 --timeout-method thread > $O/gpu_tests_35.log 2>&1 || exit 1
ROUNDS=3 STEPS=10 LIBS="nohs" CFGS="9,800,800,256 8,1024,1024,64" timeout -k 10 800 bash tools/ab.sh > $O/ab_s35.txt 2>&1
