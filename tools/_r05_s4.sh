# round-5: GPU tests, then A/B of the rounding-critical hand-over (nocrit), pixel sums (nopsum) and
# packed slabs (nopk)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out/r05
timeout -k 10 500 python3 -u -m pytest tests -m gpu -q -x --timeout 200 --timeout-method thread > gpurun_out/r05/gpu_tests_7.log 2>&1 || exit 1
export ROUNDS=2 STEPS=10 LIBS="nocrit nopsum nopk" CFGS="5,500,500,1024 9,800,800,256 8,1024,1024,64 7,2048,2048,64 0,1200,800,64"
timeout -k 10 900 bash tools/ab.sh > gpurun_out/r05/ab_s4.txt 2>&1
