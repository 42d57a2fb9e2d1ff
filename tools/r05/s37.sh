# round-5: GPU tests with the fast room + mesh kernel at 8 waves; C4's path-exact room + mesh kernel
# at 8 waves/SIMD (p8: 64 VGPRs, 9 spilled) vs 7 (in tree, 72, 1 spilled); C3 in tree for reference
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
O=gpurun_out/r05
mkdir -p $O
timeout -k 10 500 python3 -u -m pytest tests -m gpu -q -x --timeout 200 --timeout-method thread > $O/gpu_tests_37.log 2>&1 || exit 1
ROUNDS=3 STEPS=10 LIBS="p8" CFGS="8,1024,1024,64 9,800,800,256" timeout -k 10 800 bash tools/ab.sh > $O/ab_s37.txt 2>&1
