# round-5: interpreter without the box instance's own box test (now in tree); 6 waves/SIMD (in tree,
# 79 VGPRs) vs 7 (w7, 72 + 1 spilled); GPU tests
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
O=gpurun_out/r05
mkdir -p $O
timeout -k 10 500 python3 -u -m pytest tests -m gpu -q -x --timeout 200 --timeout-method thread > $O/gpu_tests_29.log 2>&1 || exit 1
MRT_NO_SIG=1 ROUNDS=3 STEPS=10 LIBS="w7" CFGS="5,500,500,1024" timeout -k 10 600 bash tools/ab.sh > $O/ab_s29.txt 2>&1
