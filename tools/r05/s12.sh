# round-5: the interpreter (MRT_NO_SIG=1) without the room op's per-lane lookup table in scratch:
# 5 waves/SIMD (in tree, 81 VGPRs) vs 6 (w6, 80) and 7 (w7, 72 + 5 spilled); C2 and scene 6
# (Cornell smoke, the catch-all machine); GPU tests
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
O=gpurun_out/r05
mkdir -p $O
timeout -k 10 500 python3 -u -m pytest tests -m gpu -q -x --timeout 200 --timeout-method thread > $O/gpu_tests_12.log 2>&1 || exit 1
MRT_NO_SIG=1 ROUNDS=2 STEPS=10 LIBS="w6 w7" CFGS="5,500,500,1024 6,500,500,256" timeout -k 10 600 bash tools/ab.sh > $O/ab_s12.txt 2>&1
