# round-5: C2's Cornell kernel at 8 waves/SIMD (l8: 64 VGPRs, 1 spilled) vs 7 (in tree, 67)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
O=gpurun_out/r05
mkdir -p $O
ROUNDS=3 STEPS=20 LIBS="l8" CFGS="5,500,500,1024" timeout -k 10 600 bash tools/ab.sh > $O/ab_s38.txt 2>&1
