# round-5: C3's room + mesh kernel at 8 waves/SIMD (m8: 62 VGPRs, no VGPR spill) vs 7 (in tree, 66)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
O=gpurun_out/r05
mkdir -p $O
ROUNDS=3 STEPS=10 LIBS="m8" CFGS="9,800,800,256" timeout -k 10 600 bash tools/ab.sh > $O/ab_s36.txt 2>&1
