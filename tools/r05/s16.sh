# round-5: the book2 variant's occupancy: in tree 6 waves/SIMD in two 12-wave groups (80 VGPRs, 39
# spilled) vs w5 = 5 in two 10-wave groups (96 VGPRs, spill-free) and w4 = 4 in one 16-wave group
# (103 VGPRs, spill-free); C5
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
O=gpurun_out/r05
mkdir -p $O
ROUNDS=3 STEPS=5 LIBS="w5 w4" CFGS="7,2048,2048,64" timeout -k 10 600 bash tools/ab.sh > $O/ab_s16.txt 2>&1
