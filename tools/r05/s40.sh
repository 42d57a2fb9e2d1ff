# round-5: book2's path-exact kernel in three 8-wave groups per CU (g8, MRT_TREE_WG=512; each its own
# LDS treelet) vs two 12-wave groups (in tree); both 6 waves/SIMD; C5
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
O=gpurun_out/r05
mkdir -p $O
ROUNDS=3 STEPS=5 LIBS="g8" CFGS="7,2048,2048,64" timeout -k 10 600 bash tools/ab.sh > $O/ab_s40.txt 2>&1
