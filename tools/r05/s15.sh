# round-5: a kernel variant shaped for book2 (bvh_node + volumes + textures + motion, no mesh / sky /
# biased sphere / generic bvh walk) vs the catch-all interpreter kernel it ran on (nob2); C5; tests
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
O=gpurun_out/r05
mkdir -p $O
timeout -k 10 500 python3 -u -m pytest tests -m gpu -q -x --timeout 200 --timeout-method thread > $O/gpu_tests_15.log 2>&1 || exit 1
ROUNDS=3 STEPS=5 LIBS="nob2" CFGS="7,2048,2048,64" timeout -k 10 600 bash tools/ab.sh > $O/ab_s15.txt 2>&1
