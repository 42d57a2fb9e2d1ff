# round-5: the async fold's shape on C2 (in tree: 8 samples in flight, one 256-thread group per CU):
# wg128 / wg64 (a 128- / 64-thread group per CU), d4 (4 samples in flight); --verify
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
O=gpurun_out/r05
mkdir -p $O
ROUNDS=3 STEPS=20 LIBS="wg128 wg64 d4" CFGS="5,500,500,1024" BENCH_ARGS="--verify" timeout -k 10 600 bash tools/ab.sh > $O/ab_s52.txt 2>&1 || exit 3
grep -o '"verify_bit_exact": [a-z]*' gpurun_out/ab_*_5_*.log >> $O/ab_s52.txt
