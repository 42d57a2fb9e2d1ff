# round-5: the async fold's shape on C2 (in tree: 8 samples in flight, one 256-thread group per CU):
# d16 (16 samples in flight, register cap 80), g2 (two groups per CU), d16g2; --verify
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
O=gpurun_out/r05
mkdir -p $O
ROUNDS=3 STEPS=20 LIBS="d16 g2 d16g2" CFGS="5,500,500,1024" BENCH_ARGS="--verify" timeout -k 10 600 bash tools/ab.sh > $O/ab_s51.txt 2>&1 || exit 3
grep -o '"verify_bit_exact": [a-z]*' gpurun_out/ab_*_5_*.log >> $O/ab_s51.txt
