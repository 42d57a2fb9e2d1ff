# round-5: the fold kernel's loads in flight per thread: FOLD_DEPTH 16 (in tree) vs 8 (fd8) and 32
# (fd32); C2 steps and a kernel trace of each
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
O=gpurun_out/r05
mkdir -p $O
ROUNDS=3 STEPS=20 LIBS="fd8 fd32" CFGS="5,500,500,1024" timeout -k 10 600 bash tools/ab.sh > $O/ab_s41.txt 2>&1 || exit 1
for t in fd8 fd32; do
  MRT_EXPERIMENT_LIB=exp/libmrt_$t.so timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $O/kt_$t -o run --output-format csv -- python3 bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-other-walk --no-parity --no-compare-numerics > $O/kt_$t.log 2>&1 || exit 1
done
