# round-5: the retrace of the listed paths on the fold's stream, ahead of the fold (MRT_RETRACE_SIDE=1:
# the next render's path kernel does not wait for it), vs in the render's stream (in tree), async fold:
# C2 at one context; the N = 8 share (rank 0) with the async fold at one and three contexts
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
O=gpurun_out/r05
mkdir -p $O
ROUNDS=3 STEPS=20 LIBS="MRT_RETRACE_SIDE=1" CFGS="5,500,500,1024" BENCH_ARGS="--verify" timeout -k 10 400 bash tools/ab.sh > $O/ab_s45.txt 2>&1 || exit 3
grep -o '"verify_bit_exact": [a-z]*' gpurun_out/ab_*_5_*.log >> $O/ab_s45.txt
for a in "--fold async --pipeline 1" "--fold async --pipeline 3"; do
  echo "== N=8 share, $a" >> $O/ab_s45.txt
  ROUNDS=2 STEPS=60 LIBS="MRT_RETRACE_SIDE=1" CFGS="5,500,500,1024" BENCH_ARGS="--emulate-world 8 --emulate-gather $a" \
      timeout -k 10 400 bash tools/ab.sh >> $O/ab_s45.txt 2>&1 || exit 4
done
