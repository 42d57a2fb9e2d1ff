# round-5: with the async fold the bench default at one context -- the rocprofv3 kernel trace of the
# default bench command; the single-GPU scale rehearsal (N = 1 / 2 shares: one context, async fold;
# N = 4 / 8: three contexts, full fold), and the N = 4 / 8 shares with the async fold at one and at
# three contexts
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
O=gpurun_out/r05
mkdir -p $O
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/s44_trace -o run --output-format csv -- python3 bench.py --steps 20 --warmup 5 \
    > $O/s44_trace.log 2>&1 || exit 3
echo "trace done $(date +%T)"
CFGS="1,0 2,0 2,1 4,0 8,0" STEPS=60 timeout -k 10 500 bash tools/scale_rehearsal.sh > $O/s44_scale.txt 2>&1 || exit 4
for a in "--fold async --pipeline 1" "--fold async --pipeline 3"; do
  echo "== $a" >> $O/s44_scale.txt
  CFGS="4,0 8,0" STEPS=60 SCALE_ARGS="$a" timeout -k 10 300 bash tools/scale_rehearsal.sh >> $O/s44_scale.txt 2>&1 || exit 5
done
