# round-5: the N = 2 share (rank 0, --emulate-gather): one context with the async fold (auto's choice)
# vs three contexts with the full fold, interleaved
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
O=gpurun_out/r05
mkdir -p $O
for r in 1 2 3; do
  for a in "--pipeline 1 --fold async" "--pipeline 3 --fold full"; do
    t=$(echo $a | tr -d ' -'); log=$O/s58_${t}_$r.log
    timeout -k 10 200 python bench.py --no-cpu-baseline --no-compare-numerics --no-other-walk --no-parity --steps 60 --warmup 4 \
        --emulate-world 2 --emulate-rank 0 --emulate-gather $a > $log 2>&1 || exit 3
    python tools/show_bench.py $log "N=2 $a round $r"
  done
done
