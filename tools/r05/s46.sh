# round-5: the N = 4 and N = 8 shares (rank 0, --emulate-gather) at three contexts: full fold (the
# default there) vs async fold, interleaved
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
O=gpurun_out/r05
mkdir -p $O
for r in 1 2 3; do
  for n in 4 8; do
    for f in full async; do
      log=$O/s46_${n}_${f}_$r.log
      timeout -k 10 200 python bench.py --no-cpu-baseline --no-compare-numerics --no-other-walk --no-parity --steps 60 --warmup 4 \
          --emulate-world $n --emulate-rank 0 --emulate-gather --pipeline 3 --fold $f > $log 2>&1 || exit 3
      python tools/show_bench.py $log "N=$n $f round $r"
    done
  done
done
