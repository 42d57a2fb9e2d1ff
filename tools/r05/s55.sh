# round-5: C3 at full size, one render each: full fold vs async fold (in tree: a 256-thread group per
# CU) vs async with a 64-thread group per CU (wg64: a quarter of the fold's memory pressure, 4x as long)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
O=gpurun_out/r05
mkdir -p $O
for r in 1 2; do
  for v in full async wg64; do
    lib=""; f=$v; [ $v = wg64 ] && { lib=exp/libmrt_wg64.so; f=async; }
    log=$O/s55_${v}_$r.log
    MRT_EXPERIMENT_LIB=$lib timeout -k 10 300 python bench.py --no-cpu-baseline --no-compare-numerics --no-other-walk --no-parity --steps 1 --warmup 0 \
        --scene 9 --width 800 --height 800 --samples 4096 --fold $f > $log 2>&1 || exit 3
    python tools/show_bench.py $log "C3 $v round $r"
  done
done
