# round-5: the interpreter's wall record from the room's data (MRT_F_ROOMREC, in tree) vs loading the
# wall's node after the walk (MRT_NO_ROOMREC=1): its GPU tests (bit-identical), then C2 through the
# interpreter (MRT_NO_SIG=1), interleaved
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
O=gpurun_out/r05
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "interpreter or linear_program" > $O/s57_test.log 2>&1 || exit 3
for r in 1 2 3; do
  for v in intree noroomrec; do
    e=""; [ $v = noroomrec ] && e="MRT_NO_ROOMREC=1"
    log=$O/s57_${v}_$r.log
    env MRT_NO_SIG=1 $e timeout -k 10 300 python bench.py --no-cpu-baseline --no-compare-numerics --no-other-walk --no-parity \
        --steps 20 --warmup 2 > $log 2>&1 || exit 4
    python tools/show_bench.py $log "interp $v round $r"
  done
done
