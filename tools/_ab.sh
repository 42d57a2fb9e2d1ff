# experiment: GPU parity tests of the in-tree build, then C2 bench A/B of exp/libmrt_<tag>.so ($LIBS),
# each variant loaded through MRT_EXPERIMENT_LIB (miniraytracer_amd/_lib.py) -- the in-tree library
# is never overwritten
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
if [ "${SKIP_TESTS:-0}" != 1 ]; then
  timeout -k 10 600 python -u -m pytest tests/ -x -q -m gpu --timeout 300 --timeout-method thread > gpurun_out/ab_tests.log 2>&1
  rc=$?; tail -3 gpurun_out/ab_tests.log; [ $rc -eq 0 ] || exit $rc
fi
for w in ${LIBS:-intree}; do
  lib=""; [ "$w" != intree ] && lib=$PWD/exp/libmrt_$w.so
  MRT_EXPERIMENT_LIB=$lib timeout -k 10 300 python bench.py --no-cpu-baseline --steps ${STEPS:-10} --warmup 1 ${BARGS:-} > gpurun_out/ab_$w.log 2>&1 || exit 3
  python tools/_show.py gpurun_out/ab_$w.log "$w"
done
