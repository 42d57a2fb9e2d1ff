# experiment: GPU parity tests of the in-tree build, then per-scene bench A/B of exp/libmrt_<tag>.so
#   LIBS="a b" CFGS="scene,W,H,spp ..."   (tag "intree" = the in-tree build)
# each variant is loaded through MRT_EXPERIMENT_LIB (miniraytracer_amd/_lib.py): the in-tree
# library is never overwritten
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
if [ "${SKIP_TESTS:-0}" != 1 ]; then
  timeout -k 10 600 python -u -m pytest tests/ -x -q -m gpu --timeout 300 --timeout-method thread > gpurun_out/ab_tests.log 2>&1
  rc=$?; tail -3 gpurun_out/ab_tests.log; [ $rc -eq 0 ] || exit $rc
fi
for cfg in ${CFGS:-8,512,512,256 9,400,400,1024 7,256,256,256}; do
  IFS=, read sid W H S <<< "$cfg"
  for w in ${LIBS:-intree}; do
    lib=""; [ "$w" != intree ] && lib=$PWD/exp/libmrt_$w.so
    MRT_EXPERIMENT_LIB=$lib timeout -k 10 300 python bench.py --no-cpu-baseline --steps ${STEPS:-3} --warmup 1 --kernel-reps 1 --scene $sid --width $W --height $H --samples $S ${BARGS:-} > gpurun_out/abs_${w}_$sid.log 2>&1 || exit 3
    python tools/_show.py gpurun_out/abs_${w}_$sid.log "$w scene $sid"
  done
done
