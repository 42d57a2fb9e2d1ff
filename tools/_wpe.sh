cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
cp exp/libmrt_w0.so miniraytracer_amd/libmrt.so
if [ -z "$SKIP" ]; then timeout -k 10 600 python -m pytest tests/ -x -q -m gpu > gpurun_out/gpu_tests.log 2>&1; rc=$?; tail -3 gpurun_out/gpu_tests.log; [ $rc -le 1 ] || exit $rc; fi
show() { python tools/_show.py "$@"; }
for spec in ${LIBS:-w0}; do
  w=${spec%%:*}; b=${spec#*:}; [ "$b" = "$spec" ] && b=""
  cp exp/libmrt_$w.so miniraytracer_amd/libmrt.so
  MRT_BLOCKS_PER_CU=$b timeout -k 10 300 python bench.py --no-cpu-baseline --steps 5 > gpurun_out/bench_$w$b.log 2>&1 || exit 3
  show gpurun_out/bench_$w$b.log "$spec"
done
cp exp/libmrt_w0.so miniraytracer_amd/libmrt.so
