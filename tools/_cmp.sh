# experiment: C2 bench for each exp/libmrt_<tag>.so in $LIBS
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
for w in ${LIBS:-w0}; do
  cp exp/libmrt_$w.so miniraytracer_amd/libmrt.so
  timeout -k 10 300 python bench.py --no-cpu-baseline --steps ${STEPS:-10} --warmup 1 ${BARGS:-} > gpurun_out/cmp_$w.log 2>&1 || exit 3
  python tools/_show.py gpurun_out/cmp_$w.log "$w"
done
cp exp/libmrt_w0.so miniraytracer_amd/libmrt.so
