cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
CFGS=${CFGS:-"0,400,200,64 7,256,256,64"}
for w in ${LIBS:-w0}; do
  cp exp/libmrt_$w.so miniraytracer_amd/libmrt.so
  for cfg in $CFGS; do
    IFS=, read sid W H S <<< "$cfg"
    timeout -k 10 300 python bench.py --no-cpu-baseline --steps 1 --warmup 1 --scene $sid --width $W --height $H --samples $S > gpurun_out/sc_${w}_$sid.log 2>&1 || exit 3
    python tools/_show.py gpurun_out/sc_${w}_$sid.log "$w scene$sid"
  done
done
cp exp/libmrt_w0.so miniraytracer_amd/libmrt.so
