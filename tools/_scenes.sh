cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
for w in ${LIBS:-w0}; do
  cp exp/libmrt_$w.so miniraytracer_amd/libmrt.so
  for cfg in "9 800 800 1024" "8 1024 1024 1024" "7 512 512 256" "0 400 200 64"; do
    set -- $cfg
    timeout -k 10 300 python bench.py --no-cpu-baseline --steps 1 --warmup 1 --scene $1 --width $2 --height $3 --samples $4 > gpurun_out/sc_$w_$1.log 2>&1 || exit 3
    python tools/_show.py gpurun_out/sc_$w_$1.log "$w scene$1"
  done
done
cp exp/libmrt_w0.so miniraytracer_amd/libmrt.so
