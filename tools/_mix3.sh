cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/mix3
for w in ${LIBS:-w0}; do
  cp exp/libmrt_$w.so miniraytracer_amd/libmrt.so
  timeout -k 10 300 rocprofv3 --pmc SQ_INSTS_VALU SQ_THREAD_CYCLES_VALU SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_INSTS_SALU SQ_WAIT_INST_ANY -d gpurun_out/mix3/$w -o run --output-format csv -- python3 bench.py --steps 1 --warmup 0 --no-cpu-baseline > gpurun_out/mix3/$w.log 2>&1 || exit 1
done
cp exp/libmrt_w0.so miniraytracer_amd/libmrt.so
