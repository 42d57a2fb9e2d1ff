# experiment: default bench invocations (the driver's), pipeline 1 vs 2
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
for a in "" "--pipeline 1" "" "--steps 20 --warmup 2"; do
  timeout -k 10 300 python bench.py --no-cpu-baseline $a > gpurun_out/bdef.log 2>&1 || exit 3
  python tools/_show.py gpurun_out/bdef.log "args[$a]"
done
