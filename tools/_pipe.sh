# experiment: bench with --pipeline 1 vs 2, at N=1 and as rank 0 of 8 (emulated)
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
for p in 1 2; do for n in 1 8; do
  timeout -k 10 300 python bench.py --no-cpu-baseline --steps 20 --warmup 2 --pipeline $p --emulate-world $n > gpurun_out/pipe_${p}_$n.log 2>&1 || exit 3
  python tools/_show.py gpurun_out/pipe_${p}_$n.log "pipeline $p world $n"
done; done
