# experiment: bench --pipeline P at N=1 and as rank 7 of 8 (emulated)
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
for p in ${PIPES:-1 2 3}; do for n in ${NS:-1 8}; do
  timeout -k 10 300 python bench.py --no-cpu-baseline --steps 20 --warmup 2 --pipeline $p --emulate-world $n --emulate-rank $((n-1)) > gpurun_out/pipe_${p}_$n.log 2>&1 || exit 3
  python tools/_show.py gpurun_out/pipe_${p}_$n.log "pipeline $p world $n"
done; done
