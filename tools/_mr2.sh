# rehearsal of bench.py's own multi-rank launch on the one-GPU box: --gpus 2 / 3 with every rank on
# GPU 0 over gloo (MRT_SAME_GPU=1), each checking the assembled image bit-exact (--verify); then the
# refusal of --gpus 8 without the override (must exit non-zero); then N=1.
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
for n in 2 3; do
  MRT_DIST_BACKEND=gloo MRT_SAME_GPU=1 timeout -k 10 240 python bench.py --gpus $n --steps 3 --warmup 1 --verify --no-cpu-baseline \
      > gpurun_out/mr2_$n.log 2>&1 || { tail -20 gpurun_out/mr2_$n.log; exit 3; }
  grep '^{' gpurun_out/mr2_$n.log | python -c "import json,sys; d=json.loads(sys.stdin.readline()); print('N=$n', d['n_gpus'], d['value'], 'verify', d.get('verify_bit_exact'))"
done
if timeout -k 10 120 python bench.py --gpus 8 --steps 1 --warmup 0 --no-cpu-baseline > gpurun_out/mr2_8.log 2>&1; then
  echo "--gpus 8 on one GPU did NOT fail"; exit 4
else
  echo "--gpus 8 refused: $(tail -1 gpurun_out/mr2_8.log)"
fi
