# rehearsal of the multi-rank bench on the one-GPU box: 2 and 3 ranks sharing GPU 0 over gloo
# (RCCL refuses two ranks on one GPU), each checking the assembled image (--verify); then N=1.
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
for n in 2 3; do
  MRT_DIST_BACKEND=gloo MRT_SAME_GPU=1 timeout -k 10 240 python -m torch.distributed.run --nnodes=1 --nproc-per-node $n \
      --master-addr 127.0.0.1 --master-port 2951$n bench.py --gpus $n --steps 5 --warmup 1 --verify --no-cpu-baseline \
      > gpurun_out/mr_$n.log 2>&1 || { tail -20 gpurun_out/mr_$n.log; exit 3; }
  grep '^{' gpurun_out/mr_$n.log | python -c "import json,sys; d=json.loads(sys.stdin.readline()); print('N=$n', d['value'], d['rays_per_step'] if 'rays_per_step' in d else d['config']['rays_per_step'], 'verify', d.get('verify_bit_exact'))"
done
timeout -k 10 240 python bench.py --steps 5 --warmup 1 --verify --no-cpu-baseline > gpurun_out/mr_1.log 2>&1 || exit 3
grep '^{' gpurun_out/mr_1.log | python -c "import json,sys; d=json.loads(sys.stdin.readline()); print('N=1', d['value'], 'verify', d.get('verify_bit_exact'))"
