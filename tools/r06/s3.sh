#!/bin/bash
# round 6 session 3: (a) A/B of the instance ray recomputed after the walk (6 LDS words per lane
# freed -> larger treelet) against the previous build (exp/libmrt_base.so), book2 / random spheres /
# C2 and C2 through the interpreter, and the branch-free stack push / pop (exp/libmrt_bf.so); (b) kernel trace of the C2 N = 8 share (three contexts) for the
# launch timeline
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out/r06
set -o pipefail
LIBS="base bf" CFGS="7,2048,2048,64 0,1200,800,64 8,1024,1024,256 9,800,800,256 5,500,500,1024" ROUNDS=2 bash tools/ab.sh || exit 3
for r in 1 2; do
  for tag in intree base; do
    lib=""; [ $tag = base ] && lib=exp/libmrt_base.so
    MRT_NO_SIG=1 MRT_EXPERIMENT_LIB=$lib timeout -k 10 300 python bench.py --no-cpu-baseline --no-compare-numerics --no-other-walk \
        --steps 10 --warmup 2 > gpurun_out/r06/s3_interp_${tag}_$r.log 2>&1 || exit 3
    python tools/show_bench.py gpurun_out/r06/s3_interp_${tag}_$r.log "interp $tag $r"
  done
done
# the exact contract's interpreter (MRT_NO_SIG=1, C2): 6 waves per SIMD with 41 spilled VGPRs (in
# tree) against 5 (96 VGPRs, 6 spilled) and 4 (107, none)
for r in 1 2; do
  for tag in intree ex5 ex4; do
    lib=""; [ $tag != intree ] && lib=exp/libmrt_$tag.so
    MRT_NO_SIG=1 MRT_EXPERIMENT_LIB=$lib timeout -k 10 300 python bench.py --numerics exact --no-cpu-baseline --no-compare-numerics \
        --no-other-walk --steps 6 --warmup 1 > gpurun_out/r06/s3_exint_${tag}_$r.log 2>&1 || exit 3
    python tools/show_bench.py gpurun_out/r06/s3_exint_${tag}_$r.log "exact interp $tag $r"
  done
done
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/r06/kt8 -o kt8 -- python bench.py --no-cpu-baseline \
    --no-compare-numerics --no-other-walk --no-parity --steps 30 --warmup 2 --emulate-world 8 --emulate-rank 6 --emulate-gather \
    --step-times > gpurun_out/r06/s3_kt8.log 2>&1 || exit 3
python tools/show_bench.py gpurun_out/r06/s3_kt8.log "N=8 share 6, kernel trace"
