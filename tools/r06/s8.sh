#!/bin/bash
# round 6 session 8: (a) the GPU suite on the tree with records made after the walk in one copy, the
# atan2 constants made at their use (book2's path-exact kernel: 0 spills), and Cornell smoke (scene 6)
# as a linear program (FT_VSUB); (b) A/B against MRT_LIN_DEFER=0 (exp/libmrt_nodefer.so) on book2,
# random spheres, C2; (c) scene 6 against the generic machine, both contracts; (d) the exact
# interpreter (MRT_NO_SIG=1, C2) at 6 (in tree) / 5 / 4 waves; (e) C2 N = 8 share step shapes with the
# retrace back on the render's stream; (f) C5 PMC
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out/r06
set -o pipefail
timeout -k 10 600 python -u -m pytest tests/ -x -v -m gpu --timeout 240 --timeout-method thread > gpurun_out/r06/s8_suite.log 2>&1
rc=$?; tail -3 gpurun_out/r06/s8_suite.log
[ $rc -eq 0 ] || exit $rc
LIBS="nodefer" CFGS="7,2048,2048,64 0,1200,800,64 5,500,500,1024" ROUNDS=2 bash tools/ab.sh || exit 3
S6="--scene 6 --width 500 --height 500 --samples 256 --no-cpu-baseline --no-compare-numerics --no-other-walk --no-parity --steps 4 --warmup 1"
for r in 1 2; do
  for num in fast exact; do
    timeout -k 10 300 python bench.py $S6 --numerics $num > gpurun_out/r06/s8_s6_lin_${num}_$r.log 2>&1 || exit 3
    python tools/show_bench.py gpurun_out/r06/s8_s6_lin_${num}_$r.log "scene 6 lin $num $r"
    MRT_FORCE_GENERIC=1 timeout -k 10 300 python bench.py $S6 --numerics $num > gpurun_out/r06/s8_s6_gen_${num}_$r.log 2>&1 || exit 3
    python tools/show_bench.py gpurun_out/r06/s8_s6_gen_${num}_$r.log "scene 6 generic $num $r"
  done
done
for r in 1 2; do
  for tag in intree ex5 ex4; do
    lib=""; [ $tag != intree ] && lib=exp/libmrt_$tag.so
    MRT_NO_SIG=1 MRT_EXPERIMENT_LIB=$lib timeout -k 10 300 python bench.py --numerics exact --no-cpu-baseline --no-compare-numerics \
        --no-other-walk --no-parity --steps 6 --warmup 1 > gpurun_out/r06/s8_exint_${tag}_$r.log 2>&1 || exit 3
    python tools/show_bench.py gpurun_out/r06/s8_exint_${tag}_$r.log "exact interp $tag $r"
  done
done
VARIANTS="1,0,n1,;8,6,n8r6_p3full,--pipeline 3 --fold full;8,6,n8r6_p2async,--pipeline 2 --fold async;8,6,n8r6_p2full,--pipeline 2 --fold full" \
    ROUNDS=2 bash tools/scale_variants.sh || exit 3
PROF_CFGS="c5:7:2048:2048:64" bash tools/prof_configs.sh || exit 3
