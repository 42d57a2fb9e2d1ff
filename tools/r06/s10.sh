#!/bin/bash
# round 6 session 10: instruction-mix PMC passes (tools/pmc_mix.sh) of C5 (book2 2048^2 x 64) and C4
# (bunny 1024^2 x 256) -- how much of the path-exact kernels' VALU issue is f64 (the project libm's
# log / sincos / atan2 evaluations)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out/r06
MIX_ARGS="--steps 1 --warmup 0 --kernel-reps 1 --pipeline 1 --no-cpu-baseline --no-other-walk --no-parity --no-compare-numerics --scene 7 --width 2048 --height 2048 --samples 64" \
    bash tools/pmc_mix.sh || exit 3
rm -rf gpurun_out/mix_c5 && mv gpurun_out/mix gpurun_out/mix_c5
MIX_ARGS="--steps 1 --warmup 0 --kernel-reps 1 --pipeline 1 --no-cpu-baseline --no-other-walk --no-parity --no-compare-numerics --scene 8 --width 1024 --height 1024 --samples 256" \
    bash tools/pmc_mix.sh || exit 3
rm -rf gpurun_out/mix_c4 && mv gpurun_out/mix gpurun_out/mix_c4
