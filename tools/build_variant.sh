#!/bin/bash
# Experiment builds: exp/libmrt_<tag>.so from the current sources with extra device defines.
#   tools/build_variant.sh <tag> "<extra hipcc flags>"
# (exp/ is git-ignored; it travels to the GPU box for A/B runs with tools/_ab.sh / tools/_abs.sh)
set -e
cd "$(dirname "$0")/.."
tag=$1; shift
flags="$*"
make -s build/obj/scene_builder.o build/obj/mrt_common.o
mkdir -p exp/obj_$tag
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -ffp-contract=off -fno-fast-math -fno-slp-vectorize -w \
    -mllvm -disable-promote-alloca-to-vector -mllvm -structurizecfg-skip-uniform-regions $flags -c miniraytracer_amd/csrc/mrt_render.hip -o exp/obj_$tag/mrt_render.o
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC exp/obj_$tag/mrt_render.o build/obj/scene_builder.o \
    build/obj/mrt_common.o -ldl -o exp/libmrt_$tag.so
echo "built exp/libmrt_$tag.so"
