#!/bin/bash
# Experiment builds: exp/libmrt_<tag>.so from the current sources, the tolerance-contract TU
# (mrt_kernels.hip, MRT_FAST build) compiled with the given flags instead of the Makefile's
# FASTFLAGS; the exact TU as in the Makefile unless EXACT_FLAGS is set.
#   tools/build_variant.sh <tag> "<fast-TU hipcc flags>"
# Load with MRT_EXPERIMENT_LIB=exp/libmrt_<tag>.so (miniraytracer_amd/_lib.py); exp/ is
# git-ignored and travels to the GPU box with the tree.
set -e
cd "$(dirname "$0")/.."
tag=$1; shift
flags="$*"
make -s build/obj/scene_builder.o build/obj/mrt_common.o build/obj/mrt_render.o build/obj/mrt_kernels_exact.o build/obj/mrt_cpu.o build/obj/mrt_comm.o
mkdir -p exp/obj_$tag
BASE="--offload-arch=gfx950 -O3 -std=c++17 -fPIC -fno-fast-math -fno-slp-vectorize -w -mllvm -disable-promote-alloca-to-vector -mllvm -structurizecfg-skip-uniform-regions -DMRT_EXPERIMENTS"
/opt/rocm/bin/hipcc $BASE -DMRT_TABLE_FAST=1 $flags -c miniraytracer_amd/csrc/mrt_kernels.hip -o exp/obj_$tag/mrt_kernels_fast.o
# the denormal-flushing build of the same flags (the kFtzVariant variants; run with MRT_FTZ=0 to A/B
# without it)
# (FTZ_PLAIN=1: the Makefile's FTZ build instead -- for flags only one translation unit may carry,
# e.g. -DMRT_PHASES; run with MRT_FTZ=0)
FZ=exp/obj_$tag/mrt_kernels_fastz.o
if [ -n "${FTZ_PLAIN:-}" ]; then
  make -s build/obj/mrt_kernels_fastz.o
  FZ=build/obj/mrt_kernels_fastz.o
else
  /opt/rocm/bin/hipcc $BASE -DMRT_TABLE_FAST=1 $flags -fgpu-flush-denormals-to-zero -DMRT_TABLE_FTZ=1 -c miniraytracer_amd/csrc/mrt_kernels.hip -o $FZ
fi
EX=build/obj/mrt_kernels_exact.o
# host defines (MRT_NPART, MRT_BATCH, ...) change PathParams / the claim protocol: the exact TU must
# be built with them too, or the exact kernel reads a foreign parameter layout (a GPU memory fault)
EXACT_FLAGS="${EXACT_FLAGS:-} ${HOST_FLAGS:-}"
if [ -n "${EXACT_FLAGS// /}" ]; then
  /opt/rocm/bin/hipcc $BASE -ffp-contract=off -DMRT_FAST=0 $EXACT_FLAGS -c miniraytracer_amd/csrc/mrt_kernels.hip -o exp/obj_$tag/mrt_kernels_exact.o
  EX=exp/obj_$tag/mrt_kernels_exact.o
fi
RO=build/obj/mrt_render.o
if [ -n "${HOST_FLAGS:-}" ]; then  # host TU too (e.g. -DMRT_PATH_WG=..., which both sides must agree on)
  /opt/rocm/bin/hipcc $BASE -ffp-contract=off $HOST_FLAGS -c miniraytracer_amd/csrc/mrt_render.hip -o exp/obj_$tag/mrt_render.o
  RO=exp/obj_$tag/mrt_render.o
fi
PX=build/obj/mrt_kernels_pex.o  # the path-exact variants as in the Makefile (run MRT_PATH_EXACT=0 to A/B them)
make -s $PX
if [ -n "${PEX_FLAGS:-}" ]; then  # ... or built with extra flags
  /opt/rocm/bin/hipcc $BASE -ffp-contract=off $(make -s -f Makefile -p 2>/dev/null | sed -n 's/^PEXFLAGS = //p') $PEX_FLAGS -c miniraytracer_amd/csrc/mrt_kernels.hip -o exp/obj_$tag/mrt_kernels_pex.o
  PX=exp/obj_$tag/mrt_kernels_pex.o
fi
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC $RO $EX $PX exp/obj_$tag/mrt_kernels_fast.o $FZ \
    build/obj/mrt_cpu.o build/obj/scene_builder.o build/obj/mrt_common.o build/obj/mrt_comm.o -ldl -o exp/libmrt_$tag.so
echo "built exp/libmrt_$tag.so"
