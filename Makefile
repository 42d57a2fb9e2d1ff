# Build of the MI355X render path (no cmake).  `make` builds:
#   miniraytracer_amd/libmrt.so   C-ABI (include/mrt.h): host scene builder + HIP kernels for gfx950
#   bin/mrt                       command-line driver with the reference's flags
#   oracle/liboracle.so           C restatement used by tests / bench cpu_baseline (test infra only)
HIPCC   ?= /opt/rocm/bin/hipcc
CC      ?= gcc
ARCH    ?= gfx950
JOBS    ?= 8
# Numerics contract: no FMA contraction, IEEE division/sqrt, denormals kept.
# No SLP vectorisation: it packed unrelated float ops into v_pk_* pairs whose constant halves
# were kept live in VGPR pairs and spilled (C2 +8%, bunny +7% without it; results identical).
HIPFLAGS = --offload-arch=$(ARCH) -O3 -std=c++17 -fPIC -ffp-contract=off -fno-fast-math -fno-slp-vectorize -Wall -Wno-unused-function
# per-lane traversal stacks stay in scratch instead of being promoted into VGPR vectors; uniform
# regions keep plain scalar branches instead of exec-mask structurisation (C2 +1.7%)
HIPDEV   = -mllvm -disable-promote-alloca-to-vector -mllvm -structurizecfg-skip-uniform-regions
CSRC     = miniraytracer_amd/csrc
OBJDIR   = build/obj

LIB_OBJS = $(OBJDIR)/mrt_render.o $(OBJDIR)/mrt_kernels_exact.o $(OBJDIR)/mrt_kernels_fast.o $(OBJDIR)/mrt_kernels_fastz.o \
           $(OBJDIR)/mrt_kernels_pex.o \
           $(OBJDIR)/mrt_cpu.o $(OBJDIR)/scene_builder.o $(OBJDIR)/mrt_common.o $(OBJDIR)/mrt_comm.o
# the path kernels twice: exact contract (no contraction, IEEE division) and tolerance contract
# (FMA contraction, reciprocal division, hardware rcp/sqrt/rsq, f32 transcendentals)
# (-fno-hip-fp32-correctly-rounded-divide-sqrt: f32 division by v_rcp_f32 + multiply instead of
# the 10-instruction IEEE sequence; -freciprocal-math alone does not lower it)
FASTFLAGS = -DMRT_FAST=1 -ffp-contract=fast -freciprocal-math -fno-hip-fp32-correctly-rounded-divide-sqrt
HDRS     = include/mrt.h include/mrt_scene.h include/mrt_mathfn.h $(wildcard $(CSRC)/*.h) Makefile

all: miniraytracer_amd/libmrt.so bin/mrt oracle/liboracle.so

$(OBJDIR)/mrt_kernels_exact.o: $(CSRC)/mrt_kernels.hip $(HDRS)
	@mkdir -p $(OBJDIR)
	$(HIPCC) $(HIPFLAGS) $(HIPDEV) -DMRT_FAST=0 -c $< -o $@

$(OBJDIR)/mrt_kernels_fast.o: $(CSRC)/mrt_kernels.hip $(HDRS)
	@mkdir -p $(OBJDIR)
	$(HIPCC) $(HIPFLAGS) $(HIPDEV) $(FASTFLAGS) -c $< -o $@

# the tolerance contract again with f32 denormals flushed, for the variants mrt_launch.h's
# kFtzVariant selects (the others are not instantiated in it)
FTZFLAGS = -fgpu-flush-denormals-to-zero -DMRT_TABLE_FTZ=1
$(OBJDIR)/mrt_kernels_fastz.o: $(CSRC)/mrt_kernels.hip $(HDRS)
	@mkdir -p $(OBJDIR)
	$(HIPCC) $(HIPFLAGS) $(HIPDEV) $(FASTFLAGS) $(FTZFLAGS) -c $< -o $@

# the tolerance contract's path-exact variants (mrt_launch.h kPathExact): the exact build's
# arithmetic with the forward fold; its bvh_node kernels in two 12-wave groups per CU (6 waves per
# SIMD, 80 VGPRs): book2 4.83 against 4.19 Grays/s in one 16-wave group, 2.90 in two 10-wave groups
# (profiles/r04_ab.txt)
PEXFLAGS = -DMRT_FAST=0 -DMRT_FWD_FOLD=1 -DMRT_TABLE_PEX=1 -DMRT_TREE_WG=768 -DMRT_WPE_WIDE=6
$(OBJDIR)/mrt_kernels_pex.o: $(CSRC)/mrt_kernels.hip $(HDRS)
	@mkdir -p $(OBJDIR)
	$(HIPCC) $(HIPFLAGS) $(HIPDEV) $(PEXFLAGS) -c $< -o $@

# the CPU backend: the same hot-path headers compiled for the host only (exact contract).
# -mfma: the reference's fused multiply-adds (mrt_device.h ref_fma) as one instruction instead of a
# libm fmaf call (same result; the reference's own build is x86 FMA too, -march=native)
HOSTFMA ?= -mfma
$(OBJDIR)/mrt_cpu.o: $(CSRC)/mrt_cpu.hip $(HDRS)
	@mkdir -p $(OBJDIR)
	$(HIPCC) $(HIPFLAGS) $(HOSTFMA) --offload-host-only -c $< -o $@

$(OBJDIR)/%.o: $(CSRC)/%.hip $(HDRS)
	@mkdir -p $(OBJDIR)
	$(HIPCC) $(HIPFLAGS) $(HIPDEV) -c $< -o $@

$(OBJDIR)/%.o: $(CSRC)/%.cpp $(HDRS)
	@mkdir -p $(OBJDIR)
	$(HIPCC) $(HIPFLAGS) $(HIPDEV) -c $< -o $@

miniraytracer_amd/libmrt.so: $(LIB_OBJS)
	$(HIPCC) --offload-arch=$(ARCH) -shared -fPIC $(LIB_OBJS) -ldl -o $@

bin/mrt: $(CSRC)/mrt_cli.cpp miniraytracer_amd/libmrt.so include/mrt.h
	@mkdir -p bin
	$(HIPCC) -O2 -std=c++17 -ffp-contract=off $(CSRC)/mrt_cli.cpp -Lminiraytracer_amd -lmrt -Wl,-rpath,'$$ORIGIN/../miniraytracer_amd' -o $@

oracle/liboracle.so: oracle/mrt_oracle.c oracle/mrt_oracle.h include/mrt_scene.h
	$(CC) -O2 -std=c11 -fPIC -shared -ffp-contract=off -fno-fast-math $(HOSTFMA) -Wall -o $@ oracle/mrt_oracle.c -lm -lpthread

clean:
	rm -rf build miniraytracer_amd/libmrt.so bin oracle/liboracle.so

.PHONY: all clean
