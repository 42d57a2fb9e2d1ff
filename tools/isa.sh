#!/bin/bash
# Dump the gfx950 ISA of the path kernels (mrt_kernels.hip) built with the Makefile's device flags
# plus extra ones: tools/isa.sh <tag> [flags...]   (e.g. tools/isa.sh fast -DMRT_FAST=1 -ffp-contract=fast -freciprocal-math)
# -> /tmp/isa_<tag>.s ; prints per path-kernel variant: VGPRs, spill counts, private segment bytes,
# the scratch instructions in the code (a private segment with none is the backend's reserved
# scavenging slot, never touched), instructions.
tag=$1; shift
d=$(mktemp -d)
( cd $d && /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -fno-fast-math -fno-slp-vectorize -Wno-unused-function \
    -mllvm -disable-promote-alloca-to-vector -mllvm -structurizecfg-skip-uniform-regions "$@" --save-temps -c /root/repo/miniraytracer_amd/csrc/mrt_kernels.hip -o k.o 2>/dev/null \
  && cp mrt_kernels-hip-amdgcn-amd-amdhsa-gfx950.s /tmp/isa_$tag.s )
rm -rf $d
awk '/^_Z(N4mrtd)?[0-9]+mrt_(path_kernel|wf_).*:/{k=$1; n=0; sc=0; inb=1} inb && /^[ \t]+[sv]_|^[ \t]+(global|ds|scratch|buffer|flat)_/{n++} inb && /^[ \t]+scratch_/{sc++} /^\.Lfunc_end/{if(inb) {ins[k]=n; scr[k]=sc}; inb=0}
     /\.amdhsa_kernel /{kk=""} /\.amdhsa_kernel _Z(N4mrtd)?[0-9]+mrt_(path|wf_)/{kk=$2":"} kk!="" && /amdhsa_private_segment_fixed_size/{ps[kk]=$2} kk!="" && /amdhsa_next_free_vgpr/{vg[kk]=$2}
     /^[ \t]+.name:/{mk=""} /^[ \t]+.name:[ \t]+_Z(N4mrtd)?[0-9]+mrt_(path|wf_)/{mk=$2":"} mk!="" && /\.sgpr_spill_count:/{ss[mk]=$2} mk!="" && /\.vgpr_spill_count:/{vs[mk]=$2}
     END{for (k in ins) printf "%-46s vgpr %4s vspill %4s sspill %4s scratch %4s (scratch insts %3d) insts %6d\n", k, vg[k], vs[k], ss[k], ps[k], scr[k], ins[k]}' /tmp/isa_$tag.s | sort
