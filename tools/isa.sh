#!/bin/bash
# Dump the gfx950 ISA of mrt_render.hip built with extra flags: tools/isa.sh <tag> [flags...]
# -> /tmp/isa_<tag>.s ; prints per path-kernel variant: VGPRs, scratch bytes, instructions.
tag=$1; shift
d=$(mktemp -d)
( cd $d && /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -fno-fast-math -ffp-contract=off -fno-slp-vectorize -Wno-unused-function \
    -mllvm -disable-promote-alloca-to-vector -mllvm -structurizecfg-skip-uniform-regions "$@" --save-temps -c /root/repo/miniraytracer_amd/csrc/mrt_render.hip -o r.o 2>/dev/null \
  && cp mrt_render-hip-amdgcn-amd-amdhsa-gfx950.s /tmp/isa_$tag.s )
rm -rf $d
awk '/^_Z15mrt_path_kernel.*:/{k=$1; n=0; inb=1} inb && /^[ \t]+[sv]_|^[ \t]+(global|ds|scratch|buffer|flat)_/{n++} /^\.Lfunc_end/{if(inb) ins[k]=n; inb=0}
     /\.amdhsa_kernel _Z15mrt_path/{kk=$2":"} /amdhsa_private_segment_fixed_size/{ps[kk]=$2} /amdhsa_next_free_vgpr/{vg[kk]=$2}
     END{for (k in ins) printf "%-48s vgpr %4s scratch %4s insts %6d\n", k, vg[k], ps[k], ins[k]}' /tmp/isa_$tag.s | sort
