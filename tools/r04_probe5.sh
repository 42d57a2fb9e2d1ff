#!/bin/bash
# Round-4 probe batch E: "exact paths, forward fold" (exp/libmrt_xpf.so: the exact arithmetic with
# the tolerance contract's forward fold) at every config's own spp, against the in-tree contracts.
mkdir -p gpurun_out
timeout -k 10 300 python -u tools/contract_parity.py fast exact > gpurun_out/r04_cp2_intree.log 2>&1 || exit 1
cut -c1-220 gpurun_out/r04_cp2_intree.log
MRT_FTZ=0 MRT_EXPERIMENT_LIB=exp/libmrt_xpf.so timeout -k 10 300 python -u tools/contract_parity.py fast > gpurun_out/r04_cp2_xpf.log 2>&1 || exit 1
cut -c1-220 gpurun_out/r04_cp2_xpf.log
