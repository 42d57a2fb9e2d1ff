#!/bin/bash
# Round-4 probe batch F: which tolerance-contract switch makes paths diverge from the exact
# contract (tools/divergence.py; exp/libmrt_n<SWITCH>.so = the fast build with MRT_FAST_<SWITCH>=0,
# exp/libmrt_xpf.so = exact arithmetic + forward fold).
mkdir -p gpurun_out
for L in xpf nDIV nSQRT nNORM nTRANS nGUARDS nSNAP nBOX nSLAB nROOM; do
  MRT_EXPERIMENT_LIB=exp/libmrt_$L.so timeout -k 10 150 python -u tools/divergence.py >> gpurun_out/r04_div3.log 2>&1 || exit 1
done
cat gpurun_out/r04_div3.log
