#!/bin/bash
# experiment: treelet size sweep (exp/libmrt_tl.so, built with the MRT_EXPERIMENTS hooks)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for n in 0 15 63 127 255 1000; do
  echo "nodes $n"
  MRT_TREELET_NODES=$n MESH_CASES="7:2048:2048:64 0:800:400:256" timeout -k 10 300 python -u tools/mesh_ab.py tl || exit 1
done
