# round-5: per-phase wave time of book2's path-exact kernel (MRT_PHASES build of the pex TU)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
O=gpurun_out/r05
mkdir -p $O
MRT_EXPERIMENT_LIB=exp/libmrt_ph.so NUMERICS=fast timeout -k 10 300 python3 -u tools/phases.py 7 1024 1024 16 > $O/phases_c5.txt 2>&1
