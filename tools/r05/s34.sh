# round-5: phase clock of C3's room + mesh kernel (MRT_PHASES build of the fast TU, MRT_FTZ=0)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
O=gpurun_out/r05
mkdir -p $O
MRT_FTZ=0 MRT_EXPERIMENT_LIB=exp/libmrt_ph.so NUMERICS=fast timeout -k 10 300 python3 -u tools/phases.py 9 800 800 64 > $O/phases_c3.txt 2>&1
