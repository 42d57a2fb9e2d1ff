# round-5: phase clock of C2 through the interpreter with the room op (slot 10) and the one-step box
# instance (slot 11) timed apart from the other ops (an experiment build; the marks are not in the tree)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
O=gpurun_out/r05
mkdir -p $O
MRT_NO_SIG=1 MRT_FTZ=0 MRT_EXPERIMENT_LIB=exp/libmrt_ph.so NUMERICS=fast timeout -k 10 300 python3 -u tools/phases.py 5 500 500 256 > $O/phases_c2_interp2.txt 2>&1
