# round-5: per-phase wave time of C2 through the interpreter and through the specialised walk
# (MRT_PHASES build of the fast TUs)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
O=gpurun_out/r05
mkdir -p $O
MRT_NO_SIG=1 MRT_FTZ=0 MRT_EXPERIMENT_LIB=exp/libmrt_ph.so NUMERICS=fast timeout -k 10 300 python3 -u tools/phases.py 5 500 500 256 > $O/phases_c2_interp.txt 2>&1 || exit 1
MRT_FTZ=0 MRT_EXPERIMENT_LIB=exp/libmrt_ph.so NUMERICS=fast timeout -k 10 300 python3 -u tools/phases.py 5 500 500 256 > $O/phases_c2_sig.txt 2>&1
