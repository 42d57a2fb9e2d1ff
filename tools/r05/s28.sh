# round-5: interpreter after the root-list drop: phase clock (room op slot 10, box instance slot 11;
# an experiment build) and the box instance without its instance box test (noaabb)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
O=gpurun_out/r05
mkdir -p $O
MRT_NO_SIG=1 MRT_FTZ=0 MRT_EXPERIMENT_LIB=exp/libmrt_ph.so NUMERICS=fast timeout -k 10 300 python3 -u tools/phases.py 5 500 500 256 > $O/phases_c2_interp3.txt 2>&1 || exit 1
MRT_NO_SIG=1 ROUNDS=3 STEPS=10 LIBS="noaabb" CFGS="5,500,500,1024" timeout -k 10 600 bash tools/ab.sh > $O/ab_s28.txt 2>&1
