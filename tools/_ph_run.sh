cd $GRAFT_REPO_ROOT
for c in ${PH_CASES:-"5 500 500 256"}; do
  MRT_EXPERIMENT_LIB=exp/libmrt_${PH_LIB:-phases}.so timeout -k 10 120 python tools/_phases.py ${c//:/ } || exit 1
done
