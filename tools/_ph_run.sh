cd $GRAFT_REPO_ROOT
for c in "7 1024 1024 64" "5 500 500 256" "8 512 512 64" "0 400 200 64"; do
  MRT_EXPERIMENT_LIB=exp/libmrt_phases.so timeout -k 10 120 python tools/_phases.py $c || exit 1
done
