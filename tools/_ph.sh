cd $GRAFT_REPO_ROOT
cp exp/libmrt_ph.so miniraytracer_amd/libmrt.so
for a in "5 500 500 256" "0 400 200 64" "7 256 256 64" "9 400 400 64"; do timeout -k 10 120 python tools/_phases.py $a || break; done
cp exp/libmrt_w0.so miniraytracer_amd/libmrt.so
