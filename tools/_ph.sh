cd $GRAFT_REPO_ROOT
cp exp/libmrt_ph.so miniraytracer_amd/libmrt.so
timeout -k 10 120 python tools/_phases.py 5 500 500 256
timeout -k 10 120 python tools/_phases.py 9 400 400 64
cp exp/libmrt_w0.so miniraytracer_amd/libmrt.so
