cd $GRAFT_REPO_ROOT
cp exp/libmrt_ph8.so miniraytracer_amd/libmrt.so
NPH=8 timeout -k 10 120 python tools/_phases.py 5 500 500 256
cp exp/libmrt_w0.so miniraytracer_amd/libmrt.so
