# experiment: per-phase wave time (exp/libmrt_ph.so, -DMRT_PHASES); PH_CFGS = "scene,W,H,spp ..."
cd $GRAFT_REPO_ROOT
cp exp/libmrt_ph.so miniraytracer_amd/libmrt.so
for a in ${PH_CFGS:-5,500,500,256 8,512,512,64 7,256,256,64}; do NPH=${NPH:-8} timeout -k 10 120 python tools/_phases.py ${a//,/ } || break; done
cp exp/libmrt_w0.so miniraytracer_amd/libmrt.so
