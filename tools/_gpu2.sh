set -e
cd $GRAFT_REPO_ROOT
PROF_SQ="SQ_WAVES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_THREAD_CYCLES_VALU SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY" bash tools/profile.sh > gpurun_out/profile.out 2>&1
STEPS=10 bash tools/scale_rehearsal.sh
bash tools/configs.sh
