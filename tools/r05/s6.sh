# round-5: A/B of the in-step hand-over (nocrit: compiled out; MRT_RETRACE=0: off at run time) and
# of the opaque scene pointer in the plain path loop (opq: bvh_node kernels), interpreter PMC,
# single-GPU scale rehearsal with step intervals
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
O=gpurun_out/r05
mkdir -p $O
export ROUNDS=2 STEPS=20 LIBS="nocrit MRT_RETRACE=0 opq" CFGS="5,500,500,1024 9,800,800,256 7,2048,2048,64 0,1200,800,64"
timeout -k 10 700 bash tools/ab.sh > $O/ab_s6.txt 2>&1 || exit 1
A="--steps 1 --warmup 0 --kernel-reps 1 --pipeline 1 --no-cpu-baseline --no-other-walk --no-parity --no-compare-numerics"
SQ="SQ_WAVES,SQ_INSTS_VALU,SQ_INSTS_SALU,SQ_INSTS_SMEM,SQ_WAIT_INST_ANY,SQ_WAVE_CYCLES,SQ_ACTIVE_INST_VALU,SQ_INSTS_LDS"
for sig in 0 1; do
  MRT_NO_SIG=$((1 - sig)) timeout -s KILL 120 rocprofv3 --pmc $SQ -d $O/pmc_interp_sig$sig -o run --output-format csv -- python3 bench.py $A > $O/pmc_interp_sig$sig.log 2>&1 || exit 1
done
unset CFGS; STEPS=60 timeout -k 10 600 bash tools/scale_rehearsal.sh > $O/scale_rehearsal.txt 2>&1
