# round-5: interpreter PMC (C2 through the linear-program interpreter), single-GPU scale
# rehearsal with per-step intervals, contract parity of the final numerics
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
O=gpurun_out/r05
mkdir -p $O
A="--steps 1 --warmup 0 --kernel-reps 1 --pipeline 1 --no-cpu-baseline --no-other-walk --no-parity --no-compare-numerics"
SQ="SQ_WAVES,SQ_INSTS_VALU,SQ_INSTS_SALU,SQ_INSTS_SMEM,SQ_WAIT_INST_ANY,SQ_WAVE_CYCLES,SQ_ACTIVE_INST_VALU,SQ_INSTS_LDS"
for sig in 0 1; do
  MRT_NO_SIG=$((1 - sig)) timeout -s KILL 120 rocprofv3 --pmc $SQ -d $O/pmc_interp_sig$sig -o run --output-format csv -- python3 bench.py $A > $O/pmc_interp_sig$sig.log 2>&1 || exit 1
done
STEPS=60 timeout -k 10 600 bash tools/scale_rehearsal.sh > $O/scale_rehearsal.txt 2>&1 || exit 1
timeout -k 10 300 python3 -u tools/contract_parity.py fast exact > $O/contract_parity_final.jsonl 2>&1
