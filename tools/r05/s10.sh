# round-5: hand-over with the list read from the argument segment and the edge criterion: GPU
# tests, contract parity, the C3 residual pixels, A/B (hand-over compiled out / no edge criterion /
# off at run time)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
O=gpurun_out/r05
mkdir -p $O $O/img
timeout -k 10 500 python3 -u -m pytest tests -m gpu -q -x --timeout 200 --timeout-method thread > $O/gpu_tests_10.log 2>&1 || exit 1
MRT_PARITY_SAVE=$O/img timeout -k 10 300 python3 -u tools/contract_parity.py fast > $O/contract_parity_6.jsonl 2>&1 || exit 1
timeout -k 10 300 python3 -u tools/handover_probe.py 9 800 800 4096 tests/golden/shipped_ownspp_full_9.npz 261,408 271,129 405,313 325,182 379,734 > $O/handover_probe_2.jsonl 2>&1 || exit 1
ROUNDS=2 STEPS=20 LIBS="nocrit noedge MRT_RETRACE=0" CFGS="5,500,500,1024 9,800,800,256" timeout -k 10 600 bash tools/ab.sh > $O/ab_s10.txt 2>&1
