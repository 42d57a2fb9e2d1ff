# round-5: the hand-over's criterion in cheaper forms (edge samples below the surface only), the
# opaque scene pointer in the shared-constructor loop (opqs); contract parity; A/B
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
O=gpurun_out/r05
mkdir -p $O $O/img
timeout -k 10 500 python3 -u -m pytest tests -m gpu -q -x --timeout 200 --timeout-method thread > $O/gpu_tests_11.log 2>&1 || exit 1
MRT_PARITY_SAVE=$O/img timeout -k 10 300 python3 -u tools/contract_parity.py fast > $O/contract_parity_7.jsonl 2>&1 || exit 1
ROUNDS=3 STEPS=20 LIBS="nocrit opqs MRT_RETRACE=0" CFGS="5,500,500,1024 9,800,800,256" timeout -k 10 900 bash tools/ab.sh > $O/ab_s11.txt 2>&1
