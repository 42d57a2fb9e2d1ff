# round-5: GPU tests, A/B of the rounding-critical hand-over (nocrit = compiled out), parity
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out/r05
timeout -k 10 500 python3 -u -m pytest tests -m gpu -q -x --timeout 200 --timeout-method thread > gpurun_out/r05/gpu_tests_8.log 2>&1 || exit 1
export ROUNDS=3 STEPS=20 LIBS="nocrit MRT_RETRACE=0" CFGS="5,500,500,1024 9,800,800,256"
timeout -k 10 600 bash tools/ab.sh > gpurun_out/r05/ab_s5.txt 2>&1 || exit 1
timeout -k 10 300 python3 -u tools/contract_parity.py fast > gpurun_out/r05/contract_parity_4.jsonl 2>&1
