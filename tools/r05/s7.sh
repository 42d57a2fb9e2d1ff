# round-5: GPU tests after the hand-over tightening (2^-18, 64 retrace groups) and the opaque scene
# default; A/B against the hand-over compiled out (nocrit), at 2^-16 (tol16) and off at run time;
# contract parity with hand-over counts; single-GPU scale rehearsal with step intervals
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
O=gpurun_out/r05
mkdir -p $O $O/img
timeout -k 10 500 python3 -u -m pytest tests -m gpu -q -x --timeout 200 --timeout-method thread > $O/gpu_tests_9.log 2>&1 || exit 1
MRT_PARITY_SAVE=$O/img timeout -k 10 300 python3 -u tools/contract_parity.py fast > $O/contract_parity_5.jsonl 2>&1 || exit 1
ROUNDS=2 STEPS=20 LIBS="nocrit tol16 MRT_RETRACE=0" CFGS="5,500,500,1024 9,800,800,256" timeout -k 10 600 bash tools/ab.sh > $O/ab_s7.txt 2>&1 || exit 1
STEPS=60 timeout -k 10 600 bash tools/scale_rehearsal.sh > $O/scale_rehearsal.txt 2>&1
