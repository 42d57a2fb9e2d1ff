# round-5: single-pixel hand-over probe of C3's dominant residual pixels
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
O=gpurun_out/r05
mkdir -p $O
timeout -k 10 300 python3 -u tools/handover_probe.py 9 800 800 4096 tests/golden/shipped_ownspp_full_9.npz 261,408 271,129 405,313 325,182 379,734 > $O/handover_probe.jsonl 2>&1
