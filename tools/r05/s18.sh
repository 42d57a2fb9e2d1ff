# round-5: single-GPU scale rehearsal of every rank share at N = 1, 2, 4, 8 (60 timed steps, the
# default three pipelined contexts), then every N = 8 share again at one context (--pipeline 1),
# whose per-step completion intervals are those of single steps
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
O=gpurun_out/r05
mkdir -p $O
CFGS="1,0 2,0 2,1 4,0 4,1 4,2 4,3 8,0 8,1 8,2 8,3 8,4 8,5 8,6 8,7" STEPS=60 timeout -k 10 900 bash tools/scale_rehearsal.sh > $O/scale_rehearsal_all.txt 2>&1 || exit 1
CFGS="8,0 8,1 8,2 8,3 8,4 8,5 8,6 8,7" STEPS=60 SCALE_ARGS="--pipeline 1" timeout -k 10 600 bash tools/scale_rehearsal.sh > $O/scale_rehearsal_p1.txt 2>&1
