# round-5: which samples of C3's dominant residual pixels end non-finite under each contract; kernel
# trace of a C2 bench (path kernel, retrace, fold per step)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
O=gpurun_out/r05
mkdir -p $O
timeout -k 10 300 python3 -u tools/nonfinite_pixels.py 9 800 800 4096 261,408 271,129 405,313 325,182 379,734 > $O/nonfinite_c3px.jsonl 2>&1 || exit 1
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $O/kt_c2 -o run --output-format csv -- python3 bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-other-walk --no-parity --no-compare-numerics > $O/kt_c2.log 2>&1
