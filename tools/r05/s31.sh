# round-5 final tree: GPU suite, smoke, contract parity (every config's own spp), the default bench
# line (CPU baselines incl. the AVX-512 reference build), kernel trace of the bench (rocprofv3 stats),
# the interpreter's PMC, the BASELINE configs at full size
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
O=gpurun_out/r05
mkdir -p $O gpurun_out/profiles
timeout -k 10 500 python3 -u -m pytest tests -m gpu -q -x --timeout 200 --timeout-method thread > $O/gpu_tests_31.log 2>&1 || exit 1
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > $O/smoke_31.log 2>&1 || exit 1
timeout -k 10 300 python3 -u tools/contract_parity.py fast > $O/contract_parity_8.jsonl 2>&1 || exit 1
timeout -k 10 400 python3 bench.py --steps 20 --warmup 5 > $O/bench_31.log 2>&1 || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/kt_bench -o run --output-format csv -- python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline > $O/kt_bench.log 2>&1 || exit 1
MRT_NO_SIG=1 PROF_OUT=gpurun_out/prof_interp timeout -k 10 600 bash tools/profile.sh > gpurun_out/prof_interp.log 2>&1 || exit 1
python3 tools/pmc_summary.py r05_v2_interp --prof gpurun_out/prof_interp --no-bench-file > gpurun_out/pmc_interp.log 2>&1 || exit 1
cp profiles/r05_v2_interp* gpurun_out/profiles/
