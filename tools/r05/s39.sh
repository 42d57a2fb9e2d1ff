# round-5 final tree (room + mesh at 8 waves, interpreter dispatch order): GPU suite, smoke, contract
# parity, PMC of C3 and C4 (summaries on the box), the BASELINE configs at full size, the bench line
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
O=gpurun_out/r05
mkdir -p $O gpurun_out/profiles
timeout -k 10 500 python3 -u -m pytest tests -m gpu -q -x --timeout 200 --timeout-method thread > $O/gpu_tests_39.log 2>&1 || exit 1
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > $O/smoke_39.log 2>&1 || exit 1
timeout -k 10 300 python3 -u tools/contract_parity.py fast > $O/contract_parity_9.jsonl 2>&1 || exit 1
PROF_CFGS="c3:9:800:800:256 c4:8:1024:1024:256" timeout -k 10 600 bash tools/prof_configs.sh > gpurun_out/prof_c34.log 2>&1 || exit 1
python3 tools/pmc_summary.py r05_v3_c3 --prof gpurun_out/prof_c3 > gpurun_out/pmc_c3.log 2>&1 || exit 1
python3 tools/pmc_summary.py r05_v3_c4 --prof gpurun_out/prof_c4 > gpurun_out/pmc_c4.log 2>&1 || exit 1
cp profiles/r05_v3_c3* profiles/r05_v3_c4* profiles/pmc_s9_800x800.json profiles/pmc_s8_1024x1024.json gpurun_out/profiles/
timeout -k 10 900 bash tools/configs.sh > $O/configs_39.txt 2>&1 || exit 1
timeout -k 10 400 python3 bench.py --steps 20 --warmup 5 > $O/bench_39.log 2>&1
