# round-5: rocprofv3 passes of the interpreter on C2 (MRT_NO_SIG=1) and of C5 with the book2
# kernel variant; summaries made on the box (tools/pmc_summary.py) and copied back
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out/profiles
MRT_NO_SIG=1 PROF_OUT=gpurun_out/prof_interp timeout -k 10 600 bash tools/profile.sh > gpurun_out/prof_interp.log 2>&1 || exit 1
python3 tools/pmc_summary.py r05_v1_interp --prof gpurun_out/prof_interp --no-bench-file > gpurun_out/pmc_interp.log 2>&1 || exit 1
PROF_CFGS="c5:7:2048:2048:64" timeout -k 10 600 bash tools/prof_configs.sh > gpurun_out/prof_c5.log 2>&1 || exit 1
python3 tools/pmc_summary.py r05_v2_c5 --prof gpurun_out/prof_c5 > gpurun_out/pmc_c5.log 2>&1 || exit 1
cp profiles/r05_v1_interp* profiles/r05_v2_c5* profiles/pmc_s7_2048x2048.json gpurun_out/profiles/
