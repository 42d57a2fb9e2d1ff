#!/bin/bash
# round-2 measurement call: contract A/B measure, C2 profile, C3/C4/C5 profiles (each step timed)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 400 python -u tools/contract_ab.py --measure > gpurun_out/contract_ab.log 2>&1 || exit 1
echo "contract_ab done $(date +%T)"
timeout -k 10 400 bash tools/profile.sh > gpurun_out/prof.log 2>&1 || exit 2
echo "prof done $(date +%T)"
timeout -k 10 600 bash tools/prof_configs.sh > gpurun_out/profcfg.log 2>&1 || exit 3
echo "prof_configs done $(date +%T)"
