#!/bin/bash
# Final-tree measurement (TAG names the record set, e.g. r04_v1), one GPU call: GPU suite + smoke; rocprofv3 kernel trace + PMC
# passes of C2 and of C3-C5 at full resolution (tools/profile.sh, tools/prof_configs.sh), summarised
# on the box (tools/pmc_summary.py) so the bench below prices its roofline by this tree's counters;
# contract A/B; parity at every config's resolution; the full-size BASELINE configs; the 8-rank
# rehearsal; the default bench line.  The new profiles/ files are copied to gpurun_out/profiles/
# (the only directory that comes back).  Every step under its own limit; any failure ends the call.
# PART=a: suite, smoke, profiles, contract A/B; PART=b: parity, configs, rehearsal, bench (after
# part a's profiles are committed); unset: both.  NO_CAB=1 leaves the contract A/B out of part a
# (a call of its own: gpurun's 20-minute limit).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/profiles
export TMPDIR=/tmp
TAG=${TAG:-r04_v1}
step() {
    local name=$1 t=$2; shift 2
    echo "== $name $(date +%T)"
    timeout -k 10 "$t" "$@" > "gpurun_out/$name.log" 2>&1
    local rc=$?
    echo "== $name rc=$rc $(date +%T)"
    tail -3 "gpurun_out/$name.log" | cut -c1-300
    if [ $rc -ne 0 ]; then echo "stopping after $name (rc=$rc)"; exit $rc; fi
    return 0
}
if [ "${PART:-ab}" != b ]; then
step gpu_tests 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread
step smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
step prof_c2 600 bash tools/profile.sh
step pmc_c2 60 python tools/pmc_summary.py $TAG
step prof_cfgs 900 bash tools/prof_configs.sh
for c in c3 c4 c5; do step pmc_$c 60 python tools/pmc_summary.py ${TAG}_$c --prof gpurun_out/prof_$c; done
cp profiles/${TAG}* profiles/pmc_s*.json gpurun_out/profiles/
[ "${NO_CAB:-0}" = 1 ] || step contract_ab 600 python tools/contract_ab.py --measure
fi
[ "${PART:-ab}" = a ] && exit 0
step parity 600 python tools/parity_record.py --out gpurun_out/profiles/${TAG}_parity.json
step configs 900 bash tools/configs.sh
CFGS="1,0 2,0 2,1 4,0 4,1 4,2 4,3 8,0 8,1 8,2 8,3 8,4 8,5 8,6 8,7" STEPS=60 step scale 900 bash tools/scale_rehearsal.sh
step bench 600 python bench.py --steps 20 --warmup 5
exit 0
