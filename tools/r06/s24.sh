#!/bin/bash
# round 6 session 24: an async-fold launch's retrace on the fold stream created at the device's
# highest stream priority (MRT_RETRACE_PRIO=1): the async GPU tests through it, then C2 at N = 1
# (one and two contexts) and the slowest N = 8 share (two contexts), with and without it
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out/r06
set -o pipefail
MRT_RETRACE_PRIO=1 timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -v -m gpu --timeout 200 --timeout-method thread \
    -k "async" > gpurun_out/r06/s24_tests.log 2>&1 || { tail -30 gpurun_out/r06/s24_tests.log; exit 3; }
tail -2 gpurun_out/r06/s24_tests.log
for r in 1 2; do
  for pr in 0 1; do
    for v in "1,0,n1p1,--pipeline 1" "1,0,n1p2,--pipeline 2" "8,6,n8r6,"; do
      IFS=, read n rk tag extra <<< "$v"
      log=gpurun_out/r06/s24_${tag}_prio${pr}_$r.log
      MRT_RETRACE_PRIO=$pr timeout -k 10 300 python bench.py --no-cpu-baseline --no-compare-numerics --no-other-walk --no-parity --steps 60 \
          --warmup 4 --emulate-world $n --emulate-rank $rk --emulate-gather --step-times $extra > $log 2>&1 || exit 3
      python - $log "$tag prio$pr" $r <<'PY'
import json, sys
j = json.loads([l for l in open(sys.argv[1]) if l.startswith("{")][-1])
st = j.get("step_times") or {}
c = j["config"]
print(f"{sys.argv[2]:>14} round {sys.argv[3]}: {j['ms_per_step']:.3f} ms/step, {j['value']:.0f} Mrays/s, kernel {j['roofline']['kernel_ms']:.3f} ms"
      f" [pipeline {c.get('pipeline')}, fold {c.get('fold')}] | intervals median {st.get('median_ms')} p90 {st.get('p90_ms')} max {st.get('max_ms')}")
PY
    done
  done
done
