#!/bin/bash
# round 6 session 25: the retrace list spread evenly over the retrace kernel's groups, and more groups
# (MRT_RETRACE_GROUPS 256 / 1024 / 4096: a few paths per wave, the longest one with little
# divergence): GPU tests of the hand-over through 4096, then C2 N = 1 under the kernel trace (the
# retrace kernel's average duration) and the slowest N = 8 share per group count
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out/r06
set -o pipefail
export TMPDIR=/tmp
MRT_RETRACE_GROUPS=4096 timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -v -m gpu --timeout 200 --timeout-method thread \
    -k "async or contract or handover or retrace or stream_5" > gpurun_out/r06/s25_tests.log 2>&1 || { tail -30 gpurun_out/r06/s25_tests.log; exit 3; }
tail -2 gpurun_out/r06/s25_tests.log
for g in 256 1024 4096; do
  MRT_RETRACE_GROUPS=$g timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r06/s25_tr_$g -o run --output-format csv -- \
      python3 bench.py --no-cpu-baseline --no-compare-numerics --no-other-walk --no-parity --steps 20 --warmup 3 > gpurun_out/r06/s25_tr_$g.log 2>&1 || exit 3
  python tools/show_bench.py gpurun_out/r06/s25_tr_$g.log "traced groups $g"
  f=$(find gpurun_out/r06/s25_tr_$g -name '*kernel_stats.csv' | head -1)
  grep -h "retrace\|fold_async" "$f" | cut -d, -f1-4
done
for r in 1 2; do
  for g in 256 1024 4096; do
    for v in "1,0,n1" "8,6,n8r6"; do
      IFS=, read n rk tag <<< "$v"
      log=gpurun_out/r06/s25_${tag}_g${g}_$r.log
      MRT_RETRACE_GROUPS=$g timeout -k 10 300 python bench.py --no-cpu-baseline --no-compare-numerics --no-other-walk --no-parity --steps 60 \
          --warmup 4 --emulate-world $n --emulate-rank $rk --emulate-gather --step-times > $log 2>&1 || exit 3
      python - $log "$tag g$g" $r <<'PY'
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
