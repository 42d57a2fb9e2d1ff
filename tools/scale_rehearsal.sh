#!/bin/bash
# Single-GPU rehearsal of the N-GPU bench: per-rank step time of rank R's tile share, N = 1, 2, 4,
# 8, with rank 0's device-side share of the gather (--emulate-gather: the scatter of all N shards;
# renders write straight into padded shard buffers, so there is no pad copy) -- only the xGMI
# transfer itself is not in it.  Predicted speed-up at N = (1-rank step) / (N-rank step).  Each run
# under its own time limit; a failure stops the script.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
CFGS=${CFGS:-1,0 2,0 4,0 8,0 8,7}
for cfg in $CFGS; do
  IFS=, read n r <<< "$cfg"
  timeout -k 10 ${RUN_TIMEOUT:-300} python bench.py --no-cpu-baseline --no-compare-numerics --no-other-walk --no-parity --steps ${STEPS:-40} --warmup ${WARMUP:-4} \
      --emulate-world $n --emulate-rank $r --emulate-gather --step-times ${SCALE_ARGS:-} > gpurun_out/scale_${n}_$r.log 2>&1 || exit 3
  python - gpurun_out/scale_${n}_$r.log $n $r <<'PY'
import json, sys
j = json.loads([l for l in open(sys.argv[1]) if l.startswith("{")][-1])
st = j.get("step_times") or {}
print(f"N={sys.argv[2]} rank {sys.argv[3]}: {j['ms_per_step']:.3f} ms/step, {j['value']:.0f} Mrays/s, kernel {j['roofline']['kernel_ms']:.3f} ms"
      f" | step intervals median {st.get('median_ms')} p90 {st.get('p90_ms')} max {st.get('max_ms')} at {st.get('max_at_step')}")
PY
done
