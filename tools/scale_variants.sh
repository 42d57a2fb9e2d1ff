#!/bin/bash
# Interleaved single-GPU rehearsal runs of per-rank shares under different step shapes:
#   VARIANTS="N,R,tag,extra bench args;..."  (tag names the run; extra args e.g. --pipeline 1 --fold async)
# ROUNDS alternations; each run: bench.py --emulate-world N --emulate-rank R --emulate-gather --step-times
# -> gpurun_out/sv_<tag>_<round>.log and one summary line (ms per step, kernel ms, step intervals).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for r in $(seq 1 "${ROUNDS:-2}"); do
  IFS=';' read -ra VS <<< "$VARIANTS"
  for v in "${VS[@]}"; do
    IFS=, read n rk tag extra <<< "$v"
    log=gpurun_out/sv_${tag}_$r.log
    timeout -k 10 ${RUN_TIMEOUT:-300} python bench.py --no-cpu-baseline --no-compare-numerics --no-other-walk --no-parity --steps ${STEPS:-60} \
        --warmup ${WARMUP:-4} --emulate-world $n --emulate-rank $rk --emulate-gather --step-times ${SCALE_ARGS:-} $extra > $log 2>&1 || exit 3
    python - $log "$tag" $r <<'PY'
import json, sys
j = json.loads([l for l in open(sys.argv[1]) if l.startswith("{")][-1])
st = j.get("step_times") or {}
c = j["config"]
print(f"{sys.argv[2]:>14} round {sys.argv[3]}: {j['ms_per_step']:.3f} ms/step, {j['value']:.0f} Mrays/s, kernel {j['roofline']['kernel_ms']:.3f} ms"
      f" [pipeline {c.get('pipeline')}, fold {c.get('fold')}] | intervals median {st.get('median_ms')} p90 {st.get('p90_ms')} max {st.get('max_ms')}")
PY
  done
done
