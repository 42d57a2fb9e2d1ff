#!/bin/bash
# Single-GPU rehearsal of the N-GPU bench: per-rank step time of rank R's tile share (no
# collectives), N = 1, 2, 4, 8.  Each run under its own time limit; a failure stops the script.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
CFGS=${CFGS:-1,0 2,0 4,0 8,0 8,7}
for cfg in $CFGS; do
  IFS=, read n r <<< "$cfg"
  timeout -k 10 300 python bench.py --no-cpu-baseline --steps ${STEPS:-20} --warmup 2 --emulate-world $n --emulate-rank $r \
      > gpurun_out/scale_${n}_$r.log 2>&1 || exit 3
  python - gpurun_out/scale_${n}_$r.log $n $r <<'PY'
import json, sys
j = json.loads([l for l in open(sys.argv[1]) if l.startswith("{")][-1])
print(f"N={sys.argv[2]} rank {sys.argv[3]}: {j['ms_per_step']:.3f} ms/step, {j['value']:.0f} Mrays/s, kernel {j['roofline']['kernel_ms']:.3f} ms")
PY
done
