#!/bin/bash
# Fixed per-launch cost of the C2 path kernel: kernel time (HIP events) at several sample counts,
# one context, fitted as t = a + b * rays.  DEPTHS / SPPS / SCALE_ARGS override the sweep.  Each
# run under its own time limit; a failure stops the script.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
out=gpurun_out/overhead_fit.txt
: > $out
for d in ${DEPTHS:-32}; do
  for s in ${SPPS:-16 64 128 256 1024}; do
    timeout -k 10 300 python bench.py --no-cpu-baseline --no-compare-numerics --no-other-walk --no-parity \
        --steps ${STEPS:-10} --warmup 3 --pipeline 1 --samples $s --depth $d ${SCALE_ARGS:-} \
        > gpurun_out/ovh_${d}_$s.log 2>&1 || exit 3
    python - gpurun_out/ovh_${d}_$s.log $d $s >> $out <<'PY'
import json, sys
j = json.loads([l for l in open(sys.argv[1]) if l.startswith("{")][-1])
r = j["config"]["rays_per_step"]
print(f"depth {sys.argv[2]} spp {sys.argv[3]} rays {r} step_ms {j['ms_per_step']:.4f} kernel_ms {j['roofline']['kernel_ms']:.4f}")
PY
  done
done
python - $out <<'PY'
import sys, numpy as np
rows = [l.split() for l in open(sys.argv[1])]
for d in sorted({r[1] for r in rows}, key=int):
    sel = [r for r in rows if r[1] == d]
    x = np.array([float(r[5]) for r in sel]); k = np.array([float(r[9]) for r in sel]); st = np.array([float(r[7]) for r in sel])
    bk, ak = np.polyfit(x, k, 1); bs, as_ = np.polyfit(x, st, 1)
    print(f"depth {d}: kernel = {ak*1e3:.1f} us + {bk*1e9:.3f} ms/Grays; step = {as_*1e3:.1f} us + {bs*1e9:.3f} ms/Grays")
PY
cat $out
