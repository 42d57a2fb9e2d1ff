#!/bin/bash
# check: bench's automatic fold choice per rank share (--emulate-world N)
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
for n in 1 2 4 8; do
  timeout -k 10 200 python bench.py --no-cpu-baseline --no-compare-numerics --steps 30 --emulate-world $n > gpurun_out/fwa_$n.log 2>&1 || exit 3
  python - gpurun_out/fwa_$n.log $n <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print("world", sys.argv[2], d["config"]["fold"], d["value"], d["ms_per_step"])
PY
done
