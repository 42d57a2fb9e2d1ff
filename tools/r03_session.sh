#!/bin/bash
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
step() {
    local name=$1 t=$2; shift 2
    echo "== $name $(date +%T)"
    timeout -k 10 "$t" "$@" > "gpurun_out/$name.log" 2>&1
    local rc=$?
    echo "== $name rc=$rc $(date +%T)"
    tail -6 "gpurun_out/$name.log"
    if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "stopping after $name (rc=$rc)"; exit $rc; fi
    return 0
}
step gpu_tests 900 python -u -m pytest tests/ -v -m gpu --timeout 300 --timeout-method thread
for tag in intree log disc logdisc; do lib=""; [ $tag != intree ] && lib=exp/libmrt_$tag.so
  MRT_EXPERIMENT_LIB=$lib step par7_$tag 300 python tools/parity_record.py --scenes 7 --out gpurun_out/par7_$tag.json; done
CFGS="7,2048,2048,64 0,1200,800,64 8,1024,1024,256 9,800,800,256" LIBS="lockstep logdisc soa" step ab 900 bash tools/ab_walk.sh
for wm in 0 16 48; do MRT_WALK_MIN=$wm CFGS="7,2048,2048,64 0,1200,800,64 1,1200,800,64" step wm_$wm 300 bash tools/ab_walk.sh; done
step scale 900 bash tools/scale_rehearsal.sh
for i in 1 2 3; do step bench_full_$i 300 python bench.py --no-cpu-baseline --no-compare-numerics --no-other-walk --steps 20 --warmup 5; done
for i in 1 2 3 4 5; do step bench_lean_$i 300 python bench.py --no-cpu-baseline --no-compare-numerics --no-other-walk --steps 20 --warmup 5 --fold lean; done
step trace_default 300 rocprofv3 --kernel-trace --stats -d gpurun_out/tr_default -o run --output-format csv -- python3 bench.py --no-cpu-baseline --no-compare-numerics --no-other-walk --no-parity --steps 20 --warmup 5
step trace_w8 300 rocprofv3 --kernel-trace --stats -d gpurun_out/tr_w8 -o run --output-format csv -- python3 bench.py --no-cpu-baseline --no-compare-numerics --no-other-walk --no-parity --steps 40 --warmup 4 --emulate-world 8 --emulate-gather
for tag in intree gen6 gen5; do lib=""; [ $tag != intree ] && lib=exp/libmrt_$tag.so
  MRT_NO_SIG=1 MRT_EXPERIMENT_LIB=$lib step nosig_$tag 300 python bench.py --no-cpu-baseline --no-compare-numerics --no-other-walk --steps 10 --warmup 2; done
exit 0
