# round-5: the fold beside the next render's path kernel (MRT_RF_FOLD_ASYNC, bench --fold async) on
# C2: in tree (full fold after the kernel), w8 (Cornell kernel capped at 64 VGPRs, launched at 7
# waves/SIMD: one slot per SIMD left for the 52-VGPR fold) with the full fold and with the async
# fold, and the in-tree kernel (no slot left) with the async fold; --verify: bit-identical image
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
O=gpurun_out/r05
mkdir -p $O
run() {  # tag env... -- bench args
  tag=$1; shift
  envs=(); while [ "$1" != "--" ]; do envs+=("$1"); shift; done; shift
  log=$O/s42_${tag}_$r.log
  env MRT_AB_TAG=$tag "${envs[@]}" timeout -k 10 300 python bench.py --no-cpu-baseline --no-compare-numerics --no-other-walk \
      --no-parity --steps 20 --warmup 2 --scene 5 --width 500 --height 500 --samples 1024 "$@" > $log 2>&1 || exit 3
  python tools/show_bench.py $log "$tag round $r"
  grep -o '"verify_bit_exact": [a-z]*' $log || true
}
for r in 1 2 3; do
  run intree -- --fold full
  run w8full MRT_EXPERIMENT_LIB=exp/libmrt_w8.so MRT_BLOCKS_PER_CU=28 -- --fold full
  run w8async MRT_EXPERIMENT_LIB=exp/libmrt_w8.so MRT_BLOCKS_PER_CU=28 -- --fold async --verify
  run async -- --fold async --verify
done
