# round-5: A/B of the rounding-critical hand-over (nocrit) and pixel sums (nopsum) builds
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out/r05
export ROUNDS=2 STEPS=10 LIBS="nocrit nopsum" CFGS="5,500,500,1024 9,800,800,256 7,2048,2048,64 0,1200,800,64"
timeout -k 10 900 bash tools/ab.sh > gpurun_out/r05/ab_s4.txt 2>&1
