#!/bin/bash
# oracle/ref/build_ref.sh -- TEST INFRASTRUCTURE ONLY.
#
# Builds the reference renderer's own translation units, where they lie under /root/reference
# (read-only), together with oracle/ref/harness.cpp into two oracle binaries in oracle/_ref/:
#
#   mrt_ref        reference as shipped: clang++ -std=c++20 -O3 -fno-exceptions -fno-rtti
#                  (clang/clang_build_linux.sh:23-29), default FP contraction (-ffp-contract=on:
#                  x86 FMA wherever one scalar expression multiplies and adds), glibc libm.
#                  -march=x86-64-v3 instead of -march=native so the binary also runs on the GPU
#                  box's host CPU (it is the cpu_baseline of bench.py); both have FMA.
#   mrt_ref_v4     the same with -march=x86-64-v4 (AVX-512): what -march=native gives on an AVX-512
#                  host; bench.py times it too where the host CPU has AVX-512F.
#   mrt_ref_exact  the same build (same flags, so the same fused multiply-adds) with the float libm
#                  calls interposed by (float)f((double)x) (harness.cpp, MRT_MATHMATCH): the
#                  reference as shipped with the project's transcendentals.  This is the bit-exact
#                  pin of the exact numerics contract: the C restatement (oracle/mrt_oracle.c), the
#                  HIP kernel and the CPU backend.  (Rounds 1-3 pinned a -ffp-contract=off build;
#                  the two differ only by the fused sites)
#
# Two compile fixes, both applied without writing into /root/reference and without copying the
# source tree: mrt_math.h:66 is an '#error INSERT LZCNT INTRINSIC HERE' placeholder for non-MSVC
# compilers -- a patched copy of that one header is mapped over the original with a clang VFS
# overlay; triangle.h:85 calls memcpy without <cstring> -- fixed with '-include cstring'.
# The SDL platform layer (platform_linux.cpp) is not compiled: the harness is headless.
# Nothing is written outside oracle/_ref/ and a private mktemp directory that is removed on exit.
set -euo pipefail
REF=${MRT_REFERENCE:-/root/reference}
HERE=$(cd "$(dirname "$0")" && pwd)
OUT=$(cd "$HERE/.." && pwd)/_ref
CXX=${CXX:-/opt/rocm/lib/llvm/bin/clang++}
if [ ! -f "$REF/main.cpp" ]; then
    echo "build_ref: reference not present at $REF; skipping (prebuilt oracle/_ref used if present)"
    exit 0
fi
mkdir -p "$OUT"
TMP=$(mktemp -d /tmp/mrtref.XXXXXX)
trap 'rm -rf "$TMP"' EXIT

sed 's|^#error INSERT LZCNT INTRINSIC HERE|        uint32 i = (uint32)__builtin_clz(v);|' "$REF/mrt_math.h" > "$TMP/mrt_math.h"
cat > "$TMP/overlay.yaml" <<EOF
{ 'version': 0, 'case-sensitive': 'true', 'roots': [ { 'name': '$REF', 'type': 'directory',
  'contents': [ { 'name': 'mrt_math.h', 'type': 'file', 'external-contents': '$TMP/mrt_math.h' } ] } ] }
EOF

SRCS="cmdline_parser.cpp mat4.cpp obj_loader.cpp pcg.cpp rect.cpp scene.cpp scene_object.cpp sphere.cpp
      stb_image.cpp texture.cpp triangle.cpp volumes.cpp work_queue.cpp"
BASE="-std=c++20 -O3 -march=x86-64-v3 -fno-exceptions -fno-rtti -w -include cstring -ivfsoverlay $TMP/overlay.yaml -I$REF -I$REF/include"

build() {  # name extra-flags
    local name=$1; shift
    local odir="$TMP/$name"; mkdir -p "$odir"
    local pids=()
    for s in $SRCS; do
        $CXX $BASE "$@" -c "$REF/$s" -o "$odir/${s%.cpp}.o" & pids+=($!)
    done
    $CXX $BASE "$@" -c "$HERE/harness.cpp" -o "$odir/harness.o" & pids+=($!)
    for p in "${pids[@]}"; do wait "$p"; done
    $CXX "$odir"/*.o -lpthread -o "$OUT/$name"
    echo "build_ref: built $OUT/$name"
    BUILT+=("$name")
}
BUILT=()

build mrt_ref
build mrt_ref_v4 -march=x86-64-v4
build mrt_ref_exact -DMRT_MATHMATCH
# numerics-diagnosis builds (MRT_REF_VARIANTS=1): the reference with no contraction at all (with
# the project's transcendentals: the rounds 1-3 pin; with glibc) and with unrestricted contraction
# (-ffp-contract=fast), to measure what each difference does to the image
if [ -n "${MRT_REF_VARIANTS:-}" ]; then
    build mrt_ref_nofma -ffp-contract=off -DMRT_MATHMATCH
    build mrt_ref_glibc -ffp-contract=off
    build mrt_ref_fastc -ffp-contract=fast
fi
# provenance of the binaries (they travel to the GPU box untracked, where /root/reference is absent):
# sha256 of each, the commit of this recipe, the compiler -- bench.py's cpu_baseline reports them
{
    echo "{"
    echo "  \"recipe\": \"oracle/ref/build_ref.sh\","
    echo "  \"recipe_commit\": \"$(git -C "$HERE" log -1 --format=%H -- build_ref.sh harness.cpp 2>/dev/null || echo unknown)\","
    echo "  \"recipe_dirty\": $( [ -n "$(git -C "$HERE" status --porcelain -- build_ref.sh harness.cpp 2>/dev/null)" ] && echo true || echo false ),"
    echo "  \"compiler\": \"$($CXX --version | head -1 | sed 's/\"/\x27/g')\","
    echo "  \"reference\": \"$REF\","
    echo "  \"built_utc\": \"$(date -u +%Y-%m-%dT%H:%M:%SZ)\","
    echo "  \"sha256\": {"
    n=${#BUILT[@]}; i=0
    for b in "${BUILT[@]}"; do
        i=$((i + 1)); sep=","; [ $i -eq $n ] && sep=""
        echo "    \"$b\": \"$(sha256sum "$OUT/$b" | cut -d' ' -f1)\"$sep"
    done
    echo "  }"
    echo "}"
} > "$OUT/BUILD_INFO.json"
echo "build_ref: provenance in $OUT/BUILD_INFO.json"
