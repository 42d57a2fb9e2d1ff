// mrt_launch.h -- the interface between the host code (mrt_render.hip) and the path-kernel
// translation unit (mrt_kernels.hip), which is compiled twice: once under the exact numerics
// contract (MRT_FAST=0, -ffp-contract=off) and once under the tolerance contract (MRT_FAST=1,
// FMA contraction, hardware reciprocal/sqrt, f32 transcendentals).  DESIGN.md "Numerics contracts".
#pragma once
#include <hip/hip_runtime.h>
#include "mrt_shade.h"

namespace mrtd {

#ifndef MRT_NPART
#define MRT_NPART 8u  // work partitions (and counters) per launch: one per XCD (mrt_kernels.hip)
#endif
#define MRT_COUNTER_STRIDE 16u  // uint64 words between two partitions' counters (128 B)
#define MRT_CNT_SLOTS MRT_NPART  // counter slots per launch (the reset kernels' unit)

struct PathParams {
    DScene sc;                            // by value: kernarg (constant) memory, scalar-loaded
    const uint2* __restrict__ pixels;     // local pixel -> (x, y), row 0 = bottom
    const float2* __restrict__ sdist;     // sample s -> grid offsets (main.cpp:324-331)
    uint32_t npix;                        // local pixel count
    double inv_npix;                      // 1.0 / npix (path index -> sample row without a divide)
    uint32_t width, height, sq, ns;
    float inv_w, inv_h;                   // RN(1/width), RN(1/height)
    uint32_t fast_uv;                     // width, height <= 2^24 and sq <= 2^16: u, v through div_core
    uint32_t s0;                          // first sample of this chunk
    uint32_t n_paths;                     // npix * chunk samples (< 2^32, enforced on the host)
    uint32_t tail_zone;                   // last paths of a partition handed out MRT_TAIL_BATCH at a time
    uint64_t part_base[MRT_NPART + 1];    // work partition k: paths [part_base[k], part_base[k+1])
    uint64_t part_dyn[MRT_NPART];         // its first path handed out by its counter (after the static claims)
    uint32_t static_first;                // every wave's first claim is static (short launches)
    uint64_t seed;
    uint32_t max_bounces;
    float* __restrict__ rad;              // n_paths * 3 floats, [s - s0][lp]
    uint32_t* __restrict__ path_rays;     // optional (debug): n_paths
    unsigned long long* __restrict__ counter;  // MRT_NPART work counters, MRT_COUNTER_STRIDE apart (paths handed out)
    unsigned long long* hprog;            // host-coherent pinned snapshots, one per partition (mrt_progress), or null
    const int* cancel;                    // device flag: non-zero makes the launch exit (G_isRunning)
    unsigned long long* __restrict__ rays;
    float4* __restrict__ lev;             // fold levels, lane-major: [slot][lev_rows]
    uint32_t lev_rows;                    // levels per lane (max_bounces, at least 1)
    uint32_t lds_frames, lds_rays, lds_mesh, lds_save;  // LDS stack slots / words per lane
    uint32_t walk_min;                    // resumable mesh walk: yield once at most this many lanes walk
    const float4* tree_src;               // TreeOf<F>::on kernels: BvhWide nodes copied to LDS at start
    uint32_t tree_n;                      // how many (the first tree_n of the breadth-first array)
    // rounding-critical paths (mrt_shade.h light_critical) listed for the exact-arithmetic retrace
    // kernel: null rt, no hand-over
    RetraceList rt;
};

typedef void (*path_kernel_t)(PathParams);

// path index -> (local pixel, sample row of the chunk): i = sl * npix + lp
MRT_DFN void path_coords(const PathParams& P, uint32_t i, uint32_t* lp_out, uint32_t* sl_out) {
    // the double estimate of i / npix is off by at most one either way
    uint32_t sl = (uint32_t)((double)i * P.inv_npix);
    uint32_t lp = i - sl * P.npix;
    if ((int32_t)lp < 0) { sl--; lp += P.npix; }
    if (lp >= P.npix) { sl++; lp -= P.npix; }
    *lp_out = lp;
    *sl_out = sl;
}

// path index -> its camera coordinates (u, v) and its PCG stream seeded from the path key
// (main.cpp:138-149 per (pixel, sample); the stream key of DESIGN.md section 2)
// (local pixel lp, sample s) -> the same
MRT_DFN void path_key_at(const PathParams& P, uint32_t lp, uint32_t s, Pcg& rng, float* uo, float* vo) {
    const uint2 xy = P.pixels[lp];
    const uint32_t x = xy.x, y = xy.y;
    const uint32_t pix = x + y * P.width;
    const float2 dd = P.sdist[s];  // ((i + 0.5) / sq, (j + 0.5) / sq), s = i*sq + j
    // (x + dx) / W with RN(1/W) from the host: numerator >= 1/(2 sq) >= 2^-17, W <= 2^24
    const float nu = (float)x + dd.x, nv = (float)y + dd.y;
    // exact for every image the host accepts (width, height <= 2^24, mrt_prepare)
    *uo = div_core(nu, (float)P.width, P.inv_w);
    *vo = div_core(nv, (float)P.height, P.inv_h);
    const uint64_t path_id = (uint64_t)pix * P.ns + s;
    pcg_seed(rng, splitmix64(P.seed ^ path_id), path_id);
}
MRT_DFN void path_key_of(const PathParams& P, uint32_t i, Pcg& rng, float* uo, float* vo) {
    uint32_t lp, sl;
    path_coords(P, i, &lp, &sl);
    path_key_at(P, lp, P.s0 + sl, rng, uo, vo);
}

// threads per path-kernel workgroup: TreeOf<F>::wg (mrt_trace.h).  One-wave groups by default
// (each wave owns its own LDS slice; a small group frees its CU slot as soon as its wave finishes,
// which matters in a launch's tail); the bvh_node kernels run one 16-wave group per CU that
// shares a treelet of hot BVH nodes.
#ifndef MRT_BATCH
#define MRT_BATCH 256u  // paths a wave claims per atomic on the work counter (one hot address)
#endif
#ifndef MRT_TAIL_BATCH
#define MRT_TAIL_BATCH 64u  // claim size within the last `tail_zone` paths of a launch
#endif
// one claim must cover a whole wave's idle lanes (the pool hands out at most 64 at once)
static_assert(MRT_TAIL_BATCH >= 64u && MRT_BATCH >= MRT_TAIL_BATCH, "claims must be at least a wave wide");

// kernel variants by scene features (the first instantiated superset is launched); FT_LIN
// variants need the scene's linear hit program (mrt_lin.h), FT_ALL runs any graph.  The same list
// in both numerics builds.
static constexpr uint32_t kVariants[] = {FT_LIN | FT_INST | FT_BIASED | MRT_SIG_BITS(SIG_CORNELL),
                                         FT_LIN | FT_MESH | FT_BIASED | MRT_SIG_BITS(SIG_ROOM_MESH),
                                         FT_LIN | FT_MESH | FT_METAL | FT_BIASED | MRT_SIG_BITS(SIG_ROOM_MESH),
                                         FT_LIN | FT_INST | FT_BIASED,
                                         FT_LIN | FT_MESH | FT_METAL | FT_BIASED,
                                         // sky-lit scenes 0-4: no light sampling compiled in (its registers
                                         // pushed this 128-VGPR kernel into a spill inside the bounce loop)
                                         FT_LIN | FT_BVHW | FT_TEX | FT_METAL | FT_MOVING | FT_SKY | FT_UV,
                                         // Cornell smoke (scene 6): box-bounded volumes as sub-programs,
                                         // instances, light sampling
                                         FT_LIN | FT_INST | FT_VOLUME | FT_VSUB | FT_ISO | FT_BIASED,
#ifndef MRT_NO_B2  // (A/B hook: book2 on the catch-all interpreter kernel)
                                         // lit bvh_node scenes with volumes, textures, motion (book2, C5): no mesh
                                         // walk, no sky, no sphere in the biased list, no generic bvh walk
                                         FT_LIN | FT_BVHW | FT_VOLUME | FT_INST | FT_TEX | FT_METAL | FT_ISO | FT_MOVING | FT_UV | FT_BIASED,
#endif
                                         FT_LIN | FT_ALL,
                                         FT_ALL};
static constexpr uint32_t kNumVariants = sizeof(kVariants) / sizeof(kVariants[0]);

// One numerics build of the path kernels: a kernel per variant and the LDS fold levels it keeps.
struct KernelTable {
    const char* numerics;  // "exact" | "fast"
    path_kernel_t kernel[kNumVariants];
    uint32_t lev_k[kNumVariants];
    uint32_t wg[kNumVariants];    // threads per workgroup
    uint32_t tree[kNumVariants];  // 1: the kernel reads the top BvhWide nodes from an LDS treelet
    uint32_t pq[kNumVariants];    // LDS words per lane slot of the kernel's queue of path starts
    uint32_t box6_walk[kNumVariants];  // 1: Cornell shape walked by cornell_fast_hit when op 8 is MRT_F_BOX6
    uint32_t rewrite[kNumVariants];    // 1: the interpreter runs the rewritten program (mrt_sig.h lin_rewrite_fast)
    // the path-exact build's retrace kernel for the tolerance variants that hand rounding-critical
    // paths over (mrt_shade.h light_critical): launched over PathParams::rt after each path kernel
    path_kernel_t retrace[kNumVariants];
};
const KernelTable& kernel_table_exact();
const KernelTable& kernel_table_fast();
// Tolerance-contract variants built with f32 denormals flushed to zero (a third build of the path
// kernels, mrt_kernels_fastz.o; DESIGN.md "Numerics contracts"): the denormal-safe reciprocal /
// sqrt sequences become single instructions.  Measured per variant (tools/ab.sh, kernel time):
// Cornell (C2) -1.0%, room + mesh -0.3..-0.4%, sky-lit bvh_node scenes -0.4%; book2 (volumes) +0.9%,
// so the variants with volumes keep the plain fast build.
#ifndef MRT_FAST_FTZ
#define MRT_FAST_FTZ 1
#endif
// Tolerance-contract variants that run the exact arithmetic with the forward fold (a fourth build,
// mrt_kernels_pex.o / mrt_path_kernel_pex<F>): scenes with volumes, and the room + mesh scenes with
// metal.  In them ANY change of rounding sends paths elsewhere -- book2 diverges on 2.9% of its
// paths under the fast arithmetic, and no single switch of it is the cause (each one reverted
// alone leaves 2.3-2.9%), the bunny on 0.015% -- and the diverged paths carry their scenes'
// fireflies (fog scattering next to the light; the light's caustics through the metal bunny): at
// the configs' own spp the fast arithmetic misses the per-pixel bar (C4 2.3e-3, one pixel 90% of
// it; C5 1.6e-3) where the exact arithmetic holds it (2.0e-5, 9.2e-6).  DESIGN.md section 2.
#ifndef MRT_PATH_EXACT
#define MRT_PATH_EXACT 1
#endif
#ifndef MRT_PEX_ALL_MESH
#define MRT_PEX_ALL_MESH 0  // A/B hook: every room + mesh variant path-exact (the teapot, C3, too)
#endif
template <uint32_t F>
static constexpr bool kPathExact =
    MRT_PATH_EXACT && ((F & FT_VOLUME) != 0 || (MRT_SIG_OF(F) == SIG_ROOM_MESH && ((F & FT_METAL) != 0 || MRT_PEX_ALL_MESH)));
template <uint32_t F>
static constexpr bool kFtzVariant = MRT_FAST_FTZ && (F & FT_VOLUME) == 0 && !kPathExact<F>;
// the FTZ build's table: a kernel for the kFtzVariant variants, null for the others
const KernelTable& kernel_table_fast_ftz();
// the path-exact build's table: a kernel for the kPathExact variants, null for the others
const KernelTable& kernel_table_fast_pex();

}  // namespace mrtd
