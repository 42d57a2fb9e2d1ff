// mrt_render.hip -- the MI355X render path behind the C-ABI (include/mrt.h).
//
// Kernels (DESIGN.md "Kernels"):
//   mrt_path_kernel   persistent waves pull 256-path batches (64 near the end of a launch) from per-XCD partition counters (one atomic
//                     per wave per batch, like work_queue::getWork pulls a tile,
//                     work_queue.cpp:158-166) and run trace() for each lane's path to completion;
//                     per-path radiance is written sample-major [s][local pixel] (coalesced).
//   mrt_fold_kernel   per pixel, folds the chunk's samples in sample order into the running
//                     accumulator with draw() (mode 0, main.cpp:161-167) or draw2() (mode 1,
//                     main.cpp:212-229) semantics -- bit-for-bit the reference's sequential sum.
//   mrt_final_kernel  mode 0: color /= ns, luminance clamp (main.cpp:168-173); writes the float4
//                     output in local-pixel order.
#include <hip/hip_runtime.h>
#include <atomic>
#include <mutex>
#include <thread>

#include <algorithm>
#include <functional>
#include <cstdio>
#include <cstring>
#include <string>
#include <vector>
#include <unistd.h>

#include "mrt_internal.h"
#include "mrt_launch.h"
#include "mrt_tables.h"
#include "mrt_cpu.h"
#include "../../include/mrt_tonemap.h"

using namespace mrtd;

#define HIPCHK(x)                                                                                   \
    do {                                                                                            \
        hipError_t e_ = (x);                                                                        \
        if (e_ != hipSuccess) return mrt_internal_fail(MRT_ERR_HIP, (std::string(#x) + ": " + hipGetErrorString(e_)).c_str()); \
    } while (0)

// The tolerance contract's kernels: the plain fast build, with the kFtzVariant variants taken
// from the denormal-flushing build (mrt_launch.h); MRT_FTZ=0 in the environment keeps the plain
// build for every variant (A/B).
// the tolerance contract's kernels: per variant the path-exact build (kPathExact), else the
// denormal-flushing build (kFtzVariant), else the plain fast build -- the variant's whole column
// (a build's workgroup shape, LDS fold levels and walk flags follow its own switches)
static void take_variant(KernelTable& m, const KernelTable& s, uint32_t i) {
    m.kernel[i] = s.kernel[i];
    m.lev_k[i] = s.lev_k[i];
    m.wg[i] = s.wg[i];
    m.tree[i] = s.tree[i];
    m.pq[i] = s.pq[i];
    m.box6_walk[i] = s.box6_walk[i];
    m.rewrite[i] = s.rewrite[i];
}
static const KernelTable& fast_table() {
    static const KernelTable t = [] {
        KernelTable m = kernel_table_fast();
        auto off = [](const char* name) {  // A/B hooks: MRT_FTZ=0, MRT_PATH_EXACT=0
            const char* e = getenv(name);
            return e && *e && atoi(e) == 0;
        };
        const KernelTable& z = kernel_table_fast_ftz();
        const KernelTable& x = kernel_table_fast_pex();
        for (uint32_t i = 0; i < kNumVariants; i++) {
            if (x.kernel[i] && !off("MRT_PATH_EXACT")) take_variant(m, x, i);
            else if (z.kernel[i] && !off("MRT_FTZ")) take_variant(m, z, i);
            // the exact arithmetic for the rounding-critical paths of the fast variants (mrt_retrace_kernel)
            m.retrace[i] = x.retrace[i];
        }
        return m;
    }();
    return t;
}

// first variant covering the scene's features: its own program shape first, then the interpreter
static uint32_t pick_variant(uint32_t features) {
    const uint32_t feat = features & 0xFFFFu, sig = MRT_SIG_OF(features);
    for (int pass = 0; pass < 2; pass++)
        for (uint32_t i = 0; i < kNumVariants; i++) {
            const uint32_t vf = kVariants[i] & 0xFFFFu, vs = MRT_SIG_OF(kVariants[i]);
            if ((feat & ~vf) != 0 || (vf & FT_LIN) != (feat & FT_LIN)) continue;
            if (pass == 0 ? (vs == sig && sig != SIG_NONE) : vs == SIG_NONE) return i;
        }
    return kNumVariants - 1;
}

// The sum is sequential per pixel (bit-exact order), so the kernel is load-latency bound when
// few pixels are local (multi-GPU shards): samples are fetched FOLD_DEPTH at a time (coalesced
// across the wave's pixels) before the dependent adds.
#ifndef FOLD_DEPTH
#define FOLD_DEPTH 16
#endif
// The render's last chunk (out != null) also finishes the pixels -- final_pixel into the caller's
// output -- and resets the counters (FoldEnd), so no separate final kernel follows it.
struct FoldEnd {
    float4* out;                     // the render's output (last chunk), or null: keep folding into acc
    uint32_t ns;                     // samples per pixel (mode 0 divides by it)
    unsigned long long* counters;    // work counters of the render's launches (MRT_COUNTER_STRIDE apart)
    unsigned long long* hprog;       // their progress snapshots in host memory (or null)
    uint32_t nreset;                 // counter slots to reset (MRT_CNT_SLOTS per launch)
    uint32_t nprog;                  // progress snapshots to reset (MRT_NPART per launch)
};
// what the render's path kernels consumed, reset for the context's next render in stream order
// after them: the counter slots (word (k * MRT_CNT_SLOTS + slot) * MRT_COUNTER_STRIDE) and the
// progress snapshots -- instead of clearing fills enqueued before each render (a blit kernel
// needs a free wave slot, which the other pipelined contexts' persistent path kernels hold)
MRT_DFN void reset_counters(const FoldEnd& e, uint32_t i) {
    if (i < e.nreset) e.counters[(size_t)i * MRT_COUNTER_STRIDE] = 0ull;
    if (i < e.nprog && e.hprog) __hip_atomic_store(e.hprog + i, 0ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}
__global__ void __launch_bounds__(256) mrt_fold_kernel(const float* __restrict__ rad, float4* __restrict__ acc, uint32_t npix, uint32_t s0,
                                                      uint32_t s1, uint32_t mode, float max_lum, FoldEnd fe) {
    uint32_t lp = blockIdx.x * blockDim.x + threadIdx.x;
    reset_counters(fe, lp);
    if (lp >= npix) return;
    // a render's first chunk starts from +0 without reading acc (no per-render clearing fill:
    // folding +0 first gives the same bits as starting from a zeroed accumulator)
    f3 c{0.0f, 0.0f, 0.0f};
    if (s0 != 0) {
        const float4 a = acc[lp];
        c = f3{a.x, a.y, a.z};
    }
    const float* q = rad + (size_t)lp * 3;
    const size_t stride = (size_t)npix * 3;
    uint32_t s = s0;
    for (; s + FOLD_DEPTH <= s1; s += FOLD_DEPTH) {
        f3 v[FOLD_DEPTH];
#pragma unroll
        for (int k = 0; k < FOLD_DEPTH; k++) {
            const float* e = q + (size_t)(s - s0 + k) * stride;
            v[k] = f3{__builtin_nontemporal_load(e), __builtin_nontemporal_load(e + 1), __builtin_nontemporal_load(e + 2)};
        }
#pragma unroll
        for (int k = 0; k < FOLD_DEPTH; k++) c = fold_sample(c, v[k], s + k, mode, max_lum);
    }
    for (; s < s1; s++) {
        const float* e = q + (size_t)(s - s0) * stride;
        c = fold_sample(c, f3{e[0], e[1], e[2]}, s, mode, max_lum);
    }
    if (fe.out) {
        c = final_pixel(c, fe.ns, mode, max_lum);
        fe.out[lp] = make_float4(c.x, c.y, c.z, 0.0f);
    } else {
        acc[lp] = make_float4(c.x, c.y, c.z, 0.0f);
    }
}

// The fold of an MRT_RF_FOLD_ASYNC launch, on the context's own stream beside the next launch's
// path kernel: one 256-thread group per CU (one wave slot per SIMD while it runs), each lane folding
// pixels grid-strided with FOLD_ASYNC_DEPTH samples in flight -- the same operations in the same
// order as mrt_fold_kernel (bit-identical): from +0 or the accumulator, into the accumulator or,
// for the render's last launch, finished into the output with the counters reset.
#ifndef MRT_FOLD_ASYNC_GROUPS
#define MRT_FOLD_ASYNC_GROUPS 1  // 256-thread groups per CU: one wave per SIMD
#endif
#ifndef FOLD_ASYNC_DEPTH
#define FOLD_ASYNC_DEPTH 8
#endif
#ifndef MRT_FOLD_ASYNC_WG
#define MRT_FOLD_ASYNC_WG 256  // threads per group
#endif
#ifndef MRT_FOLD_ASYNC_WPE
#define MRT_FOLD_ASYNC_WPE 8  // (register cap 64: FOLD_ASYNC_DEPTH 8 takes 46)
#endif
__global__ void __launch_bounds__(MRT_FOLD_ASYNC_WG) __attribute__((amdgpu_waves_per_eu(MRT_FOLD_ASYNC_WPE)))
mrt_fold_async_kernel(const float* __restrict__ rad, float4* __restrict__ acc, uint32_t npix, uint32_t s0, uint32_t s1, uint32_t mode,
                      float max_lum, FoldEnd fe) {
    const uint32_t step = gridDim.x * blockDim.x;
    const uint32_t nthr = max(npix, fe.nreset);
    for (uint32_t lp = blockIdx.x * blockDim.x + threadIdx.x; lp < nthr; lp += step) {
        reset_counters(fe, lp);
        if (lp >= npix) continue;
        f3 c{0.0f, 0.0f, 0.0f};
        if (s0 != 0) {
            const float4 a = acc[lp];
            c = f3{a.x, a.y, a.z};
        }
        const float* q = rad + (size_t)lp * 3;
        const size_t stride = (size_t)npix * 3;
        uint32_t s = s0;
        for (; s + FOLD_ASYNC_DEPTH <= s1; s += FOLD_ASYNC_DEPTH) {
            f3 v[FOLD_ASYNC_DEPTH];
#pragma unroll
            for (int k = 0; k < FOLD_ASYNC_DEPTH; k++) {
                const float* e = q + (size_t)(s - s0 + k) * stride;
                v[k] = f3{__builtin_nontemporal_load(e), __builtin_nontemporal_load(e + 1), __builtin_nontemporal_load(e + 2)};
            }
#pragma unroll
            for (int k = 0; k < FOLD_ASYNC_DEPTH; k++) c = fold_sample(c, v[k], s + k, mode, max_lum);
        }
        for (; s < s1; s++) {
            const float* e = q + (size_t)(s - s0) * stride;
            c = fold_sample(c, f3{e[0], e[1], e[2]}, s, mode, max_lum);
        }
        if (fe.out) {
            c = final_pixel(c, fe.ns, mode, max_lum);
            fe.out[lp] = make_float4(c.x, c.y, c.z, 0.0f);
        } else {
            acc[lp] = make_float4(c.x, c.y, c.z, 0.0f);
        }
    }
}

// draw()'s fold (mode 0) in 8 VGPRs: the persistent path kernel fills 7 waves per SIMD with 72
// VGPRs each (504 of 512), so only a kernel this lean fits the 8th wave slot beside it -- the fold
// of one render then runs under the next render's path kernel (bench.py --pipeline, two contexts
// on two streams) instead of after it.  Buffer loads (a scalar resource + one 32-bit VGPR offset;
// a launch chunk's radiance is < 4 GiB, mrt_prepare) keep it at 8 VGPRs: the offset, the acc
// offset, c and one sample, so one 12-B load is in flight per lane.  (Staging rows in LDS with
// buffer loads to LDS was tried: the compiler then reserves 97 VGPRs for the kernel.)  The same
// operations in the same order as mrt_fold_kernel (bit-identical).
#ifndef MRT_FOLD_LEAN_WG
#define MRT_FOLD_LEAN_WG 64  // one-wave groups take any single free wave slot (C2 step 8.44 -> 8.38 ms vs 256)
#endif
__global__ void __launch_bounds__(MRT_FOLD_LEAN_WG) __attribute__((amdgpu_num_vgpr(8)))
mrt_fold_lean_kernel(const float* __restrict__ rad, float4* __restrict__ acc, uint32_t npix, uint32_t n, uint32_t first) {
    const uint32_t lp = blockIdx.x * blockDim.x + threadIdx.x;
    if (lp >= npix) return;
    const __amdgpu_buffer_rsrc_t rr = __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(rad), 0, 0xFFFFFFFFu, 0x00020000);
    const __amdgpu_buffer_rsrc_t ra = __builtin_amdgcn_make_buffer_rsrc(acc, 0, 0xFFFFFFFFu, 0x00020000);
    f3 c{0.0f, 0.0f, 0.0f};  // the render's first chunk: from +0 (as mrt_fold_kernel)
    if (!first) {
        const auto a = __builtin_amdgcn_raw_buffer_load_b96(ra, lp * 16u, 0, 0);
        c = f3{__uint_as_float(a[0]), __uint_as_float(a[1]), __uint_as_float(a[2])};
    }
    const uint32_t stride = npix * 12u;
    uint32_t off = lp * 12u;
    for (uint32_t s = 0; s < n; s++, off += stride) {
        const auto v = __builtin_amdgcn_raw_buffer_load_b96(rr, off, 0, 2 /* nt */);
        c = fold_sample(c, f3{__uint_as_float(v[0]), __uint_as_float(v[1]), __uint_as_float(v[2])}, s, 0u, 0.0f);
    }
    using u3 = decltype(__builtin_amdgcn_raw_buffer_load_b96(ra, 0u, 0, 0));
    const u3 o = {__float_as_uint(c.x), __float_as_uint(c.y), __float_as_uint(c.z)};
    __builtin_amdgcn_raw_buffer_store_b96(o, ra, lp * 16u, 0, 0);
}

// Also resets what the render's path kernels consumed, for the context's next render, in stream
// order after them: the counter slots of its launches (word (k * MRT_CNT_SLOTS + slot) *
// MRT_COUNTER_STRIDE) and their progress snapshots in host memory -- instead of clearing fills
// enqueued before each render (a blit kernel needs a free wave slot, which the persistent path
// kernels of the other pipelined contexts hold: up to 49 ms waits in the bench trace).
// Lean like mrt_fold_lean_kernel (one-wave groups, 8 VGPRs): a 256-thread group of a 13-VGPR
// kernel needs a wave slot on every SIMD, which the other pipelined contexts' persistent path
// kernels (7 waves x 72 VGPRs per SIMD) do not leave free -- the final of one render then waited
// for another render's path kernel to end, and the next render on its stream with it (the
// bench's 3-context timeline, DESIGN.md "Pipelined renders").  Same operations, same bits.
#ifndef MRT_FINAL_WG
#define MRT_FINAL_WG 64
#endif
__global__ void __launch_bounds__(MRT_FINAL_WG) __attribute__((amdgpu_num_vgpr(8)))
mrt_final_kernel(const float4* __restrict__ acc, float4* __restrict__ out, uint32_t npix, uint32_t ns, uint32_t mode, float max_lum,
                 unsigned long long* __restrict__ counters, unsigned long long* hprog, uint32_t nreset, uint32_t nprog) {
    const uint32_t lp = blockIdx.x * blockDim.x + threadIdx.x;
    if (lp < nreset) counters[(size_t)lp * MRT_COUNTER_STRIDE] = 0ull;
    if (lp < nprog && hprog) __hip_atomic_store(hprog + lp, 0ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    if (lp >= npix) return;
    const __amdgpu_buffer_rsrc_t ra = __builtin_amdgcn_make_buffer_rsrc(const_cast<float4*>(acc), 0, 0xFFFFFFFFu, 0x00020000);
    const __amdgpu_buffer_rsrc_t ro = __builtin_amdgcn_make_buffer_rsrc(out, 0, 0xFFFFFFFFu, 0x00020000);
    const auto a = __builtin_amdgcn_raw_buffer_load_b96(ra, lp * 16u, 0, 0);
    const f3 c = final_pixel(f3{__uint_as_float(a[0]), __uint_as_float(a[1]), __uint_as_float(a[2])}, ns, mode, max_lum);
    using u4 = decltype(__builtin_amdgcn_raw_buffer_load_b128(ra, 0u, 0, 0));
    const u4 o = {__float_as_uint(c.x), __float_as_uint(c.y), __float_as_uint(c.z), 0u};
    __builtin_amdgcn_raw_buffer_store_b128(o, ro, lp * 16u, 0, 0);
}

// Image output on the device (main.cpp:416-444): global max luminance, then per-pixel Drago +
// ARGB32 -- the functions of include/mrt_tonemap.h, the same bits as the host mrt_tonemap_argb.
__global__ void __launch_bounds__(256) mrt_lum_max_kernel(const float4* __restrict__ rgb, uint32_t n, unsigned int* __restrict__ lwmax_bits) {
    float m = 0.0f;
    for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) {
        const float4 c = rgb[i];
        const float cc[3] = {c.x, c.y, c.z};
        const float l = mrt_luminance(cc);
        m = (m < l) ? l : m;  // std::max(L_wmax, lum): NaN and negative luminance never win
    }
    for (int off = 32; off > 0; off >>= 1) {
        const float o = __shfl_xor(m, off);
        m = (m < o) ? o : m;
    }
    if ((threadIdx.x & 63) == 0) atomicMax(lwmax_bits, __float_as_uint(m));  // m >= +0: bit order == value order
}
__global__ void __launch_bounds__(256) mrt_tonemap_kernel(const float4* __restrict__ rgb, uint32_t n, const float* __restrict__ lwmax,
                                                         uint32_t* __restrict__ argb) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    mrt_tonemap_params tp;
    mrt_tonemap_setup(*lwmax, &tp);
    const float4 c = rgb[i];
    const float cc[3] = {c.x, c.y, c.z};
    argb[i] = mrt_tonemap_pixel(&tp, cc);
}

extern "C" mrt_status mrt_lum_max_device(const float* d_rgb, uint32_t n, float* d_lwmax, void* stream) {
    if (!d_rgb || !d_lwmax) return mrt_internal_fail(MRT_ERR_INVALID, "mrt_lum_max_device: null");
    if (n == 0) return MRT_OK;
    const uint32_t blocks = std::min<uint32_t>((n + 255) / 256, 2048);
    hipLaunchKernelGGL(mrt_lum_max_kernel, dim3(blocks), dim3(256), 0, (hipStream_t)stream, (const float4*)d_rgb, n, (unsigned int*)d_lwmax);
    HIPCHK(hipGetLastError());
    return MRT_OK;
}
extern "C" mrt_status mrt_tonemap_device(const float* d_rgb, uint32_t n, const float* d_lwmax, uint32_t* d_argb, void* stream) {
    if (!d_rgb || !d_lwmax || !d_argb) return mrt_internal_fail(MRT_ERR_INVALID, "mrt_tonemap_device: null");
    if (n == 0) return MRT_OK;
    hipLaunchKernelGGL(mrt_tonemap_kernel, dim3((n + 255) / 256), dim3(256), 0, (hipStream_t)stream, (const float4*)d_rgb, n, d_lwmax, d_argb);
    HIPCHK(hipGetLastError());
    return MRT_OK;
}

// --------------------------------------------------------------------------------------------
// host side
// --------------------------------------------------------------------------------------------
// one numerics build of the scene's path kernel (exact / fast): kernel, grid, registers
struct PathLaunch {
    path_kernel_t fn = nullptr;
    int grid = 0;
    size_t lds_bytes = 0;
    uint32_t vgprs = 0;
    uint32_t wg = 64;     // threads per workgroup
    uint32_t tree_n = 0;  // BvhWide nodes kept in each workgroup's LDS (treelet kernels)
    uint32_t lds_save = 0;  // LDS words per lane slot for the query ray parked during instances
    uint32_t lds_mesh = 0;  // LDS words per lane of the mesh walk's stack
    bool rewrite = false;   // the kernel runs the tolerance-contract program rewrite (s->prog_fast)
    path_kernel_t retrace = nullptr;  // the exact arithmetic for its rounding-critical paths (mrt_retrace_kernel)
    size_t retrace_lds = 0;
    bool handover = false;  // the kernel hands its rounding-critical paths to it (fast arithmetic)
    uint32_t walk_min = 32;  // resumable mesh walk threshold of this build (PathParams::walk_min)
};

// Wide nodes renumbered breadth-first over all roots together (level 0 of every tree, then level
// 1, ...), so the first K nodes of the array are the top levels of the scene's BVHs -- what a
// treelet of K nodes holds.  Only the labels change: every walk visits the same nodes.
// limit: only the first `limit` nodes breadth-first, the others after them in their own order
// (pod_bvh's depth-first layout keeps a subtree's nodes together in the cache).
template <typename W>
static void bfs_order(std::vector<W>& wide, std::vector<uint32_t*> roots, uint32_t leaf_bit, uint32_t limit = 0xFFFFFFFFu) {
    const uint32_t n = (uint32_t)wide.size();
    std::vector<uint32_t> nid(n, MRT_NONE), order;
    order.reserve(n);
    for (uint32_t* r : roots)
        if (!(*r & leaf_bit) && *r < n && nid[*r] == MRT_NONE && order.size() < limit) { nid[*r] = (uint32_t)order.size(); order.push_back(*r); }
    for (size_t q = 0; q < order.size() && order.size() < limit; q++) {
        const W& w = wide[order[q]];
        for (uint32_t c : {w.lref, w.rref})
            if (!(c & leaf_bit) && c < n && nid[c] == MRT_NONE && order.size() < limit) { nid[c] = (uint32_t)order.size(); order.push_back(c); }
    }
    for (uint32_t i = 0; i < n; i++)  // the rest (and unreachable nodes) in their own order
        if (nid[i] == MRT_NONE) { nid[i] = (uint32_t)order.size(); order.push_back(i); }
    auto remap = [&](uint32_t c) { return (c & leaf_bit) || c >= n ? c : nid[c]; };
    std::vector<W> out(n);
    for (uint32_t k = 0; k < n; k++) {
        out[k] = wide[order[k]];
        out[k].lref = remap(out[k].lref);
        out[k].rref = remap(out[k].rref);
    }
    wide.swap(out);
    for (uint32_t* r : roots) *r = remap(*r);
}

struct mrt_scene {
    int device = 0;
    mrt_cpu_scene* cpu = nullptr;  // MRT_DEVICE_CPU: the CPU backend's scene (mrt_cpu.hip); nothing below is used
    DScene S{};
    DScene* d_S = nullptr;
    std::vector<void*> allocs;
    uint32_t n_nodes = 0;
    // workspace
    mrt_render_desc wdesc{};
    std::vector<uint32_t> wpixels;   // the pixel list of wdesc (mrt_render_desc.pixels), copied
    const LinOp* prog_fast = nullptr;  // the tolerance contract's program for the interpreter (lin_rewrite_fast)
    bool have_ws = false;
    uint32_t npix = 0, chunk = 0;
    uint2* d_pixels = nullptr;
    float2* d_sdist = nullptr;
    uint32_t sdist_sq = 0;
    float* d_rad = nullptr;
    uint32_t* d_path_rays = nullptr;
    float4* d_acc = nullptr;
    float4* d_lev = nullptr;
    float4* d_out = nullptr;         // mrt_render's device framebuffer (local-pixel order)
    // progressive preview (MRT_RF_PREVIEW): device staging image, pinned host copy guarded by a
    // sequence word the render's stream writes around each copy (odd = copy in flight) and the
    // sample count the copy holds
    float4* d_prev = nullptr;
    size_t prev_cap = 0;
    float4* h_prev = nullptr;
    size_t h_prev_cap = 0;
    uint32_t* h_seq = nullptr;       // [0] sequence, [1] samples folded into h_prev
    uint32_t prev_epoch = 0;
    std::vector<uint32_t> prev_px;   // local pixel -> row-major pixel of the previewed render
    uint32_t prev_w = 0, prev_h = 0;
    uint32_t lev_rows = 0;
    uint64_t* d_counter = nullptr;   // 64 B scratch: [0] paths handed to the exact arithmetic since upload, [2] ray total of mrt_render, [4] cancel flag,
                                     // [1] rounding-critical paths listed (u32), [3] retrace groups done (u32), [5] listed beyond the cap since upload,
                                     // [6] the parity-1 list's count (u32) and retrace groups done (u32)
    uint32_t* d_rt = nullptr;        // rounding-critical paths listed for the retrace kernel (path indices)
    size_t rt_cap = 0;
    uint64_t* d_counters = nullptr;  // one work counter per chunk launch (progress reads them)
    size_t cnt_cap = 0;
    std::vector<uint64_t> chunk_paths;
    hipStream_t pstream = nullptr;   // non-blocking stream for the cancel-flag copy
    // host-coherent pinned memory: per-launch snapshots of the work counters, stored by the path
    // kernel itself (mrt_progress reads them with no GPU work), and the cancel flag's source
    uint64_t* h_prog = nullptr;
    size_t h_prog_cap = 0;
    std::vector<uint64_t> h_seen;  // largest snapshot read per launch (waves store out of order)
    int* h_one = nullptr;
    std::atomic<uint32_t> n_chunks{0};  // launches of the current render (0 until all are enqueued)
    // mrt_progress may run on another host thread: it and every change to the launch bookkeeping
    // above (h_prog, h_seen, ev, chunk_paths) hold this lock
    std::mutex prog_mu;
    // recorded at the end of every mrt_render_device on the caller's stream: workspace changes
    // (relayout uploads, reallocation) wait for it, so a render still running on another stream
    // never sees its buffers rewritten or freed
    hipEvent_t ev_done = nullptr;
    bool ev_done_pending = false;
    // MRT_RF_FOLD_ASYNC: launches alternate between two radiance buffers (parity lpar), renders
    // between two sets of counter slots (rpar); the fold of parity p runs on fstream and ev_fold[p]
    // marks its end, which the next path kernel writing parity p's radiance buffer waits for (folds
    // run in order on fstream, so it also orders every earlier fold)
    hipStream_t fstream = nullptr;
    hipEvent_t ev_kern = nullptr;
    hipEvent_t ev_fold[2] = {nullptr, nullptr};
    bool fold_pending[2] = {false, false};
    uint32_t lpar = 0, rpar = 0;
    float* d_rad2 = nullptr;
    size_t rad2_cap = 0;
    uint32_t n_cu = 0;
    uint32_t prog_base = 0;  // launch slot of the current render's counters and progress snapshots
    uint32_t slot_half = 0;  // launch slots per set (renders use set rpar at rpar * slot_half; mrt_prepare)
    unsigned long long* d_rays = nullptr;
    uint32_t features = 0, variant = 0;
    uint32_t lds_frames = 0, lds_rays = 0, lds_mesh = 0, lds_save = 0;
    uint32_t walk_min = 32;  // resumable mesh walk threshold (PathParams::walk_min)
    PathLaunch pl[2];            // [0] exact contract, [1] tolerance contract (MRT_RF_FAST)
    size_t max_threads = 0;  // largest path-kernel grid in threads (per-lane level rows)
    std::vector<hipEvent_t> ev;  // [2*k]: start/stop of path-kernel launch k of the last render
    uint32_t n_launch = 0;
    size_t rad_cap = 0, acc_cap = 0, lev_cap = 0, px_cap = 0, pr_cap = 0, sd_cap = 0, out_cap = 0;
    uint64_t last_paths = 0;
    uint32_t last_numerics = 0;
    uint32_t prog_ops = 0;  // linear hit program length (0: generic machine)
};

static mrt_status dev_alloc(mrt_scene* s, void** p, size_t bytes) {
    if (bytes == 0) bytes = 16;
    hipError_t e = hipMalloc(p, bytes);
    if (e != hipSuccess) return mrt_internal_fail(e == hipErrorOutOfMemory ? MRT_ERR_OOM : MRT_ERR_HIP, "hipMalloc failed");
    s->allocs.push_back(*p);
    return MRT_OK;
}
static mrt_status upload(mrt_scene* s, const void* src, size_t bytes, void** dst) {
    void* p = nullptr;
    mrt_status st = dev_alloc(s, &p, bytes);
    if (st) return st;
    if (bytes) {
        hipError_t e = hipMemcpy(p, src, bytes, hipMemcpyHostToDevice);
        if (e != hipSuccess) return mrt_internal_fail(MRT_ERR_HIP, "hipMemcpy upload failed");
    }
    *dst = p;
    return MRT_OK;
}

extern "C" mrt_status mrt_init(int* device_count) {
    int n = 0;
    hipError_t e = hipGetDeviceCount(&n);
    if (e != hipSuccess || n == 0) {
        if (device_count) *device_count = 0;
        return mrt_internal_fail(MRT_ERR_NO_DEVICE, "no HIP device visible");
    }
    hipDeviceProp_t prop;
    HIPCHK(hipGetDeviceProperties(&prop, 0));
    if (strncmp(prop.gcnArchName, "gfx950", 6) != 0)
        return mrt_internal_fail(MRT_ERR_NO_DEVICE, (std::string("device is ") + prop.gcnArchName + ", libmrt is built for gfx950").c_str());
    if (device_count) *device_count = n;
    return MRT_OK;
}

// graph checks on the host: every device stack is sized from them, so none can overflow
static bool needs_uv_tex(const mrt_scene_view* v, uint32_t t, int guard = 0) {
    if (t == MRT_NONE || t >= v->n_textures || guard > 16) return false;
    const mrt_texture& T = v->textures[t];
    if (T.kind == MRT_T_IMAGE) return true;
    if (T.kind == MRT_T_CHECKER) return needs_uv_tex(v, T.a, guard + 1) || needs_uv_tex(v, T.b, guard + 1);
    return false;
}
struct GraphCheck {
    const std::vector<mrt_node>& nodes;
    const mrt_scene_view* v;
    int max_frames = 0, max_rays = 0, max_mesh = 0;
    int bvhw_depth = 0;  // deepest wide-node stack of the converted bvh_node subtrees
    bool ok = true;
    std::string why;
    int mesh_depth(uint32_t ni, int guard) {
        if (guard > 1000 || ni >= v->n_mesh_nodes) return 100000;
        const mrt_mesh_node& m = v->mesh_nodes[ni];
        if (m.count_order & 0xFFFFFFu) return 1;
        return 1 + std::max(mesh_depth(m.left_or_first, guard + 1), mesh_depth(m.left_or_first + 1, guard + 1));
    }
    void walk(uint32_t id, int frames, int rays, bool in_volume, int guard) {
        if (!ok) return;
        if (id >= nodes.size() || guard > 4096) { ok = false; why = "bad node index / cyclic scene graph"; return; }
        const mrt_node& n = nodes[id];
        uint32_t k = n.kind & 0xFF;
        if (k == MRT_K_SPHERE || k == MRT_K_XY || k == MRT_K_XZ || k == MRT_K_YZ) return;
        if (k == MRT_K_MESH) {
            max_mesh = std::max(max_mesh, mesh_depth(n.a, 0));
            return;
        }
        if (k == MRT_K_BVHW) {
            max_mesh = std::max(max_mesh, bvhw_depth);
            return;
        }
        frames++;
        max_frames = std::max(max_frames, frames);
        switch (k) {
        case MRT_K_LIST:
            for (uint32_t i = 0; i < n.b; i++) walk(v->children[n.a + i], frames, rays, in_volume, guard + 1);
            break;
        case MRT_K_BVH:
            walk(n.a, frames, rays, in_volume, guard + 1);
            walk(n.b, frames, rays, in_volume, guard + 1);
            break;
        case MRT_K_TRANSLATE: case MRT_K_ROTY: case MRT_K_TRROTY:
            max_rays = std::max(max_rays, rays + 1);
            walk(n.a, frames, rays + 1, in_volume, guard + 1);
            break;
        case MRT_K_VOLUME:
            if (in_volume) { ok = false; why = "nested constant_volume"; return; }
            walk(n.a, frames, rays, true, guard + 1);
            break;
        default: ok = false; why = "unknown node kind";
        }
    }
};

// Linear hit program (mrt_lin.h): object_list trees of primitives / meshes with at most one
// instance level.  Returns false (generic kernel) for bvh_node, constant_volume, nested instances.
struct LinCompiler {
    const std::vector<mrt_node>& nodes;
    const mrt_scene_view* v;
    std::vector<LinOp> prog;
    int max_lvl = 0;
    uint32_t inst_pc = MRT_NONE;  // op index of the enclosing instance while its subtree is emitted
    bool in_vsub = false;         // emitting a volume's boundary sub-program (primitives, lists, one instance level)
    bool vsub = false;            // the program has such a volume (FT_VSUB)
    // code = op | kind << 8 | flags << 16 | nesting level << 24 (the level the op is tested at)
    LinOp op_of(uint32_t code, uint32_t id, int lvl) {
        const mrt_node& n = nodes[id];
        LinOp o{};
        o.code = code | ((n.kind & 0xFFu) << 8) | (n.kind & 0xFF0000u) | ((uint32_t)lvl << 24);
        o.node = id;
        o.skip = 0;
        o.mat = n.mat;
        for (int i = 0; i < 12; i++) o.f[i] = n.f[i];
        return o;
    }
    // primitive-like ops (prim, mesh, bvh subtree, volume) also carry the enclosing instance's op
    // index in f[11] (which they do not use) for the resumable interpreter
    LinOp leaf_op(uint32_t code, uint32_t id, int lvl) {
        LinOp o = op_of(code, id, lvl);
        memcpy(&o.f[11], &inst_pc, 4);
        return o;
    }
    bool emit(uint32_t id, int inst_depth, int lvl, int guard) {
        if (id >= nodes.size() || guard > 256 || lvl > 30) return false;
        const mrt_node& n = nodes[id];
        const uint32_t k = n.kind & 0xFFu;
        max_lvl = std::max(max_lvl, lvl);
        switch (k) {
        case MRT_K_SPHERE: case MRT_K_XY: case MRT_K_XZ: case MRT_K_YZ:
            prog.push_back(leaf_op(LOP_PRIM, id, lvl));
            return true;
        case MRT_K_MESH:
            if (in_vsub) return false;
            prog.push_back(leaf_op(LOP_MESH, id, lvl));
            return true;
        case MRT_K_BVHW: {
            if (in_vsub) return false;
            LinOp o = leaf_op(LOP_BVHW, id, lvl);
            o.skip = n.a;  // the subtree's root ref (the op's f[0..5] are its box)
            prog.push_back(o);
            return true;
        }
        case MRT_K_VOLUME: {
            if (n.a >= nodes.size() || in_vsub) return false;
            const uint32_t bk = nodes[n.a].kind & 0xFFu;
            if (bk == MRT_K_SPHERE || bk == MRT_K_XY || bk == MRT_K_XZ || bk == MRT_K_YZ) {  // a primitive boundary
                prog.push_back(leaf_op(LOP_VOLUME, id, lvl));
                prog.push_back(op_of(LOP_VBOUND, n.a, lvl));
                return true;
            }
            // any other boundary (box.h lists, instances of them: cornell_smoke, scene.cpp:364-369)
            // as a sub-program after the op, walked twice per query by the volume op (lin_sub_t) and
            // skipped by the main walk; outside instances only (its instance is then the only level)
            if (inst_depth > 0) return false;
            const size_t at = prog.size();
            LinOp vo = leaf_op(LOP_VOLUME, id, lvl);
            vo.code |= MRT_F_VSUB << 16;
            prog.push_back(vo);
            in_vsub = true;
            const bool ok = emit(n.a, inst_depth, 0, guard + 1);  // (levels of the sub-program from 0)
            in_vsub = false;
            if (!ok) return false;
            prog[at].skip = (uint32_t)prog.size();
            vsub = true;
            return true;
        }
        case MRT_K_LIST: {
            size_t at = prog.size();
            prog.push_back(op_of(LOP_LIST, id, lvl));
            for (uint32_t i = 0; i < n.b; i++)
                if (!emit(v->children[n.a + i], inst_depth, lvl + 1, guard + 1)) return false;
            prog[at].skip = (uint32_t)prog.size();
            prog.push_back(op_of(LOP_LIST_END, id, lvl));
            return true;
        }
        case MRT_K_TRANSLATE: case MRT_K_ROTY: case MRT_K_TRROTY: {
            if (inst_depth > 0) return false;
            size_t at = prog.size();
            prog.push_back(op_of(LOP_INST, id, lvl));
            const uint32_t outer_pc = inst_pc;
            if (!in_vsub) inst_pc = (uint32_t)at;
            const bool ok = emit(n.a, inst_depth + 1, lvl + 1, guard + 1);
            inst_pc = outer_pc;
            if (!ok) return false;
            prog[at].skip = (uint32_t)prog.size();
            LinOp e = op_of(LOP_INST_END, id, lvl);
            e.skip = (uint32_t)at;  // its instance op
            prog.push_back(e);
            return true;
        }
        default:
            return false;
        }
    }
};

static uint32_t scene_features(const mrt_scene_view* v, const std::vector<mrt_node>& nodes, const std::vector<uint8_t>& absorbed) {
    uint32_t f = 0;
    for (size_t i = 0; i < nodes.size(); i++) {
        const mrt_node& n = nodes[i];
        switch (n.kind & 0xFF) {
        case MRT_K_BVH: if (!absorbed[i]) f |= FT_BVH; break;
        case MRT_K_BVHW: f |= FT_BVHW; break;
        case MRT_K_MESH: f |= FT_MESH; break;
        case MRT_K_VOLUME: f |= FT_VOLUME; break;
        case MRT_K_TRANSLATE: case MRT_K_ROTY: case MRT_K_TRROTY: f |= FT_INST; break;
        case MRT_K_SPHERE: if ((n.kind >> 16) & MRT_F_MOVING) f |= FT_MOVING; break;
        }
        if ((n.kind >> 16) & MRT_F_NEEDUV) f |= FT_UV;
    }
    for (uint32_t i = 0; i < v->n_textures; i++)
        if (v->textures[i].kind != MRT_T_COLOR) f |= FT_TEX;
    for (uint32_t i = 0; i < v->n_materials; i++) {
        if (v->materials[i].kind == MRT_M_METAL) f |= FT_METAL;
        if (v->materials[i].kind == MRT_M_ISOTROPIC) f |= FT_ISO;
    }
    if (v->sky) f |= FT_SKY;
    if (v->biased != MRT_NONE) {
        f |= FT_BIASED;
        const mrt_node& b = nodes[v->biased];
        if ((b.kind & 0xFF) == MRT_K_SPHERE) f |= FT_BSPHERE;
        if ((b.kind & 0xFF) == MRT_K_LIST)
            for (uint32_t i = 0; i < b.b; i++)
                if ((nodes[v->children[b.a + i]].kind & 0xFF) == MRT_K_SPHERE) f |= FT_BSPHERE;
    }
    return f;
}

// The scene's device tables (mrt_tables.h), built on the host from the caller's view; both
// backends run on them: mrt_scene_upload copies them to HBM, mrt_cpu_scene_create keeps them.
mrt_status mrt_internal_scene_tables(const mrt_scene_view* v, SceneTables* T) {
    if (!v || !T || v->root >= v->n_nodes) return mrt_internal_fail(MRT_ERR_INVALID, "mrt_scene_upload: bad view");
    // device node table: NEEDUV flags; translate(rotate_y(x)) fused into one instance node
    std::vector<mrt_node> nodes(v->nodes, v->nodes + v->n_nodes);
    for (mrt_node& n : nodes) {
        uint32_t k = n.kind & 0xFF;
        if ((k == MRT_K_SPHERE || k == MRT_K_XY || k == MRT_K_XZ || k == MRT_K_YZ) && n.mat < v->n_materials &&
            needs_uv_tex(v, v->materials[n.mat].tex))
            n.kind |= MRT_F_NEEDUV << 16;
    }
    // rect planes outside {0} U [2^-77, 2^60] keep the IEEE division in rect tests (mrt_device.h ray_nice)
    for (mrt_node& n : nodes) {
        const uint32_t k = n.kind & 0xFF;
        if (k != MRT_K_XY && k != MRT_K_XZ && k != MRT_K_YZ) continue;
        const float c = std::fabs(n.f[4]);
        if (!(c == 0.0f || (c >= 0x1p-77f && c <= 0x1p60f))) n.kind |= MRT_F_SLOWDIV << 16;
    }
    // box.h:12-20 recognised: an object_list of exactly six outward-facing rects over one box
    // (xy at max z / min z, xz at max y / min y, yz at max x / min x, bounds spanning the box, one
    // material, no uv, no slow divisions).  Flag MRT_F_BOX6, planes in f[6..11] (min xyz, max xyz):
    // the tolerance contract tests such a list as one slab test (mrt_sig.h box6_hit).
    for (size_t i = 0; i < nodes.size(); i++) {
        mrt_node& n = nodes[i];
        if ((n.kind & 0xFF) != MRT_K_LIST || n.b != 6 || n.a + 6 > v->n_children) continue;
        const mrt_node* c[6];
        bool ok = true;
        for (int j = 0; j < 6 && ok; j++) {
            const uint32_t ci = v->children[n.a + j];
            ok = ci < nodes.size();
            if (ok) c[j] = &nodes[ci];
        }
        if (!ok) continue;
        static const uint32_t kinds[6] = {MRT_K_XY, MRT_K_XY, MRT_K_XZ, MRT_K_XZ, MRT_K_YZ, MRT_K_YZ};
        for (int j = 0; j < 6 && ok; j++)
            ok = (c[j]->kind & 0xFF) == kinds[j] && c[j]->f[5] == ((j & 1) ? -1.0f : 1.0f) && c[j]->mat == c[0]->mat &&
                 !((c[j]->kind >> 16) & (MRT_F_NEEDUV | MRT_F_SLOWDIV));
        if (!ok) continue;
        const float xmin = c[5]->f[4], xmax = c[4]->f[4], ymin = c[3]->f[4], ymax = c[2]->f[4], zmin = c[1]->f[4], zmax = c[0]->f[4];
        auto span = [&](const mrt_node* r, float a0, float a1, float b0, float b1) {
            return r->f[0] == a0 && r->f[1] == a1 && r->f[2] == b0 && r->f[3] == b1;
        };
        ok = xmin < xmax && ymin < ymax && zmin < zmax && span(c[0], xmin, xmax, ymin, ymax) && span(c[1], xmin, xmax, ymin, ymax) &&
             span(c[2], xmin, xmax, zmin, zmax) && span(c[3], xmin, xmax, zmin, zmax) && span(c[4], ymin, ymax, zmin, zmax) &&
             span(c[5], ymin, ymax, zmin, zmax);
        if (!ok) continue;
        n.kind |= MRT_F_BOX6 << 16;
        n.mat = c[0]->mat;  // (an object_list has no material of its own)
        n.f[6] = xmin; n.f[7] = ymin; n.f[8] = zmin;
        n.f[9] = xmax; n.f[10] = ymax; n.f[11] = zmax;
    }
    for (mrt_node& n : nodes) {
        if ((n.kind & 0xFF) != MRT_K_TRANSLATE || n.a >= nodes.size()) continue;
        const mrt_node& c = nodes[n.a];
        if ((c.kind & 0xFF) != MRT_K_ROTY) continue;
        mrt_node f{};
        f.kind = MRT_K_TRROTY | (c.kind & (MRT_F_HASBOX << 16));
        f.a = c.a;
        f.b = MRT_NONE;
        f.mat = MRT_NONE;
        for (int i = 0; i < 8; i++) f.f[i] = c.f[i];  // bbox, sin, cos
        f.f[8] = n.f[0]; f.f[9] = n.f[1]; f.f[10] = n.f[2];
        n = f;
    }
    // pod_bvh -> wide nodes (both child boxes inline); MESH nodes get b = root ref
    std::vector<MeshWide> wide;
    {
        std::vector<uint32_t> wide_of(v->n_mesh_nodes, MRT_NONE);
        for (uint32_t i = 0; i < v->n_mesh_nodes; i++)
            if ((v->mesh_nodes[i].count_order & 0xFFFFFFu) == 0) {
                wide_of[i] = (uint32_t)wide.size();
                wide.push_back(MeshWide{});
            }
        bool ok = wide.size() < MESH_LEAF;
        auto ref_of = [&](uint32_t i) -> uint32_t {
            if (i >= v->n_mesh_nodes) { ok = false; return 0; }
            const mrt_mesh_node& m = v->mesh_nodes[i];
            const uint32_t cnt = m.count_order & 0xFFFFFFu;
            if (cnt == 0) return wide_of[i];
            if (cnt > 0x7Fu || m.left_or_first > 0xFFFFFFu) ok = false;
            if ((MESH_LEAF | (cnt << 24) | m.left_or_first) >= kMeshEmpty) ok = false;  // (the walk's marks)
            return MESH_LEAF | (cnt << 24) | m.left_or_first;
        };
        for (uint32_t i = 0; i < v->n_mesh_nodes && ok; i++) {
            if (wide_of[i] == MRT_NONE) continue;
            const mrt_mesh_node& m = v->mesh_nodes[i];
            const uint32_t l = m.left_or_first;
            if (l + 1 >= v->n_mesh_nodes) { ok = false; break; }
            MeshWide& W = wide[wide_of[i]];
            const mrt_mesh_node &L = v->mesh_nodes[l], &R = v->mesh_nodes[l + 1];
            for (int k = 0; k < 3; k++) {
                W.lmin[k] = L.bmin[k]; W.lmax[k] = L.bmax[k];
                W.rmin[k] = R.bmin[k]; W.rmax[k] = R.bmax[k];
            }
            W.lref = ref_of(l);
            W.rref = ref_of(l + 1);
            W.order = m.count_order >> 24;
        }
        for (mrt_node& n : nodes)
            if ((n.kind & 0xFF) == MRT_K_MESH) n.b = ref_of(n.a);
        if (!ok) return mrt_internal_fail(MRT_ERR_INVALID, "mesh BVH outside the device encoding (leaf > 127 triangles or > 2^24 triangles)");
        // the top 63 nodes first, breadth-first: the hot top levels share cache lines
        std::vector<uint32_t*> mroots;
        for (mrt_node& n : nodes)
            if ((n.kind & 0xFF) == MRT_K_MESH) mroots.push_back(&n.b);
        bfs_order(wide, mroots, MESH_LEAF, 63u);
    }
    // bvh_node subtrees whose leaves are primitives / object_lists of primitives (and of boxes of
    // primitives) -> wide nodes; the subtree root becomes an MRT_K_BVHW node (a = root ref)
    std::vector<BvhWide> bwide;
    std::vector<mrt_node> bprims;  // leaf primitive runs of the wide subtrees
    int bvhw_depth = 0;
    std::vector<uint8_t> absorbed(nodes.size(), 0);  // bvh_nodes now inside a wide subtree
    {
        const size_t nn = nodes.size();
        auto kind_of = [&](uint32_t i) { return nodes[i].kind & 0xFFu; };
        auto is_leaf_prim = [&](uint32_t i) {
            const uint32_t k = kind_of(i);
            return k == MRT_K_SPHERE || k == MRT_K_XY || k == MRT_K_XZ || k == MRT_K_YZ;
        };
        auto leaf_ok = [&](uint32_t i) {
            if (is_leaf_prim(i)) return true;
            if (kind_of(i) != MRT_K_LIST) return false;
            const mrt_node& l = nodes[i];
            for (uint32_t c = 0; c < l.b; c++) {
                const uint32_t ci = v->children[l.a + c];
                if (ci >= nn) return false;
                if (is_leaf_prim(ci)) continue;
                if (kind_of(ci) != MRT_K_LIST) return false;
                const mrt_node& g = nodes[ci];
                for (uint32_t j = 0; j < g.b; j++) {
                    const uint32_t gi = v->children[g.a + j];
                    if (gi >= nn || !is_leaf_prim(gi)) return false;
                }
            }
            return true;
        };
        std::vector<uint8_t> under_bvh(nn, 0);
        for (size_t i = 0; i < nn; i++)
            if (kind_of((uint32_t)i) == MRT_K_BVH) {
                if (nodes[i].a < nn) under_bvh[nodes[i].a] = 1;
                if (nodes[i].b < nn) under_bvh[nodes[i].b] = 1;
            }
        // does the subtree at i qualify (bvh_node inner nodes, qualifying leaves)?
        std::function<bool(uint32_t, int)> ok = [&](uint32_t i, int guard) -> bool {
            if (i >= nn || guard > 64) return false;
            if (kind_of(i) != MRT_K_BVH) return leaf_ok(i);
            return ok(nodes[i].a, guard + 1) && ok(nodes[i].b, guard + 1);
        };
        // a leaf's primitives as one contiguous run of node records (bprims): a primitive leaf is a
        // run of one; an object_list leaf is its children in order, a nested object_list as a LIST
        // record (its box, b = the count of its own children that follow) before its children.  The
        // walk then fetches a leaf's records at independent addresses instead of through the
        // children[] -> node chain (two dependent loads per primitive).
        bool leaves_ok = true;
        auto emit_leaf = [&](uint32_t i) -> uint32_t {
            const uint32_t first = (uint32_t)bprims.size();
            if (is_leaf_prim(i)) {
                bprims.push_back(nodes[i]);
            } else {
                const mrt_node& l = nodes[i];
                for (uint32_t c = 0; c < l.b; c++) {
                    const uint32_t ci = v->children[l.a + c];
                    if (is_leaf_prim(ci)) { bprims.push_back(nodes[ci]); continue; }
                    const mrt_node& g = nodes[ci];
                    mrt_node m = g;
                    m.b = g.b;
                    bprims.push_back(m);
                    for (uint32_t j = 0; j < g.b; j++) bprims.push_back(nodes[v->children[g.a + j]]);
                }
            }
            const uint32_t cnt = (uint32_t)bprims.size() - first;
            if (cnt > BVHW_MAX_RUN || first > BVHW_FIRST_MASK) leaves_ok = false;
            if ((BVHW_LEAF | (cnt << 24) | (first & BVHW_FIRST_MASK)) == kBvhwEmpty) leaves_ok = false;  // (the walk's empty-stack mark)
            return BVHW_LEAF | (cnt << 24) | (first & BVHW_FIRST_MASK);
        };
        std::function<uint32_t(uint32_t, int)> build = [&](uint32_t i, int depth) -> uint32_t {
            bvhw_depth = std::max(bvhw_depth, depth);
            if (kind_of(i) != MRT_K_BVH) return emit_leaf(i);
            absorbed[i] = 1;
            const uint32_t w = (uint32_t)bwide.size();
            bwide.push_back(BvhWide{});
            const mrt_node& b = nodes[i];
            const uint32_t lc = b.a, rc = b.b;
            const uint32_t lref = build(lc, depth + 1), rref = build(rc, depth + 1);
            BvhWide& W = bwide[w];
            W.lref = lref;
            W.rref = rref;
            W.order = (b.kind >> 8) & 0xFFu;
            W.flags = 0;
            const mrt_node &L = nodes[lc], &R = nodes[rc];
            auto has_box = [&](const mrt_node& c) {
                const uint32_t k = c.kind & 0xFFu;
                return k == MRT_K_BVH || (k == MRT_K_LIST && ((c.kind >> 16) & MRT_F_HASBOX));
            };
            if (has_box(L)) { W.flags |= 1u; for (int k = 0; k < 3; k++) { W.lmin[k] = L.f[k]; W.lmax[k] = L.f[3 + k]; } }
            if (has_box(R)) { W.flags |= 2u; for (int k = 0; k < 3; k++) { W.rmin[k] = R.f[k]; W.rmax[k] = R.f[3 + k]; } }
            return w;
        };
        const char* no_bvhw = getenv("MRT_NO_BVHW");  // test hook: keep the generic bvh_node walk
        if (!(no_bvhw && *no_bvhw && *no_bvhw != '0'))
            for (size_t i = 0; i < nn; i++)
                if (kind_of((uint32_t)i) == MRT_K_BVH && !under_bvh[i] && ok((uint32_t)i, 0) && bwide.size() < BVHW_LEAF / 2) {
                    const uint32_t root = build((uint32_t)i, 1);
                    mrt_node& r = nodes[i];
                    r.kind = (r.kind & ~0xFFu) | MRT_K_BVHW;
                    r.a = root;
                }
        if (!leaves_ok) return mrt_internal_fail(MRT_ERR_INVALID, "bvh_node leaf outside the device encoding (> 127 primitives or > 2^24 leaf records)");
    }
    {  // treelet kernels cache the first nodes of the wide array: the top levels
        std::vector<uint32_t*> broots;
        for (mrt_node& n : nodes)
            if ((n.kind & 0xFF) == MRT_K_BVHW) broots.push_back(&n.a);
        bfs_order(bwide, broots, BVHW_LEAF);
    }
    GraphCheck gc{nodes, v};
    // stack words: one per level for the binary walk
    gc.bvhw_depth = bvhw_depth;
    gc.walk(v->root, 0, 0, false, 0);
    if (!gc.ok) return mrt_internal_fail(MRT_ERR_INVALID, gc.why.c_str());
    if (v->biased != MRT_NONE) {
        if (v->biased >= nodes.size()) return mrt_internal_fail(MRT_ERR_INVALID, "bad biased node");
        const mrt_node& b = nodes[v->biased];
        if ((b.kind & 0xFF) == MRT_K_LIST)
            for (uint32_t i = 0; i < b.b; i++)
                if ((nodes[v->children[b.a + i]].kind & 0xFF) == MRT_K_LIST)
                    return mrt_internal_fail(MRT_ERR_INVALID, "nested biased object_list");
    }
    std::vector<DMat> dmats(v->n_materials);
    for (uint32_t i = 0; i < v->n_materials; i++) {
        const mrt_material& m = v->materials[i];
        DMat& d = dmats[i];
        d.kind = m.kind;
        d.tex = m.tex;
        d.p = m.p;
        d.flags = 0;
        if (m.tex < v->n_textures && v->textures[m.tex].kind == MRT_T_COLOR) {
            d.flags = DMAT_COLOR;
            for (int k = 0; k < 4; k++) d.col[k] = v->textures[m.tex].f[k];
        }
        if (m.kind == MRT_M_DIELECTRIC) {  // dielectric::scatter's per-material quotients (material.h:121-175)
            const float ref = m.p;
            d.col[0] = 1.0f / ref;
            float r0 = (1 - ref) / (1 + ref);
            d.col[1] = r0 * r0;
        }
    }
    // scene.biased_objects flattened: an object_list's children, or the object itself
    std::vector<mrt_node> bleaf;
    uint32_t blist = 0;
    if (v->biased != MRT_NONE) {
        const mrt_node& b = nodes[v->biased];
        if ((b.kind & 0xFF) == MRT_K_LIST) {
            blist = 1;
            for (uint32_t i = 0; i < b.b; i++) bleaf.push_back(nodes[v->children[b.a + i]]);
        } else {
            bleaf.push_back(b);
        }
    }
    if (bleaf.empty()) bleaf.push_back(mrt_node{});
    LinCompiler lc{nodes, v, {}};
    const char* force_generic = getenv("MRT_FORCE_GENERIC");  // test hook: run the generic machine
    const bool lin = !(force_generic && *force_generic && *force_generic != '0') && lc.emit(v->root, 0, 0, 0);
    if (!lin) lc.prog.clear();
    T->prog_ops = (uint32_t)lc.prog.size();
    lc.prog.push_back(LinOp{});  // LOP_END
    T->features = scene_features(v, nodes, absorbed);
    const char* no_sig = getenv("MRT_NO_SIG");  // test hook: run the interpreter on known shapes too
    if (lin) T->features |= FT_LIN;
    if (lin && lc.vsub) T->features |= FT_VSUB;
    if (lin) cornell_room_fill(lc.prog.data(), (uint32_t)lc.prog.size());  // (Cornell shape: the room into the END op)
    if (lin && !(no_sig && *no_sig && *no_sig != '0')) T->features |= MRT_SIG_BITS(lin_sig_of(lc.prog.data(), (uint32_t)lc.prog.size()));
    T->nbleaf = blist ? nodes[v->biased].b : 1u;
    T->blist = blist;
    T->max_frames = gc.max_frames;
    T->max_rays = gc.max_rays;
    T->max_mesh = gc.max_mesh;
    T->nodes.swap(nodes);
    T->wide.swap(wide);
    T->bwide.swap(bwide);
    T->bprims.swap(bprims);
    T->dmats.swap(dmats);
    T->bleaf.swap(bleaf);
    if (lin) T->prog_fast = lin_rewrite_fast(lc.prog);
    T->prog.swap(lc.prog);
    return MRT_OK;
}

extern "C" mrt_status mrt_scene_upload(int device, const mrt_scene_view* v, mrt_scene** out) {
    if (!out) return mrt_internal_fail(MRT_ERR_INVALID, "mrt_scene_upload: null");
    if (device == MRT_DEVICE_CPU) {  // the CPU backend (explicit choice only)
        mrt_cpu_scene* c = nullptr;
        mrt_status st = mrt_cpu_scene_create(v, &c);
        if (st) return st;
        mrt_scene* s = new mrt_scene();
        s->device = MRT_DEVICE_CPU;
        s->cpu = c;
        s->n_nodes = v->n_nodes;
        s->features = mrt_cpu_scene_features(c);
        *out = s;
        return MRT_OK;
    }
    if (device < 0) return mrt_internal_fail(MRT_ERR_INVALID, "mrt_scene_upload: bad device");
    SceneTables T;
    mrt_status st = mrt_internal_scene_tables(v, &T);
    if (st) return st;
    HIPCHK(hipSetDevice(device));
    mrt_scene* s = new mrt_scene();
    s->device = device;
    DScene& S = s->S;
#define UP(src, n, dst) { void* t_ = nullptr; if ((st = upload(s, src, (size_t)(n) * sizeof(*(src)), &t_))) { mrt_scene_free(s); return st; } *(dst) = (decltype(+*(dst)))t_; }
    UP(T.nodes.data(), T.nodes.size(), &S.nodes);
    UP(v->children, v->n_children, &S.children);
    UP(v->mesh_nodes, v->n_mesh_nodes, &S.mnodes);
    UP(T.wide.data(), T.wide.size(), &S.mwide);
    S.mwide_n = (uint32_t)T.wide.size();
    UP(T.bwide.data(), T.bwide.size(), &S.bwide);
    UP(T.bprims.data(), T.bprims.size(), &S.bprims);
    UP((const float4*)v->tri_geo, (size_t)v->n_tris * 3, &S.tri_geo);
    UP((const float4*)v->tri_nrm, (size_t)v->n_tris * 3, &S.tri_nrm);
    UP(T.dmats.data(), T.dmats.size(), &S.mats);
    UP(T.bleaf.data(), T.bleaf.size(), &S.bleaf);
    S.nbleaf = T.nbleaf;
    S.nbleaf_f = (float)T.nbleaf;
    S.inv_nbleaf = 1.0f / S.nbleaf_f;
    S.blist = T.blist;
    UP(v->textures, v->n_textures, &S.texs);
    UP((const float4*)v->perlin_ranvec, 256, &S.ranvec);
    UP(v->perlin_perm, 768, &S.perm);
    UP(v->texels, (size_t)v->n_texels, &S.texels);
    UP(T.prog.data(), T.prog.size(), &S.prog);
    {
        const char* e = getenv("MRT_NO_REWRITE");  // A/B hook: the interpreter on the program as compiled
        if (!T.prog_fast.empty() && !(e && *e && *e != '0')) UP(T.prog_fast.data(), T.prog_fast.size(), &s->prog_fast);
    }
    UP(&v->camera, 1, &S.camp);
#undef UP
    S.root = v->root;
    S.biased = v->biased;
    S.sky = v->sky;
    S.cam = v->camera;
    s->n_nodes = v->n_nodes;
    s->prog_ops = T.prog_ops;
    void* p;
    if ((st = upload(s, &s->S, sizeof(DScene), &p))) { mrt_scene_free(s); return st; }
    s->d_S = (DScene*)p;
    if ((st = dev_alloc(s, &p, 64))) { mrt_scene_free(s); return st; }
    s->d_counter = (uint64_t*)p;
    s->d_rays = (unsigned long long*)((char*)p + 16);
    HIPCHK(hipMemset(p, 0, 64));  // the cancel flag (d_counter + 4) starts clear
    // kernel variant + LDS stacks sized from the scene graph (top frame lives in registers)
    s->features = T.features;
    s->variant = pick_variant(s->features);
    const bool lin_kernel = (kVariants[s->variant] & FT_LIN) != 0;
    s->lds_frames = lin_kernel ? 0 : (uint32_t)std::max(T.max_frames - 1, 0);
    s->lds_rays = lin_kernel ? 0 : (uint32_t)T.max_rays;
    s->lds_mesh = (uint32_t)T.max_mesh;
    // the query ray parked in LDS: instances (scene_hit_lin)
    s->lds_save = (lin_kernel && (kVariants[s->variant] & FT_INST)) ? 9u : 0u;  // (round 6: 15 -> 9, mrt_lin.h inst_ray)
    // resumable mesh walk: deeper pod_bvh trees keep the wave walking longer
    s->walk_min = T.wide.size() >= 2048 ? 40u : 32u;  // inner nodes: bunny 2937, teapot ~1045
    bool walk_min_env = false;
    if (const char* e = getenv("MRT_WALK_MIN"))  // sweep hook (tools/ab_walk.sh)
        if (*e) {
            s->walk_min = (uint32_t)atoi(e);
            walk_min_env = true;
        }
    const std::vector<BvhWide>& bwide = T.bwide;
    hipDeviceProp_t prop;
    HIPCHK(hipGetDeviceProperties(&prop, device));
    s->n_cu = (uint32_t)prop.multiProcessorCount;
    // resident workgroups per CU: one 256-thread group = one wave per SIMD (a 64-thread group =
    // a quarter of that); VGPRs (512 per SIMD lane, granule 8) and LDS (160 KiB per CU) bound it.
    // (The runtime occupancy query under-counts gfx950 register budgets, so it is computed from
    // the kernel's attributes.)  Per numerics build: their register counts differ.
    const KernelTable* tabs[2] = {&kernel_table_exact(), &fast_table()};
    for (int k = 0; k < 2; k++) {
        PathLaunch& L = s->pl[k];
        L.fn = tabs[k]->kernel[s->variant];
        L.wg = tabs[k]->wg[s->variant];
        const uint32_t waves_per_wg = L.wg / 64u;
        // the Cornell walk of the tolerance contract (mrt_sig.h cornell_fast_hit) parks no ray
        L.lds_save = tabs[k]->box6_walk[s->variant] ? 0u : s->lds_save;
        L.lds_mesh = s->lds_mesh;
        L.rewrite = tabs[k]->rewrite[s->variant] != 0;
        L.retrace = tabs[k]->retrace[s->variant];
        // a fast-arithmetic kernel hands its rounding-critical paths to the exact arithmetic
        // (mrt_shade.h light_critical); MRT_RETRACE=0 at upload keeps them (A/B)
        {
            const char* e = getenv("MRT_RETRACE");
            L.handover = k == 1 && L.retrace && L.fn != kernel_table_fast_pex().kernel[s->variant] && !(e && *e && atoi(e) == 0);
        }
        L.retrace_lds = (size_t)64 * 4 * (s->lds_frames * 2 + s->lds_rays * 11 + s->lds_mesh + s->lds_save);
        // the path-exact build (the metal bunny under the tolerance contract) yields at 32 walking
        // lanes: 40 -1.2%, 28 -1.7%, 48 -10% (bunny 1024x1024x64, profiles/r04_ab.txt section 13)
        L.walk_min = (!walk_min_env && L.fn == kernel_table_fast_pex().kernel[s->variant]) ? 32u : s->walk_min;
        hipFuncAttributes fa{};
        HIPCHK(hipFuncGetAttributes(&fa, reinterpret_cast<const void*>(L.fn)));
        const int vg = std::max(8, (fa.numRegs + 7) & ~7);
        const int nb_vgpr = std::max(1, std::min(8, 512 / vg) * 4 / (int)waves_per_wg);  // waves per CU / waves per group
        auto groups = [&](size_t lds) { return std::max(1, lds ? std::min<int>(nb_vgpr, (int)((160u * 1024u) / lds)) : nb_vgpr); };
        const size_t lds_core = (size_t)waves_per_wg * 64 * 4 *
                                (s->lds_frames * 2 + s->lds_rays * 11 + L.lds_mesh + L.lds_save + tabs[k]->lev_k[s->variant] * 4 +
                                 tabs[k]->pq[s->variant]);
        L.lds_bytes = lds_core;
        if (L.lds_bytes > (size_t)prop.sharedMemPerBlock) {
            mrt_scene_free(s);
            return mrt_internal_fail(MRT_ERR_INVALID, "scene graph too deep for the LDS stacks");
        }
        int nb = groups(L.lds_bytes);
        if (tabs[k]->tree[s->variant]) {
            // the LDS the resident groups leave free, split among them: the treelet of each group
            const size_t per = std::min<size_t>((160u * 1024u) / nb, (size_t)prop.sharedMemPerBlock);
            const uint32_t node_bytes = 64u;  // BvhWide
            const uint32_t n_nodes = (uint32_t)bwide.size();
            uint32_t cap = per > L.lds_bytes ? (uint32_t)((per - L.lds_bytes) / node_bytes) : 0u;
#ifdef MRT_EXPERIMENTS
            if (const char* e = getenv("MRT_TREELET_NODES"))  // sweep hook
                if (*e) cap = std::min<uint32_t>(cap, (uint32_t)atoi(e));
#endif
            L.tree_n = std::min(cap, n_nodes);
            L.lds_bytes += (size_t)L.tree_n * node_bytes;
        }
        L.vgprs = (uint32_t)fa.numRegs;
#ifdef MRT_EXPERIMENTS
        if (const char* e = getenv("MRT_BLOCKS_PER_CU"))  // experiment hook
            if (*e) nb = std::max(1, atoi(e));
#endif
        L.grid = prop.multiProcessorCount * nb;
        // every work partition needs waves of its own: a wave leaves its partition only once it is
        // handed out, and visits at most MRT_STEAL_TRIES partitions (mrt_kernels.hip)
        if (L.grid < (int)MRT_NPART) return mrt_internal_fail(MRT_ERR_HIP, "path kernel grid smaller than the work partitions");
        s->max_threads = std::max(s->max_threads, (size_t)L.grid * L.wg);
    }
    *out = s;
    return MRT_OK;
}

extern "C" void mrt_scene_free(mrt_scene* s) {
    if (!s) return;
    if (s->cpu) {
        mrt_cpu_scene_free(s->cpu);
        delete s;
        return;
    }
    (void)hipSetDevice(s->device);
    if (s->ev_done_pending) (void)hipEventSynchronize(s->ev_done);
    for (void* p : s->allocs) (void)hipFree(p);
    for (hipEvent_t e : s->ev) (void)hipEventDestroy(e);
    if (s->pstream) (void)hipStreamDestroy(s->pstream);
    if (s->h_prog) (void)hipHostFree(s->h_prog);
    if (s->h_one) (void)hipHostFree(s->h_one);
    if (s->h_prev) (void)hipHostFree(s->h_prev);
    if (s->h_seq) (void)hipHostFree(s->h_seq);
    if (s->ev_done) (void)hipEventDestroy(s->ev_done);
    if (s->fstream) (void)hipStreamDestroy(s->fstream);
    for (hipEvent_t e : {s->ev_kern, s->ev_fold[0], s->ev_fold[1]})
        if (e) (void)hipEventDestroy(e);
    for (void* p : {(void*)s->d_rad2, (void*)s->d_counters, (void*)s->d_pixels, (void*)s->d_sdist, (void*)s->d_rad, (void*)s->d_path_rays, (void*)s->d_acc,
                    (void*)s->d_lev, (void*)s->d_out, (void*)s->d_prev, (void*)s->d_rt})
        if (p) (void)hipFree(p);
    delete s;
}

static uint32_t auto_chunk(uint32_t npix, uint32_t ns) {
    // keep the per-chunk radiance buffer within ~4 GiB of HBM (288 GB per MI355X)
    const size_t budget = (size_t)4 << 30;
    size_t per_sample = (size_t)npix * 12;
    size_t c = per_sample ? budget / per_sample : ns;
    if (c < 1) c = 1;
    return (uint32_t)std::min<size_t>(c, ns);
}

static bool same_layout(const mrt_render_desc& a, const std::vector<uint32_t>& a_px, const mrt_render_desc& b) {
    if (a.width != b.width || a.height != b.height || (a.pixels != nullptr) != (b.pixels != nullptr)) return false;
    if (b.pixels) return a_px.size() == b.n_pixels && std::equal(a_px.begin(), a_px.end(), b.pixels);
    return a.tile_size == b.tile_size && a.rank == b.rank && a.world == b.world;
}

// Before the workspace is rewritten or reallocated: wait for the last enqueued render of this
// context (it may still run on a caller stream that the synchronous uploads do not order against).
static mrt_status quiesce(mrt_scene* s) {
    if (s->ev_done_pending) {
        HIPCHK(hipEventSynchronize(s->ev_done));
        s->ev_done_pending = false;
    }
    return MRT_OK;
}
static mrt_status grow(mrt_scene* s, void** p, size_t* cap, size_t bytes) {
    if (*cap >= bytes && *p) return MRT_OK;
    mrt_status st = quiesce(s);
    if (st) return st;
    if (*p) (void)hipFree(*p);
    *p = nullptr;
    *cap = 0;
    hipError_t e = hipMalloc(p, bytes ? bytes : 16);
    if (e != hipSuccess) return mrt_internal_fail(MRT_ERR_OOM, "workspace allocation failed");
    *cap = bytes;
    return MRT_OK;
}

// rounding-critical paths listed per launch (mrt_shade.h light_critical; a full list loses the rest,
// which keep their fast radiance): measured ~1e-5 per path in the Cornell scenes
static constexpr uint32_t kRtCap = 1u << 20;
// one-wave groups of the retrace kernel: 16384 lanes, a path each (more loop); its time is the longest
// listed path's, plus the launch
static constexpr uint32_t kRetraceGroups = 256;
// (Round 6: the retrace of an MRT_RF_FOLD_ASYNC launch beside the next launch's path kernel -- on the
// context's fold stream, and there in one-wave slots the next kernel left free -- measured slower:
// the previous launch's fold uses the GPU during the retrace's gap on the render's stream, and behind
// the retrace on the fold stream it got only the free slots, profiles/r06_ab.txt sections 2 and 7.)

#define MRT_GPU_ONLY(s, what) \
    if ((s) && (s)->cpu) return mrt_internal_fail(MRT_ERR_INVALID, what " is a GPU-backend entry point (scene on MRT_DEVICE_CPU)")

extern "C" mrt_status mrt_prepare(mrt_scene* s, const mrt_render_desc* d) {
    MRT_GPU_ONLY(s, "mrt_prepare");
    if (!s || !d || d->width == 0 || d->height == 0 || d->sqrt_samples == 0 || (d->world && d->rank >= d->world))
        return mrt_internal_fail(MRT_ERR_INVALID, "mrt_prepare: bad desc");
    // the path kernel's u = (x + dx) / W by one reciprocal is exact up to 2^24 (mrt_kernels.hip)
    if (d->width > (1u << 24) || d->height > (1u << 24))
        return mrt_internal_fail(MRT_ERR_INVALID, "mrt_prepare: width / height above 2^24 pixels");
    // every GPU entry point renders in per-path stream order (mrt_render_device and mrt_render come here)
    if (d->flags & MRT_RF_REF_ORDER)
        return mrt_internal_fail(MRT_ERR_INVALID, "MRT_RF_REF_ORDER is a CPU-backend mode (the GPU keys its PCG streams per path)");
    mrt_status st;
    if ((st = mrt_internal_check_pixels(d))) return st;
    HIPCHK(hipSetDevice(s->device));
    bool relayout = !s->have_ws || !same_layout(s->wdesc, s->wpixels, *d);
    uint32_t ns = d->sqrt_samples * d->sqrt_samples;
    if (relayout) {
        std::vector<uint32_t> px = mrt_internal_local_pixels(d);
        std::vector<uint2> xy(px.size());
        for (size_t i = 0; i < px.size(); i++) xy[i] = make_uint2(px[i] % d->width, px[i] / d->width);
        if ((st = quiesce(s))) return st;
        if ((st = grow(s, (void**)&s->d_pixels, &s->px_cap, xy.size() * 8))) return st;
        HIPCHK(hipMemcpy(s->d_pixels, xy.data(), xy.size() * 8, hipMemcpyHostToDevice));
        s->npix = (uint32_t)px.size();
    }
    if (s->sdist_sq != d->sqrt_samples) {  // sample grid of main.cpp:319-332, in float like the reference
        const uint32_t sq = d->sqrt_samples;
        std::vector<float2> sd((size_t)sq * sq);
        for (uint32_t i = 0; i < sq; i++)
            for (uint32_t j = 0; j < sq; j++)
                sd[(size_t)i * sq + j] = make_float2(((float)i + 0.5f) / (float)sq, ((float)j + 0.5f) / (float)sq);
        if ((st = quiesce(s))) return st;
        if ((st = grow(s, (void**)&s->d_sdist, &s->sd_cap, sd.size() * 8))) return st;
        HIPCHK(hipMemcpy(s->d_sdist, sd.data(), sd.size() * 8, hipMemcpyHostToDevice));
        s->sdist_sq = sq;
    }
    uint32_t chunk = d->chunk_samples ? std::min(d->chunk_samples, ns) : auto_chunk(s->npix, ns);
    chunk = (uint32_t)std::min<uint64_t>(chunk, 0xFFFFFFFFull / std::max<uint32_t>(s->npix, 1));  // 32-bit path index
    // 32-bit byte offsets of the chunk's radiance (the path kernel's held store, mrt_kernels.hip)
    chunk = (uint32_t)std::max<uint64_t>(1, std::min<uint64_t>(chunk, 0xFFFFFFFFull / (12ull * std::max<uint32_t>(s->npix, 1))));
    if (chunk == 0) return mrt_internal_fail(MRT_ERR_INVALID, "image too large for one launch");
    if (d->flags & MRT_RF_PATH_DEBUG) chunk = ns;  // debug keeps every path
    if (chunk != s->chunk && (st = quiesce(s))) return st;  // the fold of a running render reads `chunk` rows
    s->chunk = chunk;
    size_t paths = (size_t)s->npix * s->chunk;
    if ((st = grow(s, (void**)&s->d_rad, &s->rad_cap, paths * 12))) return st;
    if (d->flags & MRT_RF_FOLD_ASYNC) {
        if (d->flags & (MRT_RF_PREVIEW | MRT_RF_PATH_DEBUG | MRT_RF_FOLD_BEHIND))
            return mrt_internal_fail(MRT_ERR_INVALID, "MRT_RF_FOLD_ASYNC: no preview, debug or lean fold");
        if ((st = grow(s, (void**)&s->d_rad2, &s->rad2_cap, paths * 12))) return st;
        if (!s->fstream) HIPCHK(hipStreamCreateWithFlags(&s->fstream, hipStreamNonBlocking));
        if (!s->ev_kern) HIPCHK(hipEventCreateWithFlags(&s->ev_kern, hipEventDisableTiming));
        for (hipEvent_t& e : s->ev_fold)
            if (!e) HIPCHK(hipEventCreateWithFlags(&e, hipEventDisableTiming));
    }
    // (two lists: one per radiance parity of the async fold)
    if ((d->flags & MRT_RF_FAST) && !(d->flags & MRT_RF_PATH_DEBUG) && s->pl[1].handover &&
        (st = grow(s, (void**)&s->d_rt, &s->rt_cap, (size_t)2 * kRtCap * sizeof(uint32_t))))
        return st;
    if ((st = grow(s, (void**)&s->d_acc, &s->acc_cap, (size_t)s->npix * 16))) return st;
    if ((st = grow(s, (void**)&s->d_out, &s->out_cap, (size_t)s->npix * 16 + 16))) return st;
    if (d->flags & MRT_RF_PREVIEW) {
        if ((st = grow(s, (void**)&s->d_prev, &s->prev_cap, (size_t)s->npix * 16 + 16))) return st;
        std::lock_guard<std::mutex> lk(s->prog_mu);
        if (s->h_prev_cap < s->npix) {
            if ((st = quiesce(s))) return st;
            if (s->h_prev) (void)hipHostFree(s->h_prev);
            s->h_prev = nullptr;
            s->h_prev_cap = 0;
            HIPCHK(hipHostMalloc((void**)&s->h_prev, (size_t)s->npix * 16 + 16, hipHostMallocPortable));
            s->h_prev_cap = s->npix;
        }
        if (!s->h_seq) {
            HIPCHK(hipHostMalloc((void**)&s->h_seq, 64, hipHostMallocPortable | hipHostMallocCoherent));
            memset(s->h_seq, 0, 64);
        }
        if (relayout || s->prev_px.size() != s->npix) {
            s->prev_px = mrt_internal_local_pixels(d);
        }
        s->prev_w = d->width;
        s->prev_h = d->height;
    }
    if (d->flags & MRT_RF_PATH_DEBUG)
        if ((st = grow(s, (void**)&s->d_path_rays, &s->pr_cap, paths * 4))) return st;
    s->lev_rows = std::max<uint32_t>(d->max_bounces, 1);
    if ((st = grow(s, (void**)&s->d_lev, &s->lev_cap, (size_t)s->lev_rows * s->max_threads * 16))) return st;
    // Two sets of counter slots / progress snapshots, `slot_half` launches each, at FIXED offsets 0
    // and slot_half: consecutive MRT_RF_FOLD_ASYNC renders alternate between them, because a render's
    // last fold still resets its set while the next render's kernels count in the other.  The stride
    // must not follow each render's own launch count: a render of 1 launch after one of 4 would
    // otherwise start its set inside the previous render's (whose reset then lands mid-claim).  The
    // set is grown only after quiesce() (no render pending), and render R+2 -- the next user of R's
    // set -- waits for R's last fold (its first launch waits for the fold of the same radiance
    // parity, and folds run in order on the context's stream).
    const uint32_t need = (ns + s->chunk - 1) / s->chunk;
    const uint32_t half = std::max(s->slot_half, need);
    const uint32_t launches = 2 * half;
    const size_t cnt_words = (size_t)MRT_CNT_SLOTS * MRT_COUNTER_STRIDE;  // per launch
    {
        void* const before = s->d_counters;
        if ((st = grow(s, (void**)&s->d_counters, &s->cnt_cap, (size_t)launches * cnt_words * 8))) return st;
        // zeroed once at allocation; afterwards every render's final kernel leaves them zero
        if (s->d_counters != before) HIPCHK(hipMemset(s->d_counters, 0, s->cnt_cap));
    }
    if (!s->pstream) HIPCHK(hipStreamCreateWithFlags(&s->pstream, hipStreamNonBlocking));
    if (!s->ev_done) HIPCHK(hipEventCreateWithFlags(&s->ev_done, hipEventDisableTiming));
    {
        std::lock_guard<std::mutex> lk(s->prog_mu);
        if (s->h_prog_cap < (size_t)launches) {
            if ((st = quiesce(s))) return st;
            if (s->h_prog) (void)hipHostFree(s->h_prog);
            s->h_prog = nullptr;
            s->h_prog_cap = 0;
            HIPCHK(hipHostMalloc((void**)&s->h_prog, (size_t)launches * MRT_NPART * 8, hipHostMallocPortable | hipHostMallocCoherent));
            memset(s->h_prog, 0, (size_t)launches * MRT_NPART * 8);  // later: reset by each render's final kernel
            s->h_prog_cap = launches;
        }
        s->slot_half = half;  // (both buffers now hold 2 * half launches)
        if (s->h_seen.size() < (size_t)launches * MRT_NPART) s->h_seen.resize((size_t)launches * MRT_NPART, 0);
        if (s->chunk_paths.size() < launches) s->chunk_paths.resize(launches, 0);
        while (s->ev.size() < 2 * (size_t)launches) {
            hipEvent_t e;
            HIPCHK(hipEventCreate(&e));
            s->ev.push_back(e);
        }
    }
    if (!s->h_one) {
        HIPCHK(hipHostMalloc((void**)&s->h_one, sizeof(int), hipHostMallocPortable));
        *s->h_one = 1;
    }
    if (relayout) s->wpixels = d->pixels ? std::vector<uint32_t>(d->pixels, d->pixels + d->n_pixels) : std::vector<uint32_t>();
    s->wdesc = *d;
    s->wdesc.pixels = nullptr;  // (the caller's list is not kept; wpixels holds a copy)
    if (d->pixels) s->wdesc.pixels = s->wpixels.data();
    s->have_ws = true;
    return MRT_OK;
}

extern "C" mrt_status mrt_render_device(mrt_scene* s, const mrt_render_desc* d, float* d_local, uint64_t* d_rays, void* stream) {
    MRT_GPU_ONLY(s, "mrt_render_device");
    if (!s || !d || !d_local) return mrt_internal_fail(MRT_ERR_INVALID, "mrt_render_device: null");
    s->n_chunks.store(0, std::memory_order_release);  // progress: a new render, not started
    mrt_status st = mrt_prepare(s, d);
    if (st) return st;
    const PathLaunch& PL = s->pl[(d->flags & MRT_RF_FAST) ? 1 : 0];
    hipStream_t q = (hipStream_t)stream;
    uint32_t ns = d->sqrt_samples * d->sqrt_samples;
    // No clearing fills enqueued here: the first fold chunk starts from +0 instead of reading the
    // accumulator, and the work counters and progress snapshots were left zero by the previous
    // render's final kernel (stream order; zeroed at allocation before the first).  The cancel flag
    // is clear unless a cancelled mrt_render set it, and that clears it again before returning.
    const uint32_t launches = (ns + s->chunk - 1) / s->chunk;
    {
        std::lock_guard<std::mutex> lk(s->prog_mu);
        for (uint32_t k = 0; k < launches; k++) {
            s->chunk_paths[k] = (uint64_t)s->npix * (std::min(ns, (k + 1) * s->chunk) - k * s->chunk);
            // the host's running maxima only: a snapshot is read only once this render's launch k
            // has started (its start event), i.e. after the previous render's final kernel reset it
            for (uint32_t j = 0; j < MRT_NPART; j++) s->h_seen[(size_t)k * MRT_NPART + j] = 0;
        }
    }
    s->n_launch = 0;
    s->last_numerics = (d->flags & MRT_RF_FAST) ? 1u : 0u;
    const bool preview = (d->flags & MRT_RF_PREVIEW) != 0;
    // MRT_RF_FOLD_ASYNC: each launch writes the radiance buffer of its parity, whose last fold (on
    // fstream) must have ended first; the render uses the counter slots of its parity (the previous
    // render's folds may still reset theirs).  Any other render waits for every pending fold.
    const bool async = (d->flags & MRT_RF_FOLD_ASYNC) != 0;
    const uint32_t rpar = async ? s->rpar : 0u;
    if (async) s->rpar ^= 1u;
    if (!async)
        for (uint32_t p = 0; p < 2; p++)
            if (s->fold_pending[p]) HIPCHK(hipStreamWaitEvent(q, s->ev_fold[p], 0));
    {
        std::lock_guard<std::mutex> lk(s->prog_mu);
        s->prog_base = rpar * s->slot_half;
    }
    unsigned long long* const d_cnt = (unsigned long long*)(s->d_counters + (size_t)rpar * s->slot_half * MRT_CNT_SLOTS * MRT_COUNTER_STRIDE);
    unsigned long long* const h_prog = (unsigned long long*)(s->h_prog + (size_t)rpar * s->slot_half * MRT_NPART);
    uint32_t seq = 0;
    if (preview) {  // a new render: no snapshot yet (sequence 0), in stream order
        std::lock_guard<std::mutex> lk(s->prog_mu);
        HIPCHK(hipStreamWriteValue32(q, s->h_seq + 1, 0u, 0));
        HIPCHK(hipStreamWriteValue32(q, s->h_seq, 0u, 0));
        s->prev_epoch++;
    }
    // the rounding-critical paths' hand-over: tolerance contract, not the per-path debug output
    // (whose radiance is the fast kernel's own)
    const bool handover = PL.handover && !(d->flags & MRT_RF_PATH_DEBUG);
    const int grid = PL.grid;
    for (uint32_t s0 = 0; s0 < ns; s0 += s->chunk) {
        uint32_t s1 = std::min(ns, s0 + s->chunk);
        const uint32_t par = async ? s->lpar : 0u;
        if (async) {
            s->lpar ^= 1u;
            if (s->fold_pending[par]) HIPCHK(hipStreamWaitEvent(q, s->ev_fold[par], 0));
        }
        float* const d_rad = par ? s->d_rad2 : s->d_rad;
        PathParams P{};
        P.sc = s->S;
        // the interpreter's tolerance-contract program (rooms and box.h lists as slab tests); the
        // shape-specialised walks read the program as compiled
        if ((d->flags & MRT_RF_FAST) && s->prog_fast && PL.rewrite) P.sc.prog = s->prog_fast;
        P.lds_frames = s->lds_frames;
        P.lds_rays = s->lds_rays;
        P.lds_mesh = PL.lds_mesh;
        P.lds_save = PL.lds_save;
        P.walk_min = PL.walk_min;
        P.tree_src = reinterpret_cast<const float4*>(s->S.bwide);
        P.tree_n = PL.tree_n;
        P.pixels = s->d_pixels;
        P.sdist = s->d_sdist;
        P.npix = s->npix;
        P.inv_npix = 1.0 / (double)std::max<uint32_t>(s->npix, 1);
        P.width = d->width;
        P.height = d->height;
        P.inv_w = 1.0f / (float)d->width;
        P.inv_h = 1.0f / (float)d->height;
        P.fast_uv = 1;  // checked by mrt_prepare (and sq < 2^16 since sq^2 fits in 32 bits)
        P.sq = d->sqrt_samples;
        P.ns = ns;
        P.s0 = s0;
        P.n_paths = s->npix * (s1 - s0);
        P.tail_zone = (uint32_t)std::min<uint64_t>((uint64_t)grid * (PL.wg / 64u) * 2 * MRT_BATCH, P.n_paths);  // ~2 big claims per wave
        P.static_first = (uint64_t)P.n_paths < (uint64_t)grid * (PL.wg / 64u) * MRT_BATCH * 64u;
        // MRT_NPART contiguous work partitions, one counter each; the waves of partition k (workgroups
        // b with b % MRT_NPART == k) take its first batches statically when P.static_first
        for (uint32_t k = 0; k <= MRT_NPART; k++) P.part_base[k] = (uint64_t)P.n_paths * k / MRT_NPART;
        for (uint32_t k = 0; k < MRT_NPART; k++) {
            const uint64_t waves_k = (uint64_t)((grid - k + MRT_NPART - 1) / MRT_NPART) * (PL.wg / 64u);
            P.part_dyn[k] = P.part_base[k] + (P.static_first ? waves_k * MRT_BATCH : 0);
        }
        P.seed = d->seed;
        P.max_bounces = d->max_bounces;
        P.rad = d_rad;
        P.path_rays = (d->flags & MRT_RF_PATH_DEBUG) ? s->d_path_rays : nullptr;
        P.counter = d_cnt + (size_t)s->n_launch * MRT_CNT_SLOTS * MRT_COUNTER_STRIDE;
        P.hprog = h_prog + (size_t)s->n_launch * MRT_NPART;
        P.cancel = (const int*)(s->d_counter + 4);
        P.rays = d_rays ? (unsigned long long*)d_rays : s->d_rays;
        P.lev = s->d_lev;
        P.lev_rows = s->lev_rows;
        // the list of the launch's radiance parity: entries at par * kRtCap, its count and its groups-done
        // word at d_counter[1] / [3] (parity 0) or the two halves of d_counter[6] (parity 1)
        if (handover)
            P.rt = RetraceList{s->d_rt + (size_t)par * kRtCap, par ? (uint32_t*)(s->d_counter + 6) : (uint32_t*)(s->d_counter + 1), kRtCap,
                               par ? (uint32_t*)(s->d_counter + 6) + 1 : (uint32_t*)(s->d_counter + 3), (unsigned long long*)s->d_counter,
                               (unsigned long long*)(s->d_counter + 5)};
        HIPCHK(hipEventRecord(s->ev[2 * s->n_launch], q));
        hipLaunchKernelGGL(PL.fn, dim3(grid), dim3(PL.wg), PL.lds_bytes, q, P);
        HIPCHK(hipGetLastError());
        HIPCHK(hipEventRecord(s->ev[2 * s->n_launch + 1], q));
        s->n_launch++;
        // this launch's rounding-critical paths, exact, into the radiance buffer before its fold (the
        // exact arithmetic walks the program as compiled: the tolerance contract's rewrite has ops -- a
        // room's slab test, one-step box instances -- only the fast builds compile)
        if (handover) {
            PathParams PR = P;
            PR.sc.prog = s->S.prog;
            hipLaunchKernelGGL(PL.retrace, dim3(kRetraceGroups), dim3(64), PL.retrace_lds, q, PR);
            HIPCHK(hipGetLastError());
        }
        if (async) {  // the fold on the fold stream, beside the next launch's path kernel
            HIPCHK(hipEventRecord(s->ev_kern, q));
            HIPCHK(hipStreamWaitEvent(s->fstream, s->ev_kern, 0));
        }
        if (async) {  // the fold beside the next launch's path kernel
            const bool last = s1 == ns;
            FoldEnd fe{last ? (float4*)d_local : nullptr, ns, last ? d_cnt : nullptr, last ? h_prog : nullptr,
                       last ? launches * MRT_CNT_SLOTS : 0u, last ? launches * MRT_NPART : 0u};
            hipLaunchKernelGGL(mrt_fold_async_kernel, dim3(s->n_cu * MRT_FOLD_ASYNC_GROUPS), dim3(MRT_FOLD_ASYNC_WG), 0, s->fstream, d_rad, s->d_acc, s->npix,
                               s0, s1, d->mode, d->max_luminance, fe);
            HIPCHK(hipGetLastError());
            HIPCHK(hipEventRecord(s->ev_fold[par], s->fstream));
            s->fold_pending[par] = true;
            s->last_paths = P.n_paths;
            continue;
        }
        // the last chunk's full fold finishes the render (no preview: no snapshot of acc needed;
        // the 8-VGPR lean fold cannot take the division as well: a final kernel follows it)
        const bool lean = (d->flags & MRT_RF_FOLD_BEHIND) && d->mode == 0;
        const bool last = s1 == ns && !preview && !lean;
        FoldEnd fe{last ? (float4*)d_local : nullptr, ns, last ? (unsigned long long*)s->d_counters : nullptr,
                   last ? (unsigned long long*)s->h_prog : nullptr, last ? launches * MRT_CNT_SLOTS : 0u, last ? launches * MRT_NPART : 0u};
        const uint32_t nthr = std::max(s->npix, fe.nreset);
        if (lean)
            hipLaunchKernelGGL(mrt_fold_lean_kernel, dim3((s->npix + MRT_FOLD_LEAN_WG - 1) / MRT_FOLD_LEAN_WG), dim3(MRT_FOLD_LEAN_WG), 0, q,
                               d_rad, s->d_acc, s->npix, s1 - s0, (uint32_t)(s0 == 0));
        else
            hipLaunchKernelGGL(mrt_fold_kernel, dim3((nthr + 255) / 256), dim3(256), 0, q, d_rad, s->d_acc, s->npix, s0, s1, d->mode,
                               d->max_luminance, fe);
        HIPCHK(hipGetLastError());
        if (preview) {  // the image after s1 samples, copied under the sequence lock
            hipLaunchKernelGGL(mrt_final_kernel, dim3((s->npix + MRT_FINAL_WG - 1) / MRT_FINAL_WG), dim3(MRT_FINAL_WG), 0, q, s->d_acc, s->d_prev,
                               s->npix, s1, d->mode, d->max_luminance,
                               (unsigned long long*)nullptr, (unsigned long long*)nullptr, 0u, 0u);
            HIPCHK(hipGetLastError());
            HIPCHK(hipStreamWriteValue32(q, s->h_seq, 2 * seq + 1, 0));
            HIPCHK(hipMemcpyAsync(s->h_prev, s->d_prev, (size_t)s->npix * 16, hipMemcpyDeviceToHost, q));
            HIPCHK(hipStreamWriteValue32(q, s->h_seq + 1, s1, 0));
            HIPCHK(hipStreamWriteValue32(q, s->h_seq, 2 * seq + 2, 0));
            seq++;
        }
        s->last_paths = P.n_paths;
    }
    if (preview || ((d->flags & MRT_RF_FOLD_BEHIND) && d->mode == 0)) {  // (otherwise the last fold wrote the output and reset the counters)
        const uint32_t nreset = launches * MRT_CNT_SLOTS;
        const uint32_t blocks = (std::max(s->npix, nreset) + MRT_FINAL_WG - 1) / MRT_FINAL_WG;
        hipLaunchKernelGGL(mrt_final_kernel, dim3(blocks), dim3(MRT_FINAL_WG), 0, q, s->d_acc, (float4*)d_local, s->npix, ns, d->mode,
                           d->max_luminance, (unsigned long long*)s->d_counters, (unsigned long long*)s->h_prog, nreset, launches * MRT_NPART);
        HIPCHK(hipGetLastError());
    }
    HIPCHK(hipEventRecord(s->ev_done, async ? s->fstream : q));
    s->ev_done_pending = true;
    s->n_chunks.store(launches, std::memory_order_release);  // progress reads start once every launch and its events are enqueued
    return MRT_OK;
}

extern "C" mrt_status mrt_render(mrt_scene* s, const mrt_render_desc* d, float* rgb_out, uint64_t* rays_out, const volatile int* cancel) {
    if (!s || !d || !rgb_out) return mrt_internal_fail(MRT_ERR_INVALID, "mrt_render: null");
    if (s->cpu) return mrt_cpu_render(s->cpu, d, rgb_out, rays_out, cancel);
    s->n_chunks.store(0, std::memory_order_release);
    if (cancel && *cancel) return mrt_internal_fail(MRT_ERR_CANCELLED, "cancelled");
    mrt_render_desc dc = *d;  // a cancellable render runs as >= 16 launches; cancel lands between them
    const uint32_t ns = d->sqrt_samples * d->sqrt_samples;
    // (so does a previewed one: each launch adds a snapshot)
    if ((cancel || (dc.flags & MRT_RF_PREVIEW)) && dc.chunk_samples == 0 && !(dc.flags & MRT_RF_PATH_DEBUG))
        dc.chunk_samples = std::max(1u, ns / 16);
    d = &dc;
    mrt_status st = mrt_prepare(s, d);
    if (st) return st;
    HIPCHK(hipMemset(s->d_rays, 0, 8));
    st = mrt_render_device(s, d, (float*)s->d_out, (uint64_t*)s->d_rays, nullptr);
    if (st) return st;
    // wait, forwarding the caller's cancel flag to the device flag the path kernel polls
    bool cancelled = false;
    if (!cancel) {
        HIPCHK(hipEventSynchronize(s->ev_done));
    } else {
        for (;;) {
            const hipError_t q = hipEventQuery(s->ev_done);
            if (q == hipSuccess) break;
            if (q != hipErrorNotReady) return mrt_internal_fail(MRT_ERR_HIP, hipGetErrorString(q));
            if (*cancel && !cancelled) {
                HIPCHK(hipMemcpyAsync(s->d_counter + 4, s->h_one, sizeof(int), hipMemcpyHostToDevice, s->pstream));
                HIPCHK(hipStreamSynchronize(s->pstream));
                cancelled = true;
            }
            usleep(200);
        }
    }
    s->ev_done_pending = false;
    if (cancelled) HIPCHK(hipMemset(s->d_counter + 4, 0, 8));  // the render is over: clear the flag for the next one
    std::vector<float> local((size_t)s->npix * 4);
    std::vector<uint32_t> px = mrt_internal_local_pixels(d);
    HIPCHK(hipMemcpy(local.data(), s->d_out, local.size() * 4, hipMemcpyDeviceToHost));
    for (size_t i = 0; i < px.size(); i++) memcpy(rgb_out + (size_t)px[i] * 4, &local[i * 4], 16);
    uint64_t rays = 0;
    HIPCHK(hipMemcpy(&rays, s->d_rays, 8, hipMemcpyDeviceToHost));
    if (rays_out) *rays_out = rays;
    if (cancelled) return mrt_internal_fail(MRT_ERR_CANCELLED, "cancelled (partial image)");
    return MRT_OK;
}

// the worker threads' join (main.cpp:490-493) as stream order: `stream` waits for the context's
// last render, including a fold on the context's own stream (MRT_RF_FOLD_ASYNC)
int mrt_internal_scene_device(const mrt_scene* s) { return s->cpu ? MRT_DEVICE_CPU : s->device; }

extern "C" mrt_status mrt_render_join(mrt_scene* s, void* stream) {
    MRT_GPU_ONLY(s, "mrt_render_join");
    if (!s) return mrt_internal_fail(MRT_ERR_INVALID, "mrt_render_join: null");
    if (!s->ev_done) return MRT_OK;  // no render yet
    HIPCHK(hipSetDevice(s->device));
    HIPCHK(hipStreamWaitEvent((hipStream_t)stream, s->ev_done, 0));
    return MRT_OK;
}

extern "C" mrt_status mrt_render_debug(mrt_scene* s, float* path_rgb, uint32_t* path_rays, uint64_t n_paths) {
    MRT_GPU_ONLY(s, "mrt_render_debug");
    if (!s || !(s->wdesc.flags & MRT_RF_PATH_DEBUG) || n_paths != s->last_paths)
        return mrt_internal_fail(MRT_ERR_INVALID, "mrt_render_debug: no debug render of that size");
    HIPCHK(hipSetDevice(s->device));
    if (path_rgb) HIPCHK(hipMemcpy(path_rgb, s->d_rad, n_paths * 12, hipMemcpyDeviceToHost));
    if (path_rays) HIPCHK(hipMemcpy(path_rays, s->d_path_rays, n_paths * 4, hipMemcpyDeviceToHost));
    return MRT_OK;
}

// work_queue::getPercentDone (work_queue.cpp:142-175): paths handed out over all paths of the
// render, callable from another host thread while the render runs.  Needs no GPU work: a finished
// launch counts whole (its stop event), a running one by the snapshot of its work counter that
// the path kernel stores into host memory, a launch not yet started as 0.
extern "C" mrt_status mrt_progress(mrt_scene* s, float* pct) {
    if (!s || !pct) return mrt_internal_fail(MRT_ERR_INVALID, "mrt_progress: null");
    *pct = 0.0f;
    if (s->cpu) return mrt_cpu_progress(s->cpu, pct);
    std::lock_guard<std::mutex> lk(s->prog_mu);
    const size_t n = s->n_chunks.load(std::memory_order_acquire);
    if (n == 0 || !s->h_prog || s->h_prog_cap < s->prog_base + n || s->ev.size() < 2 * n || s->h_seen.size() < n * MRT_NPART) return MRT_OK;  // not started
    double done = 0, total = 0;
    for (size_t k = 0; k < n; k++) {
        total += (double)s->chunk_paths[k];
        if (hipEventQuery(s->ev[2 * k + 1]) == hipSuccess) {
            done += (double)s->chunk_paths[k];
        } else if (hipEventQuery(s->ev[2 * k]) == hipSuccess) {
            // one snapshot per work partition (the paths it has handed out); snapshots from
            // different waves land out of order: report the largest seen so far
            const uint64_t np = s->chunk_paths[k];
            for (uint32_t j = 0; j < MRT_NPART; j++) {
                uint64_t c = __atomic_load_n(&s->h_prog[(s->prog_base + k) * MRT_NPART + j], __ATOMIC_RELAXED);
                c = std::max(c, s->h_seen[k * MRT_NPART + j]);
                s->h_seen[k * MRT_NPART + j] = c;
                done += (double)std::min<uint64_t>(c, np * (j + 1) / MRT_NPART - np * j / MRT_NPART);
            }
        }
    }
    *pct = total > 0 ? (float)std::min(100.0, done * 100.0 / total) : 0.0f;
    return MRT_OK;
}

// The UI thread's view of G_linearBackBuffer (main.cpp:387-444) without stopping the render: the
// newest snapshot whose sequence word was even, and unchanged, around the copy out of pinned memory.
extern "C" mrt_status mrt_preview(mrt_scene* s, float* rgb_out, uint32_t* samples_done) {
    if (!s || !rgb_out || !samples_done) return mrt_internal_fail(MRT_ERR_INVALID, "mrt_preview: null");
    *samples_done = 0;
    if (s->cpu) return mrt_cpu_preview(s->cpu, rgb_out, samples_done);
    std::lock_guard<std::mutex> lk(s->prog_mu);
    if (!s->h_seq || !s->h_prev || s->prev_px.empty()) return MRT_OK;  // no preview render yet
    std::vector<float4> snap(s->prev_px.size());
    for (int tries = 0; tries < 1000; tries++) {
        const uint32_t a = __atomic_load_n(s->h_seq, __ATOMIC_ACQUIRE);
        if (a == 0) return MRT_OK;  // nothing folded yet
        if (a & 1u) {               // a copy is landing: the previous one is being overwritten
            usleep(50);
            continue;
        }
        const uint32_t n = __atomic_load_n(s->h_seq + 1, __ATOMIC_ACQUIRE);
        memcpy(snap.data(), s->h_prev, snap.size() * 16);
        __atomic_thread_fence(__ATOMIC_ACQUIRE);
        if (__atomic_load_n(s->h_seq, __ATOMIC_ACQUIRE) != a) continue;  // torn: retry
        for (size_t i = 0; i < snap.size(); i++) memcpy(rgb_out + (size_t)s->prev_px[i] * 4, &snap[i], 16);
        *samples_done = n;
        return MRT_OK;
    }
    return MRT_OK;  // the render outran every attempt: report nothing rather than a torn image
}

extern "C" mrt_status mrt_set_worker_seeds(mrt_scene* s, uint32_t n_threads, const uint64_t* initstate, const uint64_t* initseq) {
    if (!s) return mrt_internal_fail(MRT_ERR_INVALID, "mrt_set_worker_seeds: null");
    if (!s->cpu)
        return mrt_internal_fail(MRT_ERR_INVALID, "mrt_set_worker_seeds: the reference's per-thread RNG order is a CPU-backend mode "
                                                  "(the GPU keys its PCG streams per path)");
    return mrt_cpu_set_worker_seeds(s->cpu, n_threads, initstate, initseq);
}

extern "C" mrt_status mrt_scene_kernel_info(const mrt_scene* s, mrt_kernel_info* out) {
    if (!s || !out) return mrt_internal_fail(MRT_ERR_INVALID, "mrt_scene_kernel_info: null");
    out->features = s->features;
    if (s->cpu) {  // the host instantiation that runs it (mrt_cpu.hip), threads of the last render
        float ms;
        uint32_t threads = 0;
        mrt_cpu_last_ms(s->cpu, &ms, &threads);
        *out = mrt_kernel_info{};
        out->features = s->features;
        out->kernel_features = (s->features & FT_LIN) ? (FT_LIN | FT_ALL) : FT_ALL;
        out->grid = threads;
        return MRT_OK;
    }
    out->kernel_features = kVariants[s->variant];
    const PathLaunch& L = s->pl[s->last_numerics];
    out->lds_bytes = (uint32_t)L.lds_bytes;
    out->grid = (uint32_t)L.grid;
    out->prog_ops = s->prog_ops;
    out->vgprs = L.vgprs;
    out->wg = L.wg;
    out->tree_nodes = L.tree_n;  // BvhWide nodes per workgroup
    out->build = s->last_numerics == 0 ? MRT_BUILD_EXACT
               : L.fn == kernel_table_fast_pex().kernel[s->variant] ? MRT_BUILD_PATH_EXACT
               : L.fn == kernel_table_fast_ftz().kernel[s->variant] ? MRT_BUILD_FAST_FTZ
                                                                     : MRT_BUILD_FAST;
    out->pad = 0;
    out->handed_over = 0;
    out->handover_lost = 0;
    if (s->d_counter) {
        // after the scene's last render, its fold included: ev_done is recorded on the render's
        // stream (or the context's fold stream), which the legacy null stream of a plain hipMemcpy
        // is not ordered after
        HIPCHK(hipSetDevice(s->device));
        if (s->ev_done_pending) HIPCHK(hipEventSynchronize(s->ev_done));
        uint64_t n[6] = {};
        if (hipMemcpy(n, s->d_counter, sizeof n, hipMemcpyDeviceToHost) != hipSuccess)
            return mrt_internal_fail(MRT_ERR_HIP, "mrt_scene_kernel_info: counter read");
        out->handed_over = n[0];
        out->handover_lost = n[5];
    }
    return MRT_OK;
}

extern "C" mrt_status mrt_kernel_ms(mrt_scene* s, float* path_ms, uint32_t* launches) {
    if (!s || !path_ms) return mrt_internal_fail(MRT_ERR_INVALID, "mrt_kernel_ms: null");
    if (s->cpu) {  // wall time of the last CPU render
        if (launches) *launches = 1;
        return mrt_cpu_last_ms(s->cpu, path_ms, nullptr);
    }
    HIPCHK(hipSetDevice(s->device));
    float total = 0;
    for (uint32_t k = 0; k < s->n_launch; k++) {
        HIPCHK(hipEventSynchronize(s->ev[2 * k + 1]));
        float ms = 0;
        HIPCHK(hipEventElapsedTime(&ms, s->ev[2 * k], s->ev[2 * k + 1]));
        total += ms;
    }
    *path_ms = total;
    if (launches) *launches = s->n_launch;
    return MRT_OK;
}
