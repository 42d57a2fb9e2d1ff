// mrt_kernels.hip -- the path kernel (DESIGN.md "Kernels"), built three times from this one source:
//   build/obj/mrt_kernels_exact.o  MRT_FAST=0, -ffp-contract=off: the exact numerics contract,
//                                  bit-for-bit the reference built exact (tests/golden/stream_*.npz)
//   build/obj/mrt_kernels_fast.o   MRT_FAST=1, FMA contraction + reciprocal division + hardware
//                                  rcp/sqrt/rsq + f32 transcendentals: the tolerance contract
//                                  (per-pixel RMSE < 1e-3 vs the reference as shipped)
//   build/obj/mrt_kernels_fastz.o  the tolerance contract with f32 denormals flushed, for the
//                                  variants mrt_launch.h's kFtzVariant selects
// Each build exports its KernelTable (mrt_launch.h); the host picks one per render
// (mrt_render_desc.flags & MRT_RF_FAST), the fast one merged with the FTZ build's variants.
//
// mrt_path_kernel: persistent waves pull 256-path batches (64 near the end of a launch) from
// per-XCD partition counters (one atomic per wave per batch, like work_queue::getWork pulls a tile,
// work_queue.cpp:158-166) and run trace() for each lane's path to completion; per-path radiance
// is written sample-major [s][local pixel] (coalesced).
#include <hip/hip_runtime.h>
#include <cstddef>
#include <utility>

#include "mrt_launch.h"

using namespace mrtd;

// which table this build provides (experiments may build the "fast" slot with other switches)
#ifndef MRT_TABLE_FAST
#define MRT_TABLE_FAST MRT_FAST
#endif
// the third build: the tolerance contract with f32 denormals flushed (-fgpu-flush-denormals-to-zero),
// for the variants kFtzVariant selects (mrt_launch.h)
#ifndef MRT_TABLE_FTZ
#define MRT_TABLE_FTZ 0
#endif
// the fourth: exact arithmetic + forward fold, the tolerance contract's kPathExact variants
#ifndef MRT_TABLE_PEX
#define MRT_TABLE_PEX 0
#endif
#if MRT_TABLE_PEX
#define MRT_PATH_KERNEL mrt_path_kernel_pex
#elif MRT_TABLE_FTZ
#define MRT_PATH_KERNEL mrt_path_kernel_fastz
#elif MRT_TABLE_FAST
#define MRT_PATH_KERNEL mrt_path_kernel_fast
#else
#define MRT_PATH_KERNEL mrt_path_kernel
#endif


// Persistent waves with per-lane path regeneration: every loop iteration advances each busy lane
// by one segment (one trace() call); a lane whose path ended takes the next path index from its
// wave's pool at once (ballot + mbcnt compaction), and a wave refills its pool 64 paths at a time
// with one atomic (work_queue::getWork, work_queue.cpp:158-166).  Lanes stay busy until the pool
// runs dry instead of idling until the longest path of a 64-path batch finishes.
// Waves per SIMD the register allocator must reach (caps VGPRs at 512/W): the path loop is
// latency-bound, so a few spilled registers cost less than the lost occupancy.  Tuned per
// variant on MI355X (DESIGN.md "Occupancy").
// (compact variants -- Cornell, Cornell room + mesh, plain interpreter -- reach 80 VGPRs without
// spills at 6; built without SLP vectorisation (Makefile), the wide-feature variants run best at
// 6 waves (80 VGPRs; round 4, with MRT_TREE_WG 768: 4 waves before) and the room + mesh variant
// at 7 (72 VGPRs, no LDS fold levels))
#ifndef MRT_WPE_WIDE
#define MRT_WPE_WIDE (MRT_FAST ? 6 : 4)
#endif
#ifndef MRT_WPE_LIN
#define MRT_WPE_LIN (MRT_FWD_FOLD ? 7 : 6)  // forward fold: no LDS levels, 72 VGPRs (C2 +1%)
#endif
#ifndef MRT_WPE_MESH
#define MRT_WPE_MESH 7
#endif
// the room + mesh walk of the tolerance contract, fast arithmetic (C3) and path-exact (C4): 8 waves
// (fast: 62 VGPRs, no VGPR spill; path-exact: 64, 9 spilled).  Round 5 against 7: teapot 17.01 vs
// 17.51 ms per step, bunny 40.60 vs 41.07 (profiles/r05_ab.txt sections 22-23)
#ifndef MRT_WPE_ROOM_MESH
#define MRT_WPE_ROOM_MESH ((MRT_FAST || MRT_TABLE_PEX) ? 8 : MRT_WPE_MESH)
#endif
#ifndef MRT_WPE_LIN_GEN
// the interpreter's compact variants (no program shape): 6 waves (80 VGPRs, spill-free).  Round 4
// held them at 5 (96 VGPRs): the room op's per-lane axis select had become a lookup table in
// scratch, which kept the query ray in scratch memory; with sel3 it is gone, 81 VGPRs at 5 waves
// (C2 through the interpreter 43.3 -> 46.4 Grays/s), 80 at 6 (47.7), 72 + 5 spilled at 7 (44.1;
// profiles/r05_ab.txt section 6)
// The exact contract's interpreter kernels keep 5 (96 VGPRs): at 6 the exact arithmetic spilled 39
// VGPRs (C2 through the interpreter, exact: 45.2 ms per step at 6, 40.3 at 5, 43.5 at 4 waves,
// round 6, profiles/r06_ab.txt section 4)
#define MRT_WPE_LIN_GEN (MRT_FAST || MRT_TABLE_PEX ? 6 : 5)
#endif
template <uint32_t F> struct PathOcc {
    static constexpr bool kWide = (F & (FT_BVHW | FT_TEX | FT_VOLUME)) != 0 || !(F & FT_LIN);
    static constexpr int W = kWide ? (!(F & FT_LIN) ? 4 : MRT_WPE_WIDE)
                             : ((F & FT_MESH) != 0 ? (MRT_SIG_OF(F) == SIG_ROOM_MESH ? MRT_WPE_ROOM_MESH : MRT_WPE_MESH)
                                                   : (MRT_SIG_OF(F) != SIG_NONE ? MRT_WPE_LIN : MRT_WPE_LIN_GEN));
};
#if defined(MRT_EXPERIMENTS) && defined(MRT_PHASES)  // build ONE of the two TUs with it
__device__ unsigned long long g_phases[12];
extern "C" int mrt_debug_phases(unsigned long long* out, int reset) {
    if (hipMemcpyFromSymbol(out, HIP_SYMBOL(g_phases), sizeof(g_phases)) != hipSuccess) return 1;
    if (reset) {
        unsigned long long z[12] = {0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0};
        if (hipMemcpyToSymbol(HIP_SYMBOL(g_phases), z, sizeof(z)) != hipSuccess) return 1;
    }
    return 0;
}
#endif
// Launch end.  A wave whose partition is handed out takes work from ONE other partition (chosen
// per wave group in four directions, MRT_STEAL_SPREAD), in small claims, then ends.  Visiting all
// eight (the round-2 rule) cost every wave 8 failing atomics at the launch's end, on 8 addresses
// hit by all 7168 waves at once: 3.5-4 us each against 0.6 us for a claim mid-launch (wave
// timelines, tools/wtimes.py), while the wave's in-flight lanes waited -- a fixed ~40 us per launch,
// 4% of an 8-rank share.  Every partition is still finished by its own waves.
#ifndef MRT_STEAL_SMALL
#define MRT_STEAL_SMALL 1
#endif
#ifndef MRT_STEAL_TRIES
#define MRT_STEAL_TRIES 2u  // partitions a wave takes work from (its own first) before it ends
#endif
#ifndef MRT_STEAL_SPREAD
#define MRT_STEAL_SPREAD 1
#endif
#if defined(MRT_EXPERIMENTS) && defined(MRT_WTIMES)  // build ONE of the two TUs with it
// per wave of the last launch: start, pool exhausted, end (s_memrealtime, 100 MHz), workgroup
// + time inside successful / failed claim atomics (10-ns ticks) and their counts (ok | fail << 32)
__device__ unsigned long long g_wtimes[7 * 16384];
#if (MRT_TABLE_FTZ || !MRT_TABLE_FAST) && !MRT_TABLE_PEX  // the reader in one TU only (the FTZ build runs the Cornell kernels)
extern "C" int mrt_debug_wtimes(unsigned long long* out, int n) {
    return hipMemcpyFromSymbol(out, HIP_SYMBOL(g_wtimes), sizeof(unsigned long long) * 7 * (size_t)n) != hipSuccess;
}
#endif
#define WT_MARK(v) (v) = __builtin_amdgcn_s_memrealtime()
#else
#define WT_MARK(v) (void)0
#endif
#if defined(MRT_EXPERIMENTS) && defined(MRT_BSTATS)  // build ONE of the two TUs with it
namespace mrtd { __device__ unsigned long long g_bstats[64]; }
extern "C" int mrt_debug_bstats(unsigned long long* out, int reset) {
    if (hipMemcpyFromSymbol(out, HIP_SYMBOL(mrtd::g_bstats), sizeof(g_bstats)) != hipSuccess) return 1;
    if (reset) {
        unsigned long long z[64] = {};
        if (hipMemcpyToSymbol(HIP_SYMBOL(mrtd::g_bstats), z, sizeof(z)) != hipSuccess) return 1;
    }
    return 0;
}
#endif
// resumable mesh walk (room + mesh kernels): the walk loop returns the wave to shading / new rays
// once at most P.walk_min lanes still walk (set on upload from the mesh BVH's size: 32, or 40 for
// BVHs of >= 2048 inner nodes -- measured: bunny, 2937 inner nodes, best at 40 (+4% over 32);
// teapot, ~1045, at 28-32 (40: -3%)) and at least MRT_WALK_OTHER lanes have other work
#ifndef MRT_WALK_OTHER
#define MRT_WALK_OTHER 16u
#endif
// walk steps between two yield checks of the resumable mesh walk (round 6: 2 against 1, teapot +1.5%,
// bunny +0.8%; 3: +1.0% / +0.6%, profiles/r06_ab.txt section 8)
// Path starts batched in the resumable mesh loop (round 6): the lanes whose path ended start new
// ones only once at least MRT_START_MIN of the wave's lanes are idle (or none is busy), so the path
// start (claim, PCG seeding, the camera ray with its disk-rejection draws) runs at a wider lane
// mask; the idle lanes wait for it through a walk.  Measured (profiles/r06_ab.txt section 13):
// teapot (fast) +0.6% at 8, +2.9% at 16; bunny (path-exact) +0.9% at 8, -1.2% at 16.  The plain loop
// (bvh_node scenes: book2 -0.1% / -1.0%, random spheres +0.5% / -0.3%) keeps 1 (MRT_START_MIN_PLAIN).
#ifndef MRT_START_MIN
#define MRT_START_MIN (MRT_FAST ? 16u : 8u)
#endif
#ifndef MRT_START_MIN_PLAIN
#define MRT_START_MIN_PLAIN 1u
#endif
#ifndef MRT_WALK_UNROLL
#define MRT_WALK_UNROLL 2
#endif
// Leaf postponing in the resumable mesh walk (mrt_trace.h mesh_step_spec): the path-exact build
// (the metal bunny, C4) chooses per step between a leaf step and an inner step by majority
// (MRT_SPEC_LEAF 0): bunny +0.8%; the fast build (teapot, C3) keeps mesh_step (-5.5% with it); a leaf
// step once 8 / 16 / 32 / 48 runs are parked: bunny -10% / -2.2% / -19% / -58% (profiles/r06_ab.txt
// sections 8 and 14)
#ifndef MRT_MESH_SPEC
#define MRT_MESH_SPEC MRT_TABLE_PEX
#endif
#ifndef MRT_SPEC_LEAF
#define MRT_SPEC_LEAF 0u
#endif
#if defined(MRT_EXPERIMENTS) && defined(MRT_WPE)  // experiment hook: override for every variant
#define MRT_OCC(F) MRT_WPE
#else
#define MRT_OCC(F) PathOcc<F>::W
#endif
// fold levels kept in LDS per lane (the rest in HBM): where the LDS budget at the target
// occupancy allows it
// (Cornell: 2 at 6 WGs/CU; wide variants at 3 WGs/CU: MRT_LEVK_WIDE; room + mesh: MRT_LEVK_MESH)
#ifndef MRT_LEVK_CORNELL
#define MRT_LEVK_CORNELL 2u
#endif
#ifndef MRT_LEVK_WIDE
#define MRT_LEVK_WIDE 2u
#endif
#ifndef MRT_LEVK_MESH
#define MRT_LEVK_MESH 0u
#endif
template <uint32_t F> struct PathLevLds {
    static constexpr uint32_t K = MRT_FWD_FOLD ? 0u  // no stored levels
                                  : ((F & 0xFFFFu & ~FT_BIASED) == (FT_LIN | FT_INST)) ? MRT_LEVK_CORNELL
                                  : PathOcc<F>::kWide                  ? MRT_LEVK_WIDE
                                  : ((F & FT_MESH) != 0)               ? MRT_LEVK_MESH
                                                                       : 0u;
};
// Path starts made a wave at a time (see the path loop): on in the tolerance-contract build for the
// shared-constructor loop of one-wave workgroups
#ifndef MRT_PATHQ
#define MRT_PATHQ MRT_FAST
#endif
// the plain path loop reads the scene's kernel arguments through an opaque pointer each iteration
// (round 5: book2 -1.5%, random spheres -1% per step; SGPR spills of book2's kernel 110 -> 35; in
// the Cornell kernels' shared-constructor loop it removed their 4 SGPR spills but not a step's time:
// 8.648 vs 8.655 ms, three rounds, not kept)
#ifndef MRT_OPAQUE_SCENE
#define MRT_OPAQUE_SCENE 1
#endif
// rounding-critical light samples handed to the exact arithmetic (mrt_shade.h light_critical): the
// fast-arithmetic builds' light-sampled variants (MRT_CRIT=0 builds it out: A/B)
#ifndef MRT_CRIT
#define MRT_CRIT 1
#endif
template <uint32_t F>
static constexpr bool kCrit = MRT_CRIT && MRT_FAST && (F & FT_BIASED) != 0;
// where crit_check finds the launch's list: PathParams (the kernel's only argument) starts the
// argument segment
template <uint32_t F>
static constexpr uint32_t kCritOff = kCrit<F> ? (uint32_t)offsetof(PathParams, rt) : 0u;
// the path kernel's scene arguments (P.sc) through an opaque pointer into the argument segment (P is
// the kernel's only argument: it starts the segment): read where used, not held in registers
MRT_DFN const DScene& kernarg_scene() {
    const MRT_CONST_AS DScene* sp =
        (const MRT_CONST_AS DScene*)((const MRT_CONST_AS char*)__builtin_amdgcn_kernarg_segment_ptr() + offsetof(PathParams, sc));
    asm volatile("" : "+s"(sp));
    return *(const DScene*)sp;
}
#ifndef MRT_OPAQUE_RESUME
#define MRT_OPAQUE_RESUME 0  // the same in the room + mesh kernels' resumable loop: measured C3 -0.6%, C4 0 (A/B hook)
#endif
template <uint32_t F> struct PathQ {
    static constexpr bool on = MRT_PATHQ && (F & FT_MESH) == 0 && !TreeOf<F>::on;
    // LDS words per lane slot: o, dir, time, PCG state + inc, index (12); + the wave's claim state
    static constexpr uint32_t words = on ? 13u : 0u;
};
template <uint32_t F>
__global__ void __launch_bounds__(TreeOf<F>::wg) __attribute__((amdgpu_waves_per_eu(MRT_OCC(F)))) MRT_PATH_KERNEL(PathParams P) {
    constexpr uint32_t LK = PathLevLds<F>::K;
    extern __shared__ __attribute__((aligned(16))) uint32_t lds[];
    const uint32_t lane = threadIdx.x & 63u;
    const uint32_t wave = threadIdx.x >> 6;
    // per wave: its stacks and queues ([slot][word][lane])
    const uint32_t words = (P.lds_frames * 2 + P.lds_rays * 11 + P.lds_mesh + P.lds_save + LK * 4 + PathQ<F>::words) * 64;
    uint32_t* wb = lds + wave * words;
    uint32_t* const wmesh = wb + P.lds_frames * 128 + P.lds_rays * 704;
    float4* tree = nullptr;
    if constexpr (TreeOf<F>::on) {
        // the workgroup's copy of the top wide nodes (after every wave's own region), filled once
        // before any wave starts a path; no other barrier follows in this persistent kernel
        tree = reinterpret_cast<float4*>(lds + (TreeOf<F>::wg / 64u) * words);
        for (uint32_t i = threadIdx.x; i < P.tree_n * 4u; i += blockDim.x) tree[i] = P.tree_src[i];
        __syncthreads();
    }
    const LStack Ls{wb, (float*)(wb + P.lds_frames * 128), wmesh, (float*)(wmesh + P.lds_mesh * 64), lane, tree,
                    TreeOf<F>::on ? P.tree_n : 0u};
    // the wave's queue of path starts ([word][entry], PathQ): after the fold levels
    float* const Lq = (float*)(wmesh + (P.lds_mesh + P.lds_save + LK * 4) * 64);
    const DScene& S = P.sc;
    const size_t slot = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    const LevStore<LK> lev{(MRT_GLOBAL_AS v4f*)P.lev, P.lev_rows, (uint32_t)slot,
                           (uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)(uintptr_t)(MRT_LDS_AS uint32_t*)(wmesh + (P.lds_mesh + P.lds_save) * 64))};
    // set bits of a wave mask below this lane (v_mbcnt: no per-lane 64-bit mask kept live)
    auto rank_below = [](uint64_t m) -> uint32_t {
        return __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
    };

    // main.cpp:180/235 stop on !G_isRunning: a launch of a cancelled render does no work (mrt_render
    // splits a cancellable render into several launches)
    if (__hip_atomic_load(P.cancel, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM)) return;
#if defined(MRT_EXPERIMENTS) && defined(MRT_WTIMES)
    uint64_t wt0 = 0, wt_ex = 0, wt1 = 0, wt_f = 0, wt_aok = 0, wt_afail = 0, wt_n = 0;
    WT_MARK(wt0);
#endif
    bool active = false;
    uint32_t idx = 0;
    PathState ps;
    // The launch's paths are split into MRT_NPART equal contiguous partitions, one work counter
    // each (128 B apart): the waves of workgroup b start on partition b % MRT_NPART -- the XCD the
    // workgroup is dispatched to, round robin -- and move on to the next partition once theirs is
    // handed out.  One counter for all 7168 waves serialised ~1 M claims per C2 launch on one
    // address (measured: claims 4x larger, 1024 paths, made the kernel 14% faster).
    // Every wave's first claim is static (the waves of a partition take its first batches in order);
    // its counter hands out what follows, so a launch does not open with one atomic per wave (short
    // launches only -- P.static_first, set by the host when a wave gets fewer than 64 claims: there
    // the opening atomics are a visible share; in long launches the static batch of a wave that
    // starts late in a pipelined step delays that launch's end).
    auto umin64 = [](uint64_t a, uint64_t b) -> uint64_t { return a < b ? a : b; };
    // wave-uniform values kept in SGPRs (the compiler otherwise held the pool bounds in VGPRs and
    // spilled them to scratch, reloaded every claim)
    auto uni64 = [](uint64_t x) -> uint64_t {
        return ((uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)(x >> 32)) << 32) |
               (uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)x);
    };
    const uint32_t wpb = blockDim.x >> 6;  // waves per workgroup
    uint32_t part = blockIdx.x % MRT_NPART;  // wave-uniform: the partition claims come from
    uint32_t part_tries = 0;                 // partitions found handed out
    // the partitions a wave visits after its own: every one (step odd, coprime with 8); with
    // MRT_STEAL_SPREAD the waves of one partition leave it in four directions instead of one
    const uint32_t steal_step = MRT_STEAL_SPREAD ? 1u + 2u * ((blockIdx.x / MRT_NPART) & 3u) : 1u;
    bool in_tail = false;                    // the partition's last paths: small claims
    uint64_t pool_next = 0, pool_end = 0;    // wave-uniform: the wave's claimed, not yet taken paths
    if (P.static_first) {
        pool_next = uni64(umin64(P.part_base[part] + ((uint64_t)(blockIdx.x / MRT_NPART) * wpb + wave) * MRT_BATCH, P.part_base[part + 1]));
        pool_end = uni64(umin64(pool_next + MRT_BATCH, P.part_base[part + 1]));
    }
    bool exhausted = false;  // no paths left in the pool nor in any partition
    // Queue kernels keep the claim state (pool bounds, partition) in LDS between claims -- it is
    // touched once per 64 path starts -- so it holds no registers across the path loop (held in
    // registers it cost VGPR spills to scratch: 1.2 GB/launch of extra HBM writes on C2).
    uint32_t* const Lc = reinterpret_cast<uint32_t*>(Lq + 12u * 64u);
    auto cold_store = [&]() {
        if (lane == 0) {
            Lc[0] = (uint32_t)pool_next;
            Lc[1] = (uint32_t)(pool_next >> 32);
            Lc[2] = (uint32_t)pool_end;
            Lc[3] = (uint32_t)(pool_end >> 32);
            Lc[4] = part | (part_tries << 8) | ((uint32_t)in_tail << 16);
        }
    };
    auto cold_load = [&]() {
        auto rd = [&](uint32_t k) { return (uint32_t)__builtin_amdgcn_readfirstlane((int)Lc[k]); };
        pool_next = (uint64_t)rd(0) | ((uint64_t)rd(1) << 32);
        pool_end = (uint64_t)rd(2) | ((uint64_t)rd(3) << 32);
        const uint32_t w = rd(4);
        part = w & 0xFFu;
        part_tries = (w >> 8) & 0xFFu;
        in_tail = ((w >> 16) & 1u) != 0;
    };
    if constexpr (PathQ<F>::on) cold_store();
    uint32_t done_rays = 0;
    PhaseClock ph{};
#ifdef MRT_PHASES
    ph.t = __builtin_amdgcn_s_memtime();
#endif
    // Lanes without a path take the next path indices from the wave's pool (ballot + mbcnt
    // compaction), the pool refilled by one atomic per claim (work_queue::getWork,
    // work_queue.cpp:158-166).  start(u, v) begins a lane's path at camera coordinates (u, v) with
    // its PCG stream seeded from the path key.
    // path index -> its camera coordinates (u, v) and its PCG stream seeded from the path key
    auto path_key = [&](uint32_t i, Pcg& rng, float* uo, float* vo) { path_key_of(P, i, rng, uo, vo); };
    // the next c path indices of the wave's pool, the lane of rank r taking index *i (>= n_paths:
    // none); the pool refilled by one atomic per claim (work_queue::getWork, work_queue.cpp:158-166)
    auto claim = [&](uint32_t c, uint32_t r, bool want, uint64_t* i) {
        const uint32_t have = (uint32_t)(pool_end - pool_next);
        uint64_t nb = 0, ne = 0;
        if (have < c) {
            while (part_tries < MRT_STEAL_TRIES) {  // wave-uniform
                const uint64_t pe = P.part_base[part + 1], p0 = P.part_dyn[part];
                const uint32_t batch = in_tail ? MRT_TAIL_BATCH : MRT_BATCH;
#if defined(MRT_EXPERIMENTS) && defined(MRT_WTIMES)
                uint64_t wt_a = 0;
                WT_MARK(wt_a);
#endif
                if (lane == 0) {
                    nb = p0 + atomicAdd(P.counter + part * MRT_COUNTER_STRIDE, (unsigned long long)batch);
                    // every 32nd claim: a system-scope store to host memory, read by mrt_progress
                    // without any GPU queue (a device-to-host copy could wait behind this launch)
                    if (P.hprog && (((nb - p0) / batch) & 31u) == 0)
                        __hip_atomic_store(P.hprog + part, nb + batch - P.part_base[part], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
                }
                // lane 0's claim to every lane, as a scalar (the whole wave runs claim())
                nb = ((uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)(nb >> 32)) << 32) |
                     (uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)nb);
#if defined(MRT_EXPERIMENTS) && defined(MRT_WTIMES)
                {
                    uint64_t wt_b = 0;
                    WT_MARK(wt_b);
                    if (nb < pe) { wt_aok += wt_b - wt_a; wt_n += 1; }
                    else { wt_afail += wt_b - wt_a; wt_n += 1ull << 32; }
                }
#endif
                if (nb < pe) {
                    ne = umin64(nb + batch, pe);
                    // near the partition's end, claims shrink so the last ones finish together
#if MRT_STEAL_SMALL
                    in_tail = pe - ne <= P.tail_zone / MRT_NPART;
#else
                    in_tail = in_tail || pe - ne <= P.tail_zone / MRT_NPART;
#endif
                    break;
                }
#if defined(MRT_EXPERIMENTS) && defined(MRT_WTIMES)
                if (wt_f == 0) WT_MARK(wt_f);
#endif
                part_tries++;
                part = (part + steal_step) % MRT_NPART;
                // (MRT_STEAL_SMALL: the first claim on the next partition is a small one -- it is
                // usually in its own tail zone -- and the claim's position decides the next size)
                in_tail = MRT_STEAL_SMALL;
            }
        }
        if (want) {
            const uint64_t j = nb + (r - have);
            *i = r < have ? pool_next + r : (j < ne ? j : ~0ull);
        }
        if (have < c) {
            pool_next = umin64(nb + (c - have), ne);
            pool_end = ne;
        } else {
            pool_next += c;
        }
        exhausted = part_tries >= MRT_STEAL_TRIES && pool_next >= pool_end;
#if defined(MRT_EXPERIMENTS) && defined(MRT_WTIMES)
        if (exhausted && wt_ex == 0) WT_MARK(wt_ex);
#endif
    };
    auto begin_path = [&]() {
        ps.depth = 0;
        ps.nlev = 0;
#if MRT_FWD_FOLD
        ps.T = f3{1.0f, 1.0f, 1.0f};
#endif
        active = true;
    };
    // Lanes without a path take the next path indices from the wave's pool (ballot + mbcnt
    // compaction).  start(u, v) begins a lane's path at camera coordinates (u, v).
    auto take_paths = [&](auto&& start) {
        const uint64_t need = __ballot(!active);
        if (!need || exhausted) return;
        const uint32_t c = (uint32_t)__popcll(need);
        uint64_t i = 0;
        claim(c, active ? 0u : rank_below(need), !active, &i);
        PH_MARK(ph, 0);
        if (!active && i < P.n_paths) {
            idx = (uint32_t)i;
            BSTAT(10);
            float u, v;
            path_key(idx, ps.rng, &u, &v);
            start(u, v);
            begin_path();
        }
        PH_MARK(ph, 4);
    };
    // a finished path: the recursion's fold, radiance out (sample-major, coalesced), rays counted
    auto finish_path = [&](f3 L) {
        L = end_path(ps, lev, L);
        PH_MARK(ph, 5);
        float* dst = P.rad + (size_t)idx * 3;
#if defined(MRT_EXPERIMENTS) && defined(MRT_EXP_NOSTORE)  // experiment: what the radiance store costs
        if (__float_as_uint(L.x) == 0x7fc00123u) {
#endif
        dst[0] = L.x;
        dst[1] = L.y;
        dst[2] = L.z;
#if defined(MRT_EXPERIMENTS) && defined(MRT_EXP_NOSTORE)
        }
#endif
        if (P.path_rays) P.path_rays[idx] = ps.rays();
        done_rays += ps.rays();
        active = false;
    };
    // mesh variants keep one constructor per branch: the shared-constructor loop spills there
    // (bunny -4%, teapot -5%; Cornell +1.8%, book2 0)
#ifndef MRT_SHARED_WIDE
#define MRT_SHARED_WIDE 0  // not the wide (bvh_node) variants: the plain loop has 6 spills instead of 29 there
                           // (random spheres +4.4%, scene 1 +5%; profiles/r03_ab.txt)
#endif
    constexpr bool kShared = (F & FT_MESH) == 0 && (MRT_SHARED_WIDE || !PathOcc<F>::kWide);
    constexpr bool kResume = MRT_SIG_OF(F) == SIG_ROOM_MESH;
    if constexpr (kShared) {
        // One iteration: (1) every lane with a ray traces one segment; a path that ends is folded
        // and stored; (2) lanes without a path take new ones (camera ray arguments); (3) ONE
        // make_ray for every lane with a next ray -- camera and scattered rays alike, instead of one
        // constructor per branch at partial lane occupancy; (4) diffuse scatters finish their pdfs
        // on the new ray.
        uint32_t q_head = 0, q_n = 0;  // wave-uniform: the queue's next entry, its valid entries
        // The radiance store of a path that ended is held in registers and issued in the NEXT
        // iteration, after the hit, beside the material load: the code waits for the vector memory
        // counter (stores count in vmcnt on gfx950) right after a store wherever it reuses nearby
        // registers, which stalled the wave for the store's whole round trip every iteration
        // (measured: SQ_WAIT_ANY 23 -> 36 quad-cycles per ray once the path loop had fewer
        // instructions); beside the material load the two round trips overlap.
        f3 st_v{0.0f, 0.0f, 0.0f};
        uint32_t st_off = 0;  // byte offset of the path's radiance (a launch chunk is < 4 GiB)
        bool st_pend = false;
        for (;;) {
            bool want_ray = false;
            // the next ray's arguments: written and read within one iteration (declared here, a
            // field a branch leaves unset is dead, not carried round the loop in copied registers)
            PendRay pr;
            if (active) {
                f3 L{0.0f, 0.0f, 0.0f};  // (left undefined, it was carried round the loop in copied registers)
                // (the held store is issued inside, after the hit, beside the material load)
                const bool ended = trace_split<F, LK>(S, ps, P.max_bounces, lev, Ls, &L, &pr, ph, [&]() {
                    if (st_pend) {
                        float* dst = reinterpret_cast<float*>(reinterpret_cast<char*>(P.rad) + st_off);
                        dst[0] = st_v.x;
                        dst[1] = st_v.y;
                        dst[2] = st_v.z;
                    }
                    st_pend = false;
                }, CritSink{idx, kCritOff<F>});
                PH_MARK(ph, 2);
                if (ended) {
                    st_v = end_path(ps, lev, L);
                    st_off = idx * 12u;
                    st_pend = true;
                    if (P.path_rays) P.path_rays[idx] = ps.rays();
                    done_rays += ps.rays();
                    active = false;
                } else {
                    want_ray = true;
                }
            }
            PH_MARK(ph, 3);
            if constexpr (PathQ<F>::on) {
                // new paths from the wave's queue of path starts; when it runs short, the next 64
                // starts are made at once, one per lane at full width (path key, PCG seeding, the
                // camera's disk-rejection and time draws), instead of by the ~1/3 of lanes whose
                // path just ended: the same paths with the same streams, in the same order
                auto pop = [&](uint32_t e) {
                    const float* q = Lq + e;
                    pr.o = f3{q[0], q[64], q[128]};
                    pr.dir = f3{q[192], q[256], q[320]};
                    pr.time = q[384];
                    ps.rng.state = (uint64_t)__float_as_uint(q[448]) | ((uint64_t)__float_as_uint(q[512]) << 32);
                    ps.rng.inc = (uint64_t)__float_as_uint(q[576]) | ((uint64_t)__float_as_uint(q[640]) << 32);
                    idx = __float_as_uint(q[704]);
                    pr.inside = 0;
                    pr.kind = 0;
                    want_ray = true;
                    begin_path();
                };
                const uint64_t need = __ballot(!active);
                const uint32_t c = (uint32_t)__popcll(need);
                const uint32_t avail = q_n - q_head;
                if (c != 0u && (avail != 0u || !exhausted)) {
                    const uint32_t rank = active ? 64u : rank_below(need);
                    if (rank < avail) pop(q_head + rank);
                    if (c <= avail) {
                        q_head += c;
                    } else {
                        q_head = q_n = 0;
                        if (!exhausted) {
                            uint64_t i = 0;
                            cold_load();
                            claim(64u, lane, true, &i);
                            cold_store();
                            const bool valid = i < P.n_paths;
                            if (valid) {
                                BSTAT(10);
                                Pcg rng;
                                float u, v, time;
                                f3 o, dir;
                                path_key((uint32_t)i, rng, &u, &v);
                                camera_ray_args(S, rng, u, v, &o, &dir, &time);
                                float* q = Lq + lane;
                                q[0] = o.x; q[64] = o.y; q[128] = o.z;
                                q[192] = dir.x; q[256] = dir.y; q[320] = dir.z;
                                q[384] = time;
                                q[448] = __uint_as_float((uint32_t)rng.state);
                                q[512] = __uint_as_float((uint32_t)(rng.state >> 32));
                                q[576] = __uint_as_float((uint32_t)rng.inc);
                                q[640] = __uint_as_float((uint32_t)(rng.inc >> 32));
                                q[704] = __uint_as_float((uint32_t)i);
                            }
                            q_n = (uint32_t)__popcll(__ballot(valid));  // a prefix of the lanes
                            const uint32_t r2 = rank - avail;
                            if (!active && r2 < q_n) pop(r2);
                            q_head = min(c - avail, q_n);
                        }
                    }
                }
                PH_MARK(ph, 4);
            } else {
                take_paths([&](float u, float v) {
                    camera_ray_args(S, ps.rng, u, v, &pr.o, &pr.dir, &pr.time);
                    pr.inside = 0;
                    pr.kind = 0;
                    want_ray = true;
                });
            }
            if (!__any(active)) {  // the last store
                if (st_pend) {
                    float* dst = reinterpret_cast<float*>(reinterpret_cast<char*>(P.rad) + st_off);
                    dst[0] = st_v.x;
                    dst[1] = st_v.y;
                    dst[2] = st_v.z;
                }
                break;
            }
            PH_MARK(ph, 0);
            BSTATC(15, active);
            if (want_ray) {
                BSTATC(12, pr.kind != 0);
                ps.r = make_ray(pr.o, pr.dir, pr.time, pr.inside);
                PH_MARK(ph, 8);
                if (pr.kind) finish_scatter<F, LK>(S, ps, lev, pr);
            }
            PH_MARK(ph, 7);
        }
    } else if constexpr (kResume) {
        // Cornell room + one pod_bvh mesh (scenes 8 / 9): the mesh walk is RESUMABLE.  Lanes walk
        // the BVH for different numbers of steps, so a walk run to completion inside one segment
        // leaves most lanes of the wave idle while the longest walks finish (lane utilisation
        // 0.13-0.17 measured).  Here a lane's walk state (node ref, stack depth, its LDS stack, the
        // walls' closest hit) persists across iterations; the walk loop hands the wave back once
        // few lanes still walk and enough others can shade or start new rays, and the stragglers
        // resume next iteration beside fresh rays (Aila & Laine 2009 "dynamic ray fetch", per
        // lane).  Every lane runs the same operations in the same order as mesh_hit: bit-exact.
        constexpr uint32_t PH_BEGIN = 1, PH_WALK = 2, PH_DONE = 3;
        using W = SigWalk<F, SIG_ROOM_MESH>;
        constexpr uint32_t kMeshPC = 7;  // LIST, 6 rects, MESH, LIST_END (mrt_sig.h kSigs)
        static_assert(kSigs[SIG_ROOM_MESH].op[kMeshPC] == LOP_MESH, "room + mesh program shape");
        const MRT_CONST_AS LinOp* prog = const_ptr(S.prog);
        uint32_t phase = 0, ref = 0, msp = 0;
#if MRT_MESH_SPEC
        uint32_t pref = 0;  // the parked leaf run (mesh_step_spec)
#endif
        SigState w;
        w.closest = FLT_MAX_;
        w.hnode = MRT_NONE;
        w.hinst = MRT_NONE;
        w.hdone = false;
        HitRec rec;
        for (;;) {
#if MRT_OPAQUE_RESUME
            const DScene& S = kernarg_scene();  // (shadows P.sc for this iteration)
            const MRT_CONST_AS LinOp* prog = const_ptr(S.prog);
#endif
            if (MRT_START_MIN <= 1 || (uint32_t)__popcll(__ballot(!active)) >= MRT_START_MIN || !__any(active))
                take_paths([&](float u, float v) {
                    ps.r = camera_ray(S, ps.rng, u, v);
                    phase = PH_BEGIN;
                });
            if (!__any(active)) break;
            PH_MARK(ph, 0);
            if (phase == PH_BEGIN) {  // the room's walls (scene_hit_sig's ops 0..6), then the mesh root box
                w.cur = ps.r;
                w.closest = FLT_MAX_;
                w.hnode = MRT_NONE;
                w.hinst = MRT_NONE;
                w.hdone = false;
                const MRT_CONST_AS LinOp& lo = prog[0];
                const bool in = !(LOP_FLAGS(lo) & MRT_F_HASBOX) || lin_box(lo, w.cur, 0.001f, w.closest);
#if MRT_FAST_ROOM
                // tolerance contract: the room's five walls as one slab test (cornell_room_fill; the
                // box test of the root list only skips work), then the light (op 3)
                (void)in;
                static_assert(kSigs[SIG_ROOM_MESH].op[kSigs[SIG_ROOM_MESH].n - 1] == LOP_END, "room in the END op");
                room_walls_op(prog[kSigs[SIG_ROOM_MESH].n - 1], w.cur, 0.001f, w);
                W::template run<3, 4>(S, prog, 0.001f, w, true, rec, Ls);
#else
                W::template run<1, kMeshPC>(S, prog, 0.001f, w, in, rec, Ls);
#endif
                const mrt_node mn = ld_node(const_ptr(S.nodes) + prog[kMeshPC].node);
                const MRT_CONST_AS mrt_mesh_node& rt = const_ptr(S.mnodes)[mn.a];
                const bool enter = in && aabb_hit(f3{rt.bmin[0], rt.bmin[1], rt.bmin[2]}, f3{rt.bmax[0], rt.bmax[1], rt.bmax[2]}, ps.r,
                                                  0.001f, w.closest);
                ref = mn.b;
#if MRT_MESH_SENT
                Ls.mesh[lane] = kMeshEmpty;  // the stack's bottom (mrt_trace.h kMeshEmpty)
                msp = 1;
#else
                msp = 0;
#endif
#if MRT_MESH_SPEC
                pref = 0;
#endif
                phase = enter ? PH_WALK : PH_DONE;
            }
            PH_MARK(ph, 1);
            // at least one step per iteration for every walking lane (no lane starves), then more
            // while enough lanes walk or too few have anything else to do
            while (__any(phase == PH_WALK)) {
                // some walking lane's ray is not nice (the box tests' slow path; wave-uniform)
                const bool bad = any_lane(phase == PH_WALK && !ps.r.nice);
#pragma unroll
                for (int u = 0; u < MRT_WALK_UNROLL; u++) {  // (A/B hook: steps between two yield checks)
#if MRT_MESH_SPEC
                    // the wave's choice: a leaf step once enough runs are parked or no inner step is left
                    const bool can_inner = phase == PH_WALK && ref != kMeshEnd && !((ref & MESH_LEAF) && pref != 0u);
                    // (MRT_SPEC_LEAF 0: a leaf step when at least as many lanes can take one as an inner step)
                    const uint32_t n_leaf = (uint32_t)__popcll(__ballot(phase == PH_WALK && pref != 0u));
                    const uint32_t n_inner = (uint32_t)__popcll(__ballot(can_inner));
                    const bool leaf_iter = MRT_SPEC_LEAF ? (n_leaf >= MRT_SPEC_LEAF || n_inner == 0u) : n_leaf >= n_inner;
                    if (phase == PH_WALK) {
                        const uint32_t st = mesh_step_spec<false>(S, ps.r, 0.001f, w.closest, rec, Ls, ref, pref, msp, w.hdone, leaf_iter, bad);
                        if (st == 1u) w.hnode = kMeshPC;  // w.closest = the hit's t, w.hdone set
                        phase = st != 0u ? PH_DONE : PH_WALK;
                    }
#else
                    if (phase == PH_WALK) {
                        const mrt_node mn = ld_node(const_ptr(S.nodes) + prog[kMeshPC].node);
                        const uint32_t st = mesh_step<false, true>(S, mn, ps.r, 0.001f, w.closest, rec, Ls, ref, msp, w.hdone, bad);
                        if (st == 1u) w.hnode = kMeshPC;  // w.closest = the hit's t, w.hdone set
                        phase = st != 0u ? PH_DONE : PH_WALK;
                    }
#endif
                }
                if ((uint32_t)__popcll(__ballot(phase == PH_WALK)) <= P.walk_min &&
                    (uint32_t)__popcll(__ballot(phase == PH_DONE || (!active && !exhausted))) >= MRT_WALK_OTHER)
                    break;  // others can shade / start rays: done lanes, or idle lanes with paths left
            }
            PH_MARK(ph, 6);
            if (phase == PH_DONE) {
                if (w.hnode == kMeshPC) {  // the mesh's record, deferred by the walk (mesh_step<.., true>)
                    const mrt_node mn = ld_node(const_ptr(S.nodes) + prog[kMeshPC].node);
                    mesh_hit_rec(S, mn, ps.r, w.closest, rec);
                } else if (!w.hdone && w.hnode != MRT_NONE) {
                    W::template derive<0>(prog, w, ps.r, ps.r, rec);
                }
                f3 L{0.0f, 0.0f, 0.0f};
                const bool ended = shade_hit<F, LK>(S, ps, P.max_bounces, lev, w.hnode != MRT_NONE, rec, &L, ph, CritSink{idx, kCritOff<F>});
                PH_MARK(ph, 2);
                phase = PH_BEGIN;
                if (ended) {
                    finish_path(L);
                    phase = 0;
                }
            }
            PH_MARK(ph, 3);
        }
    } else {
        for (;;) {
            if (MRT_START_MIN_PLAIN <= 1 || (uint32_t)__popcll(__ballot(!active)) >= MRT_START_MIN_PLAIN || !__any(active))
                take_paths([&](float u, float v) { ps.r = camera_ray(S, ps.rng, u, v); });
            if (!__any(active)) break;
            PH_MARK(ph, 0);
#if MRT_OPAQUE_SCENE
            // the scene's kernel arguments re-derived each iteration through an opaque constant
            // pointer: its fields are scalar-loaded at their uses in the segment instead of held in
            // SGPRs across the path loop (which spilled them into VGPR lanes)
            const DScene& Sseg = kernarg_scene();
#else
            const DScene& Sseg = S;
#endif
            if (active) {
                f3 L{0.0f, 0.0f, 0.0f};
                const bool ended = trace_segment<F, LK>(Sseg, ps, P.max_bounces, lev, Ls, &L, ph, CritSink{idx, kCritOff<F>});
                PH_MARK(ph, 2);
                if (ended) finish_path(L);
            }
            PH_MARK(ph, 3);
        }
    }
#ifdef MRT_PHASES
    if (lane == 0)
        for (int i = 0; i < 12; i++) atomicAdd(&g_phases[i], (unsigned long long)ph.a[i]);
#endif
#if defined(MRT_EXPERIMENTS) && defined(MRT_WTIMES)
    WT_MARK(wt1);
    if (lane == 0) {
        const size_t g = ((size_t)blockIdx.x * (blockDim.x >> 6) + wave) * 7;
        if (g + 6 < 7 * 16384) {
            g_wtimes[g + 4] = wt_aok;
            g_wtimes[g + 5] = wt_afail;
            g_wtimes[g + 6] = wt_n;
            g_wtimes[g] = wt0;
            g_wtimes[g + 1] = wt_ex;
            g_wtimes[g + 2] = wt1;
            g_wtimes[g + 3] = (uint64_t)blockIdx.x | ((wt_f ? wt_f - wt0 : 0ull) << 20);
        }
    }
#endif
    // one 64-bit add per wave
    uint64_t my = done_rays;
    for (int off = 32; off > 0; off >>= 1) my += __shfl_xor(my, off);
    if (lane == 0 && my) atomicAdd(P.rays, (unsigned long long)my);
}

// The exact arithmetic (the path-exact build: the reference's, forward fold) for the paths a
// fast-arithmetic launch listed as rounding-critical (mrt_shade.h light_critical; PathParams::rt):
// each traced from its camera ray to its end as the reference traces it -- including its
// non-finite end, which the fold then turns into main.cpp:162-164's doubling -- and its radiance
// written over the fast one in the launch's radiance buffer, before the fold.  A few hundred to a
// few thousand paths per launch: one-wave groups over the list, one path per lane; the last group
// to finish clears the list for the next launch.  (The launch's ray count stays the fast paths'.)
template <uint32_t F>
static constexpr bool kRetrace = MRT_TABLE_PEX && MRT_FWD_FOLD && (F & FT_BIASED) != 0 && !kPathExact<F>;
#if MRT_TABLE_PEX
template <uint32_t F>
__global__ void __launch_bounds__(64) mrt_retrace_kernel(PathParams P) {
    extern __shared__ __attribute__((aligned(16))) uint32_t lds[];
    const uint32_t lane = threadIdx.x & 63u;
    uint32_t* const wb = lds;
    uint32_t* const wmesh = wb + P.lds_frames * 128 + P.lds_rays * 704;
    const LStack Ls{wb, (float*)(wb + P.lds_frames * 128), wmesh, (float*)(wmesh + P.lds_mesh * 64), lane, nullptr, 0u};
    const LevStore<0> lev{nullptr, 0u, 0u, 0u};
    const DScene& S = P.sc;
    PhaseClock ph{};
    const uint32_t listed = __hip_atomic_load(P.rt.n, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    const uint32_t n = min(listed, P.rt.cap);
    if (blockIdx.x == 0 && lane == 0 && n) atomicAdd(P.rt.total, (unsigned long long)n);
    if (blockIdx.x == 0 && lane == 0 && listed > n) atomicAdd(P.rt.lost, (unsigned long long)(listed - n));  // (kept fast)
    for (uint32_t i = blockIdx.x * 64u + lane; i < n; i += gridDim.x * 64u) {
        const uint32_t idx = P.rt.idx[i];
        uint32_t lp, sl;
        path_coords(P, idx, &lp, &sl);
        PathState ps;
        float u, v;
        path_key_at(P, lp, P.s0 + sl, ps.rng, &u, &v);
        ps.r = camera_ray(S, ps.rng, u, v);
        ps.depth = 0;
        ps.nlev = 0;
        ps.T = f3{1.0f, 1.0f, 1.0f};
        f3 L{0.0f, 0.0f, 0.0f};
        while (!trace_segment<F, 0>(S, ps, P.max_bounces, lev, Ls, &L, ph)) {
        }
        L = end_path(ps, lev, L);
        float* dst = P.rad + (size_t)idx * 3u;
        dst[0] = L.x;
        dst[1] = L.y;
        dst[2] = L.z;
    }
    if (lane == 0 && atomicAdd(P.rt.done, 1u) == gridDim.x - 1u) {
        atomicExch(P.rt.n, 0u);  // every group has read the count: the list is empty for the next launch
        atomicExch(P.rt.done, 0u);
    }
}
#endif
template <uint32_t F>
static constexpr path_kernel_t kfn_retrace() {
#if MRT_TABLE_PEX
    if constexpr (kRetrace<F>) return mrt_retrace_kernel<F>;
#endif
    return nullptr;
}

template <uint32_t F>
static constexpr path_kernel_t kfn() {
#if MRT_TABLE_PEX
    if constexpr (!kPathExact<F>) return nullptr;  // (not instantiated: another build runs it)
    else
#elif MRT_TABLE_FTZ
    if constexpr (!kFtzVariant<F>) return nullptr;  // (not instantiated: the plain fast build runs it)
    else
#endif
    return MRT_PATH_KERNEL<F>;
}

// one entry per variant of mrt_launch.h's kVariants
template <size_t... I>
static KernelTable make_table(const char* numerics, std::index_sequence<I...>) {
    return KernelTable{numerics,
                       {kfn<kVariants[I]>()...},
                       {PathLevLds<kVariants[I]>::K...},
                       {TreeOf<kVariants[I]>::wg...},
                       {TreeOf<kVariants[I]>::on...},
                       {PathQ<kVariants[I]>::words...},
                       {kBox6Walk<kVariants[I]>...},
                       {(uint32_t)(kLinSlabOps<kVariants[I]> && MRT_SIG_OF(kVariants[I]) == SIG_NONE)...},
                       {kfn_retrace<kVariants[I]>()...}};
}
#if MRT_TABLE_PEX
const KernelTable& mrtd::kernel_table_fast_pex() {
    static const KernelTable t = make_table("fast", std::make_index_sequence<kNumVariants>{});
#elif MRT_TABLE_FTZ
const KernelTable& mrtd::kernel_table_fast_ftz() {
    static const KernelTable t = make_table("fast", std::make_index_sequence<kNumVariants>{});
#elif MRT_TABLE_FAST
const KernelTable& mrtd::kernel_table_fast() {
    static const KernelTable t = make_table("fast", std::make_index_sequence<kNumVariants>{});
#else
const KernelTable& mrtd::kernel_table_exact() {
    static const KernelTable t = make_table("exact", std::make_index_sequence<kNumVariants>{});
#endif
    return t;
}
