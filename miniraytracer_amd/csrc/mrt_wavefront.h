// mrt_wavefront.h -- the split ("wavefront") form of the path loop (mrt_launch.h WfParams), built in
// the path-exact TU (mrt_kernels.hip with MRT_TABLE_PEX) for the bvh_node scenes with volumes.
//
// The persistent path kernel runs scene_object::hit and material::scatter in one loop, so its
// register file is sized by both: book2 (C5) runs at 6 waves per SIMD, VALU busy 0.45, a third of
// its wave cycles waiting on memory.  Here a path's state stays in slot
// arrays in HBM and two kernels alternate, one launch pair per segment:
//   mrt_wf_ext<F>    for every busy slot: the hit query of trace() (main.cpp:79-82, the scene graph
//                    of scene_object.h / bvh_node / constant_volume, which draws from the path's PCG
//                    stream) -> the closest hit record; persistent waves, LDS treelet + stacks.
//   mrt_wf_shade<F>  for every busy slot: the rest of the segment (main.cpp:83-118: emission, the
//                    depth limit, material::scatter, the mixture pdf) -> the next ray, or the path's
//                    radiance; then the freed slots take new paths (work_queue::getWork,
//                    work_queue.cpp:158-166) and start them with camera::get_ray.
// Every path runs the operations of the path kernel in the same order on the same stream: the
// per-path radiance is the path kernel's bit for bit (tests/test_gpu_parity.py).
#pragma once

namespace mrtd {

#define MRT_WF_SHADE_WG 256

// Slot traffic is streamed past the caches (non-temporal loads / stores): the state arrays of one
// iteration are far larger than the L2, and the walk's BVH nodes and primitives must stay in it.
#ifndef MRT_WF_NT
#define MRT_WF_NT 1
#endif
MRT_DFN float4 wf_ld(const float4* p) {
#if MRT_WF_NT
    const v4f v = __builtin_nontemporal_load(reinterpret_cast<const v4f*>(p));
    return make_float4(v.x, v.y, v.z, v.w);
#else
    return *p;
#endif
}
MRT_DFN void wf_st(float4* p, float4 v) {
#if MRT_WF_NT
    const v4f w = {v.x, v.y, v.z, v.w};
    __builtin_nontemporal_store(w, reinterpret_cast<v4f*>(p));
#else
    *p = v;
#endif
}
MRT_DFN float2 wf_ld2(const float2* p) {
#if MRT_WF_NT
    typedef float v2f __attribute__((ext_vector_type(2)));
    const v2f v = __builtin_nontemporal_load(reinterpret_cast<const v2f*>(p));
    return make_float2(v.x, v.y);
#else
    return *p;
#endif
}
MRT_DFN void wf_st2(float2* p, float2 v) {
#if MRT_WF_NT
    typedef float v2f __attribute__((ext_vector_type(2)));
    const v2f w = {v.x, v.y};
    __builtin_nontemporal_store(w, reinterpret_cast<v2f*>(p));
#else
    *p = v;
#endif
}
MRT_DFN uint32_t wf_ldu(const uint32_t* p) {
#if MRT_WF_NT
    return __builtin_nontemporal_load(p);
#else
    return *p;
#endif
}

// the slot's ray (as make_ray left it)
MRT_DFN Ray wf_load_ray(const WfState& W, uint32_t i, uint32_t* depth) {
    const float4 a = wf_ld(W.ray0 + i), b = wf_ld(W.ray1 + i), c = wf_ld(W.ray2 + i);
    Ray r;
    r.o = f3{a.x, a.y, a.z};
    r.time = a.w;
    r.d = f3{b.x, b.y, b.z};
    const uint32_t bits = __float_as_uint(b.w);
    r.mask = bits & 0xFFu;
    r.nice = ((bits >> 8) & 1u) != 0;
    r.inside = (int)(bits >> 16);
    r.inv = f3{c.x, c.y, c.z};
    *depth = __float_as_uint(c.w);
    return r;
}
MRT_DFN void wf_store_ray(const WfState& W, uint32_t i, const Ray& r, uint32_t depth) {
    wf_st(W.ray0 + i, make_float4(r.o.x, r.o.y, r.o.z, r.time));
    wf_st(W.ray1 + i, make_float4(r.d.x, r.d.y, r.d.z, __uint_as_float(r.mask | ((uint32_t)r.nice << 8) | ((uint32_t)r.inside << 16))));
    wf_st(W.ray2 + i, make_float4(r.inv.x, r.inv.y, r.inv.z, __uint_as_float(depth)));
}
MRT_DFN Pcg wf_load_rng(const WfState& W, uint32_t i) {
    const float4 g = wf_ld(reinterpret_cast<const float4*>(W.rng) + i);
    Pcg p;
    p.state = (uint64_t)__float_as_uint(g.x) | ((uint64_t)__float_as_uint(g.y) << 32);
    p.inc = (uint64_t)__float_as_uint(g.z) | ((uint64_t)__float_as_uint(g.w) << 32);
    return p;
}
MRT_DFN void wf_store_rng(const WfState& W, uint32_t i, const Pcg& p) {
    wf_st(reinterpret_cast<float4*>(W.rng) + i, make_float4(__uint_as_float((uint32_t)p.state), __uint_as_float((uint32_t)(p.state >> 32)),
                                                           __uint_as_float((uint32_t)p.inc), __uint_as_float((uint32_t)(p.inc >> 32))));
}

// ---- the hit kernel ----------------------------------------------------------------------
template <uint32_t F>
__global__ void __launch_bounds__(MRT_WF_EXT_WG) __attribute__((amdgpu_waves_per_eu(MRT_WF_EXT_W))) mrt_wf_ext(WfParams A) {
    const PathParams& P = A.P;
    const DScene& S = P.sc;
    extern __shared__ __attribute__((aligned(16))) uint32_t lds[];
    const uint32_t lane = threadIdx.x & 63u;
    const uint32_t wave = threadIdx.x >> 6;
    const uint32_t wpb = blockDim.x >> 6;
    // per wave: its stacks ([slot][word][lane]), then the workgroup's treelet (mrt_kernels.hip)
    const uint32_t words = (P.lds_frames * 2 + P.lds_rays * 11 + P.lds_mesh + P.lds_save) * 64;
    uint32_t* wb = lds + wave * words;
    uint32_t* const wmesh = wb + P.lds_frames * 128 + P.lds_rays * 704;
    float4* tree = nullptr;
    if constexpr (TreeOf<F>::on) {
        tree = reinterpret_cast<float4*>(lds + wpb * words);
        for (uint32_t i = threadIdx.x; i < P.tree_n * 4u; i += blockDim.x) tree[i] = P.tree_src[i];
        __syncthreads();
    }
    const LStack Ls{wb, (float*)(wb + P.lds_frames * 128), wmesh, (float*)(wmesh + P.lds_mesh * 64), lane, tree,
                    TreeOf<F>::on ? P.tree_n : 0u};
    if (blockIdx.x == 0 && threadIdx.x == 0) {
        // the shade kernel of this iteration has finished (stream order): publish whether every
        // partition is handed out, and the progress snapshots (mrt_progress)
        const uint32_t e = __hip_atomic_load(A.exh, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        // (a cancelled render hands out nothing more: its loop ends as if the partitions were done)
        const bool all = e == (1u << MRT_NPART) - 1u || __hip_atomic_load(P.cancel, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) != 0;
        if (P.hprog)
            for (uint32_t k = 0; k < MRT_NPART; k++) {
                const uint64_t len = P.part_base[k + 1] - P.part_base[k];
                const uint64_t c = __hip_atomic_load(A.cnt + k * MRT_COUNTER_STRIDE, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                __hip_atomic_store(P.hprog + k, c < len ? c : len, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
            }
        __hip_atomic_store(A.h_state, (A.epoch << 32) | A.iter | (all ? 0x80000000ull : 0ull), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    }
    PhaseClock ph{};
    // 64-slot groups claimed MRT_WF_CLAIM at a time from per-XCD partitions of the slot range (the
    // walks' lengths vary: a static deal left every launch waiting on its slowest waves)
    const uint32_t groups = A.nslots >> 6;
    uint32_t part = blockIdx.x % MRT_NPART;
    for (uint32_t tries = 0; tries < MRT_NPART; tries++, part = (part + 1) % MRT_NPART) {
      const uint32_t lo = (uint32_t)((uint64_t)groups * part / MRT_NPART), hi = (uint32_t)((uint64_t)groups * (part + 1) / MRT_NPART);
      for (;;) {
        uint32_t c = 0;
        if (lane == 0) c = atomicAdd(A.gcnt + part * 32u, (uint32_t)MRT_WF_CLAIM);
        c = (uint32_t)__builtin_amdgcn_readfirstlane((int)c);
        if (c >= hi - lo) break;
        const uint32_t g1 = min(lo + c + (uint32_t)MRT_WF_CLAIM, hi);
        for (uint32_t g = lo + c; g < g1; g++) {
        const uint32_t i = (g << 6) + lane;
        if (wf_ldu(A.W.idx + i) == MRT_NONE) continue;
        uint32_t depth;
        Ray r = wf_load_ray(A.W, i, &depth);
        Pcg rng = wf_load_rng(A.W, i);
        HitRec rec;
        bool hit;
        if constexpr (MRT_SIG_OF(F) != SIG_NONE) hit = scene_hit_sig<F>(S, r, 0.001f, rec, Ls);
        else if constexpr ((F & FT_LIN) != 0) hit = scene_hit_lin<F>(S, r, 0.001f, rec, Ls, rng, ph);
        else hit = scene_hit<F>(S, r, 0.001f, rec, rng, Ls);
        wf_st(A.W.hit0 + i, make_float4(rec.t, rec.p.x, rec.p.y, rec.p.z));
        wf_st(A.W.hit1 + i, make_float4(rec.n.x, rec.n.y, rec.n.z, __uint_as_float(hit ? rec.mat : MRT_NONE)));
        wf_st2(A.W.hit2 + i, make_float2(rec.u, rec.v));
        if constexpr ((F & FT_VOLUME) != 0) wf_store_rng(A.W, i, rng);  // constant_volume draws inside hit
        }
      }
    }
}

// ---- the shade kernel --------------------------------------------------------------------
template <uint32_t F>
__global__ void __launch_bounds__(MRT_WF_SHADE_WG) mrt_wf_shade(WfParams A) {
    const PathParams& P = A.P;
    const DScene& S = P.sc;
    const uint32_t lane = threadIdx.x & 63u;
    const uint32_t i = blockIdx.x * MRT_WF_SHADE_WG + threadIdx.x;  // nslots is a multiple of the group
    const LevStore<0> lev{nullptr, 0u, 0u, 0u};  // forward fold: no stored levels
    PhaseClock ph{};
    if (i < MRT_NPART) A.gcnt[i * 32u] = 0u;  // the hit kernel's group claims of this iteration (it runs next)
    uint32_t idx = wf_ldu(A.W.idx + i);
    const uint32_t idx0 = idx;
    bool active = idx != MRT_NONE;
    PathState ps;
    uint32_t done = 0;  // rays of the path this slot ended
    if (active) {
        ps.r = wf_load_ray(A.W, i, &ps.depth);
        ps.rng = wf_load_rng(A.W, i);
        ps.nlev = 0;
        const float4 t = wf_ld(A.W.thr + i);
        ps.T = f3{t.x, t.y, t.z};
        const float4 h0 = wf_ld(A.W.hit0 + i), h1 = wf_ld(A.W.hit1 + i);
        const float2 h2 = wf_ld2(A.W.hit2 + i);
        HitRec rec;
        rec.t = h0.x;
        rec.p = f3{h0.y, h0.z, h0.w};
        rec.n = f3{h1.x, h1.y, h1.z};
        rec.mat = __float_as_uint(h1.w);
        rec.u = h2.x;
        rec.v = h2.y;
        f3 L{0.0f, 0.0f, 0.0f};
        if (shade_hit<F, 0>(S, ps, P.max_bounces, lev, rec.mat != MRT_NONE, rec, &L, ph)) {
            L = end_path(ps, lev, L);
            float* dst = P.rad + (size_t)idx * 3;
            dst[0] = L.x;
            dst[1] = L.y;
            dst[2] = L.z;
            if (P.path_rays) P.path_rays[idx] = ps.rays();
            done = ps.rays();
            active = false;
        }
    }
    // freed slots take new paths: the wave's idle lanes claim them together, one atomic per claim
    // on the partition counter of the wave's XCD (partitions found handed out are skipped)
    const bool stop = __hip_atomic_load(P.cancel, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) != 0;
    uint64_t need = __ballot(!active);
    if (need && !stop) {
        uint32_t exh = (uint32_t)__builtin_amdgcn_readfirstlane((int)__hip_atomic_load(A.exh, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
        uint32_t part = blockIdx.x % MRT_NPART;
        for (uint32_t tries = 0; need && tries < MRT_NPART; tries++, part = (part + 1) % MRT_NPART) {
            if ((exh >> part) & 1u) continue;  // (wave-uniform)
            const uint32_t c = (uint32_t)__popcll(need);
            const uint64_t len = P.part_base[part + 1] - P.part_base[part];
            uint64_t nb = 0;
            if (lane == 0) nb = atomicAdd(A.cnt + part * MRT_COUNTER_STRIDE, (unsigned long long)c);
            nb = ((uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)(nb >> 32)) << 32) |
                 (uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)nb);
            const uint32_t got = nb < len ? (uint32_t)(len - nb < c ? len - nb : c) : 0u;
            if (!active) {
                const uint32_t r = __builtin_amdgcn_mbcnt_hi((uint32_t)(need >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)need, 0u));
                if (r < got) {
                    idx = (uint32_t)(P.part_base[part] + nb + r);
                    float u, v;
                    path_key_of(P, idx, ps.rng, &u, &v);
                    ps.r = camera_ray(S, ps.rng, u, v);
                    ps.depth = 0;
                    ps.T = f3{1.0f, 1.0f, 1.0f};
                    active = true;
                }
            }
            if (got < c) {
                if (lane == 0) atomicOr(A.exh, 1u << part);
                exh |= 1u << part;
            }
            need = __ballot(!active);
        }
    }
    if (active) {
        wf_store_ray(A.W, i, ps.r, ps.depth);
        wf_store_rng(A.W, i, ps.rng);
        wf_st(A.W.thr + i, make_float4(ps.T.x, ps.T.y, ps.T.z, 0.0f));
    }
    const uint32_t nidx = active ? idx : MRT_NONE;
    if (nidx != idx0) A.W.idx[i] = nidx;
    // rays of the ended paths: one add per 64-slot group (the group's own word, no atomics)
    uint64_t my = done;
    for (int off = 32; off > 0; off >>= 1) my += __shfl_xor(my, off);
    if (lane == 0 && my) A.ray_acc[i >> 6] += my;
}

}  // namespace mrtd
