// mrt_shade.h -- textures, materials, pdfs and one trace() segment (main.cpp:66-118)
#pragma once
#include <cstddef>
#include <type_traits>
#include "mrt_sig.h"

namespace mrtd {

// perlin_noise::noise / turbulence (texture.cpp:68-165)
MRT_DFN float perlin_noise(const DScene& S, f3 p) {
    float fx = floorf(p.x), fy = floorf(p.y), fz = floorf(p.z);
    float u = p.x - fx, v = p.y - fy, w = p.z - fz;
    int i = (int)fx, j = (int)fy, k = (int)fz;
    f3 uvw = mul(mul(f3{u, v, w}, f3{u, v, w}), sub(f3{3, 3, 3}, fmul(2, f3{u, v, w})));
    float acc = 0;
#pragma unroll
    for (int di = 0; di < 2; di++) {
        int px = S.perm[(i + di) & 255];
#pragma unroll
        for (int q = 0; q < 4; q++) {
            int dj = q >> 1, dk = q & 1;
            int idx = px ^ S.perm[256 + ((j + dj) & 255)] ^ S.perm[512 + ((k + dk) & 255)];
            f3 c = ld3(S.ranvec[idx]);
            f3 ijk{(float)di, (float)dj, (float)dk};
            f3 weights = sub(f3{u, v, w}, ijk);
            f3 a = add(mul(ijk, uvw), mul(sub(f3{1, 1, 1}, ijk), sub(f3{1, 1, 1}, uvw)));
            acc = ref_fma((a.x * a.y) * a.z, dot(c, weights), acc);  // texture.cpp:82-97
        }
    }
    return acc;
}
MRT_DFN float turbulence(const DScene& S, f3 p) {
    float acc = 0, weight = 1.0f;
    for (int i = 0; i < 7; i++) {
        acc = ref_fma(weight, perlin_noise(S, p), acc);  // texture.cpp:160
        weight *= 0.5f;
        p = mulf(p, 2);
    }
    return fabsf(acc);
}

// texture::sample (texture.h:18-20, 56-62; texture.cpp:7-25, 207-224)
template <uint32_t F>
MRT_DFN f3 tex_sample(const DScene& S, uint32_t t, float u, float v, f3 p) {
    for (;;) {
        const mrt_texture& T = S.texs[t];
        if (!(F & FT_TEX)) return f3{T.f[0], T.f[1], T.f[2]};
        switch (T.kind) {
        case MRT_T_COLOR:
            return f3{T.f[0], T.f[1], T.f[2]};
        case MRT_T_CHECKER: {
            float sc = T.f[0];
            float sines = (sin_(sc * p.x) * sin_(sc * p.y)) * sin_(sc * p.z);
            t = sines < 0 ? T.b : T.a;
            continue;
        }
        case MRT_T_PERLIN: {
            float tb = turbulence(S, mulf(p, T.f[0]));
            return f3{1 * tb, 1 * tb, 1 * tb};
        }
        default: {  // image
            int32_t w = (int32_t)T.b, h = (int32_t)T.c;
            int32_t i = (int32_t)(u * w);
            int32_t j = (int32_t)((1 - v) * h);
            i = i < 0 ? 0 : (i > w - 1 ? w - 1 : i);
            j = j < 0 ? 0 : (j > h - 1 ? h - 1 : j);
            const uint8_t* d = S.texels + T.a + ((size_t)i + (size_t)w * j) * 3;
            const float f = 1.0f / 255.0f;
            return f3{(float)d[0] * f, (float)d[1] * f, (float)d[2] * f};
        }
        }
    }
}

// the material's texture at the hit (constant colours come inline with the material)
template <uint32_t F>
MRT_DFN f3 mat_color(const DScene& S, const DMat& M, const HitRec& rec) {
    if (!(F & FT_TEX) || (M.flags & DMAT_COLOR)) return f3{M.col[0], M.col[1], M.col[2]};
    return tex_sample<F>(S, M.tex, rec.u, rec.v, rec.p);
}

// onb(n) * vec (onb.h:19-27)
MRT_DFN f3 onb_apply(f3 w, f3 vec) {
    f3 a = fabsf(w.x) > 0.9f ? f3{0, 1, 0} : f3{1, 0, 0};
    f3 v = normalize(cross(w, a));
    f3 u = cross(w, v);
    return add(add(fmul(vec.x, u), fmul(vec.y, v)), fmul(vec.z, w));
}

// The next randf() values of a path's stream, two of them drawn ahead: every direction generator
// of the lambertian mix starts with two draws, so they are drawn once before the light/surface
// branch instead of inside both sides (same values, same stream order).
// (a light sample's draw this close to 0 or 1 puts its point on the rect's edge: crit_check)
#ifndef MRT_EDGE_TOL
#define MRT_EDGE_TOL 0x1p-18f
#endif
struct Draws {
    float v0, v1;
    uint32_t used;
    bool edge = false;  // a light sample drawn within MRT_EDGE_TOL of its rect's edge (crit_check)
    MRT_DFN float next(Pcg& rng) {
        if (used == 0) { used = 1; return v0; }
        if (used == 1) { used = 2; return v1; }
        return randf(rng);
    }
};

// biased object pdfs: object_list / xz_rect / sphere pdf_value & pdf_generate
// (scene_object.h:64-77, rect.cpp:92-107, sphere.cpp:63-78, scene_object.h:24-29)
template <uint32_t F>
MRT_DFN float leaf_pdf_value(const DScene& S, const mrt_node& n, f3 origin, f3 dir, float time) {
    uint32_t k = MRT_NODE_KIND(n);
    HitRec rec;
    if (k == MRT_K_XZ) {  // xz_rect::pdf_value (rect.cpp:92-102), the hit test branch-free
        const Ray r = make_ray_unit<kFastUnit<F>>(origin, dir, 0.0f, 0);  // dir: the scattered ray's unit direction
        float t;
        const bool h = lin_prim_t<F, MRT_K_XZ>(n, r, 0.001f, FLT_MAX_, &t);
        const float area = (n.f[1] - n.f[0]) * (n.f[3] - n.f[2]);
        const float dist_sq = t * t;
        const float cosine = fabsf(dot(dir, f3{0, n.f[5], 0}));
        const float pdf = dist_sq / (cosine * area);
        return h ? pdf : 0.0f;
    }
    if ((F & FT_BSPHERE) && k == MRT_K_SPHERE) {
        Ray r = make_ray_unit<kFastUnit<F>>(origin, dir, time, 0);
        if (sphere_hit<F>(n, r, 0.001f, FLT_MAX_, rec, false)) {
            float radius = n.f[8];
            float cos_theta_max = sqrt_(1 - (radius * radius) / sdot(sub(sphere_center<F>(n, time), origin)));
            float solid_angle = (2 * PI_F) * (1 - cos_theta_max);
            return 1 / solid_angle;
        }
        return 0;
    }
    return 0;
}

// object_list::pdf_value over the biased list (scene_object.h:64-70): the leaves are read through
// the constant address space (uniform index: scalar loads, no node -> children -> node chain)
template <uint32_t F>
MRT_DFN float biased_pdf_value(const DScene& S, f3 origin, f3 dir, float time) {
    const MRT_CONST_AS mrt_node* bl = const_ptr(S.bleaf);
    // one leaf (also a list of one, as the Cornell box's and book2's biased lists are,
    // scene.cpp:326-329, 456-459): (0 + v) / 1 == v for the pdf values v >= +0 leaves return;
    // one 64-B scalar load, no loop of dependent kind / field loads
    if (!S.blist || S.nbleaf == 1) {
        const mrt_node n = ld_node(bl);
        return leaf_pdf_value<F>(S, n, origin, dir, time);
    }
    float sum = 0;
    for (uint32_t i = 0; i < S.nbleaf; i++) {
        const mrt_node n = ld_node(bl + i);
        sum += leaf_pdf_value<F>(S, n, origin, dir, time);
    }
#if MRT_FAST
    return sum * S.inv_nbleaf;  // (-freciprocal-math: the division by the loop-invariant count)
#else
    return sum / S.nbleaf_f;
#endif
}
template <uint32_t F>
MRT_DFN f3 leaf_pdf_generate(const DScene& S, const mrt_node& n, f3 origin, float time, Pcg& rng, Draws& dr) {
    uint32_t k = MRT_NODE_KIND(n);
    if (k == MRT_K_XZ) {
        float a = dr.next(rng);
        float x = ref_fma(a, n.f[1] - n.f[0], n.f[0]);  // rect.cpp:105 (left to right)
        float b = dr.next(rng);
        float z = ref_fma(b, n.f[3] - n.f[2], n.f[2]);
        dr.edge = fmaxf(fabsf(a - 0.5f), fabsf(b - 0.5f)) >= 0.5f - MRT_EDGE_TOL;
        return sub(f3{x, n.f[4], z}, origin);
    }
    if ((F & FT_BSPHERE) && k == MRT_K_SPHERE) {
        f3 dir = sub(sphere_center<F>(n, time), origin);
        float dist_sq = sdot(dir);
        f3 w = normalize(dir);
        const float r1 = dr.next(rng), r2 = dr.next(rng);
        return onb_apply(w, random_towards_sphere_pre(r1, r2, n.f[8], dist_sq));
    }
    return f3{1, 0, 0};
}
template <uint32_t F>
MRT_DFN f3 biased_pdf_generate(const DScene& S, f3 origin, float time, Pcg& rng, Draws& dr) {
    if (!S.blist) {
        const mrt_node n = ld_node(const_ptr(S.bleaf));
        return leaf_pdf_generate<F>(S, n, origin, time, rng, dr);
    }
    const int i = int(dr.next(rng) * S.nbleaf_f);  // object_list::pdf_generate (scene_object.h:72-77)
    if (S.nbleaf == 1) {
        const mrt_node n = ld_node(const_ptr(S.bleaf));
        return leaf_pdf_generate<F>(S, n, origin, time, rng, dr);
    }
    return leaf_pdf_generate<F>(S, S.bleaf[i], origin, time, rng, dr);
}

// A light sample is rounding-critical (tolerance contract, DESIGN.md section 2 "Non-finite
// samples") where xz_rect::pdf_value (rect.cpp:92-102) can return a non-finite or zero pdf on one
// side of a last-bit difference, which main.cpp:162-164 turns into a doubling of the pixel's
// running colour:
//  (1) its direction is (nearly) parallel to the light's plane: from a point ON the plane the
//      sampled direction has dir.y == 0 (the sampled point's y minus the origin's), pdf_value
//      computes t = 0 / 0 and reports a hit with a NaN pdf.  Whether a wall hit lands on y == 554
//      exactly depends on the last bit of its arithmetic and on the rounding the path gathered on
//      its earlier bounces: a window of MRT_CRIT_TOL relative to the origin's height (2^-16, ~140
//      ulps at the Cornell light's 554);
//  (2) the sampled point lies on the light's edge (a draw within MRT_EDGE_TOL of 0 or 1, 2^-18:
//      5e-4 on the Cornell light's 130-wide side, ~8 ulps of 555, a few times the rounding of the
//      hit point pdf_value recomputes from the origin) and below the surface: the recomputed point
//      can fall outside the rect by rounding, pdf 0, and with the cosine pdf 0 too the sample is
//      0 / 0.
// Under the fast arithmetic these events fall on other paths than the reference's (C3 at 4096
// spp: 98% of the tolerance contract's squared error in 100 such pixels).  Such paths are traced
// again with the exact arithmetic (mrt_retrace_kernel), whose radiance replaces the fast one; the
// fast kernel only lists them and goes on.
#ifndef MRT_CRIT_TOL
#define MRT_CRIT_TOL 0x1p-16f
#endif
MRT_DFN bool light_critical(f3 origin, f3 gen) { return fabsf(gen.y) <= fabsf(origin.y) * MRT_CRIT_TOL + MRT_CRIT_TOL; }
// The list the fast-arithmetic path kernel appends such paths to (their path index in the launch);
// the retrace kernel (mrt_kernels.hip) traces each again with the exact arithmetic and overwrites
// its radiance before the fold.  A path listed at several bounces is traced once per entry.
struct RetraceList {
    uint32_t* __restrict__ idx;              // path indices of the launch (sample-major, as rad)
    uint32_t* __restrict__ n;                // entries appended (may exceed cap: the rest are lost)
    uint32_t cap;
    uint32_t* __restrict__ done;             // retrace groups finished (the last one clears n)
    unsigned long long* __restrict__ total;  // paths listed since the scene's upload (mrt_kernel_info)
    unsigned long long* __restrict__ lost;   // entries beyond cap since the upload (mrt_kernel_info.handover_lost)
};
// where a shading step lists its path when its light sample is rounding-critical: the path's index
// and the byte offset of the launch's RetraceList in the kernel's argument segment (a compile-time
// constant; 0: no hand-over compiled in).  The list is read from the argument segment only where a
// path is listed (a null list: no hand-over this launch), so nothing of it is held in registers
// across the path loop (held there, it cost the Cornell kernel 1.3% with the hand-over off).
struct CritSink {
    uint32_t idx;
    uint32_t rt_off;
};
MRT_DFN void crit_check(const CritSink& cs, bool light, f3 origin, f3 gen, bool edge, f3 n) {
#if defined(__HIP_DEVICE_COMPILE__)
    if (cs.rt_off && light && (edge || light_critical(origin, gen))) {
        // (an edge sample above the surface has a cosine pdf > 0: finite either way)
        if (!light_critical(origin, gen) && dot(gen, n) > (fabsf(gen.x) + fabsf(gen.y) + fabsf(gen.z)) * 0x1p-12f) return;
        const MRT_CONST_AS char* ka = (const MRT_CONST_AS char*)__builtin_amdgcn_kernarg_segment_ptr();
        asm volatile("" : "+s"(ka));  // (the list's fields are loaded here, not hoisted out of the loop)
        const MRT_CONST_AS RetraceList& rl = *(const MRT_CONST_AS RetraceList*)(ka + cs.rt_off);
        if (rl.idx) {
            const uint32_t k = atomicAdd(rl.n, 1u);
            if (k < rl.cap) rl.idx[k] = cs.idx;
        }
    }
#else
    (void)cs, (void)light, (void)origin, (void)gen, (void)edge, (void)n;  // (the CPU backend runs the exact contract)
#endif
}

// ------------------------------------------------------------------------------------------
// trace() (main.cpp:66-118) as a per-lane state machine advanced one segment (= one ray, one
// scene_object::hit query) per call, so a lane whose path ends can start a new one at once.
// Per-bounce (attenuation*scatter_pdf, pdf) pairs go to `lev` and are folded back deepest-first
// exactly as the recursion of trace() returns: L = emitted + ((a * L) / pdf) (diffuse),
// L = attenuation * L (metal: pdf slot < 0).  Dielectric attenuation is exactly 1 (1*L == L),
// so glass bounces store nothing.
// ------------------------------------------------------------------------------------------
struct PathState {
    Ray r;
    Pcg rng;
    uint32_t depth;  // bounces so far (trace depth)
    uint32_t nlev;   // stored fold levels | LEV_LOUD once a level could turn a black result non-zero
    // trace() calls of a finished path: every segment but the last scatters (depth++), so the count
    // is depth + 1 -- derived, not kept in a register of its own across the path loop
    MRT_DFN uint32_t rays() const { return depth + 1u; }
#if MRT_FWD_FOLD
    f3 T;            // throughput of the bounces so far (forward fold)
#endif
};
static constexpr uint32_t LEV_LOUD = 0x80000000u;

// Fold levels of one lane: the first LK in LDS ([level][lane] float4), deeper ones in HBM.
template <uint32_t LK>
struct LevStore {
    // explicit address spaces: a generic pointer here made the compiler merge the two cases into
    // one flat access, which counts against vmcnt AND lgkmcnt (every later LDS wait then waited
    // for the level store to reach memory)
    // this lane's HBM row = base + slot * rows, formed at each use: a 32-bit slot stays live across
    // the path loop instead of a 64-bit pointer (which the register allocator spilled to scratch)
    MRT_GLOBAL_AS v4f* base;  // uniform
    uint32_t rows;            // uniform: levels per lane
    uint32_t slot;
    uint32_t lds_base;        // uniform: LDS byte address of this wave's level 0 row (64 float4)
    // this lane's first LDS slot, formed at use from the lane id (a per-lane pointer kept live
    // across the path loop was spilled)
    MRT_DFN MRT_LDS_AS v4f* lds() const {
#if defined(__HIP_DEVICE_COMPILE__)
        const uint32_t lane = __builtin_amdgcn_mbcnt_hi(~0u, __builtin_amdgcn_mbcnt_lo(~0u, 0u));
#else
        const uint32_t lane = 0;
#endif
        return (MRT_LDS_AS v4f*)(uintptr_t)(lds_base + lane * 16u);
    }
    MRT_DFN MRT_GLOBAL_AS v4f* g() const {
        uint32_t sl = slot;
#if defined(__HIP_DEVICE_COMPILE__)
        asm volatile("" : "+v"(sl));  // keeps the address from being hoisted out of the loop
#endif
        return base + (uint64_t)sl * rows;
    }
    MRT_DFN void put(uint32_t d, float4 v) const {
        const v4f w = {v.x, v.y, v.z, v.w};
        if (LK > 0 && d < LK) lds()[d * 64] = w;
        else g()[d] = w;
    }
    MRT_DFN float4 get(uint32_t d) const {
        v4f w;
        if (LK > 0 && d < LK) w = lds()[d * 64];
        else w = g()[d];
        return make_float4(w.x, w.y, w.z, w.w);
    }
};
// A level is quiet when folding +0 through it gives +0 exactly: finite factors, for diffuse a
// pdf > 0 (0 + (a * 0) / pdf == +0), for metal non-negative factors (att * +0 == +0).
MRT_DFN bool quiet_level(float4 v) {
    const bool fin = isfinite(v.x) && isfinite(v.y) && isfinite(v.z);
    if (v.w < 0.0f) return fin & (((__float_as_uint(v.x) | __float_as_uint(v.y) | __float_as_uint(v.z)) >> 31) == 0);
    return fin & (v.w > 0.0f) & isfinite(v.w);
}

// One bounce's level (a, pdf; pdf < 0: metal, L = a*L): stored for the deepest-first fold, or
// (forward fold) multiplied into the path's throughput.
template <uint32_t LK>
MRT_DFN void push_level(PathState& ps, const LevStore<LK>& lev, float4 lv) {
#if MRT_FWD_FOLD
    (void)lev;
    if (lv.w < 0.0f) ps.T = f3{ps.T.x * lv.x, ps.T.y * lv.y, ps.T.z * lv.z};
    else ps.T = f3{(ps.T.x * lv.x) / lv.w, (ps.T.y * lv.y) / lv.w, (ps.T.z * lv.z) / lv.w};
#else
    lev.put(ps.nlev & ~LEV_LOUD, lv);
    ps.nlev = (ps.nlev + 1) | (quiet_level(lv) ? 0u : LEV_LOUD);
#endif
}

// camera::get_ray (camera.h:38-44)
MRT_DFN Ray camera_ray(const DScene& S, Pcg& rng, float s, float t) {
    // through a pointer the compiler cannot prove loop-invariant: the camera is re-read (scalar
    // loads, constant cache) at each path start instead of being held in ~40 SGPRs across the
    // path loop, where it spilled to VGPR lanes and cost a v_readlane per use
    const MRT_CONST_AS mrt_camera* cp = const_ptr(S.camp);
#if defined(__HIP_DEVICE_COMPILE__)
    asm volatile("" : "+s"(cp));
#endif
    const MRT_CONST_AS mrt_camera& C = *cp;
    f3 rd = fmul(C.lens_radius, random_in_disk(rng));
    f3 offset = add(mulf(ld3(C.u), rd.x), mulf(ld3(C.v), rd.y));
    float time = ref_fma(C.time1 - C.time0, randf(rng), C.time0);  // camera.h:41
    f3 origin = ld3(C.origin);
    f3 dir = sub(sub(add(add(ld3(C.llcorner), fmul(s, ld3(C.horz))), fmul(t, ld3(C.vert))), origin), offset);
    return make_ray(add(origin, offset), dir, time, 0);
}

// camera::get_ray without the ray constructor: origin, direction argument and time of the ray
// (the constructor -- normalize, 1/dir, dirMask -- runs once per iteration for every lane that
// has a new ray, see PendRay)
MRT_DFN void camera_ray_args(const DScene& S, Pcg& rng, float s, float t, f3* o, f3* dir, float* time) {
    const MRT_CONST_AS mrt_camera* cp = const_ptr(S.camp);
#if defined(__HIP_DEVICE_COMPILE__)
    asm volatile("" : "+s"(cp));
#endif
    const MRT_CONST_AS mrt_camera& C = *cp;
    f3 rd = fmul(C.lens_radius, random_in_disk(rng));
    f3 offset = add(mulf(ld3(C.u), rd.x), mulf(ld3(C.v), rd.y));
    *time = ref_fma(C.time1 - C.time0, randf(rng), C.time0);  // camera.h:41
    f3 origin = ld3(C.origin);
    *dir = sub(sub(add(add(ld3(C.llcorner), fmul(s, ld3(C.horz))), fmul(t, ld3(C.vert))), origin), offset);
    *o = add(origin, offset);
}

// The rest of one segment once scene_object::hit has answered for ps.r: emission, the bounce
// limit, material::scatter and the next ray.  Returns true when the path has ended; its radiance
// is then in *L.
template <uint32_t F, uint32_t LK>
MRT_DFN bool shade_hit(const DScene& S, PathState& ps, uint32_t max_bounces, const LevStore<LK>& lev, bool hit,
                                          const HitRec& rec, f3* L, PhaseClock& ph, const CritSink& cs = CritSink{0u, 0u}) {
    Ray& r = ps.r;
    if (!hit) {
        if ((F & FT_SKY) && S.sky) {  // main.cpp:113-115
            float tt = 0.5f * (r.d.y + 1.0f);
            float o = 1.0f - tt;
            *L = f3{o + tt * 0.5f, o + tt * 0.7f, o + tt * 1.0f};
        } else {
            *L = f3{0, 0, 0};
        }
        return true;
    }
    const DMat M = S.mats[rec.mat];
    if (M.kind == MRT_M_LIGHT) {  // diffuse_light: sampleEmissive, never scatters (material.h:190-199)
        *L = dot(rec.n, r.d) < 0.0f ? fmul(M.p, mat_color<F>(S, M, rec)) : f3{0, 0, 0};
        return true;
    }
    if (ps.depth >= max_bounces) {  // the emitted term of a non-emissive material
        *L = f3{0, 0, 0};
        return true;
    }
    ps.depth++;
    if ((F & FT_METAL) && M.kind == MRT_M_METAL) {  // metal::scatter (material.h:91-98)
        f3 reflected = sub(r.d, fmul(2.0f * dot(r.d, rec.n), rec.n));
        f3 rs = random_in_sphere(ps.rng);
        f3 nd = add(reflected, fmul(1 - M.p, rs));
        f3 att = mat_color<F>(S, M, rec);
        const float4 lv = make_float4(att.x, att.y, att.z, -1.0f);
        push_level(ps, lev, lv);
        r = make_ray(rec.p, nd, r.time, 0);
        return false;
    }
    if (M.kind == MRT_M_DIELECTRIC) {  // dielectric::scatter (material.h:121-175)
        const float ref = M.p;
        const float cosI = -dot(r.d, rec.n);
        f3 facing;
        float nio;
        if (cosI < 0) {
            facing = f3{-rec.n.x, -rec.n.y, -rec.n.z};
            nio = ref;
        } else {
            facing = rec.n;
            nio = M.col[0];  // 1.0f / ref, computed on upload (the same IEEE quotient)
        }
        f3 nd = sub(r.d, fmul(2.0f * dot(r.d, rec.n), rec.n));  // reflect (vec3.h:178-181)
        int inside = r.inside;
        // refract (vec3.h:185-198)
        const float ncosI = dot(r.d, facing);
        // the scalar expressions of refract / dielectric::scatter / fresnel_schlick, fused as
        // shipped (vec3.h:187, 191; material.h:146, 109)
        const float sinT2 = (nio * nio) * ref_fnma(ncosI, ncosI, 1.0f);
        if (sinT2 <= 1.0f) {
            const float cosT = sqrt_(1.0f - sinT2);
            const float cs = cosI < 0 ? sqrt_(ref_fnma(nio * nio, ref_fnma(cosI, cosI, 1.0f), 1.0f)) : cosI;
            const float r0 = M.col[1];  // ((1 - ref) / (1 + ref))^2, computed on upload
            const float reflect_prob = ref_fma(1 - r0, pow5_((1 - cs)), r0);
            if (!(randf(ps.rng) < reflect_prob)) {
                nd = add(fmul(nio, r.d), fmul(ref_fms(nio, -ncosI, cosT), facing));
                if (cosI < 0) {
                    inside--;
                    if (inside < 0) inside = 0;
                } else {
                    inside++;
                }
            }
        }
        r = make_ray(rec.p, nd, r.time, inside);
        return false;
    }
    // lambertian / isotropic (material.h:48-74) with mix_pdf against the biased list (main.cpp:84-102)
    const bool lamb = !(F & FT_ISO) || M.kind == MRT_M_LAMBERTIAN;
    const f3 att = mat_color<F>(S, M, rec);
    f3 gen;
    const bool light = ((F & FT_BIASED) && S.biased != MRT_NONE) && randf(ps.rng) < 0.5f;
    // both sides of the mix start with two draws when the surface side is cosine sampling
    Draws dr{0.0f, 0.0f, 2u};
    if (lamb) {
        dr.v0 = randf(ps.rng);
        dr.v1 = randf(ps.rng);
        dr.used = 0;
    }
    if (light) gen = biased_pdf_generate<F>(S, rec.p, r.time, ps.rng, dr);
    else gen = lamb ? onb_apply(rec.n, random_cosine_direction_pre(dr.v0, dr.v1)) : random_in_sphere(ps.rng);
    crit_check(cs, light, rec.p, gen, dr.edge, rec.n);  // listed: retraced with the exact arithmetic
    PH_MARK(ph, 6);
    const Ray sc = make_ray(rec.p, gen, r.time, 0);
    float sval, spdf;
    if (lamb) {
        const float cosine = dot(sc.d, rec.n);
        // cosine / PI_F through div_core: PI_F and RN(1/PI_F) are normal, cosine <= 1
        constexpr float INV_PI = 1.0f / PI_F;
        float sv = div_core(cosine, PI_F, INV_PI);
        if (!MRT_FAST_GUARDS && __builtin_expect(any_lane((cosine > 0) & (cosine < 0x1p-100f)), 0)) sv = cosine < 0x1p-100f ? cosine / PI_F : sv;
        sval = cosine > 0 ? sv : 0;
        spdf = cosine < 0 ? 0 : cosine * (1.0f / PI_F);  // dot(rec.n, dir) == dot(dir, rec.n)
    } else {
        sval = 1 / (2 * PI_F);
        spdf = 1.0f / (2.0f * PI_F);
    }
    const float pdf_v = ((F & FT_BIASED) && S.biased != MRT_NONE) ? 0.5f * (biased_pdf_value<F>(S, rec.p, sc.d, r.time) + sval) : sval;
    const float4 lv = make_float4(att.x * spdf, att.y * spdf, att.z * spdf, pdf_v);
    push_level(ps, lev, lv);
    r = sc;
    return false;
}

// One segment.  Returns true when the path has ended; its radiance is then in *L.
template <uint32_t F, uint32_t LK>
MRT_DFN bool trace_segment(const DScene& S, PathState& ps, uint32_t max_bounces, const LevStore<LK>& lev,
                                              const LStack& Ls, f3* L, PhaseClock& ph, const CritSink& cs = CritSink{0u, 0u}) {
    HitRec rec;
    bool hit;
    if constexpr (MRT_SIG_OF(F) != SIG_NONE) hit = scene_hit_sig<F>(S, ps.r, 0.001f, rec, Ls);
    else if constexpr ((F & FT_LIN) != 0) hit = scene_hit_lin<F>(S, ps.r, 0.001f, rec, Ls, ps.rng, ph);
    else hit = scene_hit<F>(S, ps.r, 0.001f, rec, ps.rng, Ls);
    PH_MARK(ph, 1);
    return shade_hit<F, LK>(S, ps, max_bounces, lev, hit, rec, L, ph, cs);
}

// The next ray of a lane, built by make_ray once per iteration for all lanes at once (camera
// rays of new paths and scattered rays alike), plus what a diffuse scatter still has to do once
// the scattered ray exists (its pdfs need the normalized direction).
struct PendRay {
    f3 o, dir;
    float time;
    int inside;
    f3 att, n;      // diffuse scatter: attenuation, normal
    uint32_t kind;  // 0: nothing after the ray; 1: lambertian mix; 2: isotropic; 3: dielectric deferred
};

// dielectric::scatter (material.h:121-175) of a hit with normal n for ray r: the next ray's
// direction and inside count in *pr (its origin and time are set by the caller)
MRT_DFN void dielectric_scatter(const DMat& M, const Ray& r, f3 n, Pcg& rng, PendRay* pr) {
    const float ref = M.p;
    const float cosI = -dot(r.d, n);
    f3 facing;
    float nio;
    if (cosI < 0) {
        facing = f3{-n.x, -n.y, -n.z};
        nio = ref;
    } else {
        facing = n;
        nio = M.col[0];  // 1.0f / ref, computed on upload (the same IEEE quotient)
    }
    f3 nd = sub(r.d, fmul(2.0f * dot(r.d, n), n));  // reflect (vec3.h:178-181)
    int inside = r.inside;
    const float ncosI = dot(r.d, facing);
    // the scalar expressions of refract / dielectric::scatter / fresnel_schlick, fused as
    // shipped (vec3.h:187, 191; material.h:146, 109)
    const float sinT2 = (nio * nio) * ref_fnma(ncosI, ncosI, 1.0f);
    if (sinT2 <= 1.0f) {
        const float cosT = sqrt_(1.0f - sinT2);
        const float cs = cosI < 0 ? sqrt_(ref_fnma(nio * nio, ref_fnma(cosI, cosI, 1.0f), 1.0f)) : cosI;
        const float r0 = M.col[1];  // ((1 - ref) / (1 + ref))^2, computed on upload
        const float reflect_prob = ref_fma(1 - r0, pow5_((1 - cs)), r0);
        if (!(randf(rng) < reflect_prob)) {
            nd = add(fmul(nio, r.d), fmul(ref_fms(nio, -ncosI, cosT), facing));
            if (cosI < 0) {
                inside--;
                if (inside < 0) inside = 0;
            } else {
                inside++;
            }
        }
    }
    pr->dir = nd;
    pr->inside = inside;
}

// trace_segment up to the next ray's constructor arguments.  Returns true when the path has
// ended (radiance in *L); otherwise *pr holds the next ray's arguments.
// `flush` runs once the hit is known, before the material is read (the path loop issues the
// previous path's radiance store there).
template <uint32_t F, uint32_t LK, typename FLUSH>
MRT_DFN bool trace_split(const DScene& S, PathState& ps, uint32_t max_bounces, const LevStore<LK>& lev,
                                            const LStack& Ls, f3* L, PendRay* pr, PhaseClock& ph, FLUSH&& flush, const CritSink& cs = CritSink{0u, 0u}) {
    HitRec rec;
    Ray& r = ps.r;
    bool hit;
    if constexpr (MRT_SIG_OF(F) != SIG_NONE) hit = scene_hit_sig<F>(S, r, 0.001f, rec, Ls);
    else if constexpr ((F & FT_LIN) != 0) hit = scene_hit_lin<F>(S, r, 0.001f, rec, Ls, ps.rng, ph);
    else hit = scene_hit<F>(S, r, 0.001f, rec, ps.rng, Ls);
    PH_MARK(ph, 1);
    flush();
    BSTAT(0);
    BSTATC(14, hit);
    if (!hit) {
        BSTAT(1);
        if ((F & FT_SKY) && S.sky) {  // main.cpp:113-115
            float tt = 0.5f * (r.d.y + 1.0f);
            float o = 1.0f - tt;
            *L = f3{o + tt * 0.5f, o + tt * 0.7f, o + tt * 1.0f};
        } else {
            *L = f3{0, 0, 0};
        }
        return true;
    }
    const DMat M = S.mats[rec.mat];
    if (M.kind == MRT_M_LIGHT) {  // diffuse_light: sampleEmissive, never scatters (material.h:190-199)
        BSTAT(2);
        *L = dot(rec.n, r.d) < 0.0f ? fmul(M.p, mat_color<F>(S, M, rec)) : f3{0, 0, 0};
        return true;
    }
    if (ps.depth >= max_bounces) {  // the emitted term of a non-emissive material
        BSTAT(3);
        *L = f3{0, 0, 0};
        return true;
    }
    ps.depth++;
    pr->o = rec.p;
    pr->time = r.time;
    pr->inside = 0;
    pr->kind = 0;
    // the diffuse scatter's attenuation and normal, set on every branch: set only on the diffuse one,
    // the merge after the material branches cost a register copy of each on every path
    constexpr bool kAttEarly = (F & FT_TEX) == 0;  // (a constant colour: no texture lookup wasted)
    if constexpr (kAttEarly) {
        pr->att = mat_color<F>(S, M, rec);
        pr->n = rec.n;
    }
    if ((F & FT_METAL) && M.kind == MRT_M_METAL) {  // metal::scatter (material.h:91-98)
        f3 reflected = sub(r.d, fmul(2.0f * dot(r.d, rec.n), rec.n));
        f3 rs = random_in_sphere(ps.rng);
        pr->dir = add(reflected, fmul(1 - M.p, rs));
        f3 att = mat_color<F>(S, M, rec);
        const float4 lv = make_float4(att.x, att.y, att.z, -1.0f);
        push_level(ps, lev, lv);
        return false;
    }
    if (M.kind == MRT_M_DIELECTRIC) {  // dielectric::scatter (material.h:121-175)
        BSTAT(5);
        dielectric_scatter(M, r, rec.n, ps.rng, pr);
        return false;
    }
    // lambertian / isotropic (material.h:48-74): the direction now, the pdfs after the ray exists
    const bool lamb = !(F & FT_ISO) || M.kind == MRT_M_LAMBERTIAN;
    if constexpr (!kAttEarly) {
        pr->att = mat_color<F>(S, M, rec);
        pr->n = rec.n;
    }
    pr->kind = lamb ? 1u : 2u;
    BSTAT(6);
    const bool light = ((F & FT_BIASED) && S.biased != MRT_NONE) && randf(ps.rng) < 0.5f;
    Draws dr{0.0f, 0.0f, 2u};
    if (lamb) {
        dr.v0 = randf(ps.rng);
        dr.v1 = randf(ps.rng);
        dr.used = 0;
    }
    BSTATC(7, light);
    if (light) pr->dir = biased_pdf_generate<F>(S, rec.p, r.time, ps.rng, dr);
    else pr->dir = lamb ? onb_apply(rec.n, random_cosine_direction_pre(dr.v0, dr.v1)) : random_in_sphere(ps.rng);
    crit_check(cs, light, rec.p, pr->dir, dr.edge, rec.n);  // listed: retraced with the exact arithmetic
    PH_MARK(ph, 6);
    return false;
}

// the rest of a diffuse scatter once ps.r = make_ray(pr): mix_pdf value (main.cpp:84-102), level
template <uint32_t F, uint32_t LK>
MRT_DFN void finish_scatter(const DScene& S, PathState& ps, const LevStore<LK>& lev, const PendRay& pr) {
    const Ray& sc = ps.r;
    float sval, spdf;
    if (pr.kind == 1u) {
        const float cosine = dot(sc.d, pr.n);
        constexpr float INV_PI = 1.0f / PI_F;
        float sv = div_core(cosine, PI_F, INV_PI);
        if (!MRT_FAST_GUARDS && __builtin_expect(any_lane((cosine > 0) & (cosine < 0x1p-100f)), 0)) sv = cosine < 0x1p-100f ? cosine / PI_F : sv;
        sval = cosine > 0 ? sv : 0;
        spdf = cosine < 0 ? 0 : cosine * (1.0f / PI_F);
    } else {
        sval = 1 / (2 * PI_F);
        spdf = 1.0f / (2.0f * PI_F);
    }
    const float pdf_v = ((F & FT_BIASED) && S.biased != MRT_NONE) ? 0.5f * (biased_pdf_value<F>(S, sc.o, sc.d, sc.time) + sval) : sval;
    const float4 lv = make_float4(pr.att.x * spdf, pr.att.y * spdf, pr.att.z * spdf, pdf_v);
    push_level(ps, lev, lv);
}

// the recursion's return path, deepest level first; the lane's levels are contiguous, so they
// are fetched four at a time (one or two cache lines) instead of one dependent load per level
MRT_DFN f3 fold_level(float4 a, f3 L) {
    if (a.w < 0.0f) return f3{a.x * L.x, a.y * L.y, a.z * L.z};
    return f3{0.0f + ((a.x * L.x) / a.w), 0.0f + ((a.y * L.y) / a.w), 0.0f + ((a.z * L.z) / a.w)};
}
template <uint32_t LK>
MRT_DFN f3 fold_levels(const LevStore<LK>& lev, uint32_t nlev, f3 L) {
    // a black end through quiet levels stays +0 (the common escaped path): nothing to fold
    if (!(nlev & LEV_LOUD) && ((__float_as_uint(L.x) | __float_as_uint(L.y) | __float_as_uint(L.z)) == 0)) return L;
    int d = (int)(nlev & ~LEV_LOUD) - 1;
#ifndef MRT_FOLD_SERIAL
    // HBM levels four at a time: the four loads (contiguous in the lane's row, indices clamped to
    // stay inside it) are in flight together, then folded deepest first: one memory round trip per
    // four levels (C2 +1.6%)
    while (d >= (int)LK) {
        const int lo = (int)LK;
        const float4 a = lev.get((uint32_t)d), b = lev.get((uint32_t)max(d - 1, lo)), c = lev.get((uint32_t)max(d - 2, lo)),
                     e = lev.get((uint32_t)max(d - 3, lo));
        L = fold_level(a, L);
        if (d - 1 >= lo) L = fold_level(b, L);
        if (d - 2 >= lo) L = fold_level(c, L);
        if (d - 3 >= lo) L = fold_level(e, L);
        d = max(d - 4, lo - 1);
    }
#endif
    for (; d >= 0; d--) L = fold_level(lev.get((uint32_t)d), L);
    return L;
}
// a path's radiance from its end's emitted (or sky / black) L
template <uint32_t LK>
MRT_DFN f3 end_path(const PathState& ps, const LevStore<LK>& lev, f3 L) {
#if MRT_FWD_FOLD
    (void)lev;
    return f3{ps.T.x * L.x, ps.T.y * L.y, ps.T.z * L.z};
#else
    return fold_levels(lev, ps.nlev, L);
#endif
}

// ---- draw() / draw2()'s per-pixel accumulation (main.cpp:150-175, 205-231), both backends ----
MRT_DFN float lum3(f3 c) { return (c.x * 0.212655f + c.y * 0.715158f) + c.z * 0.072187f; }

// one sample of draw()/draw2()'s per-pixel loop
MRT_DFN f3 fold_sample(f3 c, f3 smp, uint32_t s, uint32_t mode, float max_lum) {
    if (mode == 0) {
        if (!finite3(smp)) smp = c;
        return add(c, smp);
    }
    if (!finite3(smp)) smp = s > 0 ? c : f3{0, 0, 0};
    if (s > 0) smp = add(c, mulf(sub(smp, c), 1.0f / ((float)s + 1.0f)));
    float l = lum3(smp);
    if (l > max_lum) smp = mulf(smp, max_lum / l);
    return smp;
}
// the pixel after its last sample: mode 0 divides by the sample count and clamps the luminance
// (main.cpp:168-173); mode 1's running average is final as it is
MRT_DFN f3 final_pixel(f3 c, uint32_t ns, uint32_t mode, float max_lum) {
    if (mode == 0) {
        c = divf(c, (float)ns);
        float l = lum3(c);
        if (l > max_lum) c = mulf(c, max_lum / l);
    }
    return c;
}

}  // namespace mrtd
