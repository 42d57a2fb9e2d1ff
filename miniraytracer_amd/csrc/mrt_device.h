// mrt_device.h -- device-side restatement of the reference hot path for gfx950 (CDNA4, wave64).
//
//   PCG32 + samplers          pcg.cpp:13-136
//   ray / camera              ray.h:18-56, camera.h:38-44
//   aabb slab test            aabb.h:45-77 (SSE minps/maxps NaN semantics kept)
//   rect / sphere / triangle  rect.cpp:24-152, sphere.cpp:6-78, triangle.cpp:222-265
//   object_list / bvh_node    scene_object.h:79-103, 208-244
//   pod_bvh                   triangle.h:171-221 (first-hit DFS, closer child by node_order)
//   translate / rotate_y      scene_object.cpp:9-18, 70-98
//   constant_volume           volumes.cpp:5-35
//   materials / pdfs / onb    material.h:34-200, pdf.h:18-80, onb.h:19-30
//   textures                  texture.cpp:7-224
//
// Numerics contract (DESIGN.md "Numerics"): every float operation is written in the reference's
// order and the file is compiled with -ffp-contract=off, f32 division and sqrt correctly rounded
// (hipcc default), denormals kept; sin/cos/log/pow/atan2/asin are evaluated in double and rounded
// once, the same definition the host builder and the C restatement use.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

// One source, two backends: the hot-path functions below are compiled for gfx950 (the path
// kernels, mrt_kernels.hip) and -- in the CPU backend's translation unit, which defines
// MRT_HOST_BACKEND -- for the host as well (mrt_cpu.hip).  Device intrinsics sit behind
// __HIP_DEVICE_COMPILE__ with IEEE host forms, so the exact contract gives the same bits on both.
#ifdef MRT_HOST_BACKEND
#define MRT_DATTR __host__ __device__
#else
#define MRT_DATTR __device__
#endif
#define MRT_DFN MRT_DATTR __forceinline__
#if defined(MRT_HOST_BACKEND) && !defined(__HIP_DEVICE_COMPILE__)
#include <cmath>
#include <cstring>
// host forms of the HIP device built-ins the hot path uses (overloads by target attribute)
__host__ static inline unsigned int __float_as_uint(float x) { unsigned int u; memcpy(&u, &x, 4); return u; }
__host__ static inline float __uint_as_float(unsigned int u) { float x; memcpy(&x, &u, 4); return x; }
__host__ static inline int __float_as_int(float x) { int u; memcpy(&u, &x, 4); return u; }
__host__ static inline float __int_as_float(int u) { float x; memcpy(&x, &u, 4); return x; }
__host__ static inline bool isfinite(float x) { return std::isfinite(x); }
__host__ static inline bool signbit(double x) { return std::signbit(x); }
#endif
#include "../../include/mrt_mathfn.h"
#include "../../include/mrt_scene.h"

// MRT_FAST=1 builds the tolerance-contract kernels (DESIGN.md "Numerics contracts"): hardware
// reciprocal / square root / reciprocal square root, f32 transcendentals, no exactness range
// guards; the translation unit is compiled with FMA contraction and reciprocal division (as the
// reference as shipped contracts a*b+c).  MRT_FAST=0 (default) is the exact contract.
#ifndef MRT_FAST
#define MRT_FAST 0
#endif
// parts of the tolerance contract (all on with MRT_FAST; separable for experiments)
#ifndef MRT_FAST_DIV
#define MRT_FAST_DIV MRT_FAST    // reciprocal-based division
#endif
#ifndef MRT_FAST_SQRT
#define MRT_FAST_SQRT MRT_FAST   // v_sqrt_f32
#endif
#ifndef MRT_FAST_NORM
#define MRT_FAST_NORM MRT_FAST   // normalize by v_rsq_f32
#endif
#ifndef MRT_FAST_TRANS
#define MRT_FAST_TRANS MRT_FAST  // f32 / hardware transcendentals
#endif
#ifndef MRT_FAST_GUARDS
#define MRT_FAST_GUARDS MRT_FAST // no exactness range guards
#endif
// A rect hit's point is put ON the rect's plane (p[axis] = k).  Under the exact contract
// o + RN(t*d) with t = RN((k - o)/d) lands on the plane almost always; with FMA contraction or a
// reciprocal-based t it lands ~1e-5 off either side, and a grazing scattered ray from a point just
// outside a face of an instanced box then re-hits that face at t > tmin (0.001): +0.1-0.2% rays on
// the Cornell box (measured; DESIGN.md "Numerics contracts").  Snapping restores the exact
// contract's geometry.
#ifndef MRT_FAST_SNAP
#define MRT_FAST_SNAP MRT_FAST
#endif
// The recursion's return path (L = emitted + a*L/pdf, main.cpp:84-104) evaluated FORWARD: a
// running throughput T = (T*a)/pdf per bounce, L = T*emitted at the path's end, instead of storing
// every bounce's (a, pdf) and folding them deepest-first.  Same factors, another association (a
// rounding difference per bounce), so tolerance contract only; it needs no per-bounce level
// storage (LDS / HBM) and no fold loop.
// box.h's six rects as one slab test (mrt_sig.h box6_hit), tolerance contract only
#ifndef MRT_FAST_BOX
#define MRT_FAST_BOX MRT_FAST
#endif
#ifndef MRT_FWD_FOLD
#define MRT_FWD_FOLD MRT_FAST
#endif
// the Cornell room's five walls as one slab test (mrt_sig.h cornell_room), tolerance contract only
#ifndef MRT_FAST_ROOM
#define MRT_FAST_ROOM MRT_FAST
#endif
// slab tests as one fma per plane (aabb_hit), tolerance contract only
#ifndef MRT_FAST_SLAB
#define MRT_FAST_SLAB MRT_FAST
#endif

namespace mrtd {

struct f3 {
    float x, y, z;
};
MRT_DFN f3 mk(float x, float y, float z) { return f3{x, y, z}; }
MRT_DFN f3 add(f3 a, f3 b) { return f3{a.x + b.x, a.y + b.y, a.z + b.z}; }
MRT_DFN f3 sub(f3 a, f3 b) { return f3{a.x - b.x, a.y - b.y, a.z - b.z}; }
MRT_DFN f3 mul(f3 a, f3 b) { return f3{a.x * b.x, a.y * b.y, a.z * b.z}; }
MRT_DFN f3 mulf(f3 a, float f) { return f3{a.x * f, a.y * f, a.z * f}; }
MRT_DFN f3 fmul(float f, f3 a) { return f3{f * a.x, f * a.y, f * a.z}; }
#if MRT_FAST_DIV && defined(__HIP_DEVICE_COMPILE__)
MRT_DFN f3 divf(f3 a, float f) {
    const float y = __builtin_amdgcn_rcpf(f);
    return f3{a.x * y, a.y * y, a.z * y};
}
#else
MRT_DFN f3 divf(f3 a, float f) { return f3{a.x / f, a.y / f, a.z / f}; }
#endif
MRT_DFN float dot(f3 a, f3 b) { return (a.x * b.x + a.y * b.y) + a.z * b.z; }
MRT_DFN float sdot(f3 a) { return (a.x * a.x + a.y * a.y) + a.z * a.z; }
// a*b + c rounded the same way wherever it is inlined: one fma in the tolerance build, where
// contraction is decided per use site (a product with other uses may stay unfused), so a hit
// predicate inlined twice -- a leaf's t-only test and its record's second test -- could otherwise
// round two ways; a product then a sum in the exact build (no contraction there).  For sums the
// reference computes with SSE Vec3 operators (never fused there).
MRT_DFN float madd_det(float a, float b, float c) {
#if MRT_FAST
    return __builtin_fmaf(a, b, c);
#else
    return a * b + c;
#endif
}
// The reference's own fused multiply-adds.  Built as shipped (clang -O3 -march=native: FMA,
// -ffp-contract=on), it fuses a*b+c exactly where ONE scalar source expression holds a product
// as an operand of a sum or difference -- clang's fmuladd rule: the left operand is tried first,
// `x*y - z` -> fma(x, y, -z), `z - x*y` -> fma(-x, y, z) -- and nowhere else (its Vec3 operators are
// SSE intrinsics, never fused).  Every such site on the hot path calls one of these, naming the
// reference line; everything else is compiled with -ffp-contract=off (exact contract), so the
// exact contract reproduces the reference as shipped bit for bit (with the project's
// transcendentals, include/mrt_mathfn.h).  The tolerance contract fuses them too.
// ref_fma(a, b, c) = a*b + c; ref_fms(a, b, c) = a*b - c; ref_fnma(a, b, c) = c - a*b
MRT_DFN float ref_fma(float a, float b, float c) { return __builtin_fmaf(a, b, c); }
MRT_DFN float ref_fms(float a, float b, float c) { return __builtin_fmaf(a, b, -c); }
MRT_DFN float ref_fnma(float a, float b, float c) { return __builtin_fmaf(-a, b, c); }
// sphere::hit's quadratic (sphere.cpp:20-26): b = dot(oc, d), c = |oc|^2 - r^2, disc = b*b - c.
MRT_DFN float sphere_disc(f3 oc, f3 d, float radius, float* bout) {
#pragma clang fp contract(off)
    const float b = (oc.x * d.x + oc.y * d.y) + oc.z * d.z;
    const float s = (oc.x * oc.x + oc.y * oc.y) + oc.z * oc.z;
    *bout = b;
    // the reference's scalar tail, fused as shipped (the dot products are SSE, unfused):
    // c = sdot(oc) - radius*radius, discriminant = b*b - c (sphere.cpp:20-21)
    const float c = ref_fnma(radius, radius, s);
    return ref_fms(b, b, c);
}
// ---- exact f32 division on a short path (tools/numcheck/markstein_check.hip) ----------------------
// IEEE a/b compiles to 11 VALU (div_scale x2, rcp, 6 fma, div_fmas, div_fixup).  With y = RN(1/b)
// known, Markstein's correction q' = q + (a - b*q)*y (q = RN(a*y), residual exact by fma) IS the
// correctly rounded quotient unless something over/underflows (div_core, 4 VALU).  y itself is
// v_rcp_f32 + one Newton step (recip_nr, 3 VALU), equal to IEEE 1/b for every normal b with a
// normal reciprocal -- all 2^32 patterns checked on MI355X.  div_core == IEEE a/b was checked for
// every normal divisor x 32 numerators (9.7e10 quotients, 0 mismatches) under: b and y normal, and
// a == 0 or (q' normal and |a| >= 2^-100).  Call sites establish those conditions from cheap range
// tests on their operands (a ray's `nice` flag, normalize's own test) and take the IEEE division in
// a wave-uniform branch otherwise (never taken on real scenes).
MRT_DFN float recip_nr(float b) {
#if MRT_FAST_DIV && defined(__HIP_DEVICE_COMPILE__)
    return __builtin_amdgcn_rcpf(b);
#elif defined(__HIP_DEVICE_COMPILE__)
    const float y0 = __builtin_amdgcn_rcpf(b);
    return __builtin_fmaf(__builtin_fmaf(-b, y0, 1.0f), y0, y0);
#else
    return 1.0f / b;
#endif
}
MRT_DFN float div_core(float a, float b, float y) {
#if MRT_FAST_DIV
    return a * y;
#endif
    const float q = a * y;
    const float r = __builtin_fmaf(-b, q, a);
    return __builtin_copysignf(__builtin_fmaf(r, y, q), q);
}
MRT_DFN bool any_lane(bool p) {
#if defined(__HIP_DEVICE_COMPILE__)
    return __builtin_amdgcn_ballot_w64(p) != 0;
#else
    return p;
#endif
}
// a ? b : c for lane booleans as lane-mask logic (SALU and / andn2 / or on the wave's masks): the
// compiler's select of two booleans materialised each as 0 / 1 in a VGPR and compared it back
// (4-6 VALU per BVH child pair).  MRT_SEL_MASK 0: the plain select (A/B hook).
#ifndef MRT_SEL_MASK
#define MRT_SEL_MASK 1
#endif
MRT_DFN bool sel_b(bool a, bool b, bool c) {
#if defined(__HIP_DEVICE_COMPILE__) && MRT_SEL_MASK
    const uint64_t ma = __builtin_amdgcn_ballot_w64(a), mb = __builtin_amdgcn_ballot_w64(b), mc = __builtin_amdgcn_ballot_w64(c);
    return __builtin_amdgcn_inverse_ballot_w64((ma & mb) | (~ma & mc));
#else
    return a ? b : c;
#endif
}
// |x| as an unsigned key (sign shifted out): 2^e -> (e + 127) << 24, 0 -> 0, inf/NaN above all finite
MRT_DFN uint32_t mag2(float x) { return __float_as_uint(x) << 1; }
#define MRT_MAG2(e) ((uint32_t)((e) + 127) << 24)
// |x| in [2^lo, 2^hi)
#define MRT_MAG_IN(x, lo, hi) ((uint32_t)((mag2(x) - MRT_MAG2(lo)) < (MRT_MAG2(hi) - MRT_MAG2(lo))))
// Correctly rounded f32 square root.  hipcc's expansion is v_sqrt_f32, a one-ulp neighbour test
// by fma residuals, and a 2^32 scaling of inputs below 2^-96 (+ zero/inf fix-up); the core alone
// equals it for every input with |x| >= 2^-96 or x == +-0 (all 2^32 patterns checked on MI355X,
// tools/numcheck/sqrt_check.hip).  (RN32(v_sqrt_f64(x)) is NOT exact: v_sqrt_f64 misrounds 3.9% of
// f32 inputs, tools/numcheck/divsqrt_check.hip.)
MRT_DFN float sqrt_core(float x) {
#if MRT_FAST_SQRT && defined(__HIP_DEVICE_COMPILE__)
    return __builtin_amdgcn_sqrtf(x);
#elif defined(__HIP_DEVICE_COMPILE__)
    const float s = __builtin_amdgcn_sqrtf(x);
    const float sdn = __uint_as_float(__float_as_uint(s) - 1u), sup = __uint_as_float(__float_as_uint(s) + 1u);
    const float r = __builtin_fmaf(-sdn, s, x) <= 0.0f ? sdn : s;
    return __builtin_fmaf(-sup, s, x) > 0.0f ? sup : r;
#else
    return __builtin_sqrtf(x);
#endif
}
MRT_DFN float sqrt_(float x) {
    float r = sqrt_core(x);
    if (MRT_FAST_SQRT) return r;
    const bool ok = mag2(x) - 1u >= MRT_MAG2(-96) - 1u;  // |x| >= 2^-96 or x == +-0
    if (__builtin_expect(any_lane(!ok), 0)) r = ok ? r : __builtin_sqrtf(x);
    return r;
}
// a / |a| (Vec3::normalize, vec3.h:116-122): one reciprocal for the three quotients.  Fast path:
// |a|^2 in [2^-52, 2^52) and every component 0 or >= 2^-100 in magnitude (then each quotient is 0
// or normal, and y is normal).
MRT_DFN f3 normalize(f3 a) {
    const float dd = sdot(a);
#if MRT_FAST_NORM && defined(__HIP_DEVICE_COMPILE__)
    const float ry = __builtin_amdgcn_rsqf(dd);
    return f3{a.x * ry, a.y * ry, a.z * ry};
#endif
    const float len = sqrt_core(dd);  // |a|^2 in [2^-52, 2^52): the core is exact, |a| in [2^-26, 2^26)
    const float y = recip_nr(len);
    f3 q{div_core(a.x, len, y), div_core(a.y, len, y), div_core(a.z, len, y)};
    const uint32_t mn = min(min(mag2(a.x) - 1u, mag2(a.y) - 1u), mag2(a.z) - 1u);  // 0 -> UINT_MAX
    const bool ok = MRT_MAG_IN(dd, -52, 52) & (mn >= MRT_MAG2(-100) - 1u);
    if (__builtin_expect(any_lane(!ok), 0)) q = ok ? q : divf(a, __builtin_sqrtf(dd));
    return q;
}
MRT_DFN f3 cross(f3 a, f3 b) { return f3{a.y * b.z - a.z * b.y, a.z * b.x - a.x * b.z, a.x * b.y - a.y * b.x}; }
MRT_DFN float maxps(float a, float b) { return a > b ? a : b; }
MRT_DFN float minps(float a, float b) { return a < b ? a : b; }
MRT_DFN f3 ld3(const float* p) { return f3{p[0], p[1], p[2]}; }
MRT_DFN f3 ld3(float4 v) { return f3{v.x, v.y, v.z}; }
MRT_DFN bool finite3(f3 a) { return isfinite(a.x) && isfinite(a.y) && isfinite(a.z); }

static constexpr float PI_F = 3.14159265358979323846f;
static constexpr float FLT_MAX_ = 3.402823466e+38f;

#if MRT_FAST_TRANS && defined(__HIP_DEVICE_COMPILE__)
// tolerance contract: f32 library functions; sincos of a path angle in [0, 2 pi) by the hardware
// v_sin/v_cos (argument in revolutions), log by v_log (log2)
MRT_DFN float sin_(float x) { return sinf(x); }
MRT_DFN float cos_(float x) { return cosf(x); }
MRT_DFN void sincos_(float x, float* s, float* c) {
    const float rev = x * 0.15915494309189535f;
    *s = __builtin_amdgcn_sinf(rev);
    *c = __builtin_amdgcn_cosf(rev);
}
#ifndef MRT_FAST_LOG_LIB
#define MRT_FAST_LOG_LIB 0
#endif
#if MRT_FAST_LOG_LIB
MRT_DFN float log_(float x) { return logf(x); }  // ocml f32 log (v_log_f32 loses relative accuracy near 1)
#else
MRT_DFN float log_(float x) { return __builtin_amdgcn_logf(x) * 0.69314718055994531f; }
#endif
MRT_DFN float pow5_(float x) {
    const float x2 = x * x;
    return (x2 * x2) * x;
}
MRT_DFN float atan2_(float y, float x) { return atan2f(y, x); }
MRT_DFN float asin_(float x) { return asinf(x); }
#else
// transcendentals: the numerics contract of include/mrt_mathfn.h (same bits as host and oracle)
MRT_DFN float sin_(float x) { return mrt_sinf(x); }
MRT_DFN float cos_(float x) { return mrt_cosf(x); }
MRT_DFN void sincos_(float x, float* s, float* c) {
    double ds, dc;
    mrt_sincos_d((double)x, &ds, &dc);
    *s = (float)ds;
    *c = (float)dc;
}
MRT_DFN float log_(float x) { return mrt_logf(x); }
MRT_DFN float pow5_(float x) { return mrt_pow5f(x); }
MRT_DFN float atan2_(float y, float x) { return mrt_atan2f(y, x); }
MRT_DFN float asin_(float x) { return mrt_asinf(x); }
#endif

// ---------------------------------------------------------------- PCG32 (pcg.cpp:13-62)
struct Pcg {
    uint64_t state, inc;
};
MRT_DFN uint32_t pcg_next(Pcg& r) {
    uint64_t old = r.state;
    r.state = old * 6364136223846793005ULL + r.inc;
    uint32_t xs = (uint32_t)(((old >> 18u) ^ old) >> 27u);
    uint32_t rot = (uint32_t)(old >> 59u);
    return (xs >> rot) | (xs << ((0u - rot) & 31u));
}
MRT_DFN void pcg_seed(Pcg& r, uint64_t initstate, uint64_t initseq) {
    r.state = 0u;
    r.inc = (initseq << 1u) | 1u;
    pcg_next(r);
    r.state += initstate;
    pcg_next(r);
}
MRT_DFN float randf(Pcg& r) {
    return __uint_as_float(0x3f800000u | (pcg_next(r) & 0x007FFFFFu)) - 1.0f;
}
MRT_DFN uint64_t splitmix64(uint64_t z) {
    z += 0x9E3779B97F4A7C15ull;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}
// samplers (pcg.cpp:70-136); Vec3(randf(), randf(), ...) arguments drawn left to right
MRT_DFN f3 random_in_sphere(Pcg& r) {
    f3 p;
    do {
        float a = randf(r), b = randf(r), c = randf(r);
        p = f3{2.0f * a - 1.0f, 2.0f * b - 1.0f, 2.0f * c - 1.0f};
    } while (sdot(p) >= 1.0f);
    return p;
}
MRT_DFN f3 random_in_disk(Pcg& r) {
    f3 p;
    do {
        float a = randf(r), b = randf(r);
        p = f3{2.0f * a - 1.0f, 2.0f * b - 1.0f, 0.0f};
    } while ((p.x * p.x + p.y * p.y) >= 1.0f);
    return p;
}
// random_cosine_direction (pcg.cpp:87-95) given its two draws r1, r2 (the caller draws them, in
// that order).  NOTE: x,y scaled by 2*sqrt(r2), as the reference does (pcg.cpp:92-93).
// randf() is 0 or >= 2^-23: both radicands are 0 or in [2^-23, 1], where sqrt_core is exact.
MRT_DFN f3 random_cosine_direction_pre(float r1, float r2) {
    float z = sqrt_core(1 - r2);
    float phi = (2 * PI_F) * r1;
    float s2 = sqrt_core(r2);
    float sp, cp;
    sincos_(phi, &sp, &cp);
    return f3{(cp * 2) * s2, (sp * 2) * s2, z};
}
// random_towards_sphere (pcg.cpp:125-133) given its two draws r1, r2 (sphere::pdf_generate, sphere.cpp:63-78)
MRT_DFN f3 random_towards_sphere_pre(float r1, float r2, float radius, float dist_sq) {
    float z = ref_fma(r2, sqrt_(1 - (radius * radius) / dist_sq) - 1, 1);  // pcg.cpp:128
    float phi = (2 * PI_F) * r1;
    float q = sqrt_(ref_fnma(z, z, 1));  // pcg.cpp:130-131
    float sp, cp;
    sincos_(phi, &sp, &cp);
    return f3{cp * q, sp * q, z};
}

// ---------------------------------------------------------------- ray (ray.h:18-56)
struct Ray {
    f3 o, d, inv;  // inv = RN(1/d) per lane (aabb.h:49), hoisted out of the slab and rect tests
    float time;
    int inside;
    uint32_t mask;
    bool nice;     // operand ranges under which inv and rect-test quotients take div_core (ray_nice)
};
// A ray is `nice` when every direction component has magnitude in [2^-26, 2) and every origin
// component is 0 or in [2^-77, 2^60]: then inv = recip_nr(d) is exact, and a rect test's
// (k - o_a) / d_a may use div_core with inv (the difference of two such coordinates -- rect planes are
// checked on upload, MRT_F_SLOWDIV -- is 0 or >= 2^-100, and the quotient stays normal).
MRT_DFN bool ray_nice(f3 o, f3 d) {
    if (MRT_FAST_GUARDS) return true;  // no exactness guards: every ray takes the hardware reciprocal
    const bool dn = MRT_MAG_IN(d.x, -26, 1) & MRT_MAG_IN(d.y, -26, 1) & MRT_MAG_IN(d.z, -26, 1);
    const uint32_t mn = min(min(mag2(o.x) - 1u, mag2(o.y) - 1u), mag2(o.z) - 1u);  // 0 -> UINT_MAX
    const float mx = fmaxf(fmaxf(fabsf(o.x), fabsf(o.y)), fabsf(o.z));
    return dn & (mn >= MRT_MAG2(-77) - 1u) & (mx <= 0x1p60f);
}
// 1/d per component (aabb.h:49), exact
MRT_DFN f3 ray_inv(f3 d, bool nice) {
    f3 y{recip_nr(d.x), recip_nr(d.y), recip_nr(d.z)};
    if (__builtin_expect(any_lane(!nice), 0)) y = nice ? y : f3{1.0f / d.x, 1.0f / d.y, 1.0f / d.z};
    return y;
}
MRT_DFN Ray make_ray(f3 o, f3 dir, float time, int inside) {
    Ray r;
    r.o = o;
    r.d = normalize(dir);
    r.time = time;
    r.inside = inside;
    // ComputeDirMask runs on the constructor ARGUMENT (ray.h:51 sees the parameter `dir`)
    uint32_t X = __float_as_uint(dir.x) >> 31, Y = __float_as_uint(dir.y) >> 31, Z = __float_as_uint(dir.z) >> 31;
    r.mask = 1u << (Z | (Y << 1) | (X << 2));
    r.nice = ray_nice(r.o, r.d);
    r.inv = ray_inv(r.d, r.nice);
    return r;
}
// A ray whose direction argument is already of unit length up to rounding (a ray's normalized
// direction, rotated or reused): the exact contract runs the constructor as the reference does;
// the tolerance contract skips the renormalization (a change of at most an ulp or two).
// U: skip it (the tolerance contract's kernels without bvh_node subtrees, textures or volumes --
// kFastUnit<F>, mrt_trace.h; measured on book2 at 2048^2 x 1024 spp: renormalising keeps its
// per-pixel RMSE vs the reference as shipped at 2.1e-3 instead of 1.2e-2, DESIGN.md "Numerics")
#ifndef MRT_FAST_UNIT
#define MRT_FAST_UNIT MRT_FAST
#endif
template <bool U = MRT_FAST_UNIT>
MRT_DFN Ray make_ray_unit(f3 o, f3 dir, float time, int inside) {
    if constexpr (!U) return make_ray(o, dir, time, inside);
    Ray r;
    r.o = o;
    r.d = dir;
    r.time = time;
    r.inside = inside;
    uint32_t X = __float_as_uint(dir.x) >> 31, Y = __float_as_uint(dir.y) >> 31, Z = __float_as_uint(dir.z) >> 31;
    r.mask = 1u << (Z | (Y << 1) | (X << 2));
    r.nice = ray_nice(r.o, r.d);
    r.inv = ray_inv(r.d, r.nice);
    return r;
}
// translate::hit's moved ray (scene_object.cpp:11): the same direction, a new origin
template <bool U = MRT_FAST_UNIT>
MRT_DFN Ray moved_ray(const Ray& r0, f3 o) {
    if constexpr (!U) return make_ray(o, r0.d, r0.time, 0);
    Ray r = r0;  // direction, its reciprocal and mask reused as they are
    r.o = o;
    r.inside = 0;
    r.nice = ray_nice(r.o, r.d);
    return r;
}
// a wave-uniform value the compiler cannot prove uniform, as an SGPR (host: itself)
MRT_DFN uint32_t uniform_u32(uint32_t v) {
#if defined(__HIP_DEVICE_COMPILE__)
    return (uint32_t)__builtin_amdgcn_readfirstlane((int)v);
#else
    return v;
#endif
}
// x, y or z by a per-lane axis index, as selects (a select chain on one index was turned into a
// per-lane lookup table in scratch memory)
MRT_DFN float sel3(uint32_t a, float x, float y, float z) {
    float v = a == 1u ? y : x;
#if defined(__HIP_DEVICE_COMPILE__)
    asm volatile("" : "+v"(v));
#endif
    return a == 2u ? z : v;
}
MRT_DFN f3 eval(const Ray& r, float t) { return add(r.o, fmul(t, r.d)); }

// aabb::hit, active SSE branch (aabb.h:49-76).  `bad`: some lane of the wave may hold a ray that is
// not nice (wave-uniform; a walk computes it once for all its box tests instead of per test)
MRT_DFN bool aabb_hit_b(const float* bmin, const float* bmax, const Ray& r, float tmin, float tmax, bool bad) {
#if MRT_FAST_SLAB
    // tolerance contract: (b - o) * inv as fma(b, inv, -(o * inv)); the products o * inv are shared
    // by every box a walk step tests with the same ray (one multiply-add per slab instead of two)
    const float nox = -(r.o.x * r.inv.x), noy = -(r.o.y * r.inv.y), noz = -(r.o.z * r.inv.z);
    float t0x = __builtin_fmaf(bmin[0], r.inv.x, nox), t0y = __builtin_fmaf(bmin[1], r.inv.y, noy), t0z = __builtin_fmaf(bmin[2], r.inv.z, noz);
    float t1x = __builtin_fmaf(bmax[0], r.inv.x, nox), t1y = __builtin_fmaf(bmax[1], r.inv.y, noy), t1z = __builtin_fmaf(bmax[2], r.inv.z, noz);
#else
    float t0x = (bmin[0] - r.o.x) * r.inv.x, t0y = (bmin[1] - r.o.y) * r.inv.y, t0z = (bmin[2] - r.o.z) * r.inv.z;
    float t1x = (bmax[0] - r.o.x) * r.inv.x, t1y = (bmax[1] - r.o.y) * r.inv.y, t1z = (bmax[2] - r.o.z) * r.inv.z;
#endif
    // A nice ray (|inv| <= 2^26, |o| <= 2^60) with a box of finite coordinates gets no NaN slab
    // values, and (bmin - o) * inv <= (bmax - o) * inv exactly when inv >= 0: the blendv swap is a
    // min/max, and maxps/minps (NaN-asymmetric) are plain max/min.  The result is a comparison, so
    // the zero signs min/max may pick do not matter.
    float lo = fmaxf(fmaxf(fminf(t0x, t1x), fminf(t0z, t1z)), fmaxf(fminf(t0y, t1y), tmin));
    float hi = fminf(fminf(fmaxf(t0x, t1x), fmaxf(t0z, t1z)), fminf(fmaxf(t0y, t1y), tmax));
    if (__builtin_expect(bad, 0)) {
        bool lx = r.inv.x < 0.0f, ly = r.inv.y < 0.0f, lz = r.inv.z < 0.0f;
        float ax = lx ? t1x : t0x, bx = lx ? t0x : t1x;
        float ay = ly ? t1y : t0y, by = ly ? t0y : t1y;
        float az = lz ? t1z : t0z, bz = lz ? t0z : t1z;
        float lo2 = maxps(maxps(ax, az), maxps(ay, tmin));
        float hi2 = minps(minps(bx, bz), minps(by, tmax));
        // (the bounds merged, one comparison after the branch: a merged boolean cost two VALU
        // copies per test)
        lo = r.nice ? lo : lo2;
        hi = r.nice ? hi : hi2;
    }
    return hi > lo;
}
MRT_DFN bool aabb_hit(const float* bmin, const float* bmax, const Ray& r, float tmin, float tmax) {
    return aabb_hit_b(bmin, bmax, r, tmin, tmax, any_lane(!r.nice));
}
MRT_DFN bool aabb_hit_b(f3 bmin, f3 bmax, const Ray& r, float tmin, float tmax, bool bad) {
    const float b[6] = {bmin.x, bmin.y, bmin.z, bmax.x, bmax.y, bmax.z};
    return aabb_hit_b(b, b + 3, r, tmin, tmax, bad);
}

MRT_DFN bool aabb_hit(f3 bmin, f3 bmax, const Ray& r, float tmin, float tmax) {
    const float b[6] = {bmin.x, bmin.y, bmin.z, bmax.x, bmax.y, bmax.z};
    return aabb_hit(b, b + 3, r, tmin, tmax);
}

// uniform-address reads of scene tables through the constant address space -> s_load
#if defined(__HIP_DEVICE_COMPILE__)
#define MRT_CONST_AS __attribute__((address_space(4)))
#else
#define MRT_CONST_AS
#endif
#define MRT_F_SLOWDIV 0x8u  /* set on upload on rects whose plane coordinate is outside {0} U [2^-77, 2^60] */
#if defined(__HIP_DEVICE_COMPILE__)
#define MRT_GLOBAL_AS __attribute__((address_space(1)))
#define MRT_LDS_AS __attribute__((address_space(3)))
#else
#define MRT_GLOBAL_AS
#define MRT_LDS_AS
#endif
typedef float v4f __attribute__((ext_vector_type(4)));  // native vector: loads/stores in any address space
template <typename T>
MRT_DFN const MRT_CONST_AS T* const_ptr(const T* p) {
    return (const MRT_CONST_AS T*)p;
}
#if defined(__HIP_DEVICE_COMPILE__)  // (host: the same type as ld3(const float*))
MRT_DFN f3 ld3(const MRT_CONST_AS float* p) { return f3{p[0], p[1], p[2]}; }
#endif

// Phase clock (experiment builds with -DMRT_PHASES): wave-uniform s_memtime deltas per phase.
#ifdef MRT_PHASES
struct PhaseClock {
    uint64_t t, a[12];  // 0-7: path loop phases; 8-11: inside scene_hit_lin (lists/instances, prims, volumes, BVHs)
};
#define PH_MARK(pc, i)                                      \
    do {                                                    \
        const uint64_t n_ = __builtin_amdgcn_s_memtime();   \
        (pc).a[i] += n_ - (pc).t;                           \
        (pc).t = n_;                                        \
    } while (0)
#else
struct PhaseClock {};
#define PH_MARK(pc, i) \
    do {               \
    } while (0)
#endif
// Branch occupancy (experiment builds with -DMRT_EXPERIMENTS -DMRT_BSTATS): per counting point,
// the wave executions reaching it and the lanes active there (g_bstats[2i], g_bstats[2i+1]).
#if defined(MRT_EXPERIMENTS) && defined(MRT_BSTATS) && defined(__HIP_DEVICE_COMPILE__)
extern __device__ unsigned long long g_bstats[64];
#define BSTAT(i)                                                                      \
    do {                                                                              \
        const uint64_t m_ = __builtin_amdgcn_ballot_w64(true);                        \
        if (__builtin_amdgcn_mbcnt_hi((uint32_t)(m_ >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m_, 0u)) == 0u) { \
            atomicAdd(&g_bstats[2 * (i)], 1ull);                                      \
            atomicAdd(&g_bstats[2 * (i) + 1], (unsigned long long)__popcll(m_));      \
        }                                                                             \
    } while (0)
// lanes where cond holds, counted at an execution of the wave (all active lanes reach it)
#define BSTATC(i, cond)                                                               \
    do {                                                                              \
        const uint64_t m_ = __builtin_amdgcn_ballot_w64(true);                        \
        const uint64_t c_ = __builtin_amdgcn_ballot_w64(cond);                        \
        if (__builtin_amdgcn_mbcnt_hi((uint32_t)(m_ >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m_, 0u)) == 0u) { \
            atomicAdd(&g_bstats[2 * (i)], 1ull);                                      \
            atomicAdd(&g_bstats[2 * (i) + 1], (unsigned long long)__popcll(c_));      \
        }                                                                             \
    } while (0)
#else
#define BSTAT(i) \
    do {         \
    } while (0)
#define BSTATC(i, cond) \
    do {                \
    } while (0)
#endif

struct HitRec {
    float t;
    f3 p, n;
    float u, v;
    uint32_t mat;
};

}  // namespace mrtd
