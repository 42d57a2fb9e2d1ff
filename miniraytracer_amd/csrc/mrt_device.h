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

#include "../../include/mrt_mathfn.h"
#include "../../include/mrt_scene.h"

namespace mrtd {

struct f3 {
    float x, y, z;
};
__device__ __forceinline__ f3 mk(float x, float y, float z) { return f3{x, y, z}; }
__device__ __forceinline__ f3 add(f3 a, f3 b) { return f3{a.x + b.x, a.y + b.y, a.z + b.z}; }
__device__ __forceinline__ f3 sub(f3 a, f3 b) { return f3{a.x - b.x, a.y - b.y, a.z - b.z}; }
__device__ __forceinline__ f3 mul(f3 a, f3 b) { return f3{a.x * b.x, a.y * b.y, a.z * b.z}; }
__device__ __forceinline__ f3 mulf(f3 a, float f) { return f3{a.x * f, a.y * f, a.z * f}; }
__device__ __forceinline__ f3 fmul(float f, f3 a) { return f3{f * a.x, f * a.y, f * a.z}; }
__device__ __forceinline__ f3 divf(f3 a, float f) { return f3{a.x / f, a.y / f, a.z / f}; }
__device__ __forceinline__ float dot(f3 a, f3 b) { return (a.x * b.x + a.y * b.y) + a.z * b.z; }
__device__ __forceinline__ float sdot(f3 a) { return (a.x * a.x + a.y * a.y) + a.z * a.z; }
__device__ __forceinline__ f3 normalize(f3 a) { return divf(a, __builtin_sqrtf(sdot(a))); }
__device__ __forceinline__ f3 cross(f3 a, f3 b) { return f3{a.y * b.z - a.z * b.y, a.z * b.x - a.x * b.z, a.x * b.y - a.y * b.x}; }
__device__ __forceinline__ float maxps(float a, float b) { return a > b ? a : b; }
__device__ __forceinline__ float minps(float a, float b) { return a < b ? a : b; }
__device__ __forceinline__ f3 ld3(const float* p) { return f3{p[0], p[1], p[2]}; }
__device__ __forceinline__ f3 ld3(float4 v) { return f3{v.x, v.y, v.z}; }
__device__ __forceinline__ bool finite3(f3 a) { return isfinite(a.x) && isfinite(a.y) && isfinite(a.z); }

static constexpr float PI_F = 3.14159265358979323846f;
static constexpr float FLT_MAX_ = 3.402823466e+38f;

// transcendentals: the numerics contract of include/mrt_mathfn.h (same bits as host and oracle)
__device__ __forceinline__ float sin_(float x) { return mrt_sinf(x); }
__device__ __forceinline__ float cos_(float x) { return mrt_cosf(x); }
__device__ __forceinline__ void sincos_(float x, float* s, float* c) {
    double ds, dc;
    mrt_sincos_d((double)x, &ds, &dc);
    *s = (float)ds;
    *c = (float)dc;
}
__device__ __forceinline__ float log_(float x) { return mrt_logf(x); }
__device__ __forceinline__ float pow5_(float x) { return mrt_pow5f(x); }
__device__ __forceinline__ float atan2_(float y, float x) { return mrt_atan2f(y, x); }
__device__ __forceinline__ float asin_(float x) { return mrt_asinf(x); }

// ---------------------------------------------------------------- PCG32 (pcg.cpp:13-62)
struct Pcg {
    uint64_t state, inc;
};
__device__ __forceinline__ uint32_t pcg_next(Pcg& r) {
    uint64_t old = r.state;
    r.state = old * 6364136223846793005ULL + r.inc;
    uint32_t xs = (uint32_t)(((old >> 18u) ^ old) >> 27u);
    uint32_t rot = (uint32_t)(old >> 59u);
    return (xs >> rot) | (xs << ((0u - rot) & 31u));
}
__device__ __forceinline__ void pcg_seed(Pcg& r, uint64_t initstate, uint64_t initseq) {
    r.state = 0u;
    r.inc = (initseq << 1u) | 1u;
    pcg_next(r);
    r.state += initstate;
    pcg_next(r);
}
__device__ __forceinline__ float randf(Pcg& r) {
    return __uint_as_float(0x3f800000u | (pcg_next(r) & 0x007FFFFFu)) - 1.0f;
}
__device__ __forceinline__ uint64_t splitmix64(uint64_t z) {
    z += 0x9E3779B97F4A7C15ull;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}
// samplers (pcg.cpp:70-136); Vec3(randf(), randf(), ...) arguments drawn left to right
__device__ __forceinline__ f3 random_in_sphere(Pcg& r) {
    f3 p;
    do {
        float a = randf(r), b = randf(r), c = randf(r);
        p = f3{2.0f * a - 1.0f, 2.0f * b - 1.0f, 2.0f * c - 1.0f};
    } while (sdot(p) >= 1.0f);
    return p;
}
__device__ __forceinline__ f3 random_in_disk(Pcg& r) {
    f3 p;
    do {
        float a = randf(r), b = randf(r);
        p = f3{2.0f * a - 1.0f, 2.0f * b - 1.0f, 0.0f};
    } while ((p.x * p.x + p.y * p.y) >= 1.0f);
    return p;
}
// NOTE: x,y scaled by 2*sqrt(r2), as the reference does (pcg.cpp:92-93)
__device__ __forceinline__ f3 random_cosine_direction(Pcg& r) {
    float r1 = randf(r), r2 = randf(r);
    float z = __builtin_sqrtf(1 - r2);
    float phi = (2 * PI_F) * r1;
    float s2 = __builtin_sqrtf(r2);
    float sp, cp;
    sincos_(phi, &sp, &cp);
    return f3{(cp * 2) * s2, (sp * 2) * s2, z};
}
__device__ __forceinline__ f3 random_towards_sphere(Pcg& r, float radius, float dist_sq) {
    float r1 = randf(r), r2 = randf(r);
    float z = 1 + r2 * (__builtin_sqrtf(1 - (radius * radius) / dist_sq) - 1);
    float phi = (2 * PI_F) * r1;
    float q = __builtin_sqrtf(1 - z * z);
    float sp, cp;
    sincos_(phi, &sp, &cp);
    return f3{cp * q, sp * q, z};
}

// ---------------------------------------------------------------- ray (ray.h:18-56)
struct Ray {
    f3 o, d, inv;  // inv = 1/d per lane (aabb.h:49), hoisted out of the slab tests
    float time;
    int inside;
    uint32_t mask;
};
__device__ __forceinline__ Ray make_ray(f3 o, f3 dir, float time, int inside) {
    Ray r;
    r.o = o;
    r.d = normalize(dir);
    r.time = time;
    r.inside = inside;
    // ComputeDirMask runs on the constructor ARGUMENT (ray.h:51 sees the parameter `dir`)
    uint32_t X = __float_as_uint(dir.x) >> 31, Y = __float_as_uint(dir.y) >> 31, Z = __float_as_uint(dir.z) >> 31;
    r.mask = 1u << (Z | (Y << 1) | (X << 2));
    r.inv = f3{1.0f / r.d.x, 1.0f / r.d.y, 1.0f / r.d.z};
    return r;
}
__device__ __forceinline__ f3 eval(const Ray& r, float t) { return add(r.o, fmul(t, r.d)); }

// aabb::hit, active SSE branch (aabb.h:49-76)
__device__ __forceinline__ bool aabb_hit(const float* bmin, const float* bmax, const Ray& r, float tmin, float tmax) {
    float t0x = (bmin[0] - r.o.x) * r.inv.x, t0y = (bmin[1] - r.o.y) * r.inv.y, t0z = (bmin[2] - r.o.z) * r.inv.z;
    float t1x = (bmax[0] - r.o.x) * r.inv.x, t1y = (bmax[1] - r.o.y) * r.inv.y, t1z = (bmax[2] - r.o.z) * r.inv.z;
    bool lx = r.inv.x < 0.0f, ly = r.inv.y < 0.0f, lz = r.inv.z < 0.0f;
    float ax = lx ? t1x : t0x, bx = lx ? t0x : t1x;
    float ay = ly ? t1y : t0y, by = ly ? t0y : t1y;
    float az = lz ? t1z : t0z, bz = lz ? t0z : t1z;
    float lo = maxps(maxps(ax, az), maxps(ay, tmin));
    float hi = minps(minps(bx, bz), minps(by, tmax));
    return hi > lo;
}

__device__ __forceinline__ bool aabb_hit(f3 bmin, f3 bmax, const Ray& r, float tmin, float tmax) {
    const float b[6] = {bmin.x, bmin.y, bmin.z, bmax.x, bmax.y, bmax.z};
    return aabb_hit(b, b + 3, r, tmin, tmax);
}

// uniform-address reads of scene tables through the constant address space -> s_load
#define MRT_CONST_AS __attribute__((address_space(4)))
template <typename T>
__device__ __forceinline__ const MRT_CONST_AS T* const_ptr(const T* p) {
    return (const MRT_CONST_AS T*)p;
}

// Phase clock (experiment builds with -DMRT_PHASES): wave-uniform s_memtime deltas per phase.
#ifdef MRT_PHASES
struct PhaseClock {
    uint64_t t, a[4];
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

struct HitRec {
    float t;
    f3 p, n;
    float u, v;
    uint32_t mat;
};

}  // namespace mrtd
