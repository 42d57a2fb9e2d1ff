// host_math.h -- host-side float3 / PCG used by the scene builder.
//
// The reference does its vector math on 16-byte SSE vectors (vec3.h:11-333).  For every lane the
// results are plain IEEE single operations, so this header restates them as scalar code with the
// same operation order (no FMA contraction: the library is compiled with -ffp-contract=off):
//   dot(a,b)   = (a.x*b.x + a.y*b.y) + a.z*b.z                     vec3.h:245-248
//   sdot(v)    = (x*x + y*y) + (z*z + w*w), w == 0 on every path   vec3.h:116-122
//   normalize  = v / sqrt(sdot(v)) (true division per lane)        vec3.h:137-144
//   vmin/vmax  = SSE minps/maxps: a<b ? a : b / a>b ? a : b        vec3.h:157-171
//   cross      = (a.yzx*b.zxy) - (a.zxy*b.yzx)                     vec3.h:252-266
// Transcendentals follow the numerics contract of include/mrt_mathfn.h (DESIGN.md "Numerics").
#pragma once
#include <cmath>
#include <cstdint>
#include <cstring>

#include "../../include/mrt_mathfn.h"

namespace mrt {

struct V3 {
    float x, y, z;
};
static inline V3 v3(float x, float y, float z) { return V3{x, y, z}; }
static inline V3 operator+(V3 a, V3 b) { return V3{a.x + b.x, a.y + b.y, a.z + b.z}; }
static inline V3 operator-(V3 a, V3 b) { return V3{a.x - b.x, a.y - b.y, a.z - b.z}; }
static inline V3 operator-(V3 a) { return V3{-a.x, -a.y, -a.z}; }
static inline V3 operator*(V3 a, V3 b) { return V3{a.x * b.x, a.y * b.y, a.z * b.z}; }
static inline V3 operator*(V3 a, float f) { return V3{a.x * f, a.y * f, a.z * f}; }
static inline V3 operator*(float f, V3 a) { return V3{f * a.x, f * a.y, f * a.z}; }
static inline V3 operator/(V3 a, float f) { return V3{a.x / f, a.y / f, a.z / f}; }
static inline float dot(V3 a, V3 b) { return (a.x * b.x + a.y * b.y) + a.z * b.z; }
static inline float sdot(V3 a) { return (a.x * a.x + a.y * a.y) + a.z * a.z; }
static inline float length(V3 a) { return std::sqrt(sdot(a)); }
static inline V3 normalize(V3 a) { return a / length(a); }
static inline float fmin_ps(float a, float b) { return a < b ? a : b; }
static inline float fmax_ps(float a, float b) { return a > b ? a : b; }
static inline V3 vmin(V3 a, V3 b) { return V3{fmin_ps(a.x, b.x), fmin_ps(a.y, b.y), fmin_ps(a.z, b.z)}; }
static inline V3 vmax(V3 a, V3 b) { return V3{fmax_ps(a.x, b.x), fmax_ps(a.y, b.y), fmax_ps(a.z, b.z)}; }
static inline V3 cross(V3 a, V3 b) {
    return V3{a.y * b.z - a.z * b.y, a.z * b.x - a.x * b.z, a.x * b.y - a.y * b.x};
}
static inline float get(V3 a, int i) { return i == 0 ? a.x : (i == 1 ? a.y : a.z); }
// max_dim (vec3.h:316-324)
static inline int max_dim(V3 a) {
    bool v01 = a.x > a.y, v02 = a.x > a.z, v12 = a.y > a.z;
    return v01 ? (v02 ? 0 : 2) : (v12 ? 1 : 2);
}

static const float PI_F = 3.14159265358979323846f;  // M_PI_F (mrt_math.h:11)
static inline float rad(float a) { return a * (PI_F / 180.0f); }

static inline float sin_(float x) { return mrt_sinf(x); }
static inline float cos_(float x) { return mrt_cosf(x); }
static inline float tan_(float x) { return mrt_tanf(x); }

// PCG32 XSH-RR (pcg.cpp:13-35)
struct Pcg {
    uint64_t state, inc;
};
static inline uint32_t pcg_next(Pcg& r) {
    uint64_t old = r.state;
    r.state = old * 6364136223846793005ULL + r.inc;
    uint32_t xs = (uint32_t)(((old >> 18u) ^ old) >> 27u);
    uint32_t rot = (uint32_t)(old >> 59u);
    return (xs >> rot) | (xs << ((0u - rot) & 31u));
}
static inline void pcg_seed(Pcg& r, uint64_t initstate, uint64_t initseq) {
    r.state = 0u;
    r.inc = (initseq << 1u) | 1u;
    pcg_next(r);
    r.state += initstate;
    pcg_next(r);
}
// randf (pcg.cpp:53-62): mantissa bits under 1.0f, minus 1
static inline float randf(Pcg& r) {
    uint32_t b = 0x3f800000u | (pcg_next(r) & 0x007FFFFFu);
    float f;
    memcpy(&f, &b, 4);
    return f - 1.0f;
}
// random_in_sphere (pcg.cpp:70-77); arguments drawn left to right (clang order)
static inline V3 random_in_sphere(Pcg& r) {
    V3 p;
    do {
        float a = randf(r), b = randf(r), c = randf(r);
        p = V3{2.0f * a - 1.0f, 2.0f * b - 1.0f, 2.0f * c - 1.0f};
    } while (sdot(p) >= 1.0f);
    return p;
}

}  // namespace mrt
