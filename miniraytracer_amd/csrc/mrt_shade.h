// mrt_shade.h -- textures, materials, pdfs and the per-path bounce loop (trace(), main.cpp:66-118)
#pragma once
#include "mrt_trace.h"

namespace mrtd {

// perlin_noise::noise / turbulence (texture.cpp:68-165)
__device__ __forceinline__ float perlin_noise(const DScene& S, f3 p) {
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
            acc += ((a.x * a.y) * a.z) * dot(c, weights);
        }
    }
    return acc;
}
__device__ __forceinline__ float turbulence(const DScene& S, f3 p) {
    float acc = 0, weight = 1.0f;
    for (int i = 0; i < 7; i++) {
        acc += weight * perlin_noise(S, p);
        weight *= 0.5f;
        p = mulf(p, 2);
    }
    return fabsf(acc);
}

// texture::sample (texture.h:18-20, 56-62; texture.cpp:7-25, 207-224)
__device__ __forceinline__ f3 tex_sample(const DScene& S, uint32_t t, float u, float v, f3 p) {
    for (;;) {
        const mrt_texture& T = S.texs[t];
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

// onb(n) * vec (onb.h:19-27)
__device__ __forceinline__ f3 onb_apply(f3 w, f3 vec) {
    f3 a = fabsf(w.x) > 0.9f ? f3{0, 1, 0} : f3{1, 0, 0};
    f3 v = normalize(cross(w, a));
    f3 u = cross(w, v);
    return add(add(fmul(vec.x, u), fmul(vec.y, v)), fmul(vec.z, w));
}

// biased object pdfs: object_list / xz_rect / sphere pdf_value & pdf_generate
// (scene_object.h:64-77, rect.cpp:92-107, sphere.cpp:63-78, scene_object.h:24-29)
__device__ __forceinline__ float leaf_pdf_value(const DScene& S, const mrt_node& n, f3 origin, f3 dir, float time) {
    uint32_t k = MRT_NODE_KIND(n);
    HitRec rec;
    if (k == MRT_K_XZ) {
        Ray r = make_ray(origin, dir, 0.0f, 0);
        if (rect_hit<1>(n, r, 0.001f, FLT_MAX_, rec, true)) {
            float area = (n.f[1] - n.f[0]) * (n.f[3] - n.f[2]);
            float dist_sq = rec.t * rec.t;
            float cosine = fabsf(dot(dir, rec.n));
            return dist_sq / (cosine * area);
        }
        return 0;
    }
    if (k == MRT_K_SPHERE) {
        Ray r = make_ray(origin, dir, time, 0);
        if (sphere_hit(n, r, 0.001f, FLT_MAX_, rec, false)) {
            float radius = n.f[8];
            float cos_theta_max = __builtin_sqrtf(1 - (radius * radius) / sdot(sub(sphere_center(n, time), origin)));
            float solid_angle = (2 * PI_F) * (1 - cos_theta_max);
            return 1 / solid_angle;
        }
        return 0;
    }
    return 0;
}
__device__ __forceinline__ float biased_pdf_value(const DScene& S, uint32_t node, f3 origin, f3 dir, float time) {
    const mrt_node& n = S.nodes[node];
    if (MRT_NODE_KIND(n) != MRT_K_LIST) return leaf_pdf_value(S, n, origin, dir, time);
    float sum = 0;
    for (uint32_t i = 0; i < n.b; i++) sum += leaf_pdf_value(S, S.nodes[S.children[n.a + i]], origin, dir, time);
    return sum / (float)n.b;
}
__device__ __forceinline__ f3 leaf_pdf_generate(const DScene& S, const mrt_node& n, f3 origin, float time, Pcg& rng) {
    uint32_t k = MRT_NODE_KIND(n);
    if (k == MRT_K_XZ) {
        float a = randf(rng);
        float x = n.f[0] + a * (n.f[1] - n.f[0]);
        float b = randf(rng);
        float z = n.f[2] + b * (n.f[3] - n.f[2]);
        return sub(f3{x, n.f[4], z}, origin);
    }
    if (k == MRT_K_SPHERE) {
        f3 dir = sub(sphere_center(n, time), origin);
        float dist_sq = sdot(dir);
        f3 w = normalize(dir);
        return onb_apply(w, random_towards_sphere(rng, n.f[8], dist_sq));
    }
    return f3{1, 0, 0};
}
__device__ __forceinline__ f3 biased_pdf_generate(const DScene& S, uint32_t node, f3 origin, float time, Pcg& rng) {
    const mrt_node& n = S.nodes[node];
    if (MRT_NODE_KIND(n) != MRT_K_LIST) return leaf_pdf_generate(S, n, origin, time, rng);
    int i = int(randf(rng) * (float)n.b);
    return leaf_pdf_generate(S, S.nodes[S.children[n.a + i]], origin, time, rng);
}

// One path: camera ray -> bounce loop -> radiance.  Per-bounce (attenuation*scatter_pdf, pdf)
// pairs go to `lev` and are folded back deepest-first exactly as the recursion of trace()
// returns: L = emitted + ((a * L) / pdf) (diffuse), L = attenuation * L (specular, pdf < 0).
struct PathOut {
    f3 L;
    uint32_t rays;
};

__device__ __forceinline__ PathOut trace_path(const DScene& S, Pcg& rng, float s, float t, uint32_t max_bounces, float4* __restrict__ lev,
                                              size_t lev_stride) {
    // camera::get_ray (camera.h:38-44)
    const mrt_camera& C = S.cam;
    f3 rd = fmul(C.lens_radius, random_in_disk(rng));
    f3 offset = add(mulf(ld3(C.u), rd.x), mulf(ld3(C.v), rd.y));
    float time = C.time0 + (C.time1 - C.time0) * randf(rng);
    f3 origin = ld3(C.origin);
    f3 dir = sub(sub(add(add(ld3(C.llcorner), fmul(s, ld3(C.horz))), fmul(t, ld3(C.vert))), origin), offset);
    Ray r = make_ray(add(origin, offset), dir, time, 0);

    uint32_t depth = 0, rays = 0;
    f3 L;
    for (;;) {
        rays++;
        HitRec rec;
        if (!scene_hit(S, r, 0.001f, rec, rng)) {
            if (S.sky) {  // main.cpp:113-115
                float tt = 0.5f * (r.d.y + 1.0f);
                float o = 1.0f - tt;
                L = f3{o + tt * 0.5f, o + tt * 0.7f, o + tt * 1.0f};
            } else {
                L = f3{0, 0, 0};
            }
            break;
        }
        const mrt_material M = S.mats[rec.mat];
        if (M.kind == MRT_M_LIGHT) {  // diffuse_light: sampleEmissive, never scatters (material.h:190-199)
            if (dot(rec.n, r.d) < 0.0f) L = fmul(M.p, tex_sample(S, M.tex, rec.u, rec.v, rec.p));
            else L = f3{0, 0, 0};
            break;
        }
        if (depth >= max_bounces) {  // emitted of a non-emissive material
            L = f3{0, 0, 0};
            break;
        }
        float4* slot = lev + (size_t)depth * lev_stride;
        if (M.kind == MRT_M_METAL) {  // metal::scatter (material.h:91-98)
            f3 reflected = sub(r.d, fmul(2.0f * dot(r.d, rec.n), rec.n));
            f3 rs = random_in_sphere(rng);
            f3 nd = add(reflected, fmul(1 - M.p, rs));
            f3 att = tex_sample(S, M.tex, rec.u, rec.v, rec.p);
            *slot = make_float4(att.x, att.y, att.z, -1.0f);
            r = make_ray(rec.p, nd, r.time, 0);
        } else if (M.kind == MRT_M_DIELECTRIC) {  // dielectric::scatter (material.h:121-175)
            float ref = M.p;
            float cosI = -dot(r.d, rec.n);
            f3 facing;
            float nio;
            if (cosI < 0) {
                facing = f3{-rec.n.x, -rec.n.y, -rec.n.z};
                nio = ref;
            } else {
                facing = rec.n;
                nio = 1.0f / ref;
            }
            f3 reflected = sub(r.d, fmul(2.0f * dot(r.d, rec.n), rec.n));
            // refract (vec3.h:185-198)
            float ncosI = dot(r.d, facing);
            float sinT2 = (nio * nio) * (1.0f - ncosI * ncosI);
            int inside = r.inside;
            f3 nd;
            if (sinT2 <= 1.0f) {
                float cosT = __builtin_sqrtf(1.0f - sinT2);
                float ci = -ncosI;
                f3 refracted = add(fmul(nio, r.d), fmul(nio * ci - cosT, facing));
                float cs = cosI < 0 ? __builtin_sqrtf(1.0f - (nio * nio) * (1.0f - cosI * cosI)) : cosI;
                float r0 = (1 - ref) / (1 + ref);
                r0 = r0 * r0;
                float reflect_prob = r0 + (1 - r0) * pow5_((1 - cs));
                if (randf(rng) < reflect_prob) {
                    nd = reflected;
                } else {
                    if (cosI < 0) {
                        inside--;
                        if (inside < 0) inside = 0;
                    } else {
                        inside++;
                    }
                    nd = refracted;
                }
            } else {
                nd = reflected;
            }
            *slot = make_float4(1.0f, 1.0f, 1.0f, -1.0f);
            r = make_ray(rec.p, nd, r.time, inside);
        } else {  // lambertian / isotropic (material.h:48-74), mix_pdf with the biased list (main.cpp:84-102)
            bool lamb = M.kind == MRT_M_LAMBERTIAN;
            f3 att = tex_sample(S, M.tex, rec.u, rec.v, rec.p);
            f3 gen;
            bool surface = true;
            if (S.biased != MRT_NONE && randf(rng) < 0.5f) {
                gen = biased_pdf_generate(S, S.biased, rec.p, r.time, rng);
                surface = false;
            }
            if (surface) gen = lamb ? onb_apply(rec.n, random_cosine_direction(rng)) : random_in_sphere(rng);
            Ray sc = make_ray(rec.p, gen, r.time, 0);
            float sval;
            if (lamb) {
                float cosine = dot(sc.d, rec.n);
                sval = cosine > 0 ? cosine / PI_F : 0;
            } else {
                sval = 1 / (2 * PI_F);
            }
            float pdf_v = S.biased != MRT_NONE ? 0.5f * (biased_pdf_value(S, S.biased, rec.p, sc.d, r.time) + sval) : sval;
            float spdf;
            if (lamb) {
                float cosine = dot(rec.n, sc.d);
                spdf = cosine < 0 ? 0 : cosine * (1.0f / PI_F);
            } else {
                spdf = 1.0f / (2.0f * PI_F);
            }
            *slot = make_float4(att.x * spdf, att.y * spdf, att.z * spdf, pdf_v);
            r = sc;
        }
        depth++;
    }
    // fold back (the recursion's return path)
    for (int d = (int)depth - 1; d >= 0; d--) {
        float4 a = lev[(size_t)d * lev_stride];
        if (a.w < 0.0f) {
            L = f3{a.x * L.x, a.y * L.y, a.z * L.z};
        } else {
            L = f3{0.0f + ((a.x * L.x) / a.w), 0.0f + ((a.y * L.y) / a.w), 0.0f + ((a.z * L.z) / a.w)};
        }
    }
    return PathOut{L, rays};
}

}  // namespace mrtd
