/* oracle/mrt_oracle.c -- TEST INFRASTRUCTURE ONLY (see mrt_oracle.h).
 *
 * Plain-C restatement of the reference render path, written recursively in the shape of the
 * reference's virtual calls so that it shares no structure with the HIP kernel's explicit-stack
 * walk.  Every function cites the reference code it restates.  Float operations follow the
 * reference's order; build with -ffp-contract=off (the reference's SSE intrinsics never fuse),
 * and the reference's scalar expressions that the shipped build fuses (x86 FMA under clang's
 * -ffp-contract=on: a product operand of a sum in one expression) are explicit fmaf() calls.
 * sin/cos/log/pow/atan2/asin follow the numerics contract of include/mrt_mathfn.h -- the functions
 * the exact reference build (oracle/_ref/mrt_ref_exact) interposes, so the two agree bit for bit.
 */
#define _GNU_SOURCE
#include "mrt_oracle.h"
#include "../include/mrt_mathfn.h"

#include <float.h>
#include <math.h>
#include <pthread.h>
#include <stdlib.h>
#include <string.h>

typedef struct { float x, y, z; } V;
static V v3(float x, float y, float z) { V r = {x, y, z}; return r; }
static V vadd(V a, V b) { return v3(a.x + b.x, a.y + b.y, a.z + b.z); }
static V vsub(V a, V b) { return v3(a.x - b.x, a.y - b.y, a.z - b.z); }
static V vmul(V a, V b) { return v3(a.x * b.x, a.y * b.y, a.z * b.z); }
static V vscale(float f, V a) { return v3(f * a.x, f * a.y, f * a.z); }
static V vdivf(V a, float f) { return v3(a.x / f, a.y / f, a.z / f); }
static float vdot(V a, V b) { return (a.x * b.x + a.y * b.y) + a.z * b.z; }            /* vec3.h:245-248 */
static float vsdot(V a) { return (a.x * a.x + a.y * a.y) + (a.z * a.z + 0.0f * 0.0f); } /* vec3.h:116-122 */
static V vnorm(V a) { return vdivf(a, sqrtf(vsdot(a))); }                               /* vec3.h:137-139 */
static V vcross(V a, V b) { return v3(a.y * b.z - a.z * b.y, a.z * b.x - a.x * b.z, a.x * b.y - a.y * b.x); }
static V ld(const float* p) { return v3(p[0], p[1], p[2]); }
static float maxps(float a, float b) { return a > b ? a : b; }
static float minps(float a, float b) { return a < b ? a : b; }
static const float PI_F = 3.14159265358979323846f;

/* transcendentals: the numerics contract (include/mrt_mathfn.h) */
static float sin_(float x) { return mrt_sinf(x); }
static float cos_(float x) { return mrt_cosf(x); }
static float log_(float x) { return mrt_logf(x); }
static float pow_(float x, float y) { return y == 5.0f ? mrt_pow5f(x) : (float)pow((double)x, (double)y); }
static float atan2_(float y, float x) { return mrt_atan2f(y, x); }
static float asin_(float x) { return mrt_asinf(x); }

/* ---------------------------------------------------------------- PCG (pcg.cpp:11-136) */
typedef struct { uint64_t state, inc; } pcg;
static uint32_t pcg_next(pcg* r) {
    uint64_t old = r->state;
    r->state = old * 6364136223846793005ULL + r->inc;
    uint32_t xs = (uint32_t)(((old >> 18u) ^ old) >> 27u);
    uint32_t rot = (uint32_t)(old >> 59u);
    return (xs >> rot) | (xs << ((-rot) & 31));
}
static void pcg_srandom(pcg* r, uint64_t st, uint64_t sq) {
    r->state = 0U;
    r->inc = (sq << 1u) | 1u;
    pcg_next(r);
    r->state += st;
    pcg_next(r);
}
static float randf(pcg* r) {
    union { float f; uint32_t b; } a;
    a.b = 0x3f800000u | (pcg_next(r) & 0x007FFFFFu);
    return a.f - 1.0f;
}
static V random_in_sphere(pcg* r) {
    V p;
    do {
        float a = randf(r), b = randf(r), c = randf(r);
        p = vsub(vscale(2.0f, v3(a, b, c)), v3(1, 1, 1));
    } while (vsdot(p) >= 1.0f);
    return p;
}
static V random_in_disk(pcg* r) {
    V p;
    do {
        float a = randf(r), b = randf(r);
        p = vsub(vscale(2.0f, v3(a, b, 0)), v3(1, 1, 0));
    } while (vsdot(p) >= 1.0f);
    return p;
}
static V random_cosine_direction(pcg* r) {
    float r1 = randf(r);
    float r2 = randf(r);
    float z = sqrtf(1 - r2);
    float phi = 2 * PI_F * r1;
    float x = cos_(phi) * 2 * sqrtf(r2);
    float y = sin_(phi) * 2 * sqrtf(r2);
    return v3(x, y, z);
}
static V random_on_sphere_uniform(pcg* r) {
    float x = fmaf(randf(r), 2, -1.0f); /* pcg.cpp:101-103, fused as shipped */
    float phi = randf(r) * 2 * PI_F;
    float s = sqrtf(fmaf(-x, x, 1));
    return v3(x, cos_(phi) * s, sin_(phi) * s);
}
static V random_towards_sphere(pcg* r, float radius, float dist_sq) {
    float r1 = randf(r);
    float r2 = randf(r);
    float z = fmaf(r2, sqrtf(1 - radius * radius / dist_sq) - 1, 1);
    float phi = 2 * PI_F * r1;
    float x = cos_(phi) * sqrtf(fmaf(-z, z, 1));
    float y = sin_(phi) * sqrtf(fmaf(-z, z, 1));
    return v3(x, y, z);
}
static uint64_t splitmix64(uint64_t z) {
    z += 0x9E3779B97F4A7C15ull;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}

/* ---------------------------------------------------------------- ray (ray.h:18-56) */
typedef struct {
    V origin, dir;
    float time;
    int inside;
    uint32_t mask;
} ray;
static ray mkray(V o, V d, float time, int inside) {
    ray r;
    r.origin = o;
    r.dir = vnorm(d);
    r.time = time;
    r.inside = inside;
    union { float f; uint32_t u; } X = {d.x}, Y = {d.y}, Z = {d.z}; /* parameter, not member */
    r.mask = 1u << ((Z.u >> 31) | ((Y.u >> 31) << 1) | ((X.u >> 31) << 2));
    return r;
}
static V ray_eval(const ray* r, float t) { return vadd(r->origin, vscale(t, r->dir)); }

/* aabb::hit (aabb.h:49-76) */
static int aabb_hit(const float* b, const ray* r, float tmin, float tmax) {
    V inv = v3(1.0f / r->dir.x, 1.0f / r->dir.y, 1.0f / r->dir.z);
    V t0 = vmul(vsub(ld(b), r->origin), inv);
    V t1 = vmul(vsub(ld(b + 3), r->origin), inv);
    V a = t0, c = t1;
    if (inv.x < 0.0f) { a.x = t1.x; c.x = t0.x; }
    if (inv.y < 0.0f) { a.y = t1.y; c.y = t0.y; }
    if (inv.z < 0.0f) { a.z = t1.z; c.z = t0.z; }
    float lo0 = maxps(a.x, a.z), lo1 = maxps(a.y, tmin);
    float hi0 = minps(c.x, c.z), hi1 = minps(c.y, tmax);
    return minps(hi0, hi1) > maxps(lo0, lo1);
}

typedef struct {
    float t;
    V p, n;
    float u, v;
    uint32_t mat;
} hit_record;

typedef struct {
    const mrt_scene_view* v;
    pcg rng;
} ctx;

#define KIND(n) ((n)->kind & 0xFFu)
#define ORDER(n) (((n)->kind >> 8) & 0xFFu)
#define FLAGS(n) (((n)->kind >> 16) & 0xFFu)

static int obj_hit(ctx* C, uint32_t id, const ray* r, float tmin, float tmax, hit_record* rec);

/* sphere (sphere.cpp:6-46) */
static V sphere_center(const mrt_node* n, float time) {
    if (FLAGS(n) & MRT_F_MOVING) return vadd(ld(n->f), vscale((time - n->f[6]) / (n->f[7] - n->f[6]), vsub(ld(n->f + 3), ld(n->f))));
    return ld(n->f);
}
static void sphere_uv(V p, float* u, float* v) {
    float phi = atan2_(p.z, p.x);
    float theta = asin_(p.y);
    *u = fmaf(-phi, 1.0f / (2.0f * PI_F), 0.5f);
    *v = fmaf(theta, 1.0f / PI_F, 0.5f);
}
static int sphere_hit(const mrt_node* n, const ray* r, float tmin, float tmax, hit_record* rec) {
    rec->mat = n->mat;
    V cen = sphere_center(n, r->time);
    float radius = n->f[8];
    V oc = vsub(r->origin, cen);
    float b = vdot(oc, r->dir);
    float c = fmaf(-radius, radius, vsdot(oc));
    float disc = fmaf(b, b, -c);
    if (disc > 0) {
        float t = (-b - sqrtf(disc));
        if (t < tmax && t > tmin) {
            rec->t = t;
            rec->p = ray_eval(r, t);
            rec->n = vdivf(vsub(rec->p, cen), radius);
            sphere_uv(rec->n, &rec->u, &rec->v);
            return 1;
        }
        if (r->inside) {
            t = (-b + sqrtf(disc));
            if (t < tmax && t > tmin) {
                rec->t = t;
                rec->p = ray_eval(r, t);
                rec->n = vdivf(vsub(rec->p, cen), radius);
                sphere_uv(rec->n, &rec->u, &rec->v);
                return 1;
            }
        }
    }
    return 0;
}

/* rects (rect.cpp:24-45, 69-90, 130-151); ax = plane axis (0 yz, 1 xz, 2 xy) */
static float comp(V a, int i) { return i == 0 ? a.x : (i == 1 ? a.y : a.z); }
static int rect_hit(const mrt_node* n, int ax, const ray* r, float tmin, float tmax, hit_record* rec) {
    V nrm = v3(ax == 0 ? n->f[5] : 0, ax == 1 ? n->f[5] : 0, ax == 2 ? n->f[5] : 0);
    if (vdot(r->dir, nrm) > 0.0f) return 0;
    float t = (n->f[4] - comp(r->origin, ax)) / comp(r->dir, ax);
    if (t < tmin || t > tmax) return 0;
    int ia = ax == 0 ? 1 : 0, ib = ax == 2 ? 1 : 2;
    float a = fmaf(t, comp(r->dir, ia), comp(r->origin, ia));
    float b = fmaf(t, comp(r->dir, ib), comp(r->origin, ib));
    if (a < n->f[0] || a > n->f[1] || b < n->f[2] || b > n->f[3]) return 0;
    rec->u = (a - n->f[0]) / (n->f[1] - n->f[0]);
    rec->v = (b - n->f[2]) / (n->f[3] - n->f[2]);
    rec->t = t;
    rec->mat = n->mat;
    rec->p = ray_eval(r, t);
    rec->n = nrm;
    return 1;
}

/* triangle::hit (triangle.cpp:222-265) */
static int tri_hit(const mrt_scene_view* v, uint32_t i, uint32_t mat, const ray* r, float tmin, float tmax, hit_record* rec) {
    const float* g = v->tri_geo + (size_t)i * 12;
    const float* q = v->tri_nrm + (size_t)i * 12;
    V m = ld(g), u = ld(g + 4), w = ld(g + 8);
    V pvec = vcross(r->dir, w);
    float det = vdot(u, pvec);
    float sign = 1.0f;
    if (r->inside) {
        sign = det < 0.0f ? -1.0f : 1.0f;
        det = sign * det;
    }
    if (det < 0.00001f) return 0;
    V tvec = vsub(r->origin, m);
    float uu = vdot(tvec, pvec) * sign;
    V qvec = vcross(tvec, u);
    float vv = vdot(r->dir, qvec) * sign;
    if ((uu < 0) | (uu > det) | (vv < 0) | ((uu + vv) > det)) return 0;
    float invDet = 1 / det;
    float t = vdot(w, qvec) * invDet * sign;
    if ((t < tmin) | (t > tmax)) return 0;
    uu *= invDet;
    vv *= invDet;
    rec->t = t;
    rec->p = ray_eval(r, t);
    rec->n = vnorm(vadd(vadd(vscale(1 - uu - vv, ld(q)), vscale(uu, ld(q + 4))), vscale(vv, ld(q + 8))));
    rec->u = uu;
    rec->v = vv;
    rec->mat = mat;
    return 1;
}

/* pod_bvh::hit (triangle.h:171-213), recursive as in the reference */
static int mesh_node_hit(const mrt_scene_view* v, uint32_t ni, uint32_t mat, const ray* r, float tmin, float tmax, hit_record* rec) {
    const mrt_mesh_node* n = &v->mesh_nodes[ni];
    float box[6] = {n->bmin[0], n->bmin[1], n->bmin[2], n->bmax[0], n->bmax[1], n->bmax[2]};
    if (!aabb_hit(box, r, tmin, tmax)) return 0;
    uint32_t cnt = n->count_order & 0xFFFFFFu;
    int has_hit = 0;
    if (cnt) {
        for (uint32_t i = 0; i < cnt; i++)
            if (tri_hit(v, n->left_or_first + i, mat, r, tmin, tmax, rec)) {
                has_hit = 1;
                tmax = rec->t;
            }
    } else {
        uint32_t closer, farther;
        if ((n->count_order >> 24) & r->mask) {
            closer = n->left_or_first;
            farther = n->left_or_first + 1;
        } else {
            closer = n->left_or_first + 1;
            farther = n->left_or_first;
        }
        int hit_closer = mesh_node_hit(v, closer, mat, r, tmin, tmax, rec);
        if (hit_closer) return 1;
        return mesh_node_hit(v, farther, mat, r, tmin, tmax, rec);
    }
    return has_hit;
}

/* scene_object::hit dispatch (scene_object.h:79-103, 208-244; scene_object.cpp:9-18, 70-98;
 * volumes.cpp:5-35) */
static int obj_hit(ctx* C, uint32_t id, const ray* r, float tmin, float tmax, hit_record* rec) {
    const mrt_scene_view* v = C->v;
    const mrt_node* n = &v->nodes[id];
    switch (KIND(n)) {
    case MRT_K_LIST: {
        if (!(FLAGS(n) & MRT_F_HASBOX) || aabb_hit(n->f, r, tmin, tmax)) {
            hit_record cur;
            memset(&cur, 0, sizeof cur);
            int hit = 0;
            float closest = tmax;
            for (uint32_t i = 0; i < n->b; i++) {
                if (obj_hit(C, v->children[n->a + i], r, tmin, closest, &cur)) {
                    hit = 1;
                    closest = cur.t;
                    *rec = cur;
                }
            }
            return hit;
        }
        return 0;
    }
    case MRT_K_BVH: {
        if (aabb_hit(n->f, r, tmin, tmax)) {
            uint32_t closer, farther;
            if (ORDER(n) & r->mask) {
                closer = n->a;
                farther = n->b;
            } else {
                closer = n->b;
                farther = n->a;
            }
            if (obj_hit(C, closer, r, tmin, tmax, rec)) return 1;
            return obj_hit(C, farther, r, tmin, tmax, rec);
        }
        return 0;
    }
    case MRT_K_MESH:
        return mesh_node_hit(v, n->a, n->mat, r, tmin, tmax, rec);
    case MRT_K_TRANSLATE: {
        ray moved = mkray(vsub(r->origin, ld(n->f)), r->dir, r->time, 0);
        if (obj_hit(C, n->a, &moved, tmin, tmax, rec)) {
            rec->p = vadd(rec->p, ld(n->f));
            return 1;
        }
        return 0;
    }
    case MRT_K_ROTY: {
        if ((FLAGS(n) & MRT_F_HASBOX) && !aabb_hit(n->f, r, tmin, tmax)) return 0;
        float s = n->f[6], c = n->f[7];
        V o = r->origin, d = r->dir;
        o.x = fmaf(c, r->origin.x, -(s * r->origin.z));
        o.z = fmaf(c, r->origin.z, s * r->origin.x);
        d.x = fmaf(c, r->dir.x, -(s * r->dir.z));
        d.z = fmaf(c, r->dir.z, s * r->dir.x);
        ray rr = mkray(o, d, r->time, 0);
        if (obj_hit(C, n->a, &rr, tmin, tmax, rec)) {
            V p = rec->p, nn = rec->n;
            p.x = fmaf(c, rec->p.x, s * rec->p.z);
            p.z = fmaf(c, rec->p.z, -(s * rec->p.x));
            nn.x = fmaf(c, rec->n.x, s * rec->n.z);
            nn.z = fmaf(c, rec->n.z, -(s * rec->n.x));
            rec->p = p;
            rec->n = nn;
            return 1;
        }
        return 0;
    }
    case MRT_K_SPHERE:
        return sphere_hit(n, r, tmin, tmax, rec);
    case MRT_K_XY:
        return rect_hit(n, 2, r, tmin, tmax, rec);
    case MRT_K_XZ:
        return rect_hit(n, 1, r, tmin, tmax, rec);
    case MRT_K_YZ:
        return rect_hit(n, 0, r, tmin, tmax, rec);
    case MRT_K_VOLUME: {
        hit_record rec1, rec2;
        if (obj_hit(C, n->a, r, -FLT_MAX, FLT_MAX, &rec1)) {
            if (obj_hit(C, n->a, r, rec1.t + 0.0001f, FLT_MAX, &rec2)) {
                if (rec1.t < tmin) rec1.t = tmin;
                if (rec2.t > tmax) rec2.t = tmax;
                if (rec1.t >= rec2.t) return 0;
                if (rec1.t < 0) rec1.t = 0;
                float inside_dist = (rec2.t - rec1.t);
                float hit_dist = -(1 / n->f[0]) * log_(randf(&C->rng));
                if (hit_dist < inside_dist) {
                    rec->t = rec1.t + hit_dist;
                    rec->p = ray_eval(r, rec->t);
                    rec->n = v3(1, 0, 0);
                    rec->mat = n->mat;
                    return 1;
                }
            }
        }
        return 0;
    }
    }
    return 0;
}

/* ---------------------------------------------------------------- textures (texture.cpp) */
static float perlin_noise(const mrt_scene_view* v, V p) {
    float u = p.x - floorf(p.x), w_ = p.y - floorf(p.y), w = p.z - floorf(p.z);
    int i = (int)floorf(p.x), j = (int)floorf(p.y), k = (int)floorf(p.z);
    V c[2][2][2];
    for (int di = 0; di < 2; di++)
        for (int dj = 0; dj < 2; dj++)
            for (int dk = 0; dk < 2; dk++)
                c[di][dj][dk] = ld(v->perlin_ranvec + 4 * (v->perlin_perm[(i + di) & 255] ^ v->perlin_perm[256 + ((j + dj) & 255)] ^
                                                           v->perlin_perm[512 + ((k + dk) & 255)]));
    /* perlin_interp (texture.cpp:68-105) */
    V init = v3(u, w_, w);
    V uvw = vmul(vmul(init, init), vsub(v3(3, 3, 3), vscale(2, init)));
    float acc = 0;
    V ijk[4] = {{0, 0, 0}, {0, 0, 1}, {0, 1, 0}, {0, 1, 1}};
    for (int ii = 0; ii < 2; ii++) {
        for (int q = 0; q < 4; q++) {
            V weights = vsub(init, ijk[q]);
            V a = vadd(vmul(ijk[q], uvw), vmul(vsub(v3(1, 1, 1), ijk[q]), vsub(v3(1, 1, 1), uvw)));
            acc = fmaf(a.x * a.y * a.z, vdot(c[ii][q >> 1][q & 1], weights), acc);
        }
        for (int q = 0; q < 4; q++) ijk[q] = vadd(ijk[q], v3(1, 0, 0));
    }
    return acc;
}
static V tex_sample(const mrt_scene_view* v, uint32_t t, float u, float vv, V p) {
    const mrt_texture* T = &v->textures[t];
    switch (T->kind) {
    case MRT_T_COLOR:
        return ld(T->f);
    case MRT_T_CHECKER: {
        float sines = sin_(T->f[0] * p.x) * sin_(T->f[0] * p.y) * sin_(T->f[0] * p.z);
        return sines < 0 ? tex_sample(v, T->b, u, vv, p) : tex_sample(v, T->a, u, vv, p);
    }
    case MRT_T_PERLIN: {
        float acc = 0, weight = 1.0f;
        V pc = vscale(T->f[0], p);
        for (int i = 0; i < 7; i++) {
            acc = fmaf(weight, perlin_noise(v, pc), acc);
            weight *= 0.5f;
            pc = vscale(2, pc);
        }
        return vscale(fabsf(acc), v3(1, 1, 1));
    }
    default: {
        int32_t w = (int32_t)T->b, h = (int32_t)T->c;
        int32_t i = (int32_t)(u * w);
        int32_t j = (int32_t)((1 - vv) * h);
        i = i < 0 ? 0 : (i > w - 1 ? w - 1 : i);
        j = j < 0 ? 0 : (j > h - 1 ? h - 1 : j);
        const uint8_t* d = v->texels + T->a + ((size_t)i + (size_t)w * j) * 3;
        return vscale(1.0f / 255.0f, v3(d[0], d[1], d[2]));
    }
    }
}

/* ---------------------------------------------------------------- pdfs (pdf.h, rect.cpp, sphere.cpp) */
static float obj_pdf_value(ctx* C, uint32_t id, V origin, V dir, float time) {
    const mrt_scene_view* v = C->v;
    const mrt_node* n = &v->nodes[id];
    hit_record rec;
    switch (KIND(n)) {
    case MRT_K_LIST: {
        float sum = 0;
        for (uint32_t i = 0; i < n->b; i++) sum += obj_pdf_value(C, v->children[n->a + i], origin, dir, time);
        return sum / (float)n->b;
    }
    case MRT_K_XZ: {
        ray r = mkray(origin, dir, 0.0f, 0);
        if (rect_hit(n, 1, &r, 0.001f, FLT_MAX, &rec)) {
            float area = (n->f[1] - n->f[0]) * (n->f[3] - n->f[2]);
            float dist_sq = rec.t * rec.t;
            float cosine = fabsf(vdot(dir, rec.n));
            return dist_sq / (cosine * area);
        }
        return 0;
    }
    case MRT_K_SPHERE: {
        ray r = mkray(origin, dir, time, 0);
        if (sphere_hit(n, &r, 0.001f, FLT_MAX, &rec)) {
            float radius = n->f[8];
            float cos_theta_max = sqrtf(1 - radius * radius / vsdot(vsub(sphere_center(n, time), origin)));
            float solid_angle = 2 * PI_F * (1 - cos_theta_max);
            return 1 / solid_angle;
        }
        return 0;
    }
    }
    return 0;
}
static V onb_mul(V w, V vec) { /* onb.h:19-27 */
    V a = fabsf(w.x) > 0.9f ? v3(0, 1, 0) : v3(1, 0, 0);
    V vv = vnorm(vcross(w, a));
    V u = vcross(w, vv);
    return vadd(vadd(vscale(vec.x, u), vscale(vec.y, vv)), vscale(vec.z, w));
}
static V obj_pdf_generate(ctx* C, uint32_t id, V origin, float time) {
    const mrt_scene_view* v = C->v;
    const mrt_node* n = &v->nodes[id];
    switch (KIND(n)) {
    case MRT_K_LIST: {
        int i = (int)(randf(&C->rng) * (float)n->b);
        return obj_pdf_generate(C, v->children[n->a + i], origin, time);
    }
    case MRT_K_XZ: {
        float a = randf(&C->rng);
        float x = fmaf(a, n->f[1] - n->f[0], n->f[0]);
        float b = randf(&C->rng);
        float z = fmaf(b, n->f[3] - n->f[2], n->f[2]);
        return vsub(v3(x, n->f[4], z), origin);
    }
    case MRT_K_SPHERE: {
        V dir = vsub(sphere_center(n, time), origin);
        float dist_sq = vsdot(dir);
        return onb_mul(vnorm(dir), random_towards_sphere(&C->rng, n->f[8], dist_sq));
    }
    }
    return v3(1, 0, 0);
}

/* ---------------------------------------------------------------- trace (main.cpp:66-118) */
typedef struct { uint32_t max_bounces; uint64_t rays; } tstate;

static V trace(ctx* C, tstate* T, const ray* r, uint32_t depth) {
    const mrt_scene_view* v = C->v;
    T->rays++;
    hit_record hrec;
    memset(&hrec, 0, sizeof hrec);
    if (obj_hit(C, v->root, r, 0.001f, FLT_MAX, &hrec)) {
        const mrt_material* M = &v->materials[hrec.mat];
        V emitted = v3(0, 0, 0);
        if (M->kind == MRT_M_LIGHT && vdot(hrec.n, r->dir) < 0.0f) emitted = vscale(M->p, tex_sample(v, M->tex, hrec.u, hrec.v, hrec.p));
        if (depth < T->max_bounces && M->kind != MRT_M_LIGHT) {
            if (M->kind == MRT_M_METAL) { /* material.h:91-98 */
                float dp = 2.0f * vdot(r->dir, hrec.n);
                V reflected = vsub(r->dir, vscale(dp, hrec.n));
                ray sr = mkray(hrec.p, vadd(reflected, vscale(1 - M->p, random_in_sphere(&C->rng))), r->time, 0);
                V att = tex_sample(v, M->tex, hrec.u, hrec.v, hrec.p);
                return vmul(att, trace(C, T, &sr, depth + 1));
            }
            if (M->kind == MRT_M_DIELECTRIC) { /* material.h:121-175 */
                float ref = M->p;
                V facing;
                float nio;
                float cosI = -vdot(r->dir, hrec.n);
                if (cosI < 0) {
                    facing = v3(-hrec.n.x, -hrec.n.y, -hrec.n.z);
                    nio = ref;
                } else {
                    facing = hrec.n;
                    nio = 1.0f / ref;
                }
                float dp = 2.0f * vdot(r->dir, hrec.n);
                V reflected = vsub(r->dir, vscale(dp, hrec.n));
                ray sr;
                float ncosI = vdot(r->dir, facing);
                float sinT2 = (nio * nio) * fmaf(-ncosI, ncosI, 1.0f);
                if (sinT2 <= 1.0f) {
                    float cosT = sqrtf(1.0f - sinT2);
                    V refracted = vadd(vscale(nio, r->dir), vscale(fmaf(nio, -ncosI, -cosT), facing));
                    float cs = cosI < 0 ? sqrtf(fmaf(-(nio * nio), fmaf(-cosI, cosI, 1.0f), 1.0f)) : cosI;
                    float r0 = (1 - ref) / (1 + ref);
                    r0 = r0 * r0;
                    float reflect_prob = fmaf(1 - r0, pow_((1 - cs), 5), r0);
                    if (randf(&C->rng) < reflect_prob) {
                        sr = mkray(hrec.p, reflected, r->time, r->inside);
                    } else {
                        int inside = r->inside;
                        if (cosI < 0) {
                            inside--;
                            if (inside < 0) inside = 0;
                        } else {
                            inside++;
                        }
                        sr = mkray(hrec.p, refracted, r->time, inside);
                    }
                } else {
                    sr = mkray(hrec.p, reflected, r->time, r->inside);
                }
                return vmul(v3(1.0f, 1.0f, 1.0f), trace(C, T, &sr, depth + 1));
            }
            /* lambertian / isotropic + mix_pdf (main.cpp:84-102) */
            int lamb = M->kind == MRT_M_LAMBERTIAN;
            V att = tex_sample(v, M->tex, hrec.u, hrec.v, hrec.p);
            ray scattered;
            float pdf_v;
            V gen;
            if (v->biased != MRT_NONE) {
                if (randf(&C->rng) < 0.5f) gen = obj_pdf_generate(C, v->biased, hrec.p, r->time);
                else gen = lamb ? onb_mul(hrec.n, random_cosine_direction(&C->rng)) : random_in_sphere(&C->rng);
            } else {
                gen = lamb ? onb_mul(hrec.n, random_cosine_direction(&C->rng)) : random_in_sphere(&C->rng);
            }
            scattered = mkray(hrec.p, gen, r->time, 0);
            float sv;
            if (lamb) {
                float cosine = vdot(scattered.dir, hrec.n);
                sv = cosine > 0 ? cosine / PI_F : 0;
            } else {
                sv = 1 / (2 * PI_F);
            }
            pdf_v = v->biased != MRT_NONE ? 0.5f * (obj_pdf_value(C, v->biased, hrec.p, scattered.dir, r->time) + sv) : sv;
            float spdf;
            if (lamb) {
                float cosine = vdot(hrec.n, scattered.dir);
                spdf = cosine < 0 ? 0 : cosine * (1.0f / PI_F);
            } else {
                spdf = 1.0f / (2.0f * PI_F);
            }
            V col = trace(C, T, &scattered, depth + 1);
            V a = vscale(spdf, att);
            V x = vmul(a, col);
            return vadd(emitted, vdivf(x, pdf_v));
        }
        return emitted;
    }
    if (v->sky) {
        float t = 0.5f * (r->dir.y + 1.0f);
        return vadd(v3(1.0f - t, 1.0f - t, 1.0f - t), vscale(t, v3(0.5f, 0.7f, 1.0f)));
    }
    return v3(0, 0, 0);
}

/* camera::get_ray (camera.h:38-44) */
static ray get_ray(ctx* C, float s, float t) {
    const mrt_camera* c = &C->v->camera;
    V rd = vscale(c->lens_radius, random_in_disk(&C->rng));
    V offset = vadd(vscale(rd.x, ld(c->u)), vscale(rd.y, ld(c->v)));
    float time = fmaf(c->time1 - c->time0, randf(&C->rng), c->time0);
    V dir = vsub(vsub(vadd(vadd(ld(c->llcorner), vscale(s, ld(c->horz))), vscale(t, ld(c->vert))), ld(c->origin)), offset);
    return mkray(vadd(ld(c->origin), offset), dir, time, 0);
}

/* one path whose draws come from C->rng as it stands (the caller seeds it) */
static V path_with(ctx* C, const oracle_desc* d, uint32_t x, uint32_t y, uint32_t s, uint32_t* rays) {
    uint32_t sq = d->sqrt_samples;
    uint32_t i = s / sq, j = s % sq;
    float dx = (i + 0.5f) / (float)sq, dy = (j + 0.5f) / (float)sq; /* main.cpp:324-331 */
    float u = (x + dx) / (float)d->width;
    float vv = (y + dy) / (float)d->height;
    ray r = get_ray(C, u, vv);
    tstate T = {d->max_bounces, 0};
    V c = trace(C, &T, &r, 0);
    *rays = (uint32_t)T.rays;
    return c;
}

static V one_path(const mrt_scene_view* v, const oracle_desc* d, uint32_t x, uint32_t y, uint32_t s, uint32_t* rays) {
    uint32_t sq = d->sqrt_samples, ns = sq * sq;
    uint32_t i = s / sq, j = s % sq;
    float dx = (i + 0.5f) / (float)sq, dy = (j + 0.5f) / (float)sq; /* main.cpp:324-331 */
    uint64_t path = ((uint64_t)x + (uint64_t)y * d->width) * ns + s;
    ctx C;
    C.v = v;
    pcg_srandom(&C.rng, splitmix64(d->seed ^ path), path);
    float u = (x + dx) / (float)d->width;
    float vv = (y + dy) / (float)d->height;
    ray r = get_ray(&C, u, vv);
    tstate T = {d->max_bounces, 0};
    V c = trace(&C, &T, &r, 0);
    *rays = (uint32_t)T.rays;
    return c;
}

uint32_t oracle_path(const mrt_scene_view* v, const oracle_desc* d, uint32_t x, uint32_t y, uint32_t s, float* out) {
    uint32_t rays;
    V c = one_path(v, d, x, y, s, &rays);
    out[0] = c.x;
    out[1] = c.y;
    out[2] = c.z;
    return rays;
}

static float lum(V c) { return (c.x * 0.212655f + c.y * 0.715158f) + c.z * 0.072187f; }

typedef struct {
    const mrt_scene_view* v;
    const oracle_desc* d;
    float* rgb;
    float* path_rgb;
    uint32_t* path_rays;
    uint32_t* next_row;
    pthread_mutex_t* mu;
    uint64_t rays;
} job;

static void* worker(void* arg) {
    job* J = (job*)arg;
    const oracle_desc* d = J->d;
    uint32_t ns = d->sqrt_samples * d->sqrt_samples, y1 = d->y1 ? d->y1 : d->height;
    for (;;) {
        pthread_mutex_lock(J->mu);
        uint32_t y = (*J->next_row)++;
        pthread_mutex_unlock(J->mu);
        if (y >= y1) break;
        for (uint32_t x = 0; x < d->width; x++) {
            size_t pix = (size_t)x + (size_t)y * d->width;
            V color = v3(0, 0, 0);
            for (uint32_t s = 0; s < ns; s++) {
                uint32_t rr;
                V smp = one_path(J->v, d, x, y, s, &rr);
                J->rays += rr;
                if (J->path_rgb) {
                    float* q = J->path_rgb + (pix * ns + s) * 3;
                    q[0] = smp.x; q[1] = smp.y; q[2] = smp.z;
                }
                if (J->path_rays) J->path_rays[pix * ns + s] = rr;
                if (d->mode == 0) { /* draw(), main.cpp:161-167 */
                    if (!isfinite(smp.x) || !isfinite(smp.y) || !isfinite(smp.z)) smp = color;
                    color = vadd(color, smp);
                } else { /* draw2(), main.cpp:212-229 */
                    if (!isfinite(smp.x) || !isfinite(smp.y) || !isfinite(smp.z)) smp = s > 0 ? color : v3(0, 0, 0);
                    if (s > 0) smp = vadd(color, vscale(1.0f / (s + 1.0f), vsub(smp, color)));
                    float l = lum(smp);
                    if (l > d->max_luminance) smp = vscale(d->max_luminance / l, smp);
                    color = smp;
                }
            }
            if (d->mode == 0) { /* main.cpp:168-173 */
                color = vdivf(color, (float)ns);
                float l = lum(color);
                if (l > d->max_luminance) color = vscale(d->max_luminance / l, color);
            }
            float* o = J->rgb + pix * 4;
            o[0] = color.x; o[1] = color.y; o[2] = color.z; o[3] = 0;
        }
    }
    return NULL;
}

uint64_t oracle_render(const mrt_scene_view* v, const oracle_desc* d, float* rgb, float* path_rgb, uint32_t* path_rays) {
    uint32_t nt = d->threads ? d->threads : 1;
    if (nt > 256) nt = 256;
    uint32_t next = d->y0;
    pthread_mutex_t mu = PTHREAD_MUTEX_INITIALIZER;
    job jobs[256];
    pthread_t th[256];
    for (uint32_t i = 0; i < nt; i++) {
        jobs[i].v = v; jobs[i].d = d; jobs[i].rgb = rgb; jobs[i].path_rgb = path_rgb; jobs[i].path_rays = path_rays;
        jobs[i].next_row = &next; jobs[i].mu = &mu; jobs[i].rays = 0;
        if (nt == 1) worker(&jobs[0]);
        else pthread_create(&th[i], NULL, worker, &jobs[i]);
    }
    uint64_t rays = 0;
    for (uint32_t i = 0; i < nt; i++) {
        if (nt > 1) pthread_join(th[i], NULL);
        rays += jobs[i].rays;
    }
    return rays;
}

/* ---- the reference's own RNG order (-threads 1): one worker, one PCG stream ------------------
 * work_queue tiles (work_queue.cpp:64-128): row-major tiles re-ordered along the inverted Hilbert
 * curve over the next power of two, tiles outside the image skipped. */
static void hil_d2xy(uint32_t n, uint32_t d, uint32_t* x, uint32_t* y) { /* work_queue.cpp:6-30 */
    uint32_t rx, ry, s, t = d;
    *x = *y = 0;
    for (s = 1; s < n; s *= 2) {
        rx = 1 & (t / 2);
        ry = 1 & (t ^ rx);
        if (ry == 0) {
            if (rx == 1) {
                *x = s - 1 - *x;
                *y = s - 1 - *y;
            }
            uint32_t tmp = *x;
            *x = *y;
            *y = tmp;
        }
        *x += s * rx;
        *y += s * ry;
        t /= 4;
    }
}
static uint32_t rev32(uint32_t v) { /* work_queue.cpp:33-45 */
    v = ((v >> 1) & 0x55555555u) | ((v & 0x55555555u) << 1);
    v = ((v >> 2) & 0x33333333u) | ((v & 0x33333333u) << 2);
    v = ((v >> 4) & 0x0F0F0F0Fu) | ((v & 0x0F0F0F0Fu) << 4);
    v = ((v >> 8) & 0x00FF00FFu) | ((v & 0x00FF00FFu) << 8);
    return (v >> 16) | (v << 16);
}
typedef struct { uint32_t x0, x1, y0, y1; } otile;
static uint32_t work_tiles(uint32_t W, uint32_t H, uint32_t ts, otile** out) {
    uint32_t xc = (W + ts - 1) / ts, yc = (H + ts - 1) / ts, n = xc * yc, po2 = 1, lg = 0;
    otile* rm = (otile*)malloc(sizeof(otile) * n);
    otile* fin = (otile*)malloc(sizeof(otile) * n);
    for (uint32_t y = 0; y < yc; y++)
        for (uint32_t x = 0; x < xc; x++) {
            otile t = {x * ts, x * ts + ts < W ? x * ts + ts : W, y * ts, y * ts + ts < H ? y * ts + ts : H};
            rm[x + y * xc] = t;
        }
    uint32_t m = xc > yc ? xc : yc;
    while (po2 < m) po2 *= 2; /* MRT::nextPo2 */
    while ((1u << lg) < po2) lg++;
    uint32_t idx = 0;
    for (uint32_t d = 0; d < po2 * po2 && idx < n; d++) {
        uint32_t x, y;
        hil_d2xy(po2, d, &x, &y);
        x = lg ? rev32(x) >> (32u - lg) : 0; /* INVERT (work_queue.cpp:104-108) */
        y = lg ? rev32(y) >> (32u - lg) : 0;
        if (x < xc && y < yc) fin[idx++] = rm[x + y * xc];
    }
    free(rm);
    *out = fin;
    return n;
}

uint64_t oracle_render_ref_order(const mrt_scene_view* v, const oracle_desc* d, uint32_t tile_size, uint64_t initstate, uint64_t initseq,
                                 float* rgb) {
    ctx C;
    C.v = v;
    pcg_srandom(&C.rng, initstate, initseq); /* Init_Thread_RNG(args.initstate, args.initseq), main.cpp:143/198 */
    otile* tiles;
    uint32_t nt = work_tiles(d->width, d->height, tile_size, &tiles);
    uint32_t ns = d->sqrt_samples * d->sqrt_samples;
    uint64_t rays = 0;
    if (d->mode == 0) { /* draw() over work_queue_seq (main.cpp:138-188, work_queue.cpp:133-140) */
        for (uint32_t k = 0; k < nt; k++)
            for (uint32_t y = tiles[k].y0; y < tiles[k].y1; y++)
                for (uint32_t x = tiles[k].x0; x < tiles[k].x1; x++) {
                    V color = v3(0, 0, 0);
                    for (uint32_t s = 0; s < ns; s++) {
                        uint32_t rr;
                        V smp = path_with(&C, d, x, y, s, &rr);
                        rays += rr;
                        if (!isfinite(smp.x) || !isfinite(smp.y) || !isfinite(smp.z)) smp = color;
                        color = vadd(color, smp);
                    }
                    color = vdivf(color, (float)ns);
                    float l = lum(color);
                    if (l > d->max_luminance) color = vscale(d->max_luminance / l, color);
                    float* o = rgb + ((size_t)x + (size_t)y * d->width) * 4;
                    o[0] = color.x; o[1] = color.y; o[2] = color.z; o[3] = 0;
                }
    } else { /* draw2() over work_queue_dynamic: item c -> tile c % nt, sample c / nt (main.cpp:193-243, work_queue.cpp:157-166) */
        for (uint64_t c = 0; c < (uint64_t)nt * ns; c++) {
            const otile* t = &tiles[c % nt];
            uint32_t s = (uint32_t)(c / nt);
            for (uint32_t y = t->y0; y < t->y1; y++)
                for (uint32_t x = t->x0; x < t->x1; x++) {
                    float* o = rgb + ((size_t)x + (size_t)y * d->width) * 4;
                    V old = v3(o[0], o[1], o[2]);
                    uint32_t rr;
                    V color = path_with(&C, d, x, y, s, &rr);
                    rays += rr;
                    if (!isfinite(color.x) || !isfinite(color.y) || !isfinite(color.z)) color = s > 0 ? old : v3(0, 0, 0);
                    if (s > 0) color = vadd(old, vscale(1.0f / (s + 1.0f), vsub(color, old)));
                    float l = lum(color);
                    if (l > d->max_luminance) color = vscale(d->max_luminance / l, color);
                    o[0] = color.x; o[1] = color.y; o[2] = color.z; o[3] = 0;
                }
        }
    }
    free(tiles);
    return rays;
}

int oracle_hit(const mrt_scene_view* v, const float* o, const float* dir, float time, int inside, uint64_t seed, float* out) {
    ctx C;
    C.v = v;
    pcg_srandom(&C.rng, seed, 4242);
    ray r = mkray(ld(o), ld(dir), time, inside);
    hit_record rec;
    memset(&rec, 0, sizeof rec);
    int h = obj_hit(&C, v->root, &r, 0.001f, FLT_MAX, &rec);
    if (h) {
        out[0] = rec.t;
        out[1] = rec.p.x; out[2] = rec.p.y; out[3] = rec.p.z;
        out[4] = rec.n.x; out[5] = rec.n.y; out[6] = rec.n.z;
    }
    return h;
}

void oracle_pcg_stream(uint64_t st, uint64_t sq, uint32_t n, uint32_t* out) {
    pcg r;
    pcg_srandom(&r, st, sq);
    for (uint32_t i = 0; i < n; i++) out[i] = pcg_next(&r);
}

void oracle_samplers(uint64_t st, uint64_t sq, uint32_t n, uint32_t which, float* out) {
    pcg r;
    pcg_srandom(&r, st, sq);
    for (uint32_t i = 0; i < n; i++) {
        V p;
        switch (which) {
        case 0: p = v3(randf(&r), 0, 0); break;
        case 1: p = random_in_sphere(&r); break;
        case 2: p = random_in_disk(&r); break;
        case 3: p = random_cosine_direction(&r); break;
        default: p = random_on_sphere_uniform(&r); break;
        }
        out[i * 3 + 0] = p.x; out[i * 3 + 1] = p.y; out[i * 3 + 2] = p.z;
    }
}
