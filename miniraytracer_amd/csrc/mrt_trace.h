// mrt_trace.h -- scene traversal (scene_object::hit tree), shading and one full path (trace()).
#pragma once
#include "mrt_device.h"

namespace mrtd {

// Device-side scene: the mrt_scene_view arrays resident in HBM.
struct DScene {
    const mrt_node* __restrict__ nodes;
    const uint32_t* __restrict__ children;
    const mrt_mesh_node* __restrict__ mnodes;
    const float4* __restrict__ tri_geo;
    const float4* __restrict__ tri_nrm;
    const mrt_material* __restrict__ mats;
    const mrt_texture* __restrict__ texs;
    const float4* __restrict__ ranvec;
    const int32_t* __restrict__ perm;
    const uint8_t* __restrict__ texels;
    uint32_t root, biased, sky;
    mrt_camera cam;
};

#define MRT_NODE_KIND(n) ((n).kind & 0xFFu)
#define MRT_NODE_ORDER(n) (((n).kind >> 8) & 0xFFu)
#define MRT_NODE_FLAGS(n) (((n).kind >> 16) & 0xFFu)
#define MRT_F_NEEDUV 0x4u /* set by the device upload when the node's material samples uv */

__device__ __forceinline__ bool is_prim(uint32_t kind) { return kind == MRT_K_SPHERE || kind == MRT_K_XY || kind == MRT_K_XZ || kind == MRT_K_YZ || kind == MRT_K_MESH; }

// get_sphere_uv (sphere.cpp:6-11)
__device__ __forceinline__ void sphere_uv(f3 p, float* u, float* v) {
    float phi = atan2_(p.z, p.x);
    float theta = asin_(p.y);
    *u = 0.5f - phi * (1.0f / (2.0f * PI_F));
    *v = 0.5f + theta * (1.0f / PI_F);
}

__device__ __forceinline__ f3 sphere_center(const mrt_node& n, float time) {
    f3 c0 = ld3(n.f);
    if (MRT_NODE_FLAGS(n) & MRT_F_MOVING) return add(c0, fmul((time - n.f[6]) / (n.f[7] - n.f[6]), sub(ld3(n.f + 3), c0)));
    return c0;
}

// sphere::hit (sphere.cpp:13-46).  `full` = write p/n/uv (false inside volume boundary queries).
__device__ __forceinline__ bool sphere_hit(const mrt_node& n, const Ray& r, float tmin, float tmax, HitRec& rec, bool full) {
    f3 cen = sphere_center(n, r.time);
    float radius = n.f[8];
    f3 oc = sub(r.o, cen);
    float b = dot(oc, r.d);
    float c = sdot(oc) - radius * radius;
    float disc = b * b - c;
    if (disc > 0) {
        float sq = __builtin_sqrtf(disc);
        float t = (-b - sq);
        bool ok = t < tmax && t > tmin;
        if (!ok && r.inside) {
            t = (-b + sq);
            ok = t < tmax && t > tmin;
        }
        if (ok) {
            rec.t = t;
            if (full) {
                rec.p = eval(r, t);
                rec.n = divf(sub(rec.p, cen), radius);
                rec.mat = n.mat;
                if (MRT_NODE_FLAGS(n) & MRT_F_NEEDUV) sphere_uv(rec.n, &rec.u, &rec.v);
            }
            return true;
        }
    }
    return false;
}

// xy/xz/yz_rect::hit (rect.cpp:24-152): axis a (plane normal), b, c (in-plane)
template <int AX>
__device__ __forceinline__ bool rect_hit(const mrt_node& n, const Ray& r, float tmin, float tmax, HitRec& rec, bool full) {
    const float ns = n.f[5];
    // dot(r.dir, normal) with the zero lanes kept (NaN directions behave as in the reference)
    float dn = AX == 2 ? (r.d.x * 0.0f + r.d.y * 0.0f) + r.d.z * ns
             : AX == 1 ? (r.d.x * 0.0f + r.d.y * ns) + r.d.z * 0.0f
                       : (r.d.x * ns + r.d.y * 0.0f) + r.d.z * 0.0f;
    if (dn > 0.0f) return false;
    float oa = AX == 2 ? r.o.z : AX == 1 ? r.o.y : r.o.x;
    float da = AX == 2 ? r.d.z : AX == 1 ? r.d.y : r.d.x;
    float t = (n.f[4] - oa) / da;
    if (t < tmin || t > tmax) return false;
    // in-plane axes: xy -> (x,y), xz -> (x,z), yz -> (y,z)
    float ob = AX == 0 ? r.o.y : r.o.x, db = AX == 0 ? r.d.y : r.d.x;
    float oc = AX == 2 ? r.o.y : r.o.z, dc = AX == 2 ? r.d.y : r.d.z;
    float pb = ob + t * db;
    float pc = oc + t * dc;
    if (pb < n.f[0] || pb > n.f[1] || pc < n.f[2] || pc > n.f[3]) return false;
    rec.t = t;
    if (full) {
        if (MRT_NODE_FLAGS(n) & MRT_F_NEEDUV) {
            rec.u = (pb - n.f[0]) / (n.f[1] - n.f[0]);
            rec.v = (pc - n.f[2]) / (n.f[3] - n.f[2]);
        }
        rec.mat = n.mat;
        rec.p = eval(r, t);
        rec.n = AX == 2 ? f3{0, 0, ns} : AX == 1 ? f3{0, ns, 0} : f3{ns, 0, 0};
    }
    return true;
}

// triangle::hit (triangle.cpp:222-265) without the normal (deferred to the closest hit)
__device__ __forceinline__ bool tri_hit(const DScene& S, uint32_t i, const Ray& r, float tmin, float tmax, float* tout, float* uout, float* vout) {
    f3 m = ld3(S.tri_geo[i * 3 + 0]), u = ld3(S.tri_geo[i * 3 + 1]), v = ld3(S.tri_geo[i * 3 + 2]);
    f3 pvec = cross(r.d, v);
    float det = dot(u, pvec);
    float sign = 1.0f;
    if (r.inside) {
        sign = det < 0.0f ? -1.0f : 1.0f;
        det = sign * det;
    }
    if (det < 0.00001f) return false;
    f3 tvec = sub(r.o, m);
    float uu = dot(tvec, pvec) * sign;
    f3 qvec = cross(tvec, u);
    float vv = dot(r.d, qvec) * sign;
    if ((uu < 0) | (uu > det) | (vv < 0) | ((uu + vv) > det)) return false;
    float invDet = 1 / det;
    float t = (dot(v, qvec) * invDet) * sign;
    if ((t < tmin) | (t > tmax)) return false;
    *tout = t;
    *uout = uu * invDet;
    *vout = vv * invDet;
    return true;
}

// pod_bvh::hit (triangle.h:171-221): DFS, closer child first (node_order & dirMask); the first
// leaf that reports a hit ends the walk (every ancestor returns on hit_closer / hit_farther).
#define MRT_MESH_STACK 48
__device__ __noinline__ bool mesh_hit(const DScene& S, const mrt_node& n, const Ray& r, float tmin, float tmax, HitRec& rec, bool full) {
    uint32_t stack[MRT_MESH_STACK];
    int sp = 0;
    stack[sp++] = n.a;
    while (sp > 0) {
        uint32_t ni = stack[--sp];
        const mrt_mesh_node& mn = S.mnodes[ni];
        if (!aabb_hit(mn.bmin, mn.bmax, r, tmin, tmax)) continue;
        uint32_t cnt = mn.count_order & 0xFFFFFFu;
        if (cnt) {
            bool has = false;
            uint32_t best = 0;
            float bu = 0, bv = 0, tt = tmax;
            for (uint32_t k = 0; k < cnt; k++) {
                float t, uu, vv;
                if (tri_hit(S, mn.left_or_first + k, r, tmin, tt, &t, &uu, &vv)) {
                    has = true;
                    tt = t;
                    best = mn.left_or_first + k;
                    bu = uu;
                    bv = vv;
                }
            }
            if (has) {
                rec.t = tt;
                if (full) {
                    f3 nm = ld3(S.tri_nrm[best * 3 + 0]), nu = ld3(S.tri_nrm[best * 3 + 1]), nv = ld3(S.tri_nrm[best * 3 + 2]);
                    rec.p = eval(r, tt);
                    rec.n = normalize(add(add(mulf(nm, (1 - bu) - bv), mulf(nu, bu)), mulf(nv, bv)));
                    rec.u = bu;
                    rec.v = bv;
                    rec.mat = n.mat;
                }
                return true;
            }
        } else {
            uint32_t l = mn.left_or_first;
            bool left_first = ((mn.count_order >> 24) & r.mask) != 0;
            if (sp + 2 > MRT_MESH_STACK) __builtin_trap();
            stack[sp++] = left_first ? l + 1 : l;  // farther
            stack[sp++] = left_first ? l : l + 1;  // closer (popped first)
        }
    }
    return false;
}

__device__ __forceinline__ bool prim_hit(const DScene& S, const mrt_node& n, uint32_t kind, const Ray& r, float tmin, float tmax, HitRec& rec, bool full) {
    switch (kind) {
    case MRT_K_SPHERE: return sphere_hit(n, r, tmin, tmax, rec, full);
    case MRT_K_XY: return rect_hit<2>(n, r, tmin, tmax, rec, full);
    case MRT_K_XZ: return rect_hit<1>(n, r, tmin, tmax, rec, full);
    case MRT_K_YZ: return rect_hit<0>(n, r, tmin, tmax, rec, full);
    default: return mesh_hit(S, n, r, tmin, tmax, rec, full);
    }
}

// ------------------------------------------------------------------------------------------
// scene_object::hit as an explicit-stack machine.  One running `closest` per query replaces the
// per-call tmax: every hit narrows it and every consumer passes it on (object_list children get
// the list's closest, bvh_node children its tmax, which is unchanged until a hit ends the node).
// constant_volume runs its two boundary queries as a nested context whose hits only record t;
// volumes never nest (checked on upload).  The top frame lives in registers; frames below it and
// saved instance rays live in per-lane scratch.  Primitives have exactly one evaluation site.
// ------------------------------------------------------------------------------------------
#define MRT_FRAMES 32
#define MRT_RAYS 6
enum : uint32_t { ST_ENTER = 0xFFFFFFFFu, ST_PH1 = 0x40000000u, ST_PH2 = 0x40000001u };

__device__ __forceinline__ bool scene_hit(const DScene& S, Ray ray, float tmin0, HitRec& rec, Pcg& rng) {
    uint32_t fnode[MRT_FRAMES], fstate[MRT_FRAMES];
    Ray rstk[MRT_RAYS];
    int depth = 0, rsp = 0;
    uint32_t tnode = 0, tstate = 0;  // top frame
    float closest = FLT_MAX_, tmin = tmin0;
    bool insub = false;  // inside a constant_volume boundary query
    float save_closest = 0, save_tmin = 0, vt1 = 0;
    HitRec subrec;
    bool ret = false;
    uint32_t req = S.root;

    for (;;) {
        if (req != MRT_NONE) {
            const mrt_node& C = S.nodes[req];
            const uint32_t ck = MRT_NODE_KIND(C);
            req = MRT_NONE;
            if (is_prim(ck)) {
                HitRec* R = insub ? &subrec : &rec;
                ret = prim_hit(S, C, ck, ray, tmin, closest, *R, !insub);
                if (ret) closest = R->t;
                if (depth == 0) break;
            } else {
                if (depth > 0) {
                    fnode[depth - 1] = tnode;
                    fstate[depth - 1] = tstate;
                }
                tnode = (uint32_t)(&C - S.nodes);
                tstate = ST_ENTER;
                depth++;
            }
        }
        const mrt_node& N = S.nodes[tnode];
        const uint32_t kind = MRT_NODE_KIND(N);
        const uint32_t st = tstate;
        bool pop = false;
        switch (kind) {
        case MRT_K_LIST: {  // object_list::hit (scene_object.h:79-103)
            uint32_t cursor, flag;
            if (st == ST_ENTER) {
                if ((MRT_NODE_FLAGS(N) & MRT_F_HASBOX) && !aabb_hit(N.f, N.f + 3, ray, tmin, closest)) {
                    ret = false;
                    pop = true;
                    break;
                }
                cursor = 0;
                flag = 0;
            } else {
                cursor = st & 0x3FFFFFFFu;
                flag = (st >> 31) | (ret ? 1u : 0u);
            }
            if (cursor < N.b) {
                req = S.children[N.a + cursor];
                tstate = (cursor + 1) | (flag << 31);
            } else {
                ret = flag != 0;
                pop = true;
            }
            break;
        }
        case MRT_K_BVH: {  // bvh_node::hit (scene_object.h:208-244)
            const bool left_first = (MRT_NODE_ORDER(N) & ray.mask) != 0;
            if (st == ST_ENTER) {
                if (!aabb_hit(N.f, N.f + 3, ray, tmin, closest)) {
                    ret = false;
                    pop = true;
                    break;
                }
                req = left_first ? N.a : N.b;
                tstate = ST_PH1;
            } else if (st == ST_PH1 && !ret) {
                req = left_first ? N.b : N.a;
                tstate = ST_PH2;
            } else {
                pop = true;  // closer hit (ret true) or farther done
            }
            break;
        }
        case MRT_K_TRANSLATE:
        case MRT_K_ROTY: {  // scene_object.cpp:9-18, 70-98
            const bool roty = kind == MRT_K_ROTY;
            if (st == ST_ENTER) {
                if (roty && (MRT_NODE_FLAGS(N) & MRT_F_HASBOX) && !aabb_hit(N.f, N.f + 3, ray, tmin, closest)) {
                    ret = false;
                    pop = true;
                    break;
                }
                rstk[rsp++] = ray;
                if (!roty) {
                    ray = make_ray(sub(ray.o, ld3(N.f)), ray.d, ray.time, 0);
                } else {
                    const float s = N.f[6], c = N.f[7];
                    f3 o = ray.o, d = ray.d;
                    o.x = c * ray.o.x - s * ray.o.z;
                    o.z = c * ray.o.z + s * ray.o.x;
                    d.x = c * ray.d.x - s * ray.d.z;
                    d.z = c * ray.d.z + s * ray.d.x;
                    ray = make_ray(o, d, ray.time, 0);
                }
                req = N.a;
                tstate = ST_PH1;
            } else {
                ray = rstk[--rsp];
                if (ret && !insub) {
                    if (!roty) {
                        rec.p = add(rec.p, ld3(N.f));
                    } else {
                        const float s = N.f[6], c = N.f[7];
                        f3 p = rec.p, nn = rec.n;
                        p.x = c * rec.p.x + s * rec.p.z;
                        p.z = c * rec.p.z - s * rec.p.x;
                        nn.x = c * rec.n.x + s * rec.n.z;
                        nn.z = c * rec.n.z - s * rec.n.x;
                        rec.p = p;
                        rec.n = nn;
                    }
                }
                pop = true;
            }
            break;
        }
        case MRT_K_VOLUME: {  // constant_volume::hit (volumes.cpp:5-35)
            if (st == ST_ENTER) {
                save_closest = closest;
                save_tmin = tmin;
                insub = true;
                closest = FLT_MAX_;
                tmin = -FLT_MAX_;  // numeric_limits<float>::lowest()
                req = N.a;
                tstate = ST_PH1;
            } else if (st == ST_PH1 && ret) {
                vt1 = subrec.t;
                closest = FLT_MAX_;
                tmin = vt1 + 0.0001f;
                req = N.a;
                tstate = ST_PH2;
            } else {
                insub = false;
                closest = save_closest;
                tmin = save_tmin;
                pop = true;
                if (!ret) break;
                float t1 = vt1, t2 = subrec.t;
                if (t1 < tmin) t1 = tmin;
                if (t2 > closest) t2 = closest;
                if (t1 >= t2) {
                    ret = false;
                    break;
                }
                if (t1 < 0) t1 = 0;
                const float inside_dist = t2 - t1;
                const float hit_dist = -(1 / N.f[0]) * log_(randf(rng));
                ret = hit_dist < inside_dist;
                if (ret) {
                    rec.t = t1 + hit_dist;
                    rec.p = eval(ray, rec.t);
                    rec.n = f3{1, 0, 0};
                    rec.mat = N.mat;
                    closest = rec.t;
                }
            }
            break;
        }
        default:
            ret = false;
            pop = true;
        }
        if (pop) {
            depth--;
            if (depth == 0) break;
            tnode = fnode[depth - 1];
            tstate = fstate[depth - 1];
        }
    }
    return ret;
}

}  // namespace mrtd
