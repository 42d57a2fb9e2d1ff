// mrt_trace.h -- scene traversal: the scene_object::hit virtual-call tree as a per-lane
// explicit-stack machine with its stacks in LDS.
#pragma once
#include "mrt_device.h"

namespace mrtd {

struct LinOp;  // mrt_lin.h

// pod_bvh inner node with both children's boxes inline (built on upload from mrt_mesh_node[]):
// one 64 B load tests both children.  Child ref: inner -> index into the wide array; leaf ->
// MESH_LEAF | count << 24 | first triangle.
struct MeshWide {
    float lmin[3];
    uint32_t lref;
    float lmax[3];
    uint32_t rref;
    float rmin[3];
    uint32_t order;  // the node's node_order byte (triangle.h:282-322)
    float rmax[3];
    uint32_t pad;
};
#define MESH_LEAF 0x80000000u

// device material: mrt_material plus, when its texture is a constant colour, that colour inline
// (one load per shading instead of material -> texture)
struct DMat {
    uint32_t kind, tex;
    float p;
    uint32_t flags;  // DMAT_COLOR: col holds the texture's colour
    float col[4];
};
#define DMAT_COLOR 0x1u

// bvh_node (scene_object.h:138-244) subtree as wide nodes: both children's boxes inline.  flags:
// bit 0 / 1 = the left / right child has a box (bvh_node, object_list with hasBox); primitives
// are hit() directly.  Child ref: inner -> index into the wide array; leaf -> BVHW_LEAF |
// count << 24 | first: a run of `count` node records in DScene::bprims (the leaf primitive, or an
// object_list leaf's children in order, nested object_lists as a LIST record before their children).
struct BvhWide {
    float lmin[3];
    uint32_t lref;
    float lmax[3];
    uint32_t rref;
    float rmin[3];
    uint32_t order;
    float rmax[3];
    uint32_t flags;
};
#define BVHW_LEAF 0x80000000u
#define BVHW_MAX_RUN 0x7Fu
#define BVHW_FIRST_MASK 0xFFFFFFu
// the bvh_node walk's empty-stack mark (bvhw_hit): a leaf ref no scene emits (the host refuses a
// run of BVHW_MAX_RUN records starting at BVHW_FIRST_MASK)
static constexpr uint32_t kBvhwEmpty = 0xFFFFFFFFu;
#ifndef MRT_BVHW_SENT
#define MRT_BVHW_SENT 1
#endif
#ifndef MRT_BVHW_PUSH_ALWAYS
#define MRT_BVHW_PUSH_ALWAYS 0
#endif
// The resumable mesh walk's empty-stack mark (MRT_MESH_SENT, as kBvhwEmpty): the caller starts a
// walk with it at the stack's bottom (msp 1), so a pop needs no empty-stack test first; popping it
// ends the walk.  A leaf ref no mesh emits (the host refuses a run of 127 triangles at 0xFFFFFE).
static constexpr uint32_t kMeshEmpty = 0xFFFFFFFEu;
#ifndef MRT_MESH_SENT
#define MRT_MESH_SENT 0  // (A/B hook: profiles/r06_ab.txt section 25)
#endif

// A wide node (MeshWide / BvhWide: both children's boxes, refs, order, flags) fetched whole: four
// 16-byte loads issued together, so one memory round trip per node visit.  (Read field by field,
// the compiler split the node into dependent loads -- left box, right box, order, then the child
// ref at a computed offset -- four round trips per visit.)
struct WideNode {
    f3 lmin, lmax, rmin, rmax;
    uint32_t lref, rref, order, flags;
};
template <typename W>
MRT_DFN WideNode load_wide(const W* p) {
    static_assert(sizeof(W) == 64, "wide node is 64 B");
    const float4* q = reinterpret_cast<const float4*>(p);
    const float4 a = q[0], b = q[1], c = q[2], d = q[3];
    WideNode n;
    n.lmin = f3{a.x, a.y, a.z};
    n.lref = __float_as_uint(a.w);
    n.lmax = f3{b.x, b.y, b.z};
    n.rref = __float_as_uint(b.w);
    n.rmin = f3{c.x, c.y, c.z};
    n.order = __float_as_uint(c.w);
    n.rmax = f3{d.x, d.y, d.z};
    n.flags = __float_as_uint(d.w);
    return n;
}

// The same from any address space: with a treelet (MRT_TREELET) the top wide nodes of the scene's
// BVHs are copied into the workgroup's LDS at kernel start, and a node ref below the treelet size
// reads there -- one flat load per 16 B that the hardware routes to LDS or memory per lane.
MRT_DFN WideNode load_wide_q(const float4* q) {
    float4 a = q[0], b = q[1], c = q[2], d = q[3];
#if defined(__HIP_DEVICE_COMPILE__)
    // all four 16-B pieces in flight together: otherwise the compiler sinks a child's box load
    // below the test of its flag word (`!(flags & 1) || aabb_hit(...)`), a second dependent round
    // trip per node visit
    asm volatile("" : "+v"(a.x), "+v"(a.y), "+v"(a.z), "+v"(a.w), "+v"(b.x), "+v"(b.y), "+v"(b.z), "+v"(b.w));
    asm volatile("" : "+v"(c.x), "+v"(c.y), "+v"(c.z), "+v"(c.w), "+v"(d.x), "+v"(d.y), "+v"(d.z), "+v"(d.w));
#endif
    WideNode n;
    n.lmin = f3{a.x, a.y, a.z};
    n.lref = __float_as_uint(a.w);
    n.lmax = f3{b.x, b.y, b.z};
    n.rref = __float_as_uint(b.w);
    n.rmin = f3{c.x, c.y, c.z};
    n.order = __float_as_uint(c.w);
    n.rmax = f3{d.x, d.y, d.z};
    n.flags = __float_as_uint(d.w);
    return n;
}

// a node record read through the constant address space (scalar loads at a uniform address)
MRT_DFN mrt_node ld_node(const MRT_CONST_AS mrt_node* p) {
    mrt_node n;
    n.kind = p->kind;
    n.a = p->a;
    n.b = p->b;
    n.mat = p->mat;
    for (int k = 0; k < 12; k++) n.f[k] = p->f[k];
    return n;
}

// a per-lane node record fetched whole (four 16-byte loads in flight together)
MRT_DFN mrt_node ld_node_v(const mrt_node* p) {
    const float4* q = reinterpret_cast<const float4*>(p);
    const float4 a = q[0], b = q[1], c = q[2], d = q[3];
    mrt_node n;
    n.kind = __float_as_uint(a.x);
    n.a = __float_as_uint(a.y);
    n.b = __float_as_uint(a.z);
    n.mat = __float_as_uint(a.w);
    n.f[0] = b.x; n.f[1] = b.y; n.f[2] = b.z; n.f[3] = b.w;
    n.f[4] = c.x; n.f[5] = c.y; n.f[6] = c.z; n.f[7] = c.w;
    n.f[8] = d.x; n.f[9] = d.y; n.f[10] = d.z; n.f[11] = d.w;
    return n;
}

// Device-side scene: the mrt_scene_view arrays resident in HBM.
struct DScene {
    const mrt_node* __restrict__ nodes;
    const uint32_t* __restrict__ children;
    const mrt_mesh_node* __restrict__ mnodes;
    const MeshWide* __restrict__ mwide;
    uint32_t mwide_n;
    const BvhWide* __restrict__ bwide;
    const mrt_node* __restrict__ bprims;  // leaf primitive runs of the wide subtrees
    const float4* __restrict__ tri_geo;
    const float4* __restrict__ tri_nrm;
    const DMat* __restrict__ mats;
    const mrt_texture* __restrict__ texs;
    const float4* __restrict__ ranvec;
    const int32_t* __restrict__ perm;
    const uint8_t* __restrict__ texels;
    const LinOp* __restrict__ prog;  // linear hit program (FT_LIN kernels), mrt_lin.h
    const mrt_node* __restrict__ bleaf;  // leaves of scene.biased_objects (the list's children, or the object)
    uint32_t nbleaf, blist;              // leaf count; 1 if biased_objects is an object_list
    float nbleaf_f, inv_nbleaf;          // (float)nbleaf and RN(1 / (float)nbleaf), from the host: kernarg
                                         // scalars (converted on the device they held two VGPRs, spilled)
    uint32_t root, biased, sky;
    mrt_camera cam;
    const mrt_camera* __restrict__ camp;  // the camera in HBM, read at each path start (scalar loads)
};



#define MRT_NODE_KIND(n) ((n).kind & 0xFFu)
#define MRT_NODE_ORDER(n) (((n).kind >> 8) & 0xFFu)
#define MRT_NODE_FLAGS(n) (((n).kind >> 16) & 0xFFu)
#define MRT_F_NEEDUV 0x4u   /* set on upload when the node's material samples uv */
#define MRT_F_BOX6 0x10u    /* set on upload on an object_list that is box.h's six rects (planes in f[6..11]) */
#define MRT_F_BOXINST 0x20u /* tolerance-contract program: an instance outside instances whose body is one MRT_F_BOX6 list */
#define MRT_F_LAST 0x40u    /* tolerance-contract program: the op after which the interpreter reaches the END op */
#define MRT_F_VSUB 0x80u    /* linear program: a constant_volume op whose boundary is the sub-program [op + 1, skip) */
#define MRT_K_TRROTY 11u    /* upload fuses translate(rotate_y(x)) into one instance node */
#define MRT_K_BVHW 12u      /* upload: a bvh_node subtree over primitives / object_lists as wide nodes */

// Scene features; kernels are instantiated for feature subsets so that Cornell-like scenes run
// without the code (and registers) of BVH/mesh/volume/texture paths they never take.
enum : uint32_t {
    FT_BVH = 1u << 0,
    FT_MESH = 1u << 1,
    FT_VOLUME = 1u << 2,
    FT_INST = 1u << 3,
    FT_TEX = 1u << 4,      // checker / perlin / image textures
    FT_METAL = 1u << 5,
    FT_ISO = 1u << 6,      // isotropic phase function
    FT_MOVING = 1u << 7,   // moving spheres
    FT_SKY = 1u << 8,
    FT_BSPHERE = 1u << 9,  // sphere in the biased (light-sampling) list
    FT_UV = 1u << 10,      // uv sampled on spheres / rects
    FT_LIN = 1u << 11,     // scene graph compiled to a linear hit program (mrt_lin.h)
    FT_BVHW = 1u << 12,    // bvh_node subtrees as wide nodes (MRT_K_BVHW)
    FT_BIASED = 1u << 13,  // a biased (light-sampling) list: the mixture pdf of main.cpp:86-101
    FT_ALL = ((1u << 14) - 1) & ~FT_LIN,
    // linear programs only: a constant_volume bounded by an object_list / instance subtree (box.h
    // boundaries, cornell_smoke, scene.cpp:334-376), walked as a sub-program (mrt_lin.h lin_sub_t)
    FT_VSUB = 1u << 14,
};

// Per-wave LDS stacks, lane-interleaved ([slot][word][lane]) so every access is conflict-free.
struct LStack {
    uint32_t* frames;  // 2 words per slot: node, state
    float* rays;       // 11 words per slot: o.xyz, d.xyz, inv.xyz, inside, mask
    uint32_t* mesh;    // 1 word per slot
    float* save;       // 9 words: query ray parked by the linear program (mrt_lin.h)
    uint32_t lane;
    const float4* tree;  // the workgroup's LDS copy of BvhWide nodes [0, tree_b) (TreeOf<F>::on kernels)
    uint32_t tree_b;
};

// Hot BVH nodes in LDS (north star): kernels of the bvh_node scenes run two 12-wave workgroups
// per CU (6 waves per SIMD, MRT_WPE_WIDE), and each group keeps the top levels of the scene's
// bvh_node subtrees (breadth-first wide-node numbering: the first tree_b nodes) in the LDS its
// waves' stacks leave free.  Measured on MI355X (DESIGN.md "Hot nodes in LDS"): random spheres
// +14%, book2 +3.6%; for the pod_bvh kernels (7 waves per SIMD, no LDS to spare at one-wave
// groups) bigger groups cost more than the treelet gained, so they keep one-wave groups and no
// treelet.  (Round 4: 2 x 12 waves over 1 x 16 -- book2 +7.4%, random spheres +9%; 2 x 10, 2 x 14
// and 2 x 16 waves slower: book2 -29%, -19%, -32%, profiles/r04_ab.txt.)
#ifndef MRT_TREELET
#define MRT_TREELET 1
#endif
#ifndef MRT_TREE_WG
#define MRT_TREE_WG (MRT_FAST ? 768 : 1024)  // the exact contract's kernels keep 1 x 16 waves (no A/B there)
#endif
// the tolerance contract's sky-lit bvh_node kernels (scenes 0-4): six 4-wave groups per CU, each
// with its own smaller treelet (random spheres +10% per step against 2 x 12 waves; book2, the
// volume variant, keeps 2 x 12: 3 x 8 -25%, 6 x 4 -12%; profiles/r04_ab.txt section 10)
#ifndef MRT_TREE_WG_SKY
#define MRT_TREE_WG_SKY (MRT_FAST ? 256 : MRT_TREE_WG)
#endif
template <uint32_t F>
struct TreeOf {
    // the kernels of bvh_node scenes (wide-node walks); the same test as PathOcc::kWide
    static constexpr bool on = MRT_TREELET && (F & FT_BVHW) != 0 &&
                               ((F & (FT_BVHW | FT_TEX | FT_VOLUME)) != 0 || !(F & FT_LIN));
    // threads per path-kernel workgroup (the generic machine, no linear program, keeps 1 x 16
    // waves: at 6 waves per SIMD it spills)
    static constexpr uint32_t wg = !on ? 64u : !(F & FT_LIN) ? 1024u : (F & FT_VOLUME) ? (uint32_t)(MRT_TREE_WG) : (uint32_t)(MRT_TREE_WG_SKY);
};
// A treelet node through LDS instructions (ds_read_b128: LDS latency, lgkmcnt only), instead of
// the flat load that can reach LDS or memory per lane (a flat access waits on both counters)
#ifndef MRT_TREE_DS
#define MRT_TREE_DS 1
#endif
MRT_DFN WideNode load_wide_lds(const float4* tree, uint32_t ref) {
#if defined(__HIP_DEVICE_COMPILE__)
    const MRT_LDS_AS float4* q = (const MRT_LDS_AS float4*)tree + (size_t)ref * 4;
#else
    const float4* q = tree + (size_t)ref * 4;
#endif
    float4 a = q[0], b = q[1], c = q[2], d = q[3];
#if defined(__HIP_DEVICE_COMPILE__)
    asm volatile("" : "+v"(a.x), "+v"(a.y), "+v"(a.z), "+v"(a.w), "+v"(b.x), "+v"(b.y), "+v"(b.z), "+v"(b.w));
    asm volatile("" : "+v"(c.x), "+v"(c.y), "+v"(c.z), "+v"(c.w), "+v"(d.x), "+v"(d.y), "+v"(d.z), "+v"(d.w));
#endif
    WideNode n;
    n.lmin = f3{a.x, a.y, a.z};
    n.lref = __float_as_uint(a.w);
    n.lmax = f3{b.x, b.y, b.z};
    n.rref = __float_as_uint(b.w);
    n.rmin = f3{c.x, c.y, c.z};
    n.order = __float_as_uint(c.w);
    n.rmax = f3{d.x, d.y, d.z};
    n.flags = __float_as_uint(d.w);
    return n;
}
#ifndef MRT_WIDE_OFF32
#define MRT_WIDE_OFF32 1  // (C4 +3.7% with the mask-logic selects, +1.6% alone; profiles/r06_ab.txt section 21)
#endif
// wide node `ref` of a BvhWide / MeshWide array: from the LDS treelet when it holds it
template <bool TREE, typename W>
MRT_DFN WideNode wide_at(const W* base, uint32_t ref, const LStack& L) {
    if constexpr (TREE) {
#if MRT_TREE_DS
        // (a lane-divergent branch only when the treelet does not hold the whole tree)
        if (ref < L.tree_b) return load_wide_lds(L.tree, ref);
        return load_wide_q(reinterpret_cast<const float4*>(base + ref));
#else
        const float4* q = ref < L.tree_b ? L.tree + (size_t)ref * 4 : reinterpret_cast<const float4*>(base + ref);
        return load_wide_q(q);
#endif
    } else {
        (void)L;
#if MRT_WIDE_OFF32
        // the node's byte offset as 32 bits (refs < 2^24): a scalar base plus a per-lane 32-bit
        // offset, one shift per visit instead of a 64-bit shift and add
        return load_wide(reinterpret_cast<const W*>(reinterpret_cast<const char*>(base) + (size_t)(ref * 64u)));
#else
        return load_wide(base + ref);
#endif
    }
}

// the tolerance contract's unit-direction shortcut (make_ray_unit) per kernel variant: not for
// scenes with bvh_node subtrees, textures or volumes (book2's numerics are too sensitive to it)
template <uint32_t F>
static constexpr bool kFastUnit = MRT_FAST_UNIT && (F & (FT_BVHW | FT_TEX | FT_VOLUME)) == 0;

template <uint32_t F>
MRT_DFN bool is_prim(uint32_t kind) {
    return kind == MRT_K_SPHERE || kind == MRT_K_XY || kind == MRT_K_XZ || kind == MRT_K_YZ || ((F & FT_MESH) && kind == MRT_K_MESH) ||
           ((F & FT_BVHW) && kind == MRT_K_BVHW);
}

// a mesh wide node (one 64-B record, four 16-B loads in flight together; a four-plane SoA layout
// was measured slower)
template <bool TREE>
MRT_DFN WideNode mesh_wide(const DScene& S, uint32_t ref, const LStack& L) {
    return wide_at<TREE>(S.mwide, ref, L);
}

// get_sphere_uv (sphere.cpp:6-11)
MRT_DFN void sphere_uv(f3 p, float* u, float* v) {
    float phi = atan2_(p.z, p.x);
    float theta = asin_(p.y);
    *u = ref_fnma(phi, 1.0f / (2.0f * PI_F), 0.5f);  // sphere.cpp:9
    *v = ref_fma(theta, 1.0f / PI_F, 0.5f);           // sphere.cpp:10
}

template <uint32_t F>
MRT_DFN f3 sphere_center(const mrt_node& n, float time) {
    f3 c0 = ld3(n.f);
    if ((F & FT_MOVING) && (MRT_NODE_FLAGS(n) & MRT_F_MOVING)) {
        const float s = (time - n.f[6]) / (n.f[7] - n.f[6]);
        const f3 dc = sub(ld3(n.f + 3), c0);
        return f3{madd_det(s, dc.x, c0.x), madd_det(s, dc.y, c0.y), madd_det(s, dc.z, c0.z)};
    }
    return c0;
}

// sphere::hit (sphere.cpp:13-46).  `full` = write p/n/uv (false inside volume boundary queries).
template <uint32_t F>
MRT_DFN bool sphere_hit(const mrt_node& n, const Ray& r, float tmin, float tmax, HitRec& rec, bool full) {
    f3 cen = sphere_center<F>(n, r.time);
    float radius = n.f[8];
    f3 oc = sub(r.o, cen);
    float b;
    float disc = sphere_disc(oc, r.d, radius, &b);
    if (disc > 0) {
        float sq = sqrt_(disc);
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
                if ((F & FT_UV) && (MRT_NODE_FLAGS(n) & MRT_F_NEEDUV)) sphere_uv(rec.n, &rec.u, &rec.v);
            }
            return true;
        }
    }
    return false;
}

// xy/xz/yz_rect::hit (rect.cpp:24-152); AX = plane axis (2: xy, 1: xz, 0: yz)
template <uint32_t F, int AX>
MRT_DFN bool rect_hit(const mrt_node& n, const Ray& r, float tmin, float tmax, HitRec& rec, bool full) {
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
    float ob = AX == 0 ? r.o.y : r.o.x, db = AX == 0 ? r.d.y : r.d.x;
    float oc = AX == 2 ? r.o.y : r.o.z, dc = AX == 2 ? r.d.y : r.d.z;
    float pb = ref_fma(t, db, ob);  // rect.cpp:32-33, 77-78, 138-139
    float pc = ref_fma(t, dc, oc);
    if (pb < n.f[0] || pb > n.f[1] || pc < n.f[2] || pc > n.f[3]) return false;
    rec.t = t;
    if (full) {
        if ((F & FT_UV) && (MRT_NODE_FLAGS(n) & MRT_F_NEEDUV)) {
            rec.u = (pb - n.f[0]) / (n.f[1] - n.f[0]);
            rec.v = (pc - n.f[2]) / (n.f[3] - n.f[2]);
        }
        rec.mat = n.mat;
        rec.p = eval(r, t);
        if (MRT_FAST_SNAP) {  // tolerance contract: the hit point on the rect's plane (see mrt_device.h)
            if (AX == 2) rec.p.z = n.f[4];
            else if (AX == 1) rec.p.y = n.f[4];
            else rec.p.x = n.f[4];
        }
        rec.n = AX == 2 ? f3{0, 0, ns} : AX == 1 ? f3{0, ns, 0} : f3{ns, 0, 0};
    }
    return true;
}

// triangle::hit (triangle.cpp:222-265) without the normal (deferred to the closest hit)
MRT_DFN bool tri_hit(const DScene& S, uint32_t i, const Ray& r, float tmin, float tmax, float* tout, float* uout, float* vout) {
    const float4* g = S.tri_geo + (size_t)i * 3;
    f3 m = ld3(g[0]), u = ld3(g[1]), v = ld3(g[2]);
#if defined(__HIP_DEVICE_COMPILE__)
    // the three rows in one round trip: otherwise m's load sinks below the det test and becomes a
    // second dependent fetch for every triangle that passes it
    asm volatile("" ::"v"(m.x), "v"(m.y), "v"(m.z));
#endif
    f3 pvec = cross(r.d, v);
    float det = dot(u, pvec);
    float sign = 1.0f;
    if (r.inside) {
        sign = det < 0.0f ? -1.0f : 1.0f;
        det = sign * det;
    }
    // Branch-free: every value is computed whatever the early tests say and the outcome is one
    // predicate (the reference's early returns only skip work whose result is unused, so the
    // results are the same bits); a wave's lanes rarely all fail a test, and the nested
    // branches cost more in exec-mask bookkeeping than they saved (room + mesh kernels)
    const bool ok_det = !(det < 0.00001f);
    f3 tvec = sub(r.o, m);
    float uu = dot(tvec, pvec) * sign;
    f3 qvec = cross(tvec, u);
    float vv = dot(r.d, qvec) * sign;
    const bool ok_uv = !((uu < 0) | (uu > det) | (vv < 0) | ((uu + vv) > det));
#if MRT_FAST_DIV && defined(__HIP_DEVICE_COMPILE__)
    float invDet = __builtin_amdgcn_rcpf(det);
#else
    float invDet = 1 / det;
#endif
    float t = (dot(v, qvec) * invDet) * sign;
    const bool ok_t = !((t < tmin) | (t > tmax));
    *tout = t;
    *uout = uu * invDet;
    *vout = vv * invDet;
    return ok_det & ok_uv & ok_t;
}

// pod_bvh::hit (triangle.h:171-221): depth-first, closer child first (node_order & dirMask); the
// first leaf that reports a hit ends the walk (every ancestor returns on hit_closer/hit_farther).
// Both children's boxes are tested when their parent is reached -- with the same (tmin, tmax) the
// reference uses when it visits them, since nothing narrows tmax before the walk ends -- and only
// a farther child whose box was hit is pushed (short stack in LDS).  n.a = root node, n.b = root ref.
MRT_DFN bool mesh_leaf(const DScene& S, uint32_t ref, const mrt_node& n, const Ray& r, float tmin, float tmax, HitRec& rec,
                                          bool full) {
    const uint32_t first = ref & 0xFFFFFFu, cnt = (ref >> 24) & 0x7Fu;
    bool has = false;
    uint32_t best = 0;
    float bu = 0, bv = 0, tt = tmax;
    for (uint32_t k = 0; k < cnt; k++) {
        float t, uu, vv;
        if (tri_hit(S, first + k, r, tmin, tt, &t, &uu, &vv)) {
            has = true;
            tt = t;
            best = first + k;
            bu = uu;
            bv = vv;
        }
    }
    if (has) {
        rec.t = tt;
        if (full) {
            const float4* q = S.tri_nrm + (size_t)best * 3;
            f3 nm = ld3(q[0]), nu = ld3(q[1]), nv = ld3(q[2]);
            rec.p = eval(r, tt);
            rec.n = normalize(add(add(mulf(nm, (1 - bu) - bv), mulf(nu, bu)), mulf(nv, bv)));
            rec.u = bu;
            rec.v = bv;
            rec.mat = n.mat;
        }
    }
    return has;
}
// UNIFORM: the mesh node is the same for the whole wave (linear programs): the root box is read
// through the constant address space (scalar loads) instead of by a per-lane load chain.
template <bool UNIFORM = false>
MRT_DFN bool mesh_hit(const DScene& S, const mrt_node& n, const Ray& r, float tmin, float tmax, HitRec& rec, bool full,
                                         const LStack& L) {
    if constexpr (UNIFORM) {
        const MRT_CONST_AS mrt_mesh_node& root = const_ptr(S.mnodes)[n.a];
        if (!aabb_hit(f3{root.bmin[0], root.bmin[1], root.bmin[2]}, f3{root.bmax[0], root.bmax[1], root.bmax[2]}, r, tmin, tmax)) return false;
    } else {
        const mrt_mesh_node& root = S.mnodes[n.a];
        if (!aabb_hit(root.bmin, root.bmax, r, tmin, tmax)) return false;
    }
    uint32_t ref = n.b, msp = 0;
    const bool bad = any_lane(!r.nice);  // (once per walk: aabb_hit_b)
#ifdef MRT_MESH_WW
    // "while-while" (Aila & Laine 2009), as bvhw_hit: measured 20% slower on the bunny (C4) and 1%
    // on the teapot (C3) than the one-step-per-iteration walk below, so kept as an experiment.
    for (;;) {
        while (!(ref & MESH_LEAF)) {
            const WideNode W = mesh_wide<false>(S, ref, L);
            const bool hl = aabb_hit_b(W.lmin, W.lmax, r, tmin, tmax, bad);
            const bool hr = aabb_hit_b(W.rmin, W.rmax, r, tmin, tmax, bad);
            const bool left_first = (W.order & r.mask) != 0;
            const uint32_t cref = left_first ? W.lref : W.rref, fref = left_first ? W.rref : W.lref;
            const bool hc = sel_b(left_first, hl, hr), hf = sel_b(left_first, hr, hl);
            if (hc) {
                if (hf) L.mesh[(msp++) * 64 + L.lane] = fref;
                ref = cref;
            } else if (hf) {
                ref = fref;
            } else {
                if (msp == 0) return false;
                ref = L.mesh[(--msp) * 64 + L.lane];
            }
        }
        if (mesh_leaf(S, ref, n, r, tmin, tmax, rec, full)) return true;
        if (msp == 0) return false;
        ref = L.mesh[(--msp) * 64 + L.lane];
    }
#else
    for (;;) {
        if (ref & MESH_LEAF) {
            if (mesh_leaf(S, ref, n, r, tmin, tmax, rec, full)) return true;
        } else {
            const WideNode W = mesh_wide<false>(S, ref, L);
            const bool hl = aabb_hit_b(W.lmin, W.lmax, r, tmin, tmax, bad);
            const bool hr = aabb_hit_b(W.rmin, W.rmax, r, tmin, tmax, bad);
            const bool left_first = (W.order & r.mask) != 0;
            const uint32_t cref = left_first ? W.lref : W.rref, fref = left_first ? W.rref : W.lref;
            const bool hc = sel_b(left_first, hl, hr), hf = sel_b(left_first, hr, hl);
            if (hc) {
                if (hf) L.mesh[(msp++) * 64 + L.lane] = fref;
                ref = cref;
                continue;
            }
            if (hf) {
                ref = fref;
                continue;
            }
        }
        if (msp == 0) return false;
        ref = L.mesh[(--msp) * 64 + L.lane];
    }
#endif
}

// One step of mesh_hit's walk for a lane whose state persists between calls (ref, msp and its LDS
// stack; inside a leaf: the triangles left in ref, the leaf's running closest in tt, the best
// triangle so far in rec.mat / rec.u / rec.v, `in_hit` set once one hit).  A step is an inner
// node's two boxes or ONE triangle of a leaf, so lanes in leaves of different sizes (up to 25
// triangles) and lanes at inner nodes cost about the same per step.  Returns 0: keep walking,
// 1: hit (rec complete, tt = its t; the walk is over: first-hit early-out), 2: no hit.  Every lane
// performs mesh_hit's operations in mesh_hit's order: the results are bit-identical.
// DEFER: on a hit, return 1 with the record's triangle (rec.mat), barycentrics (rec.u, rec.v) and
// tt only -- mesh_hit_rec completes it once the walk is over.  Completed inside the step, the point
// and normal were carried round every walk step of the wave (the compiler copied all six registers
// in and out of each step's branches).
template <bool TREE = false, bool DEFER = false>
MRT_DFN uint32_t mesh_step(const DScene& S, const mrt_node& n, const Ray& r, float tmin, float& tt, HitRec& rec,
                                              const LStack& L, uint32_t& ref, uint32_t& msp, bool& in_hit, bool bad) {
    if constexpr (DEFER) {
        // the same step with the walk state updated by selects where mesh_step branches and
        // returns: each branch's results otherwise merged in copies of every state register
        uint32_t res = 0u;
        bool pop;
        if (ref & MESH_LEAF) {
            const uint32_t first = ref & 0xFFFFFFu, cnt = (ref >> 24) & 0x7Fu;
            float t = 0.0f, uu = 0.0f, vv = 0.0f;
            const bool h = cnt > 0 && tri_hit(S, first, r, tmin, tt, &t, &uu, &vv);
            in_hit = in_hit || h;
            tt = h ? t : tt;
            rec.mat = h ? first : rec.mat;
            rec.u = h ? uu : rec.u;
            rec.v = h ? vv : rec.v;
            const bool more = cnt > 1;
            ref = more ? (MESH_LEAF | ((cnt - 1) << 24) | (first + 1)) : ref;
            res = (!more && in_hit) ? 1u : 0u;
            pop = !more && !in_hit;
        } else {
            const WideNode W = mesh_wide<TREE>(S, ref, L);
            const bool hl = aabb_hit_b(W.lmin, W.lmax, r, tmin, tt, bad);
            const bool hr = aabb_hit_b(W.rmin, W.rmax, r, tmin, tt, bad);
            const bool left_first = (W.order & r.mask) != 0;
            const uint32_t cref = left_first ? W.lref : W.rref, fref = left_first ? W.rref : W.lref;
            const bool hc = sel_b(left_first, hl, hr), hf = sel_b(left_first, hr, hl);
            if (hc && hf) L.mesh[(msp++) * 64 + L.lane] = fref;
            ref = hc ? cref : (hf ? fref : ref);
            pop = !hc && !hf;
        }
        if (pop) {
#if MRT_MESH_SENT
            ref = L.mesh[(--msp) * 64 + L.lane];
            res = ref == kMeshEmpty ? 2u : res;
#else
            if (msp == 0) res = 2u;
            else ref = L.mesh[(--msp) * 64 + L.lane];
#endif
        }
        return res;
    }
    if (ref & MESH_LEAF) {
        const uint32_t first = ref & 0xFFFFFFu, cnt = (ref >> 24) & 0x7Fu;
        float t, uu, vv;
        if (cnt > 0 && tri_hit(S, first, r, tmin, tt, &t, &uu, &vv)) {
            in_hit = true;
            tt = t;
            rec.mat = first;
            rec.u = uu;
            rec.v = vv;
        }
        if (cnt > 1) {
            ref = MESH_LEAF | ((cnt - 1) << 24) | (first + 1);
            return 0u;
        }
        if (in_hit) {  // mesh_leaf's record of the leaf's closest triangle
            const uint32_t best = rec.mat;
            const float bu = rec.u, bv = rec.v;
            const float4* q = S.tri_nrm + (size_t)best * 3;
            f3 nm = ld3(q[0]), nu = ld3(q[1]), nv = ld3(q[2]);
            rec.t = tt;
            rec.p = eval(r, tt);
            rec.n = normalize(add(add(mulf(nm, (1 - bu) - bv), mulf(nu, bu)), mulf(nv, bv)));
            rec.mat = n.mat;
            return 1u;
        }
    } else {
        const WideNode W = mesh_wide<TREE>(S, ref, L);
        const bool hl = aabb_hit_b(W.lmin, W.lmax, r, tmin, tt, bad);
        const bool hr = aabb_hit_b(W.rmin, W.rmax, r, tmin, tt, bad);
        const bool left_first = (W.order & r.mask) != 0;
        const uint32_t cref = left_first ? W.lref : W.rref, fref = left_first ? W.rref : W.lref;
        const bool hc = sel_b(left_first, hl, hr), hf = sel_b(left_first, hr, hl);
        if (hc) {
            if (hf) L.mesh[(msp++) * 64 + L.lane] = fref;
            ref = cref;
            return 0u;
        }
        if (hf) {
            ref = fref;
            return 0u;
        }
    }
    if (msp == 0) return 2u;
    ref = L.mesh[(--msp) * 64 + L.lane];
    return 0u;
}
// Leaf postponing (Aila & Laine 2009's speculative traversal) for the resumable mesh walk, as an
// A/B variant of mesh_step<TREE, true> (MRT_MESH_SPEC): a lane that reaches a leaf run parks it in
// `pref` and walks on through inner nodes in DFS order (the stack's next entries), stopping at a
// second leaf or the stack's end; the WAVE chooses per iteration between an inner step (every lane
// that can take one) and a leaf step (one triangle of every parked run), so an iteration runs one of
// the two codes instead of both.  Same results: the nodes walked past a parked leaf are the ones DFS
// visits after it, tested with the same tt (a parked run that hits ends the walk, and the steps
// taken beyond it are dropped).  kMeshEnd: the stack ran out while a run is parked.
static constexpr uint32_t kMeshEnd = 0xFFFFFFFFu;
template <bool TREE = false>
MRT_DFN uint32_t mesh_step_spec(const DScene& S, const Ray& r, float tmin, float& tt, HitRec& rec, const LStack& L, uint32_t& ref,
                                uint32_t& pref, uint32_t& msp, bool& in_hit, bool leaf_iter, bool bad) {
    uint32_t res = 0u;
    if (leaf_iter) {  // one triangle of the parked run (mesh_step's leaf step)
        if (pref != 0u) {
            const uint32_t first = pref & 0xFFFFFFu, cnt = (pref >> 24) & 0x7Fu;
            float t = 0.0f, uu = 0.0f, vv = 0.0f;
            const bool h = cnt > 0 && tri_hit(S, first, r, tmin, tt, &t, &uu, &vv);
            in_hit = in_hit || h;
            tt = h ? t : tt;
            rec.mat = h ? first : rec.mat;
            rec.u = h ? uu : rec.u;
            rec.v = h ? vv : rec.v;
            const bool more = cnt > 1;
            pref = more ? (MESH_LEAF | ((cnt - 1) << 24) | (first + 1)) : 0u;
            res = (!more && in_hit) ? 1u : ((!more && ref == kMeshEnd) ? 2u : 0u);
        }
        return res;
    }
    if (ref == kMeshEnd) return 0u;  // waits for its parked run
    if (ref & MESH_LEAF) {
        if (pref != 0u) return 0u;  // a second leaf: waits
        pref = ref;                  // parked; the walk goes on with the stack's next entry
#if MRT_MESH_SENT
        ref = L.mesh[(--msp) * 64 + L.lane];
        ref = ref == kMeshEmpty ? kMeshEnd : ref;
#else
        ref = msp == 0u ? kMeshEnd : L.mesh[(--msp) * 64 + L.lane];
#endif
        return 0u;
    }
    const WideNode W = mesh_wide<TREE>(S, ref, L);
    const bool hl = aabb_hit_b(W.lmin, W.lmax, r, tmin, tt, bad);
    const bool hr = aabb_hit_b(W.rmin, W.rmax, r, tmin, tt, bad);
    const bool left_first = (W.order & r.mask) != 0;
    const uint32_t cref = left_first ? W.lref : W.rref, fref = left_first ? W.rref : W.lref;
    const bool hc = sel_b(left_first, hl, hr), hf = sel_b(left_first, hr, hl);
    if (hc && hf) L.mesh[(msp++) * 64 + L.lane] = fref;
    ref = hc ? cref : (hf ? fref : ref);
    if (!hc && !hf) {
#if MRT_MESH_SENT
        ref = L.mesh[(--msp) * 64 + L.lane];
        const bool end = ref == kMeshEmpty;
        ref = end && pref != 0u ? kMeshEnd : ref;
        res = end && pref == 0u ? 2u : res;
#else
        if (msp != 0u) ref = L.mesh[(--msp) * 64 + L.lane];
        else if (pref != 0u) ref = kMeshEnd;
        else res = 2u;
#endif
    }
    return res;
}

// the record mesh_step<TREE, true> left for mesh_leaf: its closest triangle's point and normal,
// the mesh's material (the same operations as mesh_step's own completion)
MRT_DFN void mesh_hit_rec(const DScene& S, const mrt_node& n, const Ray& r, float tt, HitRec& rec) {
    const uint32_t best = rec.mat;
    const float bu = rec.u, bv = rec.v;
    const float4* q = S.tri_nrm + (size_t)best * 3;
    f3 nm = ld3(q[0]), nu = ld3(q[1]), nv = ld3(q[2]);
    rec.t = tt;
    rec.p = eval(r, tt);
    rec.n = normalize(add(add(mulf(nm, (1 - bu) - bv), mulf(nu, bu)), mulf(nv, bv)));
    rec.mat = n.mat;
}

template <uint32_t F>
MRT_DFN bool leaf_prim_hit(const mrt_node& n, uint32_t kind, const Ray& r, float tmin, float tmax, HitRec& rec, bool full) {
    switch (kind) {
    case MRT_K_SPHERE: return sphere_hit<F>(n, r, tmin, tmax, rec, full);
    case MRT_K_XY: return rect_hit<F, 2>(n, r, tmin, tmax, rec, full);
    case MRT_K_XZ: return rect_hit<F, 1>(n, r, tmin, tmax, rec, full);
    default: return rect_hit<F, 0>(n, r, tmin, tmax, rec, full);
    }
}

// Tolerance contract: an object_list flagged MRT_F_BOX6 (box.h's six outward-facing rects, planes
// in f[6..11], the rects' material in mat) as one slab test -- the entry face is the one
// front-facing rect a ray from outside can hit (mrt_sig.h box6_hit); its record is the rect's
// (rect.cpp:40-44: p on the plane, n = the face's axis and sign).  Its own bounding-box test is
// implied by the slab test.
MRT_DFN bool box6_leaf_hit(const mrt_node& c, const Ray& r, float tmin, float tmax, HitRec& rec, bool full) {
    const float t0x = (c.f[6] - r.o.x) * r.inv.x, t1x = (c.f[9] - r.o.x) * r.inv.x;
    const float t0y = (c.f[7] - r.o.y) * r.inv.y, t1y = (c.f[10] - r.o.y) * r.inv.y;
    const float t0z = (c.f[8] - r.o.z) * r.inv.z, t1z = (c.f[11] - r.o.z) * r.inv.z;
    const float nx = fminf(t0x, t1x), ny = fminf(t0y, t1y), nz = fminf(t0z, t1z);
    const float tn = fmaxf(fmaxf(nx, ny), nz);
    const float tf = fminf(fminf(fmaxf(t0x, t1x), fmaxf(t0y, t1y)), fmaxf(t0z, t1z));
    if (!((tn <= tf) & (tn >= tmin) & (tn <= tmax))) return false;
    rec.t = tn;
    if (full) {
        rec.mat = c.mat;
        rec.p = eval(r, tn);
        // ties go to the later rect of box.h's order (x faces, then y, then z)
        if (tn == nx) {
            const bool lo = r.d.x > 0.0f;
            rec.p.x = lo ? c.f[6] : c.f[9];
            rec.n = f3{lo ? -1.0f : 1.0f, 0, 0};
        } else if (tn == ny) {
            const bool lo = r.d.y > 0.0f;
            rec.p.y = lo ? c.f[7] : c.f[10];
            rec.n = f3{0, lo ? -1.0f : 1.0f, 0};
        } else {
            const bool lo = r.d.z > 0.0f;
            rec.p.z = lo ? c.f[8] : c.f[11];
            rec.n = f3{0, 0, lo ? -1.0f : 1.0f};
        }
    }
    return true;
}

// a bvh_node leaf: a primitive, or an object_list (its box already tested by the parent) of
// primitives and object_lists of primitives (box, box.h:6-30) -- object_list::hit semantics,
// the running closest narrowing across children (scene_object.h:79-103).  The leaf is a run of
// node records (BVHW_LEAF ref); a nested list's record carries its box and child count.
template <uint32_t F>
MRT_DFN bool bvhw_leaf(const DScene& S, uint32_t ref, const Ray& r, float tmin, float tmax, HitRec& rec, bool full) {
    const uint32_t first = ref & BVHW_FIRST_MASK, cnt = (ref >> 24) & BVHW_MAX_RUN;
    const mrt_node* run = S.bprims + first;
    if (cnt == 1) {  // a primitive leaf (or a list of one): hit() with the bvh_node's (tmin, tmax)
        const mrt_node n = ld_node_v(run);
        const uint32_t k = MRT_NODE_KIND(n);
        // t alone first, the record by a second test of a hit with the same (tmin, tmax): the
        // record written inside the primitive-kind switch merged its registers at the switch's end
        // (book2 117 -> 105 VGPRs, kernel -1.6%; random spheres -4.5%)
        if (k == MRT_K_LIST) return false;
        HitRec tr;
        if (!leaf_prim_hit<F>(n, k, r, tmin, tmax, tr, false)) return false;
        if (!full) {  // t, and what bvhw_leaf_rec needs to make the record later
            rec.t = tr.t;
            rec.mat = first;
            rec.u = tmax;
            return true;
        }
        // the second test repeats the first's predicate with the same operands and range: its
        // arithmetic is contraction-proof (explicit ref_f* / madd_det fusions, the rest unfused), so it
        // hits again.  (Returning its result instead of true changed the register allocation of the
        // whole walk: book2's fast kernel 40 -> 204 spilled VGPRs, round 4.  MRT_CHECK_LEAF builds
        // assert it.)
        const bool again = leaf_prim_hit<F>(n, k, r, tmin, tmax, rec, true);
#ifdef MRT_CHECK_LEAF
        if (!again) __builtin_trap();
#endif
        (void)again;
        return true;
    }
    // The run's primitives are tested for t alone; the closest one's full record is computed once
    // after the loop, by the same test with the same (tmin, tmax) it passed with -- the same bits.
    // (Each hit writing the whole record inside the loop merged all its registers at every
    // primitive-kind branch: 132 of the loop's 233 VALU instructions were copies.)
    float closest = tmax, t_before = tmax;
    uint32_t best = ~0u;
    for (uint32_t i = 0; i < cnt; i++) {
        const mrt_node c = ld_node_v(run + i);
        const uint32_t ck = MRT_NODE_KIND(c);
        HitRec tr;
        if (ck == MRT_K_LIST) {
            if (MRT_FAST_BOX && (MRT_NODE_FLAGS(c) & MRT_F_BOX6)) {  // box.h's six rects as one slab test
                const bool h = box6_leaf_hit(c, r, tmin, closest, tr, false);
                t_before = h ? closest : t_before;
                best = h ? i : best;
                closest = h ? tr.t : closest;
                i += c.b;
                continue;
            }
            if ((MRT_NODE_FLAGS(c) & MRT_F_HASBOX) && !aabb_hit(c.f, c.f + 3, r, tmin, closest)) i += c.b;
            continue;
        }
        const bool h = leaf_prim_hit<F>(c, ck, r, tmin, closest, tr, false);
        t_before = h ? closest : t_before;
        best = h ? i : best;
        closest = h ? tr.t : closest;
    }
    if (best == ~0u) return false;
    if (!full) {  // t, and what bvhw_leaf_rec needs to make the record later
        rec.t = closest;
        rec.mat = first + best;
        rec.u = t_before;
        return true;
    }
    const mrt_node c = ld_node_v(run + best);
    const uint32_t ck = MRT_NODE_KIND(c);
    bool again;  // (the same test with the same range: it hits again; see the one-primitive case)
    if (MRT_FAST_BOX && ck == MRT_K_LIST) again = box6_leaf_hit(c, r, tmin, t_before, rec, true);
    else again = leaf_prim_hit<F>(c, ck, r, tmin, t_before, rec, true);
#ifdef MRT_CHECK_LEAF
    if (!again) __builtin_trap();
#endif
    (void)again;
    return true;
}

// The record of a bvh_node leaf hit that bvhw_leaf(.., full = false) found: primitive `prim` of
// S.bprims (its rec.mat) hit at or before tlim (its rec.u) -- bvhw_leaf's own second test, with the
// same ray and range, made after the scene's walk instead of inside it (mrt_lin.h MRT_LIN_DEFER).
template <uint32_t F>
MRT_DFN void bvhw_leaf_rec(const DScene& S, uint32_t prim, const Ray& r, float tmin, float tlim, HitRec& rec) {
    const mrt_node c = ld_node_v(S.bprims + prim);
    const uint32_t ck = MRT_NODE_KIND(c);
    bool again;  // (the same test with the same range: it hits again)
    if (MRT_FAST_BOX && ck == MRT_K_LIST) again = box6_leaf_hit(c, r, tmin, tlim, rec, true);
    else again = leaf_prim_hit<F>(c, ck, r, tmin, tlim, rec, true);
#ifdef MRT_CHECK_LEAF
    if (!again) __builtin_trap();
#endif
    (void)again;
}

// bvh_node::hit (scene_object.h:208-244) over wide nodes: the root's own box, then depth-first,
// closer child first (node_order & dirMask), the first child subtree that hits ends the walk.
// A child's box is tested at its parent with the (tmin, tmax) the reference uses when it visits
// it; only a farther child whose box was hit is pushed (short stack in LDS, shared with meshes).
// n.a = root ref, n.f[0..5] = the root bvh_node's box.
template <uint32_t F>
MRT_DFN bool bvhw_hit(const DScene& S, const mrt_node& n, const Ray& r, float tmin, float tmax, HitRec& rec, bool full,
                                         const LStack& L) {
    if (!aabb_hit(n.f, n.f + 3, r, tmin, tmax)) return false;
#if MRT_BVHW_SENT
    // the stack's bottom holds kBvhwEmpty, popped when the walk is over: a lane leaves the inner
    // loop by its leaf test alone, with no `return` inside it (the host sizes the stack with the
    // slot to spare: the deepest leaf's inner ancestors are bvhw_depth - 1)
    uint32_t ref = n.a, sp = 1;
    L.mesh[L.lane] = kBvhwEmpty;
#else
    uint32_t ref = n.a, sp = 0;
#endif
    const bool bad = any_lane(!r.nice);  // (once per walk: aabb_hit_b)
    // (Leaf postponing by majority -- a lane parks its first leaf and walks on, as the path-exact
    // mesh walk does -- measured and removed: scene 2 +7.3%, random spheres +0.5% / -2.1% exact,
    // scenes 1 / 3 / 4 -3.2% / -1% / -1%, book2 -5.7%, profiles/r06_ab.txt section 17.)
    // "while-while" (Aila & Laine 2009): each lane descends through inner nodes until it holds a
    // leaf, and the leaves are tested together, instead of one inner-or-leaf step per iteration
    // with the two branches serialised whenever lanes disagree (book2, C5: +14%).  Each lane
    // visits the same nodes in the same order as the reference's recursion: results unchanged.
    for (;;) {
        while (!(ref & BVHW_LEAF)) {
            const WideNode W = wide_at<TreeOf<F>::on>(S.bwide, ref, L);
            // (both boxes tested on every lane, `|` rather than `||`: a box-less slot's test is
            // ignored, and the walk keeps no branch around each test)
            const bool hl = !(W.flags & 1u) | aabb_hit_b(W.lmin, W.lmax, r, tmin, tmax, bad);
            const bool hr = !(W.flags & 2u) | aabb_hit_b(W.rmin, W.rmax, r, tmin, tmax, bad);
            const bool left_first = (W.order & r.mask) != 0;
            const uint32_t cref = left_first ? W.lref : W.rref, fref = left_first ? W.rref : W.lref;
            const bool hc = sel_b(left_first, hl, hr), hf = sel_b(left_first, hr, hl);
#if MRT_BVHW_PUSH_ALWAYS
            // (A/B hook: the far child stored by every lane above its stack's top, kept by the
            // pointer's increment alone -- an inner node's lane has sp <= its depth < the stack's size)
            L.mesh[sp * 64 + L.lane] = fref;
            sp += (hc && hf && fref != cref) ? 1u : 0u;
#else
            if (hc && hf && fref != cref) L.mesh[(sp++) * 64 + L.lane] = fref;  // n == 1: left == right, a repeat misses again
#endif
            ref = hc ? cref : fref;
#if MRT_BVHW_SENT
            if (!hc && !hf) ref = L.mesh[(--sp) * 64 + L.lane];
#else
            if (!hc && !hf) {
                if (sp == 0) return false;
                ref = L.mesh[(--sp) * 64 + L.lane];
            }
#endif
        }
#if MRT_BVHW_SENT
        if (ref == kBvhwEmpty) return false;
        if (bvhw_leaf<F>(S, ref, r, tmin, tmax, rec, full)) return true;
#else
        if (bvhw_leaf<F>(S, ref, r, tmin, tmax, rec, full)) return true;
        if (sp == 0) return false;
#endif
        ref = L.mesh[(--sp) * 64 + L.lane];
    }
}

template <uint32_t F>
MRT_DFN bool bvhw_walk(const DScene& S, const mrt_node& n, const Ray& r, float tmin, float tmax, HitRec& rec, bool full,
                                          const LStack& L) {
    return bvhw_hit<F>(S, n, r, tmin, tmax, rec, full, L);
}

template <uint32_t F>
MRT_DFN bool prim_hit(const DScene& S, const mrt_node& n, uint32_t kind, const Ray& r, float tmin, float tmax, HitRec& rec,
                                         bool full, const LStack& L) {
    switch (kind) {
    case MRT_K_SPHERE: return sphere_hit<F>(n, r, tmin, tmax, rec, full);
    case MRT_K_XY: return rect_hit<F, 2>(n, r, tmin, tmax, rec, full);
    case MRT_K_XZ: return rect_hit<F, 1>(n, r, tmin, tmax, rec, full);
    case MRT_K_YZ: return rect_hit<F, 0>(n, r, tmin, tmax, rec, full);
    default:
        if constexpr ((F & FT_BVHW) != 0)
            if (kind == MRT_K_BVHW) return bvhw_walk<F>(S, n, r, tmin, tmax, rec, full, L);
        if constexpr ((F & FT_MESH) != 0) return mesh_hit(S, n, r, tmin, tmax, rec, full, L);
        return false;
    }
}

MRT_DFN void push_ray(const LStack& L, uint32_t slot, const Ray& r) {
    float* b = L.rays + slot * 11 * 64 + L.lane;
    b[0] = r.o.x; b[64] = r.o.y; b[128] = r.o.z;
    b[192] = r.d.x; b[256] = r.d.y; b[320] = r.d.z;
    b[384] = r.inv.x; b[448] = r.inv.y; b[512] = r.inv.z;
    b[576] = __int_as_float(r.inside);
    b[640] = __uint_as_float(r.mask | ((uint32_t)r.nice << 31));
}
MRT_DFN void pop_ray(const LStack& L, uint32_t slot, Ray& r) {
    const float* b = L.rays + slot * 11 * 64 + L.lane;
    r.o = f3{b[0], b[64], b[128]};
    r.d = f3{b[192], b[256], b[320]};
    r.inv = f3{b[384], b[448], b[512]};
    r.inside = __float_as_int(b[576]);
    const uint32_t m = __float_as_uint(b[640]);
    r.mask = m & 0xFFu;
    r.nice = (m >> 31) != 0;
}

// rotate_y::hit ray transform (scene_object.cpp:75-82)
template <bool U = MRT_FAST_UNIT>
MRT_DFN Ray rotate_ray(const Ray& ray, float s, float c) {
    f3 o = ray.o, d = ray.d;
    o.x = ref_fms(c, ray.o.x, s * ray.o.z);  // scene_object.cpp:77-80
    o.z = ref_fma(c, ray.o.z, s * ray.o.x);
    d.x = ref_fms(c, ray.d.x, s * ray.d.z);
    d.z = ref_fma(c, ray.d.z, s * ray.d.x);
    return make_ray_unit<U>(o, d, ray.time, 0);
}
// ... and the record back (scene_object.cpp:85-93)
MRT_DFN void unrotate_rec(HitRec& rec, float s, float c) {
    f3 p = rec.p, nn = rec.n;
    p.x = ref_fma(c, rec.p.x, s * rec.p.z);  // scene_object.cpp:87-91
    p.z = ref_fms(c, rec.p.z, s * rec.p.x);
    nn.x = ref_fma(c, rec.n.x, s * rec.n.z);
    nn.z = ref_fms(c, rec.n.z, s * rec.n.x);
    rec.p = p;
    rec.n = nn;
}

// ------------------------------------------------------------------------------------------
// scene_object::hit as an explicit-stack machine.  One running `closest` per query replaces the
// per-call tmax: every hit narrows it and every consumer passes it on (object_list children get
// the list's closest, bvh_node children its tmax, which is unchanged until a hit ends the node).
// constant_volume runs its two boundary queries as a nested context whose hits only record t;
// volumes never nest (checked on upload).  The top frame lives in registers; frames below it and
// saved instance rays live in LDS.  Primitives have exactly one evaluation site.
// ------------------------------------------------------------------------------------------
enum : uint32_t { ST_ENTER = 0xFFFFFFFFu, ST_PH1 = 0x40000000u, ST_PH2 = 0x40000001u };

template <uint32_t F>
MRT_DFN bool scene_hit(const DScene& S, Ray ray, float tmin0, HitRec& rec, Pcg& rng, const LStack& L) {
    uint32_t depth = 0, rsp = 0;
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
            if (is_prim<F>(ck)) {
                HitRec* R = ((F & FT_VOLUME) && insub) ? &subrec : &rec;
                ret = prim_hit<F>(S, C, ck, ray, tmin, closest, *R, !((F & FT_VOLUME) && insub), L);
                if (ret) closest = R->t;
                req = MRT_NONE;
                if (depth == 0) break;
            } else {
                if (depth > 0) {
                    L.frames[(depth - 1) * 128 + L.lane] = tnode;
                    L.frames[(depth - 1) * 128 + 64 + L.lane] = tstate;
                }
                tnode = req;
                tstate = ST_ENTER;
                depth++;
                req = MRT_NONE;
            }
        }
        const mrt_node& N = S.nodes[tnode];
        const uint32_t kind = MRT_NODE_KIND(N);
        const uint32_t st = tstate;
        bool pop = false;
        if (kind == MRT_K_LIST) {  // object_list::hit (scene_object.h:79-103)
            uint32_t cursor, flag;
            if (st == ST_ENTER) {
                if ((MRT_NODE_FLAGS(N) & MRT_F_HASBOX) && !aabb_hit(N.f, N.f + 3, ray, tmin, closest)) {
                    ret = false;
                    pop = true;
                }
                cursor = 0;
                flag = 0;
            } else {
                cursor = st & 0x3FFFFFFFu;
                flag = (st >> 31) | (ret ? 1u : 0u);
            }
            if (!pop) {
                if (cursor < N.b) {
                    req = S.children[N.a + cursor];
                    tstate = (cursor + 1) | (flag << 31);
                } else {
                    ret = flag != 0;
                    pop = true;
                }
            }
        } else if ((F & FT_INST) && kind == MRT_K_TRROTY) {  // translate(rotate_y(x)) fused
            const float s = N.f[6], c = N.f[7];
            if (st == ST_ENTER) {
                Ray moved = moved_ray<kFastUnit<F>>(ray, sub(ray.o, ld3(N.f + 8)));  // translate::hit
                if ((MRT_NODE_FLAGS(N) & MRT_F_HASBOX) && !aabb_hit(N.f, N.f + 3, moved, tmin, closest)) {
                    ret = false;
                    pop = true;
                } else {
                    push_ray(L, rsp++, ray);
                    ray = rotate_ray<kFastUnit<F>>(moved, s, c);
                    req = N.a;
                    tstate = ST_PH1;
                }
            } else {
                pop_ray(L, --rsp, ray);
                if (ret && !insub) {
                    unrotate_rec(rec, s, c);
                    rec.p = add(rec.p, ld3(N.f + 8));
                }
                pop = true;
            }
        } else if ((F & FT_INST) && (kind == MRT_K_TRANSLATE || kind == MRT_K_ROTY)) {  // scene_object.cpp:9-18, 70-98
            const bool roty = kind == MRT_K_ROTY;
            if (st == ST_ENTER) {
                if (roty && (MRT_NODE_FLAGS(N) & MRT_F_HASBOX) && !aabb_hit(N.f, N.f + 3, ray, tmin, closest)) {
                    ret = false;
                    pop = true;
                } else {
                    push_ray(L, rsp++, ray);
                    ray = roty ? rotate_ray<kFastUnit<F>>(ray, N.f[6], N.f[7]) : moved_ray<kFastUnit<F>>(ray, sub(ray.o, ld3(N.f)));
                    req = N.a;
                    tstate = ST_PH1;
                }
            } else {
                pop_ray(L, --rsp, ray);
                if (ret && !insub) {
                    if (!roty) rec.p = add(rec.p, ld3(N.f));
                    else unrotate_rec(rec, N.f[6], N.f[7]);
                }
                pop = true;
            }
        } else if ((F & FT_BVH) && kind == MRT_K_BVH) {  // bvh_node::hit (scene_object.h:208-244)
            const bool left_first = (MRT_NODE_ORDER(N) & ray.mask) != 0;
            if (st == ST_ENTER) {
                if (!aabb_hit(N.f, N.f + 3, ray, tmin, closest)) {
                    ret = false;
                    pop = true;
                } else {
                    req = left_first ? N.a : N.b;
                    tstate = ST_PH1;
                }
            } else if (st == ST_PH1 && !ret) {
                req = left_first ? N.b : N.a;
                tstate = ST_PH2;
            } else {
                pop = true;  // closer hit (ret true) or farther done
            }
        } else if ((F & FT_VOLUME) && kind == MRT_K_VOLUME) {  // constant_volume::hit (volumes.cpp:5-35)
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
                if (ret) {
                    float t1 = vt1, t2 = subrec.t;
                    if (t1 < tmin) t1 = tmin;
                    if (t2 > closest) t2 = closest;
                    if (t1 >= t2) {
                        ret = false;
                    } else {
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
                }
            }
        } else {
            ret = false;
            pop = true;
        }
        if (pop) {
            depth--;
            if (depth == 0) break;
            tnode = L.frames[(depth - 1) * 128 + L.lane];
            tstate = L.frames[(depth - 1) * 128 + 64 + L.lane];
        }
    }
    return ret;
}

}  // namespace mrtd
