// mrt_lin.h -- scene_object::hit for scene graphs WITHOUT per-ray traversal order (object_list
// trees, instances, primitives, meshes; no bvh_node and no constant_volume) compiled on upload
// into a linear program that every lane of a wave walks in lockstep.
//
// In such graphs the reference visits children in a fixed order (object_list::hit,
// scene_object.h:79-103); only which subtrees a ray enters differs per lane (list / rotate_y boxes).
// The program is that visit order, flattened: the op index is wave-uniform, so op and node data
// come through scalar loads and every branch on the op is a scalar branch; a lane that failed a
// box is masked until the matching END op (its bit in `act` is clear), and the whole wave jumps
// over a subtree no lane entered.  Hits record only (t, node); p/n/uv are derived once from the
// winning primitive in its own instance frame -- the same operations on the same inputs as the
// primitive's hit() (rect.cpp:24-45, sphere.cpp:13-46), so the record is bit-identical.
#pragma once
#include "mrt_trace.h"

namespace mrtd {

enum : uint32_t {
    LOP_END = 0,
    LOP_PRIM = 1,      // sphere / rect
    LOP_MESH = 2,      // pod_bvh<triangle> (per-lane traversal, mesh_hit)
    LOP_LIST = 3,      // object_list enter (box test), skip = index of its LOP_LIST_END
    LOP_LIST_END = 4,
    LOP_INST = 5,      // translate / rotate_y / fused translate(rotate_y) enter, skip = its LOP_INST_END
    LOP_INST_END = 6,
    LOP_BVHW = 7,      // bvh_node subtree as wide nodes (per-lane traversal, bvhw_hit)
    LOP_VOLUME = 8,    // constant_volume; the next op (LOP_VBOUND) is its primitive boundary
    LOP_VBOUND = 9,
    // tolerance-contract program only (lin_rewrite_fast, mrt_sig.h): the inward-facing rects of one
    // object_list that bound a box (a room's walls) as one slab test; the next op (LOP_ROOMDATA)
    // holds each face's node
    LOP_ROOM = 10,
    LOP_ROOMDATA = 11,
};

// one op = the node's own record (no second load): code = op | kind << 8 | flags << 16 | level << 24
// (the nesting level the op is tested at).  Host-filled extras: prim / mesh / bvh / volume ops
// carry the enclosing instance's op index in f[11] (MRT_NONE outside instances), a BVHW op its
// subtree's root ref in skip, an INST_END op its instance op's index in skip.
struct LinOp {
    uint32_t code, node, skip, mat;
    float f[12];
};
static_assert(sizeof(LinOp) == 64, "LinOp is one 64 B scalar load");

#define LOP_OP(o) ((o).code & 0xFFu)
#define LOP_KIND(o) (((o).code >> 8) & 0xFFu)
#define LOP_FLAGS(o) (((o).code >> 16) & 0xFFu)

MRT_DFN uint32_t op_flags(const LinOp& o) { return LOP_FLAGS(o); }
#if defined(__HIP_DEVICE_COMPILE__)
MRT_DFN uint32_t op_flags(const MRT_CONST_AS LinOp& o) { return LOP_FLAGS(o); }
#endif
MRT_DFN uint32_t op_flags(const mrt_node& n) { return MRT_NODE_FLAGS(n); }

// t of the primitive's hit() or a miss; no record written.  KIND is wave-uniform at the call.
// Branch-free: every lane evaluates the whole test and the outcome is a predicate (the early
// returns of the reference only skip work whose result is unused, so the outcome is the same).
template <uint32_t F, uint32_t KIND, typename OP>
MRT_DFN bool lin_prim_t(const OP& o, const Ray& r, float tmin, float tmax, float* tout) {
    if constexpr (KIND == MRT_K_SPHERE) {  // sphere::hit (sphere.cpp:13-46)
        f3 cen = f3{o.f[0], o.f[1], o.f[2]};
        if ((F & FT_MOVING) && (LOP_FLAGS(o) & MRT_F_MOVING))
            cen = add(cen, fmul((r.time - o.f[6]) / (o.f[7] - o.f[6]), sub(f3{o.f[3], o.f[4], o.f[5]}, cen)));
        const float radius = o.f[8];
        const f3 oc = sub(r.o, cen);
        float b;
        const float disc = sphere_disc(oc, r.d, radius, &b);
        const float sq = sqrt_(disc);
        const float t1 = (-b - sq), t2 = (-b + sq);
        const bool ok1 = (t1 < tmax) & (t1 > tmin);
        const bool ok2 = (r.inside != 0) & (t2 < tmax) & (t2 > tmin);
        *tout = ok1 ? t1 : t2;
        return (disc > 0) & (ok1 | ok2);
    } else {
        // xy/xz/yz_rect::hit (rect.cpp:24-45, 69-90, 130-151)
        constexpr int AX = KIND == MRT_K_XY ? 2 : KIND == MRT_K_XZ ? 1 : 0;
        const float ns = o.f[5];
        const float oa = AX == 2 ? r.o.z : AX == 1 ? r.o.y : r.o.x;
        const float da = AX == 2 ? r.d.z : AX == 1 ? r.d.y : r.d.x;
        const float ia = AX == 2 ? r.inv.z : AX == 1 ? r.inv.y : r.inv.x;
        const float num = o.f[4] - oa;
        // nice ray (make_ray): (k - o_a) / d_a through div_core, and the one-sided test
        // dot(dir, n) > 0 reduces to d_a * ns > 0 (the other products are zeros of finite values)
        float t = div_core(num, da, ia);
        bool back = da * ns > 0.0f;
        const bool slow = !MRT_FAST_GUARDS && (op_flags(o) & MRT_F_SLOWDIV) != 0;  // uniform
        if (__builtin_expect(slow || any_lane(!r.nice), 0)) {  // the reference's forms
            const float dn = AX == 2 ? (r.d.x * 0.0f + r.d.y * 0.0f) + r.d.z * ns
                           : AX == 1 ? (r.d.x * 0.0f + r.d.y * ns) + r.d.z * 0.0f
                                     : (r.d.x * ns + r.d.y * 0.0f) + r.d.z * 0.0f;
            const bool ex = slow || !r.nice;
            t = ex ? num / da : t;
            back = ex ? dn > 0.0f : back;
        }
        const float ob = AX == 0 ? r.o.y : r.o.x, db = AX == 0 ? r.d.y : r.d.x;
        const float oc = AX == 2 ? r.o.y : r.o.z, dc = AX == 2 ? r.d.y : r.d.z;
        const float pb = ref_fma(t, db, ob);  // rect.cpp:32-33, 77-78, 138-139 (fused as shipped)
        const float pc = ref_fma(t, dc, oc);
        *tout = t;
        return !back & !((t < tmin) | (t > tmax)) & !((pb < o.f[0]) | (pb > o.f[1]) | (pc < o.f[2]) | (pc > o.f[3]));
    }
}

// lin_prim_rec for a primitive op whose kind is known at compile time, its data read through the
// constant address space (wave-uniform op: scalar loads).  Same arithmetic as lin_prim_rec.
template <uint32_t F, uint32_t KIND>
MRT_DFN void lin_prim_rec_op(const MRT_CONST_AS LinOp& o, const Ray& r, float t, HitRec& rec) {
    const uint32_t fl = LOP_FLAGS(o);
    const bool needuv = (F & FT_UV) && (fl & MRT_F_NEEDUV);
    rec.t = t;
    rec.mat = o.mat;
    rec.p = eval(r, t);
    if constexpr (KIND == MRT_K_SPHERE) {
        f3 cen = f3{o.f[0], o.f[1], o.f[2]};
        if ((F & FT_MOVING) && (fl & MRT_F_MOVING))
            cen = add(cen, fmul((r.time - o.f[6]) / (o.f[7] - o.f[6]), sub(f3{o.f[3], o.f[4], o.f[5]}, cen)));
        rec.n = divf(sub(rec.p, cen), o.f[8]);
        if (needuv) sphere_uv(rec.n, &rec.u, &rec.v);
    } else {
        const float ns = o.f[5];
        float pb = 0, pc = 0;
        if constexpr (KIND == MRT_K_XY) {
            rec.n = f3{0, 0, ns};
            if (MRT_FAST_SNAP) rec.p.z = o.f[4];
            if (needuv) { pb = ref_fma(t, r.d.x, r.o.x); pc = ref_fma(t, r.d.y, r.o.y); }
        } else if constexpr (KIND == MRT_K_XZ) {
            rec.n = f3{0, ns, 0};
            if (MRT_FAST_SNAP) rec.p.y = o.f[4];
            if (needuv) { pb = ref_fma(t, r.d.x, r.o.x); pc = ref_fma(t, r.d.z, r.o.z); }
        } else {
            rec.n = f3{ns, 0, 0};
            if (MRT_FAST_SNAP) rec.p.x = o.f[4];
            if (needuv) { pb = ref_fma(t, r.d.y, r.o.y); pc = ref_fma(t, r.d.z, r.o.z); }
        }
        if (needuv) {
            rec.u = (pb - o.f[0]) / (o.f[1] - o.f[0]);
            rec.v = (pc - o.f[2]) / (o.f[3] - o.f[2]);
        }
    }
}

// the record the primitive's hit() writes for a hit at t.  The node is per lane; its 64 B are
// fetched whole (four 16-byte loads in flight together) rather than field by field, which the
// compiler turned into two dependent round trips (kind/mat, then the kind's fields).
template <uint32_t F>
MRT_DFN void lin_prim_rec(const DScene& S, uint32_t node, const Ray& r, float t, HitRec& rec) {
#ifndef MRT_REC_FIELDWISE
    const float4* q = reinterpret_cast<const float4*>(S.nodes + node);
    const float4 q0 = q[0], q1 = q[1], q2 = q[2], q3 = q[3];
    const uint32_t code = __float_as_uint(q0.x), nmat = __float_as_uint(q0.w);
    const float nf[12] = {q1.x, q1.y, q1.z, q1.w, q2.x, q2.y, q2.z, q2.w, q3.x, q3.y, q3.z, q3.w};
#else
    const mrt_node* n = S.nodes + node;
    const uint32_t code = n->kind, nmat = n->mat;
    const float* nf = n->f;
#endif
    const uint32_t kind = code & 0xFFu;
    const bool needuv = (F & FT_UV) && ((code >> 16) & MRT_F_NEEDUV);
    rec.t = t;
    rec.mat = nmat;
    rec.p = eval(r, t);
    if (kind == MRT_K_SPHERE) {
        f3 cen = f3{nf[0], nf[1], nf[2]};
        if ((F & FT_MOVING) && ((code >> 16) & MRT_F_MOVING))
            cen = add(cen, fmul((r.time - nf[6]) / (nf[7] - nf[6]), sub(f3{nf[3], nf[4], nf[5]}, cen)));
        rec.n = divf(sub(rec.p, cen), nf[8]);
        if (needuv) sphere_uv(rec.n, &rec.u, &rec.v);
        return;
    }
    const float ns = nf[5];
    // the rect's in-plane hit coordinates (rect.cpp:32-33: o + t * d on its two axes, one fused
    // scalar expression each as shipped), chosen by selects (a kind-indexed choice had become a
    // per-lane lookup table in scratch memory)
    const f3 p0 = rec.p;
    const bool xy = kind == MRT_K_XY, xz = kind == MRT_K_XZ;
    const float pb = kind == MRT_K_YZ ? ref_fma(t, r.d.y, r.o.y) : ref_fma(t, r.d.x, r.o.x);
    const float pc = xy ? ref_fma(t, r.d.y, r.o.y) : ref_fma(t, r.d.z, r.o.z);
    rec.n = f3{xy || xz ? 0.0f : ns, xz ? ns : 0.0f, xy ? ns : 0.0f};
    if (MRT_FAST_SNAP) {
        rec.p.x = xy || xz ? p0.x : nf[4];
        rec.p.y = xz ? nf[4] : p0.y;
        rec.p.z = xy ? nf[4] : p0.z;
    }
    if (needuv) {
        rec.u = (pb - nf[0]) / (nf[1] - nf[0]);
        rec.v = (pc - nf[2]) / (nf[3] - nf[2]);
    }
}

// the query ray parked in LDS while an instance ray occupies the registers ([word][lane])
MRT_DFN void lin_save_ray(const LStack& L, const Ray& r) {
    float* b = L.save + L.lane;
    b[0] = r.o.x; b[64] = r.o.y; b[128] = r.o.z;
    b[192] = r.d.x; b[256] = r.d.y; b[320] = r.d.z;
    b[384] = r.time;
    b[448] = __int_as_float(r.inside);
    b[512] = __uint_as_float(r.mask);
}
MRT_DFN Ray lin_load_ray(const LStack& L) {
    const float* b = L.save + L.lane;
    Ray r;
    r.o = f3{b[0], b[64], b[128]};
    r.d = f3{b[192], b[256], b[320]};
    r.time = b[384];
    r.inside = __float_as_int(b[448]);
    r.mask = __float_as_uint(b[512]);
    r.nice = ray_nice(r.o, r.d);  // recomputed where used (cheaper than parking them in LDS)
    r.inv = ray_inv(r.d, r.nice);
    return r;
}
// An op's 64 B as one batch of scalar loads with a single wait: the asm makes every word live at
// one point, so the loads cannot be sunk to their uses (the compiler otherwise split each op into
// three load + s_waitcnt round trips to the scalar cache).
template <uint32_t F, uint32_t KIND>
MRT_DFN LinOp lin_fetch_op(const MRT_CONST_AS LinOp& o) {
    const MRT_CONST_AS uint32_t* q = reinterpret_cast<const MRT_CONST_AS uint32_t*>(&o);
    LinOp r;
    r.code = q[0];
    r.node = q[1];
    r.skip = 0;
    r.mat = 0;
    if constexpr (KIND == MRT_K_SPHERE) {  // centre, radius (+ the moving centre's fields)
        uint32_t c0 = q[4], c1 = q[5], c2 = q[6], rad = q[12];
#if defined(__HIP_DEVICE_COMPILE__)
        asm volatile("" : "+s"(r.code), "+s"(r.node), "+s"(c0), "+s"(c1), "+s"(c2), "+s"(rad));
#endif
        r.f[0] = __uint_as_float(c0); r.f[1] = __uint_as_float(c1); r.f[2] = __uint_as_float(c2); r.f[8] = __uint_as_float(rad);
        if (F & FT_MOVING)
            for (int k = 3; k < 8; k++) r.f[k] = o.f[k];
    } else {  // rect: bounds, plane, normal sign
        uint32_t b0 = q[4], b1 = q[5], b2 = q[6], b3 = q[7], k = q[8], ns = q[9];
#if defined(__HIP_DEVICE_COMPILE__)
        asm volatile("" : "+s"(r.code), "+s"(r.node), "+s"(b0), "+s"(b1), "+s"(b2), "+s"(b3), "+s"(k), "+s"(ns));
#endif
        r.f[0] = __uint_as_float(b0); r.f[1] = __uint_as_float(b1); r.f[2] = __uint_as_float(b2); r.f[3] = __uint_as_float(b3);
        r.f[4] = __uint_as_float(k); r.f[5] = __uint_as_float(ns);
    }
    return r;
}
// The whole 64-B op as ONE batch of scalar loads and one wait (the compact interpreter kernels):
// the op's fields are then read from SGPRs; read in place, an op cost the loop several load + wait
// round trips to the scalar cache (the instance op's box, its rotation, its list's planes ...).
MRT_DFN LinOp lin_fetch_all(const MRT_CONST_AS LinOp& o) {
    const MRT_CONST_AS uint32_t* q = reinterpret_cast<const MRT_CONST_AS uint32_t*>(&o);
    uint32_t w[16];
#pragma unroll
    for (int k = 0; k < 16; k++) w[k] = q[k];
#if defined(__HIP_DEVICE_COMPILE__)
    asm volatile("" : "+s"(w[0]), "+s"(w[1]), "+s"(w[2]), "+s"(w[3]), "+s"(w[4]), "+s"(w[5]), "+s"(w[6]), "+s"(w[7]), "+s"(w[8]),
                 "+s"(w[9]), "+s"(w[10]), "+s"(w[11]), "+s"(w[12]), "+s"(w[13]), "+s"(w[14]), "+s"(w[15]));
#endif
    LinOp r;
    r.code = w[0];
    r.node = w[1];
    r.skip = w[2];
    r.mat = w[3];
#pragma unroll
    for (int k = 0; k < 12; k++) r.f[k] = __uint_as_float(w[4 + k]);
    return r;
}
// (measured slower: C2 through the interpreter 49.5 vs 50.6 Grays/s with the ops read in place,
// three interleaved rounds, profiles/r05_ab.txt section 7; kept as an A/B switch)
#ifndef MRT_LIN_FETCH_ALL
#define MRT_LIN_FETCH_ALL 0
#endif

// LOP_ROOM (tolerance contract): the room's walls -- one-sided rects facing into the box
// [f[0..2], f[3..5]], face k = axis * 2 + side present when bit k of o.node is set -- as one slab
// test: a ray that meets the box leaves it through the face of its smallest far-plane distance,
// and that face, if the room has it, is the wall hit (a face crossed going in is back-facing and
// missed, rect.cpp:26-30).  *face = the exit face.
template <typename OP>
MRT_DFN bool lin_room_hit(const OP& o, const Ray& r, float tmin, float tmax, float* t, uint32_t* face) {
    const float t0x = (o.f[0] - r.o.x) * r.inv.x, t1x = (o.f[3] - r.o.x) * r.inv.x;
    const float t0y = (o.f[1] - r.o.y) * r.inv.y, t1y = (o.f[4] - r.o.y) * r.inv.y;
    const float t0z = (o.f[2] - r.o.z) * r.inv.z, t1z = (o.f[5] - r.o.z) * r.inv.z;
    const float fx = fmaxf(t0x, t1x), fy = fmaxf(t0y, t1y), fz = fmaxf(t0z, t1z);
    const float tn = fmaxf(fmaxf(fminf(t0x, t1x), fminf(t0y, t1y)), fminf(t0z, t1z));
    const float tf = fminf(fminf(fx, fy), fz);
    const uint32_t a = tf == fz ? 2u : (tf == fy ? 1u : 0u);  // ties to the later axis
    const float da = sel3(a, r.d.x, r.d.y, r.d.z);
    const uint32_t k = a * 2u + (da > 0.0f ? 1u : 0u);
    *t = tf;
    *face = k;
    return (tn <= tf) & (((o.node >> k) & 1u) != 0u) & (tf >= tmin) & (tf <= tmax);
}
// an object_list flagged MRT_F_BOX6 (box.h:12-20, planes in f[6..11]) as one slab test
// (tolerance contract, box6_leaf_hit); *child = the entry face's position among its six rects
// (box.h order: xy at max z, xy at min z, xz at max y, xz at min y, yz at max x, yz at min x)
template <typename OP>
MRT_DFN bool lin_box6_hit(const OP& o, const Ray& r, float tmin, float tmax, float* t, uint32_t* child) {
    const float t0x = (o.f[6] - r.o.x) * r.inv.x, t1x = (o.f[9] - r.o.x) * r.inv.x;
    const float t0y = (o.f[7] - r.o.y) * r.inv.y, t1y = (o.f[10] - r.o.y) * r.inv.y;
    const float t0z = (o.f[8] - r.o.z) * r.inv.z, t1z = (o.f[11] - r.o.z) * r.inv.z;
    const float nx = fminf(t0x, t1x), ny = fminf(t0y, t1y), nz = fminf(t0z, t1z);
    const float tn = fmaxf(fmaxf(nx, ny), nz);
    const float tf = fminf(fminf(fmaxf(t0x, t1x), fmaxf(t0y, t1y)), fmaxf(t0z, t1z));
    const uint32_t c = tn == nx ? (r.d.x > 0.0f ? 5u : 4u) : tn == ny ? (r.d.y > 0.0f ? 3u : 2u) : (r.d.z > 0.0f ? 1u : 0u);
    *t = tn;
    *child = c;
    return (tn <= tf) & (tn >= tmin) & (tn <= tmax);
}

// aabb::hit (invDir = 1/dir of the ray, aabb.h:49)
template <typename OP>
MRT_DFN bool lin_box(const OP& o, const Ray& r, float tmin, float tmax) {
    const float b[6] = {o.f[0], o.f[1], o.f[2], o.f[3], o.f[4], o.f[5]};
    return aabb_hit(b, b + 3, r, tmin, tmax);
}

// The instance-frame ray of instance op `io` for the query ray r -- the walk's own operations at
// LOP_INST and at the one-step box instance (translate::hit / rotate_y::hit, scene_object.cpp:9-18,
// 70-98) -- recomputed after the walk for the record of a hit inside the instance, instead of
// parking the 6 words of the instance ray in LDS at the hit (round 6: the LDS freed holds more
// treelet nodes).  Only its origin and direction are read; from the same query ray and op they are
// the walk's bits.
template <bool U, typename OP>
MRT_DFN Ray inst_ray(const OP& io, const Ray& r) {
    const uint32_t kind = LOP_KIND(io);
    if (kind == MRT_K_TRROTY) return rotate_ray<U>(moved_ray<U>(r, sub(r.o, f3{io.f[8], io.f[9], io.f[10]})), io.f[6], io.f[7]);
    if (kind == MRT_K_ROTY) return rotate_ray<U>(r, io.f[6], io.f[7]);
    return moved_ray<U>(r, sub(r.o, f3{io.f[0], io.f[1], io.f[2]}));
}

// record frames of instance hits, back to the world (scene_object.cpp:13-16, 85-93)
template <typename OP>
MRT_DFN void lin_untransform(const OP& io, HitRec& rec) {
    const uint32_t kind = LOP_KIND(io);
    if (kind == MRT_K_TRROTY) {
        unrotate_rec(rec, io.f[6], io.f[7]);
        rec.p = add(rec.p, f3{io.f[8], io.f[9], io.f[10]});
    } else if (kind == MRT_K_ROTY) {
        unrotate_rec(rec, io.f[6], io.f[7]);
    } else {
        rec.p = add(rec.p, f3{io.f[0], io.f[1], io.f[2]});
    }
}

// r: the query ray; on return it holds the same values (reloaded from LDS when instances exist).
// LDS per lane (L.save): [0..8] the query ray (the instance ray of the closest hit is recomputed
// after the walk, inst_ray).
// The interpreter's slab-test ops (LOP_ROOM of the tolerance contract's program rewrite, an
// object_list flagged MRT_F_BOX6) are compiled into the kernels of scenes without bvh_node
// subtrees, volumes, textures or motion only: in the catch-all interpreter kernel their two cases
// tripled book2's register spills (C5 2.7x slower, profiles/r04_ab.txt).  The other kernels run
// the program as compiled (the host uploads the rewrite only where KernelTable::rewrite says so).
#ifndef MRT_BOXINST
#define MRT_BOXINST 1  // the one-step box instance (MRT_F_BOXINST)
#endif
#ifndef MRT_LIN_LAST
#define MRT_LIN_LAST 1  // the walk ends at the op flagged MRT_F_LAST (0: at the END op)
#endif
#ifndef MRT_BOXINST_AABB
#define MRT_BOXINST_AABB 0  // 1: the one-step box instance tests its instance's box first (measured 2.7% slower, A/B hook)
#endif
#ifndef MRT_LIN_PREFETCH_INST
#define MRT_LIN_PREFETCH_INST 1
#endif
template <uint32_t F>
static constexpr bool kLinSlabOps = MRT_FAST && (F & FT_LIN) != 0 && (F & (FT_BVHW | FT_VOLUME | FT_TEX | FT_MOVING)) == 0;
// Round 6: the records of bvh_node leaf hits and constant_volume hits made after the walk, like a
// primitive op's, from what the walk keeps of the hit (the leaf primitive and the range it passed
// with; the volume op), instead of inside it: the 10-word record is then not live across the rest
// of the walk (book2's bvh_node walks ran with the ground's record held while the spheres' tree was
// walked).  The same tests with the same rays and ranges: the same bits.
#ifndef MRT_LIN_DEFER
#define MRT_LIN_DEFER 1
#endif
enum : uint32_t { HK_PRIM = 0, HK_DONE = 1, HK_VOL = 2, HK_BVHW = 3 };  // how the record is made after the walk

// t of the closest hit in [tmin, tmax] of a volume's boundary sub-program [b, e) (MRT_F_VSUB: box.h
// lists and one level of instances, emitted after the volume op) for the volume-frame ray r0 --
// object_list::hit / translate::hit / rotate_y::hit as the main walk runs them (scene_object.h:79-103,
// scene_object.cpp:9-18, 70-98), the running closest narrowing, with its own nesting mask.  Only t is
// kept: constant_volume::hit reads rec1.t / rec2.t alone (volumes.cpp:10-21).
template <uint32_t F, typename PROG>
MRT_DFN bool lin_sub_t(PROG prog, uint32_t b, uint32_t e, const Ray& r0, float tmin, float tmax, float* tout) {
    Ray cur = r0;
    float closest = tmax;
    bool hit = false;
    uint32_t act = 1u, lvl = 0;  // (lvl wave-uniform)
    for (uint32_t pc = b; pc < e; pc++) {
        const auto& o = prog[pc];
        const uint32_t op = LOP_OP(o);
        const bool on = (act >> lvl) & 1u;
        if (op == LOP_PRIM) {
            float t;
            bool h;
            switch (LOP_KIND(o)) {  // uniform: a scalar branch
            case MRT_K_SPHERE: h = lin_prim_t<F, MRT_K_SPHERE>(o, cur, tmin, closest, &t); break;
            case MRT_K_XY: h = lin_prim_t<F, MRT_K_XY>(o, cur, tmin, closest, &t); break;
            case MRT_K_XZ: h = lin_prim_t<F, MRT_K_XZ>(o, cur, tmin, closest, &t); break;
            default: h = lin_prim_t<F, MRT_K_YZ>(o, cur, tmin, closest, &t); break;
            }
            h = h & on;
            closest = h ? t : closest;
            hit = hit | h;
        } else if (op == LOP_LIST) {
            bool in = on;
            if (in && (LOP_FLAGS(o) & MRT_F_HASBOX)) in = lin_box(o, cur, tmin, closest);
            lvl++;
            act = (act & ~(1u << lvl)) | ((uint32_t)in << lvl);
            if (!any_lane(in)) pc = o.skip - 1;
        } else if (op == LOP_LIST_END) {
            lvl--;
        } else if (op == LOP_INST) {  // as scene_hit_lin's LOP_INST, from the volume-frame ray
            const uint32_t kind = LOP_KIND(o);
            bool in = on;
            if (kind == MRT_K_TRROTY) {
                cur = moved_ray<kFastUnit<F>>(r0, sub(r0.o, f3{o.f[8], o.f[9], o.f[10]}));
                if (in && (LOP_FLAGS(o) & MRT_F_HASBOX)) in = lin_box(o, cur, tmin, closest);
            } else if (kind == MRT_K_ROTY) {
                cur = r0;
                if (in && (LOP_FLAGS(o) & MRT_F_HASBOX)) in = lin_box(o, cur, tmin, closest);
            }
            lvl++;
            act = (act & ~(1u << lvl)) | ((uint32_t)in << lvl);
            if (!any_lane(in)) {
                pc = o.skip - 1;  // (its INST_END next)
                continue;
            }
            if (kind == MRT_K_TRROTY || kind == MRT_K_ROTY) cur = rotate_ray<kFastUnit<F>>(cur, o.f[6], o.f[7]);
            else cur = moved_ray<kFastUnit<F>>(r0, sub(r0.o, f3{o.f[0], o.f[1], o.f[2]}));
        } else if (op == LOP_INST_END) {
            cur = r0;
            lvl--;
        }
    }
    *tout = closest;
    return hit;
}

// the record of a primitive op's hit (HK_PRIM: node `h`) or a constant_volume's (HK_VOL: op `h`,
// volumes.cpp:24-31: the point at t, normal (1, 0, 0), the volume's phase-function material) for the
// ray of the hit's frame
template <uint32_t F, typename PROG>
MRT_DFN void lin_hit_rec(const DScene& S, PROG prog, uint32_t hk, uint32_t h, const Ray& r, float t, HitRec& rec) {
    if (MRT_LIN_DEFER && (F & FT_VOLUME) && hk == HK_VOL) {
        rec.t = t;
        rec.p = eval(r, t);
        rec.n = f3{1, 0, 0};
        rec.mat = prog[h].mat;
        return;
    }
    lin_prim_rec<F>(S, h, r, t, rec);
}

template <uint32_t F>
MRT_DFN bool scene_hit_lin(const DScene& S, Ray& r, float tmin, HitRec& rec, const LStack& L, Pcg& rng, PhaseClock& ph) {
    constexpr bool INST = (F & FT_INST) != 0;
    // (parked even when every instance is a one-step box instance, which never displaces it: skipping
    // the park there measured 0.8% slower, C2 through the interpreter, profiles/r05_ab.txt section 10)
    if (INST) lin_save_ray(L, r);
    Ray cur = r;
    float closest = FLT_MAX_;
    uint32_t act = 1u;            // bit l: this lane takes part at nesting level l
    uint32_t lvl = 0;             // wave-uniform
    uint32_t inst = MRT_NONE;     // wave-uniform: op index of the enclosing instance
    uint32_t hnode = MRT_NONE;    // node of the closest hit so far (MRT_NONE: none)
    uint32_t hinst = MRT_NONE;    // op index of the instance it lies in (MRT_NONE: world frame)
    // how the record is made after the walk: HK_PRIM from hnode's primitive; HK_DONE rec holds it
    // (mesh_hit writes it); HK_VOL from volume op hnode; HK_BVHW from bvh leaf primitive hprim < htlim
    uint32_t hk = HK_PRIM;
    uint32_t hprim = 0;
    float htlim = 0.0f;
    const MRT_CONST_AS LinOp* prog = const_ptr(S.prog);
    // one op: `o` is the op in place (constant memory) or its register copy (MRT_LIN_FETCH_ALL);
    // false at the program's end
    constexpr bool kFetch = MRT_LIN_FETCH_ALL && kLinSlabOps<F>;
    uint32_t pc = 0;
    auto op_at = [&](uint32_t k) -> decltype(auto) {
        if constexpr (kFetch) return lin_fetch_all(prog[k]);
        else return (prog[k]);
    };
    auto step = [&](const auto& o) __attribute__((always_inline)) -> bool {
        const uint32_t op = LOP_OP(o);
        if (op == LOP_END) return false;
        const bool on = (act >> lvl) & 1u;
        if (op == LOP_PRIM) {
            float t;
            bool h;
            switch (LOP_KIND(o)) {  // uniform: a scalar branch
            case MRT_K_SPHERE: h = lin_prim_t<F, MRT_K_SPHERE>(o, cur, tmin, closest, &t); break;
            case MRT_K_XY: h = lin_prim_t<F, MRT_K_XY>(o, cur, tmin, closest, &t); break;
            case MRT_K_XZ: h = lin_prim_t<F, MRT_K_XZ>(o, cur, tmin, closest, &t); break;
            default: h = lin_prim_t<F, MRT_K_YZ>(o, cur, tmin, closest, &t); break;
            }
            h = h & on;
            closest = h ? t : closest;
            hnode = h ? o.node : hnode;
            hinst = h ? inst : hinst;
            hk = h ? HK_PRIM : hk;
            PH_MARK(ph, 9);
        } else if (MRT_FAST_ROOM && kLinSlabOps<F> && op == LOP_ROOM) {
            float t;
            uint32_t face;
            const bool h = on & lin_room_hit(o, cur, tmin, closest, &t, &face);
            // LOP_ROOMDATA (the next op): each face's node, read at a per-lane index (selecting it
            // from the op's six uniform words instead measured 3.5% slower, profiles/r05_ab.txt 17)
            const MRT_CONST_AS uint32_t* fnode = reinterpret_cast<const MRT_CONST_AS uint32_t*>(prog[pc + 1].f);
            closest = h ? t : closest;
            hnode = h ? fnode[face] : hnode;
            hinst = h ? inst : hinst;
            hk = h ? HK_PRIM : hk;
            pc++;
        } else if (MRT_BOXINST && kLinSlabOps<F> && INST && op == LOP_INST && (LOP_FLAGS(o) & MRT_F_BOXINST)) {  // uniform
            // an instance of one box.h list, outside instances (cur is the query ray): the instance
            // ray from it in registers, the instance's box test and the list's slab test, the body
            // skipped -- the operations of the INST / LIST / LIST_END / INST_END steps below, without
            // parking and reloading the query ray
            const uint32_t kind = LOP_KIND(o);
            Ray ci = cur;
            bool in = on;
            if (kind == MRT_K_TRROTY) {
                ci = moved_ray<kFastUnit<F>>(cur, sub(cur.o, f3{o.f[8], o.f[9], o.f[10]}));
                if (MRT_BOXINST_AABB && in && (LOP_FLAGS(o) & MRT_F_HASBOX)) in = lin_box(o, ci, tmin, closest);
                ci = rotate_ray<kFastUnit<F>>(ci, o.f[6], o.f[7]);
            } else if (kind == MRT_K_ROTY) {
                if (MRT_BOXINST_AABB && in && (LOP_FLAGS(o) & MRT_F_HASBOX)) in = lin_box(o, ci, tmin, closest);
                ci = rotate_ray<kFastUnit<F>>(ci, o.f[6], o.f[7]);
            } else {
                ci = moved_ray<kFastUnit<F>>(cur, sub(cur.o, f3{o.f[0], o.f[1], o.f[2]}));
            }
            const auto lo = op_at(pc + 1);
            float t;
            uint32_t c;
            const bool h = in & lin_box6_hit(lo, ci, tmin, closest, &t, &c);
            closest = h ? t : closest;
            hnode = h ? prog[pc + 2 + c].node : hnode;
            hinst = h ? pc : hinst;
            hk = h ? HK_PRIM : hk;
            pc = o.skip;  // its LOP_INST_END
        } else if (MRT_FAST_BOX && kLinSlabOps<F> && op == LOP_LIST && (LOP_FLAGS(o) & MRT_F_BOX6)) {  // uniform
            // box.h's six rects as one slab test (its own box test implied), the list skipped
            float t;
            uint32_t c;
            const bool h = on & lin_box6_hit(o, cur, tmin, closest, &t, &c);
            closest = h ? t : closest;
            hnode = h ? prog[pc + 1 + c].node : hnode;
            hinst = h ? inst : hinst;
            hk = h ? HK_PRIM : hk;
            pc = o.skip;  // past its LOP_LIST_END
        } else if ((F & FT_MESH) && op == LOP_MESH) {
            if (on && mesh_hit<true>(S, ld_node(const_ptr(S.nodes) + o.node), cur, tmin, closest, rec, true, L)) {
                closest = rec.t;
                hnode = o.node;
                hinst = inst;
                hk = HK_DONE;
            }
        } else if ((F & FT_VOLUME) && op == LOP_VOLUME) {
            // constant_volume::hit (volumes.cpp:5-35): two boundary queries, then a free-flight
            // distance drawn from the path's RNG (inside hit(), in list order)
            const MRT_CONST_AS LinOp& bo = prog[pc + 1];
            float t1, t2;
            bool h1, h2;
            if ((F & FT_VSUB) && (LOP_FLAGS(o) & MRT_F_VSUB)) {  // uniform: the boundary is the sub-program
                h1 = lin_sub_t<F>(prog, pc + 1, o.skip, cur, -FLT_MAX_, FLT_MAX_, &t1);
                h2 = lin_sub_t<F>(prog, pc + 1, o.skip, cur, t1 + 0.0001f, FLT_MAX_, &t2);
            } else if (LOP_KIND(bo) == MRT_K_SPHERE) {
                h1 = lin_prim_t<F, MRT_K_SPHERE>(bo, cur, -FLT_MAX_, FLT_MAX_, &t1);
                h2 = lin_prim_t<F, MRT_K_SPHERE>(bo, cur, t1 + 0.0001f, FLT_MAX_, &t2);
            } else if (LOP_KIND(bo) == MRT_K_XY) {
                h1 = lin_prim_t<F, MRT_K_XY>(bo, cur, -FLT_MAX_, FLT_MAX_, &t1);
                h2 = lin_prim_t<F, MRT_K_XY>(bo, cur, t1 + 0.0001f, FLT_MAX_, &t2);
            } else if (LOP_KIND(bo) == MRT_K_XZ) {
                h1 = lin_prim_t<F, MRT_K_XZ>(bo, cur, -FLT_MAX_, FLT_MAX_, &t1);
                h2 = lin_prim_t<F, MRT_K_XZ>(bo, cur, t1 + 0.0001f, FLT_MAX_, &t2);
            } else {
                h1 = lin_prim_t<F, MRT_K_YZ>(bo, cur, -FLT_MAX_, FLT_MAX_, &t1);
                h2 = lin_prim_t<F, MRT_K_YZ>(bo, cur, t1 + 0.0001f, FLT_MAX_, &t2);
            }
            if (on && h1 && h2) {
                float a = t1 < tmin ? tmin : t1;
                const float b = t2 > closest ? closest : t2;
                if (a < b) {
                    if (a < 0) a = 0;
                    const float inside_dist = b - a;
                    const float hit_dist = -(1 / o.f[0]) * log_(randf(rng));
                    if (hit_dist < inside_dist) {
                        closest = a + hit_dist;
#if MRT_LIN_DEFER
                        hnode = pc;  // the volume op: its record after the walk
                        hk = HK_VOL;
#else
                        rec.t = closest;
                        rec.p = eval(cur, closest);
                        rec.n = f3{1, 0, 0};
                        rec.mat = o.mat;
                        hnode = o.node;
                        hk = HK_DONE;
#endif
                        hinst = inst;
                    }
                }
            }
            pc = ((F & FT_VSUB) && (LOP_FLAGS(o) & MRT_F_VSUB)) ? o.skip - 1 : pc + 1;  // past the boundary
            PH_MARK(ph, 10);
        } else if ((F & FT_BVHW) && op == LOP_BVHW) {
#if MRT_LIN_DEFER
            HitRec tr;  // t, the leaf primitive (mat) and the range it passed with (u)
            if (on && bvhw_walk<F>(S, S.nodes[o.node], cur, tmin, closest, tr, false, L)) {
                closest = tr.t;
                hnode = o.node;
                hinst = inst;
                hk = HK_BVHW;
                hprim = tr.mat;
                htlim = tr.u;
            }
#else
            if (on && bvhw_walk<F>(S, S.nodes[o.node], cur, tmin, closest, rec, true, L)) {
                closest = rec.t;
                hnode = o.node;
                hinst = inst;
                hk = HK_DONE;
            }
#endif
            PH_MARK(ph, 11);
        } else if (op == LOP_LIST) {  // object_list::hit box reject (scene_object.h:83)
            bool in = on;
            if (in && (LOP_FLAGS(o) & MRT_F_HASBOX)) in = lin_box(o, cur, tmin, closest);
            lvl++;
            act = (act & ~(1u << lvl)) | ((uint32_t)in << lvl);
            if (!any_lane(in)) pc = o.skip - 1;
        } else if (INST && op == LOP_INST) {
            const uint32_t kind = LOP_KIND(o);
            bool in = on;
            const Ray r0 = lin_load_ray(L);
            if (kind == MRT_K_TRROTY) {  // translate::hit then rotate_y::hit (scene_object.cpp:9-18, 70-98)
                cur = moved_ray<kFastUnit<F>>(r0, sub(r0.o, f3{o.f[8], o.f[9], o.f[10]}));
                if (in && (LOP_FLAGS(o) & MRT_F_HASBOX)) in = lin_box(o, cur, tmin, closest);
            } else if (kind == MRT_K_ROTY) {
                cur = r0;
                if (in && (LOP_FLAGS(o) & MRT_F_HASBOX)) in = lin_box(o, cur, tmin, closest);
            }
            lvl++;
            act = (act & ~(1u << lvl)) | ((uint32_t)in << lvl);
            inst = pc;
            if (!any_lane(in)) {
                pc = o.skip - 1;
                return true;
            }
            if (kind == MRT_K_TRROTY || kind == MRT_K_ROTY) cur = rotate_ray<kFastUnit<F>>(cur, o.f[6], o.f[7]);
            else cur = moved_ray<kFastUnit<F>>(r0, sub(r0.o, f3{o.f[0], o.f[1], o.f[2]}));
        } else if (INST && op == LOP_INST_END) {
            cur = lin_load_ray(L);
            inst = MRT_NONE;
            lvl--;
        } else if (op == LOP_LIST_END) {
            lvl--;
        }
        PH_MARK(ph, 8);
        // (the tolerance contract's program marks the op after which the END op comes)
        return !(MRT_LIN_LAST && kLinSlabOps<F> && (LOP_FLAGS(o) & MRT_F_LAST));
    };
    for (;; pc++) {
        if constexpr (kFetch) {
            pc = uniform_u32(pc);  // (wave-uniform: the op's words go to SGPRs)
            if (!step(lin_fetch_all(prog[pc]))) break;
        } else {
            if (!step(prog[pc])) break;
        }
    }
    if (INST) r = lin_load_ray(L);
    if (hnode == MRT_NONE) return false;
    // one copy of each record's code for hits in both frames: the ray of the hit's frame first (the
    // instance ray recomputed, inst_ray), then the record, then the instance's transform back
    const bool in_inst = INST && hinst != MRT_NONE;
#if MRT_LIN_PREFETCH_INST
    // the instance op's words (per lane: vector loads) fetched before the record's node, so the
    // two sets of loads are in flight together instead of one round trip after the other
    // (only the words inst_ray and lin_untransform read: its code, the offset f[0..2], rotate_y's
    // f[6..7], the fused translation f[8..10])
    LinOp io;
    if (in_inst) {
        const LinOp* ip = S.prog + hinst;
        io.code = ip->code;
        for (int k = 0; k < 3; k++) io.f[k] = ip->f[k];
        for (int k = 6; k < 11; k++) io.f[k] = ip->f[k];
    }
#else
    const LinOp& io = S.prog[in_inst ? hinst : 0u];
#endif
    if (hk != HK_DONE) {
        const Ray hr = in_inst ? inst_ray<kFastUnit<F>>(io, r) : r;
        if (MRT_LIN_DEFER && (F & FT_BVHW) && hk == HK_BVHW) bvhw_leaf_rec<F>(S, hprim, hr, tmin, htlim, rec);
        else lin_hit_rec<F>(S, prog, hk, hnode, hr, closest, rec);
    }
    if (in_inst) lin_untransform(io, rec);
    return true;
}

}  // namespace mrtd
