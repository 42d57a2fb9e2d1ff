// mrt_sig.h -- linear hit programs of known shape, walked by code generated at compile time.
//
// The reference builds a fixed set of scenes (select_scene, scene.cpp:25-49).  Their linear
// programs (mrt_lin.h) have a handful of distinct SHAPES -- the sequence of (op, kind, skip)
// with the data left out.  For a shape listed here the kernel is instantiated with the walk
// unrolled by template recursion: no op fetch/dispatch loop, every op kind and jump target a
// compile-time constant, only the primitive data read (scalar loads at constant offsets).  The
// semantics are exactly scene_hit_lin's: same tests, same order, same record.  Programs of any
// other shape run the scene_hit_lin interpreter.
#pragma once
#include "mrt_lin.h"

namespace mrtd {

struct LinSig {
    uint32_t n;         // ops, including the final LOP_END
    uint8_t op[32];     // LOP_*
    uint8_t kind[32];   // node kind (MRT_K_*)
    uint8_t skip[32];   // matching END op of a LIST / INST
};

// shape ids (bits 16.. of a kernel's feature word; 0 = interpreter)
enum : uint32_t { SIG_NONE = 0, SIG_CORNELL = 1, SIG_ROOM_MESH = 2, SIG_COUNT = 3 };
#define MRT_SIG_OF(F) (((F) >> 16) & 0xFFu)
#define MRT_SIG_BITS(id) ((uint32_t)(id) << 16)

// clang-format off
static constexpr LinSig kSigs[SIG_COUNT] = {
    {0, {}, {}, {}},
    // scene 5 (cornell_box, scene.cpp:286-330): walls + light, translate(rotate_y(box)), glass sphere
    {20,
     {LOP_LIST, LOP_PRIM, LOP_PRIM, LOP_PRIM, LOP_PRIM, LOP_PRIM, LOP_PRIM, LOP_INST, LOP_LIST, LOP_PRIM, LOP_PRIM, LOP_PRIM, LOP_PRIM,
      LOP_PRIM, LOP_PRIM, LOP_LIST_END, LOP_INST_END, LOP_PRIM, LOP_LIST_END, LOP_END},
     {MRT_K_LIST, MRT_K_YZ, MRT_K_YZ, MRT_K_XZ, MRT_K_XZ, MRT_K_XZ, MRT_K_XY, MRT_K_TRROTY, MRT_K_LIST, MRT_K_XY, MRT_K_XY, MRT_K_XZ,
      MRT_K_XZ, MRT_K_YZ, MRT_K_YZ, MRT_K_LIST, MRT_K_TRROTY, MRT_K_SPHERE, MRT_K_LIST, 0},
     {18, 0, 0, 0, 0, 0, 0, 16, 15, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0}},
    // scenes 8 / 9 (bunny / teapot in the Cornell room): walls + light + one pod_bvh mesh
    {10,
     {LOP_LIST, LOP_PRIM, LOP_PRIM, LOP_PRIM, LOP_PRIM, LOP_PRIM, LOP_PRIM, LOP_MESH, LOP_LIST_END, LOP_END},
     {MRT_K_LIST, MRT_K_YZ, MRT_K_YZ, MRT_K_XZ, MRT_K_XZ, MRT_K_XZ, MRT_K_XY, MRT_K_MESH, MRT_K_LIST, 0},
     {8, 0, 0, 0, 0, 0, 0, 0, 0, 0}},
};
// clang-format on

// host: the shape id of a compiled program (SIG_NONE if it matches no entry)
inline uint32_t lin_sig_of(const LinOp* prog, uint32_t n) {
    for (uint32_t id = 1; id < SIG_COUNT; id++) {
        const LinSig& g = kSigs[id];
        if (g.n != n) continue;
        bool ok = true;
        for (uint32_t i = 0; i < n && ok; i++) {
            const uint32_t op = prog[i].code & 0xFFu, kind = (prog[i].code >> 8) & 0xFFu;
            ok = op == g.op[i] && (op == LOP_END || kind == g.kind[i]) &&
                 ((op != LOP_LIST && op != LOP_INST) || prog[i].skip == g.skip[i]);
        }
        // the Cornell shape's box must be box.h's six rects (MRT_F_BOX6, set on upload): the
        // tolerance-contract kernel walks it as one slab test with no fallback (cornell_fast_hit)
        if (ok && id == SIG_CORNELL) ok = ((prog[8].code >> 16) & MRT_F_BOX6) != 0;
        if (ok) return id;
    }
    return SIG_NONE;
}

struct SigState {
    Ray cur;
    float closest;
    uint32_t hnode, hinst;
    bool hdone;
};

template <uint32_t F, uint32_t SIG>
struct SigWalk {
    static constexpr const LinSig& G = kSigs[SIG];
    // room + mesh: the record is derived op by op with scalar loads (teapot +1.4%); the Cornell
    // walk keeps the per-lane node record (neutral there, shorter code)
    static constexpr bool kDerive = SIG == SIG_ROOM_MESH;

    // ops [PC, END) of the program, lanes `on` taking part
    template <uint32_t PC, uint32_t END>
    MRT_DATTR static __forceinline__ void run(const DScene& S, const MRT_CONST_AS LinOp* prog, float tmin, SigState& w, bool on,
                                               HitRec& rec, const LStack& L) {
        if constexpr (PC < END) {
            constexpr uint32_t op = G.op[PC];
            constexpr uint32_t kind = G.kind[PC];
            const MRT_CONST_AS LinOp& o = prog[PC];
            if constexpr (op == LOP_PRIM) {
                float t;
                bool h;
                uint32_t node;
                if constexpr (SIG == SIG_ROOM_MESH) {
                    // each op's words by one batch of scalar loads (+2% on the mesh scenes; -2% on
                    // the Cornell box, whose walk is short of SGPRs: there the loads stay lazy)
                    const LinOp ov = lin_fetch_op<F, kind>(o);
                    h = lin_prim_t<F, kind>(ov, w.cur, tmin, w.closest, &t) & on;
                    node = ov.node;
                } else {
                    h = lin_prim_t<F, kind>(o, w.cur, tmin, w.closest, &t) & on;
                    node = o.node;
                }
                w.closest = h ? t : w.closest;
                if constexpr (kDerive) w.hnode = h ? PC : w.hnode;  // op index: the record is derived op by op
                else w.hnode = h ? node : w.hnode;  // the op's node (scalar operand): no per-lane lookup later
                w.hinst = h ? cur_inst<PC>() : w.hinst;
                w.hdone = h ? false : w.hdone;
                run<PC + 1, END>(S, prog, tmin, w, on, rec, L);
            } else if constexpr (op == LOP_MESH) {
                if (on && mesh_hit<true>(S, ld_node(const_ptr(S.nodes) + o.node), w.cur, tmin, w.closest, rec, true, L)) {
                    w.closest = rec.t;
                    w.hnode = kDerive ? PC : o.node;
                    w.hinst = cur_inst<PC>();
                    w.hdone = true;
                }
                run<PC + 1, END>(S, prog, tmin, w, on, rec, L);
            } else if constexpr (op == LOP_LIST) {  // object_list::hit box reject (scene_object.h:83)
                constexpr uint32_t skip = G.skip[PC];
                const bool in = on && (!(LOP_FLAGS(o) & MRT_F_HASBOX) || lin_box(o, w.cur, tmin, w.closest));
                if constexpr (MRT_FAST_BOX && is_box6<PC>()) {
                    if (LOP_FLAGS(o) & MRT_F_BOX6) {  // uniform: box.h's six rects as one slab test
                        BSTATC(11, in);
                        if (any_lane(in)) box6_hit<PC>(prog, w, in, tmin);
                        run<skip + 1, END>(S, prog, tmin, w, on, rec, L);
                        return;
                    }
                }
                if (any_lane(in)) run<PC + 1, skip>(S, prog, tmin, w, in, rec, L);
                run<skip + 1, END>(S, prog, tmin, w, on, rec, L);
            } else if constexpr (op == LOP_INST) {  // scene_object.cpp:9-18, 70-98
                constexpr uint32_t skip = G.skip[PC];
                const Ray r0 = lin_load_ray(L);
                bool in = on;
                if constexpr (kind == MRT_K_TRROTY) {
                    w.cur = moved_ray(r0, sub(r0.o, f3{o.f[8], o.f[9], o.f[10]}));
                    if (in && (LOP_FLAGS(o) & MRT_F_HASBOX)) in = lin_box(o, w.cur, tmin, w.closest);
                } else if constexpr (kind == MRT_K_ROTY) {
                    w.cur = r0;
                    if (in && (LOP_FLAGS(o) & MRT_F_HASBOX)) in = lin_box(o, w.cur, tmin, w.closest);
                }
                BSTATC(8, in);
                if (any_lane(in)) {
                    BSTATC(9, in);
                    if constexpr (kind == MRT_K_TRROTY || kind == MRT_K_ROTY) w.cur = rotate_ray(w.cur, o.f[6], o.f[7]);
                    else w.cur = moved_ray(r0, sub(r0.o, f3{o.f[0], o.f[1], o.f[2]}));
                    run<PC + 1, skip>(S, prog, tmin, w, in, rec, L);
                    if (w.hinst == PC) {  // keep the instance-frame ray of the hit for the record
                        float* b = L.save + L.lane + 9 * 64;
                        b[0] = w.cur.o.x; b[64] = w.cur.o.y; b[128] = w.cur.o.z;
                        b[192] = w.cur.d.x; b[256] = w.cur.d.y; b[320] = w.cur.d.z;
                    }
                }
                w.cur = lin_load_ray(L);
                run<skip + 1, END>(S, prog, tmin, w, on, rec, L);
            } else {
                run<PC + 1, END>(S, prog, tmin, w, on, rec, L);
            }
        }
    }

    // ops PC+1..PC+6 are the six rects of box.h in its order (the list at PC ends at PC+7)
    template <uint32_t PC>
    MRT_DATTR static constexpr bool is_box6() {
        if (PC + 7 >= G.n || G.op[PC] != LOP_LIST || G.skip[PC] != PC + 7) return false;
        constexpr uint32_t k[6] = {MRT_K_XY, MRT_K_XY, MRT_K_XZ, MRT_K_XZ, MRT_K_YZ, MRT_K_YZ};
        for (uint32_t j = 0; j < 6; j++)
            if (G.op[PC + 1 + j] != LOP_PRIM || G.kind[PC + 1 + j] != k[j]) return false;
        return true;
    }
    // Tolerance contract: box.h's object_list of six outward-facing one-sided rects (MRT_F_BOX6)
    // as one slab test.  From outside the box the one front-facing face a ray can hit is where it
    // enters, at the slab entry t (the same (k - o) * 1/d the rect test forms); from inside or from
    // the surface every face is behind or back-facing, and so is the entry (t < tmin).  Ties
    // (edges) go to the later rect of box.h's order, as object_list::hit's closest narrowing does.
    // Differs from the six tests only by rounding at edges.
    template <uint32_t PC>
    MRT_DATTR static __forceinline__ void box6_hit(const MRT_CONST_AS LinOp* prog, SigState& w, bool in, float tmin) {
        const MRT_CONST_AS LinOp& o = prog[PC];
        const Ray& r = w.cur;
        const float t0x = (o.f[6] - r.o.x) * r.inv.x, t1x = (o.f[9] - r.o.x) * r.inv.x;
        const float t0y = (o.f[7] - r.o.y) * r.inv.y, t1y = (o.f[10] - r.o.y) * r.inv.y;
        const float t0z = (o.f[8] - r.o.z) * r.inv.z, t1z = (o.f[11] - r.o.z) * r.inv.z;
        const float nx = fminf(t0x, t1x), ny = fminf(t0y, t1y), nz = fminf(t0z, t1z);
        const float tn = fmaxf(fmaxf(nx, ny), nz);
        const float tf = fminf(fminf(fmaxf(t0x, t1x), fmaxf(t0y, t1y)), fmaxf(t0z, t1z));
        const bool h = in & (tn <= tf) & (tn >= tmin) & (tn <= w.closest);
        // the entry face: rects 0/1 = z max/min, 2/3 = y max/min, 4/5 = x max/min
        const uint32_t nz_node = r.d.z > 0.0f ? prog[PC + 2].node : prog[PC + 1].node;
        const uint32_t ny_node = r.d.y > 0.0f ? prog[PC + 4].node : prog[PC + 3].node;
        const uint32_t nx_node = r.d.x > 0.0f ? prog[PC + 6].node : prog[PC + 5].node;
        const uint32_t node = tn == nx ? nx_node : (tn == ny ? ny_node : nz_node);
        w.closest = h ? tn : w.closest;
        w.hnode = h ? (kDerive ? PC + 1 : node) : w.hnode;
        w.hinst = h ? cur_inst<PC + 1>() : w.hinst;
        w.hdone = h ? false : w.hdone;
    }

    // the record of the closest hit, op by op: for each primitive op some lane hit, that op's
    // data by scalar loads and its compile-time kind (no per-lane node loads or kind switch)
    template <uint32_t PC>
    MRT_DATTR static __forceinline__ void derive(const MRT_CONST_AS LinOp* prog, const SigState& w, const Ray& r, const Ray& ir,
                                                  HitRec& rec) {
        if constexpr (PC < G.n) {
            if constexpr (G.op[PC] == LOP_PRIM) {
                if (any_lane(w.hnode == PC)) {
                    if (w.hnode == PC) lin_prim_rec_op<F, G.kind[PC]>(prog[PC], cur_inst<PC>() != MRT_NONE ? ir : r, w.closest, rec);
                }
            }
            derive<PC + 1>(prog, w, r, ir, rec);
        }
    }
    // the program's only instance op (MRT_NONE if it has none or several)
    MRT_DATTR static constexpr uint32_t only_inst() {
        uint32_t found = MRT_NONE, count = 0;
        for (uint32_t i = 0; i < G.n; i++)
            if (G.op[i] == LOP_INST) { found = i; count++; }
        return count == 1 ? found : MRT_NONE;
    }
    // op index of the instance enclosing op PC (MRT_NONE: world frame)
    template <uint32_t PC>
    MRT_DATTR static constexpr uint32_t cur_inst() {
        uint32_t found = MRT_NONE;
        for (uint32_t i = 0; i < PC; i++)
            if (G.op[i] == LOP_INST && G.skip[i] > PC) found = i;
        return found;
    }
};

// Tolerance contract, Cornell box shape (scene 5, scene.cpp:286-330) whose box is box.h's six rects
// (MRT_F_BOX6 on op 8): the walk written out for the ops the shape fixes, with the closest hit's
// record carried per lane through the walk (a code, a plane, a sign, a material: a few selects per
// primitive) instead of derived afterwards from the winning op (per-lane node loads and a switch on
// its kind) -- no branch, no LDS.
//   * the root list's and the instance's bounding boxes are not tested: every primitive test below
//     is exact geometry, a box test only skips work (object_list::hit, scene_object.h:83;
//     rotate_y::hit, scene_object.cpp:72);
//   * translate(rotate_y(box)) (scene_object.cpp:9-18, 70-98) is ONE slab test of the box in its own
//     frame (the ray moved and rotated; box6_hit's entry-face rule), the record taken in the world
//     frame: p = o + t d (t is frame-independent: translate keeps d, rotate_y keeps |d|), the entry
//     face's outward normal rotated back (scene_object.cpp:85-93).  Differs from the reference's
//     per-face tests and frame round trip by rounding only.
// Walls and sphere are lin_prim_t's tests in op order (ties to the later op, as closest narrowing).
#ifndef MRT_CORNELL_BATCHES
#define MRT_CORNELL_BATCHES 2
#endif
struct CornellRec {
    float closest, k, ns;
    uint32_t code, mat;  // code: 0 none; 1-3 world rect of axis code-1 (plane k); 4-6 box face of axis code-4; 7 sphere
};
// A rect op's words (its LinOp's mat and f[0..5]) loaded into SGPRs.  The walk loads all six rects'
// words as one batch and takes them at one point (the asms, issued back to back after the loads): one
// scalar-cache round trip for the walls -- the compiler otherwise loaded each op's fields in two
// dependent rounds, the material lazily inside a branch on the hit (12 round trips for the walls).
struct CornellRect {
    uint32_t mat, b0, b1, b2, b3, k, ns;
};
MRT_DFN CornellRect cornell_load(const MRT_CONST_AS LinOp& o) {
    const MRT_CONST_AS uint32_t* q = reinterpret_cast<const MRT_CONST_AS uint32_t*>(&o);
    return CornellRect{q[3], q[4], q[5], q[6], q[7], q[8], q[9]};
}
MRT_DFN void cornell_take1(CornellRect& d) {
#if defined(__HIP_DEVICE_COMPILE__)
    asm volatile("" : "+s"(d.mat), "+s"(d.b0), "+s"(d.b1), "+s"(d.b2), "+s"(d.b3), "+s"(d.k), "+s"(d.ns));
#else
    (void)d;
#endif
}
// translate(rotate_y(box)): rotate_y's (sin, cos), translate's offset (op 7), the box's planes
// and material (op 8); the sphere's centre, radius and material (op 17)
struct CornellBox {
    uint32_t s, c, o0, o1, o2, lo0, lo1, lo2, hi0, hi1, hi2, mat;
};
struct CornellSphere {
    uint32_t c0, c1, c2, rad, mat;
};
MRT_DFN CornellBox cornell_load_box(const MRT_CONST_AS LinOp& io, const MRT_CONST_AS LinOp& bo) {
    const MRT_CONST_AS uint32_t* qi = reinterpret_cast<const MRT_CONST_AS uint32_t*>(&io);
    const MRT_CONST_AS uint32_t* qb = reinterpret_cast<const MRT_CONST_AS uint32_t*>(&bo);
    return CornellBox{qi[10], qi[11], qi[12], qi[13], qi[14], qb[10], qb[11], qb[12], qb[13], qb[14], qb[15], qb[3]};
}
MRT_DFN CornellSphere cornell_load_sphere(const MRT_CONST_AS LinOp& so) {
    const MRT_CONST_AS uint32_t* q = reinterpret_cast<const MRT_CONST_AS uint32_t*>(&so);
    return CornellSphere{q[4], q[5], q[6], q[12], q[3]};
}
MRT_DFN void cornell_take1(CornellBox& d) {
#if defined(__HIP_DEVICE_COMPILE__)
    asm volatile("" : "+s"(d.s), "+s"(d.c), "+s"(d.o0), "+s"(d.o1), "+s"(d.o2), "+s"(d.mat));
    asm volatile("" : "+s"(d.lo0), "+s"(d.lo1), "+s"(d.lo2), "+s"(d.hi0), "+s"(d.hi1), "+s"(d.hi2));
#else
    (void)d;
#endif
}
MRT_DFN void cornell_take1(CornellSphere& d) {
#if defined(__HIP_DEVICE_COMPILE__)
    asm volatile("" : "+s"(d.c0), "+s"(d.c1), "+s"(d.c2), "+s"(d.rad), "+s"(d.mat));
#else
    (void)d;
#endif
}
template <typename... D>
MRT_DFN void cornell_take(D&... d) {
    (cornell_take1(d), ...);
}
template <uint32_t F, uint32_t PC>
MRT_DFN void cornell_rect(const CornellRect& d, const Ray& r, float tmin, CornellRec& w) {
    constexpr uint32_t KIND = kSigs[SIG_CORNELL].kind[PC];
    static_assert(kSigs[SIG_CORNELL].op[PC] == LOP_PRIM && KIND != MRT_K_SPHERE, "Cornell shape: world rect");
    constexpr uint32_t AX = KIND == MRT_K_XY ? 2u : KIND == MRT_K_XZ ? 1u : 0u;
    LinOp o;
    o.code = 0;  // (lin_prim_t reads the flags only under the exact contract's guards)
    o.f[0] = __uint_as_float(d.b0);
    o.f[1] = __uint_as_float(d.b1);
    o.f[2] = __uint_as_float(d.b2);
    o.f[3] = __uint_as_float(d.b3);
    o.f[4] = __uint_as_float(d.k);
    o.f[5] = __uint_as_float(d.ns);
    float t;
    const bool h = lin_prim_t<F, KIND>(o, r, tmin, w.closest, &t);
    w.closest = h ? t : w.closest;
    w.code = h ? 1u + AX : w.code;
    w.k = h ? o.f[4] : w.k;
    w.ns = h ? o.f[5] : w.ns;
    w.mat = h ? d.mat : w.mat;
}
template <uint32_t F>
MRT_DFN bool cornell_fast_hit(const MRT_CONST_AS LinOp* prog, const Ray& r, float tmin, HitRec& rec) {
    constexpr const LinSig& G = kSigs[SIG_CORNELL];
    static_assert(G.op[7] == LOP_INST && G.kind[7] == MRT_K_TRROTY && G.op[8] == LOP_LIST && G.skip[8] == 15 &&
                      G.op[17] == LOP_PRIM && G.kind[17] == MRT_K_SPHERE,
                  "Cornell shape: translate(rotate_y(box)) at op 7, its six rects under op 8, the sphere at op 17");
    CornellRec w{FLT_MAX_, 0.0f, 0.0f, 0u, 0u};
    // the six rects' words in one batch of scalar loads, one wait
    CornellRect d1 = cornell_load(prog[1]), d2 = cornell_load(prog[2]), d3 = cornell_load(prog[3]);
    CornellRect d4 = cornell_load(prog[4]), d5 = cornell_load(prog[5]), d6 = cornell_load(prog[6]);
#if MRT_CORNELL_BATCHES == 2  // walls, then box + sphere (fewer SGPRs live at once, one more wait)
    cornell_take(d1, d2, d3, d4, d5, d6);
    cornell_rect<F, 1>(d1, r, tmin, w);
    cornell_rect<F, 2>(d2, r, tmin, w);
    cornell_rect<F, 3>(d3, r, tmin, w);
    cornell_rect<F, 4>(d4, r, tmin, w);
    cornell_rect<F, 5>(d5, r, tmin, w);
    cornell_rect<F, 6>(d6, r, tmin, w);
    CornellBox db = cornell_load_box(prog[7], prog[8]);
    CornellSphere dsp = cornell_load_sphere(prog[17]);
    cornell_take(db, dsp);
#else
    CornellBox db = cornell_load_box(prog[7], prog[8]);
    CornellSphere dsp = cornell_load_sphere(prog[17]);
    cornell_take(d1, d2, d3, d4, d5, d6, db, dsp);
    cornell_rect<F, 1>(d1, r, tmin, w);
    cornell_rect<F, 2>(d2, r, tmin, w);
    cornell_rect<F, 3>(d3, r, tmin, w);
    cornell_rect<F, 4>(d4, r, tmin, w);
    cornell_rect<F, 5>(d5, r, tmin, w);
    cornell_rect<F, 6>(d6, r, tmin, w);
#endif
    // the box in its own frame: o' = R(o - offset), d' = R d, R = rotate_y's (s, c)
    const float s = __uint_as_float(db.s), c = __uint_as_float(db.c);
    const float off0 = __uint_as_float(db.o0), off1 = __uint_as_float(db.o1), off2 = __uint_as_float(db.o2);
    const float lo0 = __uint_as_float(db.lo0), lo1 = __uint_as_float(db.lo1), lo2 = __uint_as_float(db.lo2);
    const float hi0 = __uint_as_float(db.hi0), hi1 = __uint_as_float(db.hi1), hi2 = __uint_as_float(db.hi2);
    const float mx = r.o.x - off0, my = r.o.y - off1, mz = r.o.z - off2;
    const float ox = c * mx - s * mz, oz = c * mz + s * mx;
    const float dx = c * r.d.x - s * r.d.z, dz = c * r.d.z + s * r.d.x;
    const float ix = recip_nr(dx), iz = recip_nr(dz);
    const float t0x = (lo0 - ox) * ix, t1x = (hi0 - ox) * ix;
    const float t0y = (lo1 - my) * r.inv.y, t1y = (hi1 - my) * r.inv.y;
    const float t0z = (lo2 - oz) * iz, t1z = (hi2 - oz) * iz;
    const float nx = fminf(t0x, t1x), ny = fminf(t0y, t1y), nz = fminf(t0z, t1z);
    const float tn = fmaxf(fmaxf(nx, ny), nz);
    const float tf = fminf(fminf(fmaxf(t0x, t1x), fmaxf(t0y, t1y)), fmaxf(t0z, t1z));
    const bool hb = (tn <= tf) & (tn >= tmin) & (tn <= w.closest);
    // the entry face: its axis, and its outward normal's sign (against the ray's direction there)
    const uint32_t bax = tn == nx ? 0u : (tn == ny ? 1u : 2u);
    const float bd = bax == 0u ? dx : (bax == 1u ? r.d.y : dz);
    w.closest = hb ? tn : w.closest;
    w.code = hb ? 4u + bax : w.code;
    w.ns = hb ? (bd > 0.0f ? -1.0f : 1.0f) : w.ns;
    w.mat = hb ? db.mat : w.mat;
    // the sphere (op 17)
    LinOp so;
    so.code = 0;  // (a static sphere: F has no FT_MOVING)
    so.f[0] = __uint_as_float(dsp.c0);
    so.f[1] = __uint_as_float(dsp.c1);
    so.f[2] = __uint_as_float(dsp.c2);
    so.f[8] = __uint_as_float(dsp.rad);
    {
        float t;
        const bool h = lin_prim_t<F, MRT_K_SPHERE>(so, r, tmin, w.closest, &t);
        w.closest = h ? t : w.closest;
        w.code = h ? 7u : w.code;
        w.mat = h ? dsp.mat : w.mat;
    }
    if (w.code == 0u) return false;
    rec.t = w.closest;
    rec.mat = w.mat;
    f3 p = eval(r, w.closest);
    // world rects: the point on the rect's plane (MRT_FAST_SNAP, lin_prim_rec_op)
    p.x = w.code == 1u ? w.k : p.x;
    p.y = w.code == 2u ? w.k : p.y;
    p.z = w.code == 3u ? w.k : p.z;
    if (w.code >= 4u && w.code <= 6u) {
        // a box face: the point in the box frame put on the face's plane, then back to the world
        // (as lin_prim_rec_op + lin_untransform do).  o + t d in the world frame lands up to ~1e-4
        // off the face (t from a reciprocal, |t| ~ 1e3), and a grazing inward light-sampling ray
        // from there re-enters the box at t > tmin: +0.35% rays (measured).
        const float t = w.closest;
        float px = ox + t * dx, py = my + t * r.d.y, pz = oz + t * dz;
        const float pl = w.code == 4u ? (w.ns < 0.0f ? lo0 : hi0)
                       : w.code == 5u ? (w.ns < 0.0f ? lo1 : hi1)
                                      : (w.ns < 0.0f ? lo2 : hi2);
        px = w.code == 4u ? pl : px;
        py = w.code == 5u ? pl : py;
        pz = w.code == 6u ? pl : pz;
        p = f3{(c * px + s * pz) + off0, py + off1, (c * pz - s * px) + off2};
    }
    rec.p = p;
    const uint32_t a = w.code >= 4u ? w.code - 4u : w.code - 1u;
    const float lx = a == 0u ? w.ns : 0.0f, ly = a == 1u ? w.ns : 0.0f, lz = a == 2u ? w.ns : 0.0f;
    f3 n{lx, ly, lz};
    if (w.code >= 4u) n = f3{c * lx + s * lz, ly, c * lz - s * lx};  // unrotate_rec's normal
    if (w.code == 7u) n = divf(sub(p, f3{so.f[0], so.f[1], so.f[2]}), so.f[8]);
    rec.n = n;
    return true;
}

// the kernels that walk the Cornell shape by cornell_fast_hit (the host sizes LDS by it)
template <uint32_t F>
static constexpr uint32_t kBox6Walk = (MRT_FAST_BOX && MRT_SIG_OF(F) == SIG_CORNELL && !(F & (FT_UV | FT_MOVING))) ? 1u : 0u;

// scene_object::hit for a program of shape SIG (same contract as scene_hit_lin)
template <uint32_t F>
MRT_DFN bool scene_hit_sig(const DScene& S, Ray& r, float tmin, HitRec& rec, const LStack& L) {
    constexpr uint32_t SIG = MRT_SIG_OF(F);
    constexpr bool INST = (F & FT_INST) != 0;
    if constexpr (kBox6Walk<F>) {  // (the shape implies MRT_F_BOX6 on op 8: lin_sig_of)
        return cornell_fast_hit<F>(const_ptr(S.prog), r, tmin, rec);
    } else {
    if (INST) lin_save_ray(L, r);
    const MRT_CONST_AS LinOp* prog = const_ptr(S.prog);
    SigState w;
    w.cur = r;
    w.closest = FLT_MAX_;
    w.hnode = MRT_NONE;
    w.hinst = MRT_NONE;
    w.hdone = false;
    SigWalk<F, SIG>::template run<0, kSigs[SIG].n - 1>(S, prog, tmin, w, true, rec, L);
    if (INST) r = lin_load_ray(L);
    if (w.hnode == MRT_NONE) return false;
    if constexpr (SigWalk<F, SIG>::kDerive) {
        Ray ir = r;
        if (INST && any_lane(w.hinst != MRT_NONE && !w.hdone)) {  // instance-frame ray of the hit (LDS)
            const float* b = L.save + L.lane + 9 * 64;
            ir.o = f3{b[0], b[64], b[128]};
            ir.d = f3{b[192], b[256], b[320]};
        }
        if (!w.hdone) SigWalk<F, SIG>::template derive<0>(prog, w, r, ir, rec);
        if (INST && w.hinst != MRT_NONE) {
            constexpr uint32_t IPC = SigWalk<F, SIG>::only_inst();
            if constexpr (IPC != MRT_NONE) lin_untransform(prog[IPC], rec);
            else lin_untransform(S.prog[w.hinst], rec);
        }
    } else {
        const uint32_t node = w.hnode;
        if (INST && w.hinst != MRT_NONE) {
            if (!w.hdone) {
                const float* b = L.save + L.lane + 9 * 64;
                Ray ir = r;
                ir.o = f3{b[0], b[64], b[128]};
                ir.d = f3{b[192], b[256], b[320]};
                lin_prim_rec<F>(S, node, ir, w.closest, rec);
            }
            constexpr uint32_t IPC = SigWalk<F, SIG>::only_inst();
            if constexpr (IPC != MRT_NONE) lin_untransform(prog[IPC], rec);  // known instance: scalar loads
            else lin_untransform(S.prog[w.hinst], rec);
        } else if (!w.hdone) {
            lin_prim_rec<F>(S, node, r, w.closest, rec);
        }
    }
    return true;
    }
}

}  // namespace mrtd
