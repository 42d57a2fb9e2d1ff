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
                if (any_lane(in)) {
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

// scene_object::hit for a program of shape SIG (same contract as scene_hit_lin)
template <uint32_t F>
MRT_DFN bool scene_hit_sig(const DScene& S, Ray& r, float tmin, HitRec& rec, const LStack& L) {
    constexpr uint32_t SIG = MRT_SIG_OF(F);
    constexpr bool INST = (F & FT_INST) != 0;
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

}  // namespace mrtd
