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
#include <algorithm>
#include <cstdlib>
#include <vector>
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

// host: the Cornell shapes' room (scene 5, and the room + mesh scenes 8 / 9, scene.cpp:489-495) --
// ops 1, 2, 4, 5, 6 (two yz, two xz, one xy rect) one-sided rects
// facing INTO one box and spanning its faces (scene.cpp:311-318; op 3 is the light) -- written into
// the program's END op: f[0..5] the box's min / max corners, f[6..11] the material of face
// 2*axis + side (side 1: the max plane), node = the mask of the faces present, skip = the op index
// of each face (4 bits per face).  The tolerance
// contract's Cornell walk tests the room as ONE slab test: a ray inside (or entering) the box hits
// the face it leaves through; a face seen from outside is back-facing.  Returns false (no room) if
// the rects do not form such a box.
inline bool cornell_room_fill(LinOp* prog, uint32_t n) {
    if (n != kSigs[SIG_CORNELL].n && n != kSigs[SIG_ROOM_MESH].n) return false;
    static const uint32_t ops[5] = {1, 2, 4, 5, 6};
    float lo[3] = {0, 0, 0}, hi[3] = {0, 0, 0};
    bool has[3][2] = {{false, false}, {false, false}, {false, false}};
    uint32_t mats[6] = {0, 0, 0, 0, 0, 0}, mask = 0, face_ops = 0;
    // in-plane axes of a rect of axis a (mrt_lin.h lin_prim_t): f[0..1] along b, f[2..3] along c
    auto in_plane = [](uint32_t a, uint32_t* b, uint32_t* c) { *b = a == 0 ? 1u : 0u; *c = a == 2 ? 1u : 2u; };
    for (uint32_t j = 0; j < 5; j++) {
        const LinOp& o = prog[ops[j]];
        const uint32_t kind = (o.code >> 8) & 0xFFu;
        if ((o.code & 0xFFu) != LOP_PRIM || (kind != MRT_K_XY && kind != MRT_K_XZ && kind != MRT_K_YZ)) return false;
        if (((o.code >> 16) & (MRT_F_NEEDUV | MRT_F_SLOWDIV)) != 0) return false;
        const uint32_t a = kind == MRT_K_YZ ? 0u : kind == MRT_K_XZ ? 1u : 2u;
        const uint32_t side = o.f[5] > 0.0f ? 0u : 1u;  // a normal along +axis faces into a box from its min plane
        if (o.f[5] != (side ? -1.0f : 1.0f) || has[a][side]) return false;
        has[a][side] = true;
        (side ? hi : lo)[a] = o.f[4];
        mats[a * 2 + side] = o.mat;
        mask |= 1u << (a * 2 + side);
        face_ops |= ops[j] << (4 * (a * 2 + side));
    }
    // the box's extent along every axis: the face planes there, and the in-plane bounds of the
    // faces that span it, must all agree
    float blo[3], bhi[3];
    bool set[3] = {false, false, false};
    auto agree = [&](uint32_t a, float l, float h) {
        if (!set[a]) { blo[a] = l; bhi[a] = h; set[a] = true; return true; }
        return blo[a] == l && bhi[a] == h;
    };
    for (uint32_t j = 0; j < 5; j++) {
        const LinOp& o = prog[ops[j]];
        const uint32_t kind = (o.code >> 8) & 0xFFu;
        const uint32_t a = kind == MRT_K_YZ ? 0u : kind == MRT_K_XZ ? 1u : 2u;
        uint32_t b, c;
        in_plane(a, &b, &c);
        if (!agree(b, o.f[0], o.f[1]) || !agree(c, o.f[2], o.f[3])) return false;
    }
    for (uint32_t a = 0; a < 3; a++) {
        if (!set[a] || !(blo[a] < bhi[a])) return false;
        if ((has[a][0] && lo[a] != blo[a]) || (has[a][1] && hi[a] != bhi[a])) return false;
    }
    LinOp& e = prog[n - 1];  // the END op: nothing else reads its fields
    for (uint32_t a = 0; a < 3; a++) {
        e.f[a] = blo[a];
        e.f[3 + a] = bhi[a];
    }
    for (uint32_t k = 0; k < 6; k++) {
        float fm;
        __builtin_memcpy(&fm, &mats[k], 4);
        e.f[6 + k] = fm;
    }
    e.node = mask;
    e.skip = face_ops;  // op index of face k in bits 4k..4k+3
    return true;
}

// host: the tolerance contract's program (the interpreter's, for graphs without a shape-
// specialised walk): in every object_list, the inward-facing rects that bound one box -- a room's
// walls, at least three of them -- become ONE LOP_ROOM op (at the first wall's position; closest-
// hit order only matters for exact ties) followed by LOP_ROOMDATA (each face's node); box.h lists
// (MRT_F_BOX6) are tested as one slab test by the interpreter itself.  Returns the rewritten
// program (the input when nothing applies).
inline std::vector<LinOp> lin_rewrite_fast(const std::vector<LinOp>& prog) {
    const uint32_t n = (uint32_t)prog.size();
    std::vector<uint8_t> del(n, 0);
    std::vector<LinOp> room(n);          // the ROOM op replacing wall op i (when i is a room's first wall)
    std::vector<LinOp> roomdata(n);
    std::vector<uint8_t> is_first(n, 0);
    for (uint32_t L = 0; L < n; L++) {
        if ((prog[L].code & 0xFFu) != LOP_LIST) continue;
        // direct children of the list: nested lists / instances skipped whole
        std::vector<uint32_t> kids;
        for (uint32_t i = L + 1; i < prog[L].skip && i < n;) {
            const uint32_t op = prog[i].code & 0xFFu;
            if (op == LOP_LIST || op == LOP_INST) { i = prog[i].skip + 1; continue; }
            if (op == LOP_VOLUME) { i = ((prog[i].code >> 16) & MRT_F_VSUB) ? prog[i].skip : i + 2; continue; }
            kids.push_back(i);
            i++;
        }
        // candidate walls per face (axis, side): one-sided rects, no uv, exact divisions; the
        // widest rect of each face (a light below the ceiling is not the ceiling)
        int64_t pick[6] = {-1, -1, -1, -1, -1, -1};
        for (uint32_t i : kids) {
            const LinOp& o = prog[i];
            const uint32_t kind = (o.code >> 8) & 0xFFu;
            if ((o.code & 0xFFu) != LOP_PRIM || (kind != MRT_K_XY && kind != MRT_K_XZ && kind != MRT_K_YZ)) continue;
            if (((o.code >> 16) & (MRT_F_NEEDUV | MRT_F_SLOWDIV)) != 0 || (o.f[5] != 1.0f && o.f[5] != -1.0f)) continue;
            const uint32_t a = kind == MRT_K_YZ ? 0u : kind == MRT_K_XZ ? 1u : 2u;
            const uint32_t k = a * 2u + (o.f[5] > 0.0f ? 0u : 1u);  // normal along +axis: the min plane
            auto area = [&](const LinOp& x) { return (double)(x.f[1] - x.f[0]) * (double)(x.f[3] - x.f[2]); };
            if (pick[k] < 0 || area(o) > area(prog[pick[k]])) pick[k] = i;
        }
        // the box: along every axis its extent from the in-plane bounds of the walls spanning it,
        // which must agree, and the planes of the walls there must be its faces
        float lo[3], hi[3];
        bool set[3] = {false, false, false}, ok = true;
        uint32_t mask = 0, walls = 0;
        for (uint32_t k = 0; k < 6 && ok; k++) {
            if (pick[k] < 0) continue;
            const LinOp& o = prog[pick[k]];
            const uint32_t a = k / 2u, b = a == 0 ? 1u : 0u, c = a == 2 ? 1u : 2u;
            const float in[2][2] = {{o.f[0], o.f[1]}, {o.f[2], o.f[3]}};
            const uint32_t ax[2] = {b, c};
            for (int j = 0; j < 2 && ok; j++) {
                if (!set[ax[j]]) { lo[ax[j]] = in[j][0]; hi[ax[j]] = in[j][1]; set[ax[j]] = true; }
                else ok = lo[ax[j]] == in[j][0] && hi[ax[j]] == in[j][1];
            }
            mask |= 1u << k;
            walls++;
        }
        for (uint32_t a = 0; a < 3 && ok; a++) ok = set[a] && lo[a] < hi[a];
        for (uint32_t k = 0; k < 6 && ok; k++)
            if (pick[k] >= 0) ok = prog[pick[k]].f[4] == ((k & 1u) ? hi[k / 2u] : lo[k / 2u]);
        if (!ok || walls < 3) continue;
        uint32_t first = n;
        for (uint32_t k = 0; k < 6; k++)
            if (pick[k] >= 0) first = std::min(first, (uint32_t)pick[k]);
        LinOp r{}, d{};
        r.code = LOP_ROOM | (prog[first].code & 0xFF000000u);
        r.node = mask;
        r.skip = 0;
        r.mat = MRT_NONE;
        for (uint32_t a = 0; a < 3; a++) { r.f[a] = lo[a]; r.f[3 + a] = hi[a]; }
        d.code = LOP_ROOMDATA | (prog[first].code & 0xFF000000u);
        for (uint32_t k = 0; k < 6; k++) {
            const uint32_t node = pick[k] >= 0 ? prog[pick[k]].node : MRT_NONE;
            __builtin_memcpy(&d.f[k], &node, 4);
            if (pick[k] >= 0) del[pick[k]] = 1;
        }
        room[first] = r;
        roomdata[first] = d;
        is_first[first] = 1;
    }
    // an instance outside instances whose body is exactly one box.h list (INST, LIST flagged
    // MRT_F_BOX6, its six rects, LIST_END, INST_END): MRT_F_BOXINST, the interpreter's one-step box
    const char* nb = getenv("MRT_NO_BOXINST");  // A/B hook
    std::vector<uint8_t> boxinst(n, 0);
    for (uint32_t i = 0, depth = 0; i < n && !(nb && *nb && *nb != '0'); i++) {
        const uint32_t op = prog[i].code & 0xFFu;
        if (op == LOP_INST) {
            const uint32_t e = prog[i].skip;
            const bool ok = depth == 0 && e == i + 9 && e < n && (prog[i + 1].code & 0xFFu) == LOP_LIST &&
                            ((prog[i + 1].code >> 16) & MRT_F_BOX6) && prog[i + 1].skip == i + 8 &&
                            (prog[i + 8].code & 0xFFu) == LOP_LIST_END && (prog[e].code & 0xFFu) == LOP_INST_END;
            boxinst[i] = ok;
            depth++;
        } else if (op == LOP_INST_END && depth > 0) {
            depth--;
        }
    }
    // the root object_list (op 0, its LIST_END just before the END op): its box test only rejects
    // rays that miss the whole scene, and its two ops cost the lockstep walk two dispatch steps per
    // ray; dropped (the children are tested by every lane anyway, at level 0)
#ifndef MRT_REWRITE_ROOT
#define MRT_REWRITE_ROOT 1
#endif
    if (MRT_REWRITE_ROOT && n >= 3 && (prog[0].code & 0xFFu) == LOP_LIST && prog[0].skip == n - 2 &&
        (prog[n - 2].code & 0xFFu) == LOP_LIST_END && (prog[n - 1].code & 0xFFu) == LOP_END) {
        del[0] = 1;
        del[n - 2] = 1;
    }
    // compact: each room's first wall becomes ROOM + ROOMDATA, the other walls go; skips re-linked
    std::vector<uint32_t> at(n + 1, 0);
    std::vector<LinOp> out;
    for (uint32_t i = 0; i < n; i++) {
        at[i] = (uint32_t)out.size();
        if (is_first[i]) { out.push_back(room[i]); out.push_back(roomdata[i]); }
        else if (!del[i]) {
            out.push_back(prog[i]);
            if (boxinst[i]) out.back().code |= MRT_F_BOXINST << 16;
        }
    }
    at[n] = (uint32_t)out.size();
    for (LinOp& o : out) {
        const uint32_t op = o.code & 0xFFu;
        if ((op == LOP_LIST || op == LOP_INST || op == LOP_INST_END) && o.skip <= n) o.skip = at[o.skip];
    }
    // MRT_F_LAST on the op the interpreter leaves for the END op (the room op steps over its data op,
    // a one-step box instance or box.h list over its body): the walk ends there without one more
    // dispatch step
    for (uint32_t i = 0; i < out.size(); i++) {
        const uint32_t op = out[i].code & 0xFFu, fl = (out[i].code >> 16) & 0xFFu;
        uint32_t next = i + 1;
        if (op == LOP_ROOM) next = i + 2;
        else if ((op == LOP_INST && (fl & MRT_F_BOXINST)) || (op == LOP_LIST && (fl & MRT_F_BOX6))) next = out[i].skip + 1;
        if (op != LOP_END && next < out.size() && (out[next].code & 0xFFu) == LOP_END) out[i].code |= MRT_F_LAST << 16;
    }
    return out;
}

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
        if (ok && id == SIG_CORNELL) ok = ((prog[8].code >> 16) & MRT_F_BOX6) != 0 && prog[n - 1].node != 0;  // + cornell_room_fill
        if (ok && id == SIG_ROOM_MESH) ok = prog[n - 1].node != 0;  // the room (cornell_room_fill)
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
// the room (cornell_room_fill): box corners, face materials, face mask -- from the END op
struct CornellRoom {
    uint32_t lo0, lo1, lo2, hi0, hi1, hi2, m0, m1, m2, m3, m4, m5, mask;
};
MRT_DFN CornellRoom cornell_load_room(const MRT_CONST_AS LinOp& e) {
    const MRT_CONST_AS uint32_t* q = reinterpret_cast<const MRT_CONST_AS uint32_t*>(&e);
    return CornellRoom{q[4], q[5], q[6], q[7], q[8], q[9], q[10], q[11], q[12], q[13], q[14], q[15], q[1]};
}
MRT_DFN void cornell_take1(CornellRoom& d) {
#if defined(__HIP_DEVICE_COMPILE__)
    asm volatile("" : "+s"(d.lo0), "+s"(d.lo1), "+s"(d.lo2), "+s"(d.hi0), "+s"(d.hi1), "+s"(d.hi2), "+s"(d.mask));
    asm volatile("" : "+s"(d.m0), "+s"(d.m1), "+s"(d.m2), "+s"(d.m3), "+s"(d.m4), "+s"(d.m5));
#else
    (void)d;
#endif
}
// The room's walls (ops 1, 2, 4, 5, 6) as one slab test: a ray that meets the box leaves it
// through the face of its smallest far-plane distance; that face, if the room has it, is the
// wall hit (front-facing: the walls face inward; any face the ray crosses going in is back-facing
// and missed, rect.cpp:26-30).  Differs from the five rect tests by rounding at the room's edges.
// (kRec false: the caller reads only the hit's code, distance and side -- room_walls_op -- so the
// face's plane and material are not selected: sel3's asm would keep the dead selects alive)
template <uint32_t F, bool kRec = true>
MRT_DFN void cornell_room(const CornellRoom& d, const Ray& r, float tmin, CornellRec& w) {
    const float lo0 = __uint_as_float(d.lo0), lo1 = __uint_as_float(d.lo1), lo2 = __uint_as_float(d.lo2);
    const float hi0 = __uint_as_float(d.hi0), hi1 = __uint_as_float(d.hi1), hi2 = __uint_as_float(d.hi2);
    const float t0x = (lo0 - r.o.x) * r.inv.x, t1x = (hi0 - r.o.x) * r.inv.x;
    const float t0y = (lo1 - r.o.y) * r.inv.y, t1y = (hi1 - r.o.y) * r.inv.y;
    const float t0z = (lo2 - r.o.z) * r.inv.z, t1z = (hi2 - r.o.z) * r.inv.z;
    const float fx = fmaxf(t0x, t1x), fy = fmaxf(t0y, t1y), fz = fmaxf(t0z, t1z);
    const float tn = fmaxf(fmaxf(fminf(t0x, t1x), fminf(t0y, t1y)), fminf(t0z, t1z));
    const float tf = fminf(fminf(fx, fy), fz);
    // the exit face: its axis (ties to the later axis: z, then y, as the later rects win), and its
    // side (the max plane when the ray goes up that axis)
    const uint32_t a = tf == fz ? 2u : (tf == fy ? 1u : 0u);
    const float da = sel3(a, r.d.x, r.d.y, r.d.z);
    const uint32_t side = da > 0.0f ? 1u : 0u;
    const uint32_t face = a * 2u + side;
    const bool h = (tn <= tf) & (((d.mask >> face) & 1u) != 0u) & (tf >= tmin) & (tf <= w.closest);
    // plane and material of the face by selects (a chain of compares with one index became a
    // per-lane lookup table in scratch memory)
    w.closest = h ? tf : w.closest;
    w.code = h ? 1u + a : w.code;
    w.ns = h ? (side ? -1.0f : 1.0f) : w.ns;
    if constexpr (kRec) {
        const bool up = side != 0u;
        const float k = up ? sel3(a, hi0, hi1, hi2) : sel3(a, lo0, lo1, lo2);
        const uint32_t m = __float_as_uint(up ? sel3(a, __uint_as_float(d.m1), __uint_as_float(d.m3), __uint_as_float(d.m5))
                                              : sel3(a, __uint_as_float(d.m0), __uint_as_float(d.m2), __uint_as_float(d.m4)));
        w.k = h ? k : w.k;
        w.mat = h ? m : w.mat;
    }
}
// The room + mesh walk's walls (scenes 8 / 9, tolerance build): the room's slab test as above,
// the hit face's op index as the hit op (the record is then derived op by op, SigWalk::derive)
MRT_DFN void room_walls_op(const MRT_CONST_AS LinOp& e, const Ray& r, float tmin, SigState& w) {
    CornellRoom d = cornell_load_room(e);
    uint32_t face_ops = e.skip;
#if defined(__HIP_DEVICE_COMPILE__)
    asm volatile("" : "+s"(face_ops));
#endif
    cornell_take1(d);
    CornellRec c{w.closest, 0.0f, 0.0f, 0u, 0u};
    cornell_room<0u, false>(d, r, tmin, c);
    if (c.code != 0u) {  // per lane: the exit face's axis from the code, its side from the sign
        const uint32_t face = (c.code - 1u) * 2u + (c.ns < 0.0f ? 1u : 0u);
        w.closest = c.closest;
        w.hnode = (face_ops >> (4u * face)) & 15u;
        w.hinst = MRT_NONE;
        w.hdone = false;
    }
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
    // the room's walls as one slab test (ops 1, 2, 4, 5, 6; cornell_room_fill), then the light
    // (op 3), the box and the sphere: their words in two batches of scalar loads
    static_assert(G.op[G.n - 1] == LOP_END, "the room is kept in the END op");
    CornellRoom dr = cornell_load_room(prog[G.n - 1]);
    CornellRect d3 = cornell_load(prog[3]);
    cornell_take(dr, d3);
    cornell_room<F>(dr, r, tmin, w);
    cornell_rect<F, 3>(d3, r, tmin, w);
    CornellBox db = cornell_load_box(prog[7], prog[8]);
    CornellSphere dsp = cornell_load_sphere(prog[17]);
    cornell_take(db, dsp);
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
    const float bd = sel3(bax, dx, r.d.y, dz);
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
    // the instance-frame ray of a hit inside an instance: recomputed from the query ray (inst_ray,
    // the walk's own operations; no longer parked in LDS at the hit)
    auto inst_ray_of = [&](Ray ir) -> Ray {
        constexpr uint32_t IPC = SigWalk<F, SIG>::only_inst();
        const Ray ci = IPC != MRT_NONE ? inst_ray<MRT_FAST_UNIT>(prog[IPC == MRT_NONE ? 0 : IPC], r) : inst_ray<MRT_FAST_UNIT>(S.prog[w.hinst], r);
        ir.o = ci.o;
        ir.d = ci.d;
        return ir;
    };
    if constexpr (SigWalk<F, SIG>::kDerive) {
        Ray ir = r;
        if (INST && any_lane(w.hinst != MRT_NONE && !w.hdone) && w.hinst != MRT_NONE) ir = inst_ray_of(ir);
        if (!w.hdone) SigWalk<F, SIG>::template derive<0>(prog, w, r, ir, rec);
        if (INST && w.hinst != MRT_NONE) {
            constexpr uint32_t IPC = SigWalk<F, SIG>::only_inst();
            if constexpr (IPC != MRT_NONE) lin_untransform(prog[IPC], rec);
            else lin_untransform(S.prog[w.hinst], rec);
        }
    } else {
        const uint32_t node = w.hnode;
        if (INST && w.hinst != MRT_NONE) {
            if (!w.hdone) lin_prim_rec<F>(S, node, inst_ray_of(r), w.closest, rec);
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
