// mrt_resume.h -- scene_object::hit for linear hit programs with bvh_node subtrees (the random
// spheres of C1, book2's final scene of C5), RESUMABLE: each lane carries its own position in the
// program and in the BVH walk across iterations of the persistent path loop.
//
// scene_hit_lin (mrt_lin.h) walks the program in lockstep: at a LOP_BVHW op every lane runs
// bvhw_hit to completion, and a wave waits for its longest walk (measured lane utilisation 0.24
// on book2, 52% of wave time in the walk).  Here a lane's intersection is a state machine:
//
//   RS_SWEEP  at op `pc`: the wave sweeps the program once per iteration (op index uniform, scalar
//             loads as in scene_hit_lin); lanes whose pc is the swept op execute it, the others wait
//             for their op to come round.  Reaching a BVHW op whose root box it hits, a lane
//             leaves the sweep and walks (RS_WALK); reaching the END op, it is RS_DONE.
//   RS_WALK   one bvh_node subtree walk (bvhw_hit's while-while: descend to a leaf, test it; the
//             first leaf that hits ends the walk), its position (node ref, LDS stack) kept per lane.
//             The walk loop hands the wave back once few lanes still walk and enough others can
//             sweep, shade or start paths; the stragglers resume next iteration beside them
//             (the pattern of the resumable mesh walk, mrt_kernels.hip).
//   RS_DONE   the closest hit's record is derived and the hit shaded (shade_hit).
//
// Every lane performs scene_hit_lin's operations on its own ray in scene_hit_lin's order (the
// volumes' RNG draws included), so the results are bit-identical (tests/test_gpu_parity.py; the
// CPU backend, which runs scene_hit_lin, is the cross-check).
#pragma once
#include "mrt_shade.h"

namespace mrtd {

enum : uint32_t { RS_IDLE = 0, RS_SWEEP = 1, RS_WALK = 2, RS_DONE = 3 };

struct ResumeState {
    Ray cur;         // the query ray in the frame of the current op (an instance's frame inside it)
    float closest;
    uint32_t pc;     // RS_SWEEP: the next op; RS_WALK: the BVHW op being walked
    uint32_t act;    // bit l: the lane takes part at nesting level l
    uint32_t hnode;  // node of the closest hit so far (MRT_NONE: none)
    uint32_t hinst;  // op index of the instance it lies in (MRT_NONE: world frame)
    uint32_t ref, sp;  // RS_WALK: the walk's current node / leaf ref and LDS stack depth
    uint32_t st;
    bool hdone;      // rec already holds the closest hit (a BVH leaf or mesh wrote it)
};

// A new trace() segment for ps.r (main.cpp:66-71: tmin 0.001, tmax FLT_MAX): the query ray is
// parked in LDS (instance ops and the shading reload it), the sweep starts at op 0.
MRT_DFN void rs_begin(ResumeState& w, const Ray& r, const LStack& L) {
    lin_save_ray(L, r);
    w.cur = r;
    w.closest = FLT_MAX_;
    w.pc = 0;
    w.act = 1u;
    w.hnode = MRT_NONE;
    w.hinst = MRT_NONE;
    w.hdone = false;
    w.st = RS_SWEEP;
}

// One step of a lane's bvh_node walk (bvhw_hit, mrt_trace.h; scene_object.h:208-244): descend
// through inner nodes to a leaf (closer child first by node_order & dirMask, a farther child whose
// box was hit pushed), then test the leaf.  Returns 0: keep walking, 1: the leaf hit (rec written;
// the walk is over: first-hit early-out), 2: the walk found nothing.
template <uint32_t F>
MRT_DFN uint32_t bvhw_step(const DScene& S, ResumeState& w, HitRec& rec, const LStack& L, float tmin) {
    while (!(w.ref & BVHW_LEAF)) {
        const WideNode W = wide_at<TreeOf<F>::on>(S.bwide, w.ref, L);
        const bool hl = !(W.flags & 1u) || aabb_hit(W.lmin, W.lmax, w.cur, tmin, w.closest);
        const bool hr = !(W.flags & 2u) || aabb_hit(W.rmin, W.rmax, w.cur, tmin, w.closest);
        const bool left_first = (W.order & w.cur.mask) != 0;
        const uint32_t cref = left_first ? W.lref : W.rref, fref = left_first ? W.rref : W.lref;
        const bool hc = left_first ? hl : hr, hf = left_first ? hr : hl;
        if (hc) {
            if (hf && fref != cref) L.mesh[(w.sp++) * 64 + L.lane] = fref;  // n == 1: left == right, a repeat misses again
            w.ref = cref;
        } else if (hf) {
            w.ref = fref;
        } else {
            if (w.sp == 0) return 2u;
            w.ref = L.mesh[(--w.sp) * 64 + L.lane];
        }
    }
    if (bvhw_leaf<F>(S, w.ref, w.cur, tmin, w.closest, rec, true)) return 1u;
    if (w.sp == 0) return 2u;
    w.ref = L.mesh[(--w.sp) * 64 + L.lane];
    return 0u;
}

// A finished walk: a hit becomes the closest so far (in the frame of the op's instance, if any);
// the lane continues the sweep after the op.
template <uint32_t F>
MRT_DFN void rs_walk_end(const DScene& S, ResumeState& w, const HitRec& rec, uint32_t res) {
    if (res == 1u) {
        // the walked op's node and enclosing instance: per lane (lanes walk different ops)
        const LinOp* o = S.prog + w.pc;
        w.closest = rec.t;
        w.hnode = o->node;
        w.hinst = LOP_INST_OF(*o);
        w.hdone = true;
    }
    w.pc += 1u;
    w.st = RS_SWEEP;
}

// One sweep over the program for the lanes in RS_SWEEP (scene_hit_lin's ops, mrt_lin.h, lane by
// lane from each one's pc): afterwards every such lane is walking a BVHW op or done.
template <uint32_t F>
MRT_DFN void rs_sweep(const DScene& S, ResumeState& w, HitRec& rec, const LStack& L, Pcg& rng, float tmin) {
    constexpr bool INST = (F & FT_INST) != 0;
    const MRT_CONST_AS LinOp* prog = const_ptr(S.prog);
    for (uint32_t pc = 0;;) {
        const bool sweeping = w.st == RS_SWEEP;
        if (!any_lane(sweeping)) return;
        const MRT_CONST_AS LinOp& o = prog[pc];
        const uint32_t op = LOP_OP(o);
        const bool here = sweeping & (w.pc == pc);
        if (op == LOP_END) {  // every sweeping lane is here now
            if (here) w.st = RS_DONE;
            return;
        }
        if (!any_lane(here)) {
            pc += op == LOP_VOLUME ? 2u : 1u;
            continue;
        }
        const uint32_t lvl = LOP_LVL(o);
        const bool on = here & (((w.act >> lvl) & 1u) != 0);
        uint32_t next = pc + 1u;
        if (op == LOP_PRIM) {
            float t;
            bool h;
            switch (LOP_KIND(o)) {  // uniform: a scalar branch
            case MRT_K_SPHERE: h = lin_prim_t<F, MRT_K_SPHERE>(o, w.cur, tmin, w.closest, &t); break;
            case MRT_K_XY: h = lin_prim_t<F, MRT_K_XY>(o, w.cur, tmin, w.closest, &t); break;
            case MRT_K_XZ: h = lin_prim_t<F, MRT_K_XZ>(o, w.cur, tmin, w.closest, &t); break;
            default: h = lin_prim_t<F, MRT_K_YZ>(o, w.cur, tmin, w.closest, &t); break;
            }
            h = h & on;
            w.closest = h ? t : w.closest;
            w.hnode = h ? o.node : w.hnode;
            w.hinst = h ? LOP_INST_OF(o) : w.hinst;
            w.hdone = h ? false : w.hdone;
        } else if ((F & FT_BVHW) && op == LOP_BVHW) {
            // bvhw_hit's root box (scene_object.h:211); a lane that enters walks from the root
            if (on && aabb_hit(f3{o.f[0], o.f[1], o.f[2]}, f3{o.f[3], o.f[4], o.f[5]}, w.cur, tmin, w.closest)) {
                w.st = RS_WALK;
                w.ref = o.skip;
                w.sp = 0;
            }
        } else if ((F & FT_MESH) && op == LOP_MESH) {
            if (on && mesh_hit<true>(S, ld_node(const_ptr(S.nodes) + o.node), w.cur, tmin, w.closest, rec, true, L)) {
                w.closest = rec.t;
                w.hnode = o.node;
                w.hinst = LOP_INST_OF(o);
                w.hdone = true;
            }
        } else if ((F & FT_VOLUME) && op == LOP_VOLUME) {
            // constant_volume::hit (volumes.cpp:5-35), as scene_hit_lin
            const MRT_CONST_AS LinOp& bo = prog[pc + 1];
            float t1, t2;
            bool h1, h2;
            if (LOP_KIND(bo) == MRT_K_SPHERE) {
                h1 = lin_prim_t<F, MRT_K_SPHERE>(bo, w.cur, -FLT_MAX_, FLT_MAX_, &t1);
                h2 = lin_prim_t<F, MRT_K_SPHERE>(bo, w.cur, t1 + 0.0001f, FLT_MAX_, &t2);
            } else if (LOP_KIND(bo) == MRT_K_XY) {
                h1 = lin_prim_t<F, MRT_K_XY>(bo, w.cur, -FLT_MAX_, FLT_MAX_, &t1);
                h2 = lin_prim_t<F, MRT_K_XY>(bo, w.cur, t1 + 0.0001f, FLT_MAX_, &t2);
            } else if (LOP_KIND(bo) == MRT_K_XZ) {
                h1 = lin_prim_t<F, MRT_K_XZ>(bo, w.cur, -FLT_MAX_, FLT_MAX_, &t1);
                h2 = lin_prim_t<F, MRT_K_XZ>(bo, w.cur, t1 + 0.0001f, FLT_MAX_, &t2);
            } else {
                h1 = lin_prim_t<F, MRT_K_YZ>(bo, w.cur, -FLT_MAX_, FLT_MAX_, &t1);
                h2 = lin_prim_t<F, MRT_K_YZ>(bo, w.cur, t1 + 0.0001f, FLT_MAX_, &t2);
            }
            if (on && h1 && h2) {
                float a = t1 < tmin ? tmin : t1;
                const float b = t2 > w.closest ? w.closest : t2;
                if (a < b) {
                    if (a < 0) a = 0;
                    const float inside_dist = b - a;
                    const float hit_dist = -(1 / o.f[0]) * log_(randf(rng));
                    if (hit_dist < inside_dist) {
                        w.closest = a + hit_dist;
                        rec.t = w.closest;
                        rec.p = eval(w.cur, w.closest);
                        rec.n = f3{1, 0, 0};
                        rec.mat = o.mat;
                        w.hnode = o.node;
                        w.hinst = LOP_INST_OF(o);
                        w.hdone = true;
                    }
                }
            }
            next = pc + 2u;  // past the boundary op
        } else if (op == LOP_LIST) {  // object_list::hit box reject (scene_object.h:83)
            bool in = on;
            if (in && (LOP_FLAGS(o) & MRT_F_HASBOX)) in = lin_box(o, w.cur, tmin, w.closest);
            if (here) {
                w.act = (w.act & ~(2u << lvl)) | ((uint32_t)in << (lvl + 1u));
                next = in ? pc + 1u : o.skip;  // a lane that did not enter goes to the list's end
            }
        } else if (INST && op == LOP_INST) {
            const uint32_t kind = LOP_KIND(o);
            bool in = on;
            const Ray r0 = lin_load_ray(L);
            Ray c = r0;
            if (kind == MRT_K_TRROTY) {  // translate::hit then rotate_y::hit (scene_object.cpp:9-18, 70-98)
                c = moved_ray<kFastUnit<F>>(r0, sub(r0.o, f3{o.f[8], o.f[9], o.f[10]}));
                if (in && (LOP_FLAGS(o) & MRT_F_HASBOX)) in = lin_box(o, c, tmin, w.closest);
            } else if (kind == MRT_K_ROTY) {
                if (in && (LOP_FLAGS(o) & MRT_F_HASBOX)) in = lin_box(o, c, tmin, w.closest);
            }
            if (kind == MRT_K_TRROTY || kind == MRT_K_ROTY) c = rotate_ray<kFastUnit<F>>(c, o.f[6], o.f[7]);
            else c = moved_ray<kFastUnit<F>>(r0, sub(r0.o, f3{o.f[0], o.f[1], o.f[2]}));
            if (here) {
                w.act = (w.act & ~(2u << lvl)) | ((uint32_t)in << (lvl + 1u));
                if (in) w.cur = c;
                next = in ? pc + 1u : o.skip;
            }
        } else if (INST && op == LOP_INST_END) {
            if (here) {
                if (w.hinst == o.skip) {  // keep the instance-frame ray of the hit for the record
                    float* b = L.save + L.lane + 9 * 64;
                    b[0] = w.cur.o.x; b[64] = w.cur.o.y; b[128] = w.cur.o.z;
                    b[192] = w.cur.d.x; b[256] = w.cur.d.y; b[320] = w.cur.d.z;
                }
                w.cur = lin_load_ray(L);
            }
        }
        if (here && w.st == RS_SWEEP) w.pc = next;
        // the wave's next op: past the subtree of a list / instance that no sweeping lane needs
        if ((op == LOP_LIST || (INST && op == LOP_INST)) && !any_lane((w.st == RS_SWEEP) & (w.pc > pc) & (w.pc < o.skip)))
            pc = o.skip;
        else
            pc += op == LOP_VOLUME ? 2u : 1u;
    }
}

// RS_DONE: the query ray back from LDS and the closest hit's record (scene_hit_lin's tail:
// p / n / uv derived from the winning primitive in its own frame, then back to the world).
// Returns whether anything was hit.
template <uint32_t F>
MRT_DFN bool rs_finish_hit(const DScene& S, const ResumeState& w, Ray& r, HitRec& rec, const LStack& L) {
    constexpr bool INST = (F & FT_INST) != 0;
    r = lin_load_ray(L);
    if (w.hnode == MRT_NONE) return false;
    if (INST && w.hinst != MRT_NONE) {
        if (!w.hdone) {
            const float* b = L.save + L.lane + 9 * 64;
            Ray ir = r;
            ir.o = f3{b[0], b[64], b[128]};
            ir.d = f3{b[192], b[256], b[320]};
            lin_prim_rec<F>(S, w.hnode, ir, w.closest, rec);
        }
        lin_untransform(S.prog[w.hinst], rec);  // per-lane instance: vector loads
    } else if (!w.hdone) {
        lin_prim_rec<F>(S, w.hnode, r, w.closest, rec);
    }
    return true;
}

}  // namespace mrtd
