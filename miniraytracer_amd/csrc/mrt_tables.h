// mrt_tables.h -- the device-side scene tables, built on the host from a mrt_scene_view
// (mrt_render.hip) and used by both backends: the GPU uploads them to HBM (mrt_scene_upload), the
// CPU backend keeps them in host memory (mrt_cpu.hip) and walks them with the same hot-path code.
#pragma once
#include <vector>
#include "mrt_shade.h"
#include "mrt_internal.h"

struct SceneTables {
    std::vector<mrt_node> nodes;        // the view's nodes (+ NEEDUV / SLOWDIV flags, fused TRROTY, BVHW roots)
    std::vector<mrtd::MeshWide> wide;   // pod_bvh inner nodes, both child boxes inline
    std::vector<mrtd::BvhWide> bwide;   // bvh_node subtrees as wide nodes, breadth-first
    std::vector<mrt_node> bprims;       // their leaves' primitive runs
    std::vector<mrtd::DMat> dmats;      // materials (+ inline constant colour, dielectric quotients)
    std::vector<mrt_node> bleaf;        // leaves of scene.biased_objects
    uint32_t blist = 0, nbleaf = 1;
    std::vector<mrtd::LinOp> prog;      // linear hit program (empty + LOP_END when the graph has none)
    std::vector<mrtd::LinOp> prog_fast; // its tolerance-contract rewrite (lin_rewrite_fast: rooms, box.h lists)
    uint32_t prog_ops = 0;
    uint32_t features = 0;              // FT_* | FT_LIN | shape id (mrt_sig.h)
    int max_frames = 0, max_rays = 0, max_mesh = 0;  // deepest stacks of the scene graph
};
mrt_status mrt_internal_scene_tables(const mrt_scene_view* v, SceneTables* t);
