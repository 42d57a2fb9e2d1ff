// mrt_internal.h -- library-internal helpers shared by the host translation units.
#pragma once
#include <string>
#include <vector>
#include "../../include/mrt.h"

mrt_status mrt_internal_fail(mrt_status s, const char* msg);
std::string mrt_internal_package_dir();

// work_queue tile list in the reference order: row-major tiles re-ordered along the inverted
// Hilbert curve (work_queue.cpp:64-128).  Each entry: xMin, xMax, yMin, yMax.
struct mrt_tile {
    uint32_t xmin, xmax, ymin, ymax;
};
std::vector<mrt_tile> mrt_internal_tiles(uint32_t width, uint32_t height, uint32_t tile_size);
// The rank of each work_queue tile: rounds of `world` consecutive tiles, each dealt in the order of
// its own pseudo-random permutation of the ranks (mrt_common.cpp).
std::vector<uint32_t> mrt_internal_tile_owners(size_t ntiles, uint32_t world);
// Pixels (row-major index, row 0 = bottom) owned by `rank` of `world`: the tiles
// mrt_internal_tile_owners gives it, each scanned row by row (the order draw() visits them,
// main.cpp:148-149).
std::vector<uint32_t> mrt_internal_local_pixels(const mrt_render_desc* d);
// The work items of one render call: the rank's tiles in work_queue order, or (d->pixels) one 1x1
// tile per listed pixel in list order.
std::vector<mrt_tile> mrt_internal_render_tiles(const mrt_render_desc* d);
// d->pixels, if set, is non-empty, inside the image and free of repeats; d->flags has no unknown bits
mrt_status mrt_internal_check_pixels(const mrt_render_desc* d);
// the HIP device of a GPU-backend scene (MRT_DEVICE_CPU for the CPU backend)
int mrt_internal_scene_device(const mrt_scene* s);
