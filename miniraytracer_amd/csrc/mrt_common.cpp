// mrt_common.cpp -- host side of the C-ABI that needs no GPU: parameters (MRT_Params /
// ParseArgv), the work_queue tile order, the per-rank pixel ownership, the Drago tone map and
// error reporting.
#include <dlfcn.h>

#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <limits>
#include <new>
#include <string>
#include <vector>

#include "mrt_internal.h"
#include "../../include/mrt_tonemap.h"

static thread_local std::string g_last_error;

mrt_status mrt_internal_fail(mrt_status s, const char* msg) {
    g_last_error = msg ? msg : "";
    return s;
}

std::string mrt_internal_package_dir() {
    Dl_info info;
    if (dladdr((void*)&mrt_internal_package_dir, &info) && info.dli_fname) {
        std::string p = info.dli_fname;
        size_t k = p.rfind('/');
        if (k != std::string::npos) return p.substr(0, k);
    }
    return ".";
}

extern "C" const char* mrt_last_error(void) { return g_last_error.c_str(); }

extern "C" uint32_t mrt_abi_version(void) { return MRT_ABI_VERSION; }

extern "C" const char* mrt_strerror(mrt_status s) {
    switch (s) {
    case MRT_OK: return "ok";
    case MRT_ERR_INVALID: return "invalid argument";
    case MRT_ERR_NO_DEVICE: return "no gfx950 device";
    case MRT_ERR_HIP: return "HIP runtime error";
    case MRT_ERR_OOM: return "out of device memory";
    case MRT_ERR_IO: return "asset not found";
    case MRT_ERR_CANCELLED: return "cancelled";
    }
    return "unknown";
}

// MRT_Params defaults (cmdline_parser.h:5-18)
extern "C" void mrt_default_params(mrt_params* p) {
    memset(p, 0, sizeof *p);
    p->window_width = 500;
    p->window_height = 500;
    p->buffer_width = 500;
    p->buffer_height = 500;
    p->samples_per_pixel = 128;
    p->tile_size = 32;
    p->num_threads = 0;
    p->max_bounces = 32;
    p->scene_select = 8;  // SCENE_TRIANGLES
    p->threading_mode = 1;
    p->max_luminance = 1000;
    p->delay = 0;
    p->seed = 11350390909718046443ull;  // main.cpp:302
    p->gpus = 0;
    p->numerics = 1;  // tolerance contract (DESIGN.md "Numerics contracts"); -numerics exact for bit-exact
    p->backend = 0;
    p->order = 0;
}

// ReadParameter (cmdline_parser.cpp:41-62): first occurrence wins, value range-checked, a bad
// value prints the reference's warning and keeps the default.
template <typename T>
static int read_param(int argc, char** argv, const char* name, T* res, T lo, T hi);
template <>
int read_param<uint32_t>(int argc, char** argv, const char* name, uint32_t* res, uint32_t lo, uint32_t hi) {
    for (int i = 1; i < argc; i++) {
        if (strcmp(name, argv[i]) == 0) {
            if (i + 1 == argc) {
                printf("Warning: Missing value for parameter '%s'.\n", name);
                return 0;
            }
            uint32_t v = (uint32_t)strtoul(argv[i + 1], nullptr, 0);
            if (v < lo || v > hi) {
                printf("Warning: Invalid value for parameter '%s', must be in [%u, %u].\n", name, lo, hi);
                return 0;
            }
            *res = v;
            return i;
        }
    }
    return 0;
}
template <>
int read_param<float>(int argc, char** argv, const char* name, float* res, float lo, float hi) {
    for (int i = 1; i < argc; i++) {
        if (strcmp(name, argv[i]) == 0) {
            if (i + 1 == argc) {
                printf("Warning: Missing value for parameter '%s'.\n", name);
                return 0;
            }
            float v = strtof(argv[i + 1], nullptr);
            if (v < lo || v > hi) {
                printf("Warning: Invalid value for parameter '%s', must be in [%g, %g].\n", name, lo, hi);
                return 0;
            }
            *res = v;
            return i;
        }
    }
    return 0;
}
static int check_param(int argc, char** argv, const char* name) {
    for (int i = 1; i < argc; i++)
        if (strcmp(name, argv[i]) == 0) return i;
    return 0;
}

extern "C" mrt_status mrt_parse_argv(int argc, char** argv, mrt_params* out) {
    mrt_params p;
    mrt_default_params(&p);
    if (check_param(argc, argv, "-help") || check_param(argc, argv, "--help") || check_param(argc, argv, "-?")) {
        printf("\nPARAMETERS:\n"
               "  -width    \t<value>\t\tWindow width\n"
               "  -height   \t<value>\t\tWindow height\n"
               "  -samples  \t<value>\t\tSamples per pixel\n"
               "  -depth    \t<value>\t\tMaximum bounce depth per primary ray\n"
               "  -maxlum   \t<value>\t\tClamp maximum luminance (introduces bias)\n"
               "  -threads  \t<value>\t\tNumber of CPU threads (0 selects all; CPU backend only)\n"
               "  -backend  \t[gpu, cpu]\tRender on the MI355X(s) (default) or on the host CPU\n"
               "            \t\t\t(the same hot-path code, exact numerics, -threads workers)\n"
               "  -gpus     \t<value>\t\tNumber of GPUs to shard tiles over (0 selects all)\n"
               "  -order    \t[ref, path]\tRNG order: ref = the reference's (one stream per worker thread,\n"
               "            \t\t\twork_queue order; CPU backend default: -threads 1 reproduces the\n"
               "            \t\t\treference's deterministic run), path = per-path stream keys (GPU)\n"
               "  -numerics \t[exact, fast]\tArithmetic contract (exact: bit-for-bit the reference built\n"
               "            \t\t\twithout contraction; fast: per-pixel RMSE < 1e-3, default)\n"
               "  -tilesize \t<value>\t\tSize of image tiles (GPUs own interleaved tiles)\n"
               "  -mode     \t[0, 1]\t\tAccumulation mode (0 per-pixel mean, 1 progressive average)\n"
               "  -scene    \t[0, 9]\t\tSelect the scene (9 = wt_teapot in the Cornell box)\n"
               "  -seed     \t<value>\t\tPath stream-key seed\n"
               "  -gather   \t[rccl, host]\tMulti-GPU frame assembly: one RCCL gather to GPU 0 (default\n"
               "            \t\t\twhen every rank has its own GPU) or per-rank host copies\n"
               "  -o        \t<file>\t\tOutput image (.pfm linear, .ppm tone-mapped)\n"
               "  -delay    \t\t\tAccepted for compatibility (no window)\n");
        if (out) *out = p;
        return mrt_internal_fail(MRT_ERR_INVALID, "help");
    }
    const uint32_t UMAX = std::numeric_limits<uint32_t>::max();
    if (read_param<uint32_t>(argc, argv, "-width", &p.window_width, 1u, UMAX)) p.buffer_width = p.window_width;
    if (read_param<uint32_t>(argc, argv, "-height", &p.window_height, 1u, UMAX)) p.buffer_height = p.window_height;
    read_param<uint32_t>(argc, argv, "-samples", &p.samples_per_pixel, 1u, UMAX);
    read_param<uint32_t>(argc, argv, "-tilesize", &p.tile_size, 1u, UMAX);
    read_param<uint32_t>(argc, argv, "-threads", &p.num_threads, 0u, UMAX);
    read_param<uint32_t>(argc, argv, "-depth", &p.max_bounces, 0u, UMAX);
    read_param<uint32_t>(argc, argv, "-scene", &p.scene_select, 0u, 9u);
    read_param<uint32_t>(argc, argv, "-mode", &p.threading_mode, 0u, 1u);
    read_param<float>(argc, argv, "-maxlum", &p.max_luminance, std::numeric_limits<float>::min(), std::numeric_limits<float>::max());
    if (int i = check_param(argc, argv, "-seed"))
        if (i + 1 < argc) p.seed = strtoull(argv[i + 1], nullptr, 0);
    if (check_param(argc, argv, "-delay")) p.delay = 1;
    read_param<uint32_t>(argc, argv, "-gpus", &p.gpus, 0u, UMAX);
    if (int i = check_param(argc, argv, "-numerics")) {
        const char* v = i + 1 < argc ? argv[i + 1] : "";
        if (!strcmp(v, "exact") || !strcmp(v, "0")) p.numerics = 0;
        else if (!strcmp(v, "fast") || !strcmp(v, "1")) p.numerics = 1;
        else printf("Warning: Invalid value for parameter '-numerics', must be exact or fast.\n");
    }
    if (int i = check_param(argc, argv, "-backend")) {
        const char* v = i + 1 < argc ? argv[i + 1] : "";
        if (!strcmp(v, "gpu")) p.backend = 0;
        else if (!strcmp(v, "cpu")) p.backend = 1;
        else printf("Warning: Invalid value for parameter '-backend', must be gpu or cpu.\n");
    }
    if (p.backend == 1) p.numerics = 0;  // the CPU backend runs the exact contract
    p.order = p.backend == 1 ? 1u : 0u;  // the reference's own RNG order where it can run
    if (int i = check_param(argc, argv, "-order")) {
        const char* v = i + 1 < argc ? argv[i + 1] : "";
        if (!strcmp(v, "ref")) p.order = 1;
        else if (!strcmp(v, "path")) p.order = 0;
        else printf("Warning: Invalid value for parameter '-order', must be ref or path.\n");
    }
    if (out) *out = p;
    return MRT_OK;
}

extern "C" void mrt_default_render_desc(const mrt_params* p, mrt_render_desc* d) {
    memset(d, 0, sizeof *d);
    d->width = p->buffer_width;
    d->height = p->buffer_height;
    d->sqrt_samples = (uint32_t)std::sqrt((float)p->samples_per_pixel);  // main.cpp:319
    d->max_bounces = p->max_bounces;
    d->max_luminance = p->max_luminance;
    d->mode = p->threading_mode;
    d->seed = p->seed;
    d->tile_size = p->tile_size;
    d->rank = 0;
    d->world = 1;
    d->flags = (p->numerics ? MRT_RF_FAST : 0u) | (p->order == 1 ? MRT_RF_REF_ORDER : 0u);
    d->threads = p->num_threads;
}

// ---- work_queue tile order (work_queue.cpp:6-128) ----
static void hil_rot(uint32_t n, uint32_t* x, uint32_t* y, uint32_t rx, uint32_t ry) {
    if (ry == 0) {
        if (rx == 1) {
            *x = n - 1 - *x;
            *y = n - 1 - *y;
        }
        std::swap(*x, *y);
    }
}
static void hilbert_d2xy(uint32_t n, uint32_t d, uint32_t* x, uint32_t* y) {
    uint32_t rx, ry, s, t = d;
    *x = *y = 0;
    for (s = 1; s < n; s *= 2) {
        rx = 1 & (t / 2);
        ry = 1 & (t ^ rx);
        hil_rot(s, x, y, rx, ry);
        *x += s * rx;
        *y += s * ry;
        t /= 4;
    }
}
static uint32_t reverse_u32(uint32_t v) {
    v = ((v >> 1) & 0x55555555u) | ((v & 0x55555555u) << 1);
    v = ((v >> 2) & 0x33333333u) | ((v & 0x33333333u) << 2);
    v = ((v >> 4) & 0x0F0F0F0Fu) | ((v & 0x0F0F0F0Fu) << 4);
    v = ((v >> 8) & 0x00FF00FFu) | ((v & 0x00FF00FFu) << 8);
    return (v >> 16) | (v << 16);
}

std::vector<mrt_tile> mrt_internal_tiles(uint32_t W, uint32_t H, uint32_t ts) {
    uint32_t xc = (W + (ts - 1u)) / ts, yc = (H + (ts - 1u)) / ts;
    std::vector<mrt_tile> rm((size_t)xc * yc), out;
    for (uint32_t y = 0; y < yc; y++)
        for (uint32_t x = 0; x < xc; x++)
            rm[x + y * xc] = mrt_tile{x * ts, std::min(x * ts + ts, W), y * ts, std::min(y * ts + ts, H)};
    uint32_t m = std::max(xc, yc), po2 = m - 1;  // nextPo2 (mrt_math.h:49-58)
    po2 |= po2 >> 1; po2 |= po2 >> 2; po2 |= po2 >> 4; po2 |= po2 >> 8; po2 |= po2 >> 16;
    po2++;
    uint32_t log2size = po2 ? 31u - (uint32_t)__builtin_clz(po2) : 0u;
    out.reserve(rm.size());
    for (uint64_t d = 0; d < (uint64_t)po2 * po2; d++) {
        uint32_t x, y;
        hilbert_d2xy(po2, (uint32_t)d, &x, &y);
        // x86 masks a shift count of 32 to 0 (single-tile case, log2size == 0: x = y = 0)
        x = log2size ? reverse_u32(x) >> (32u - log2size) : reverse_u32(x);
        y = log2size ? reverse_u32(y) >> (32u - log2size) : reverse_u32(y);
        if (x < xc && y < yc) out.push_back(rm[x + y * xc]);
        if (out.size() == rm.size()) break;
    }
    return out;
}

// Tile k of the work_queue order -> its rank.  The tiles are dealt in rounds of `world` consecutive
// tiles; round b goes to the ranks in the order of its own permutation (Fisher-Yates, draws
// splitmix64^i(b)).  Dealing every round in rank order (k % world) gave one rank the same position of
// every small Hilbert block, a systematic share: on the Cornell box at 8 ranks up to 2.8% more rays
// than the mean rank (per-tile ray counts); permuted rounds leave the statistical spread.
static uint64_t owner_mix(uint64_t z) {
    z += 0x9E3779B97F4A7C15ull;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}
std::vector<uint32_t> mrt_internal_tile_owners(size_t ntiles, uint32_t world) {
    std::vector<uint32_t> own(ntiles, 0u), perm(world);
    if (world <= 1) return own;
    for (size_t b = 0; b * world < ntiles; b++) {
        for (uint32_t i = 0; i < world; i++) perm[i] = i;
        uint64_t st = b;
        for (uint32_t i = world - 1; i > 0; i--) {
            st = owner_mix(st);
            std::swap(perm[i], perm[st % (i + 1u)]);
        }
        for (uint32_t j = 0; j < world && b * world + j < ntiles; j++) own[b * world + j] = perm[j];
    }
    return own;
}

std::vector<mrt_tile> mrt_internal_render_tiles(const mrt_render_desc* d) {
    std::vector<mrt_tile> out;
    if (d->pixels) {  // a pixel list: one 1x1 "tile" per listed pixel, in list order
        out.reserve(d->n_pixels);
        for (uint32_t i = 0; i < d->n_pixels; i++) {
            const uint32_t x = d->pixels[i] % d->width, y = d->pixels[i] / d->width;
            out.push_back(mrt_tile{x, x + 1u, y, y + 1u});
        }
        return out;
    }
    const std::vector<mrt_tile> all = mrt_internal_tiles(d->width, d->height, d->tile_size ? d->tile_size : 32u);
    const std::vector<uint32_t> own = mrt_internal_tile_owners(all.size(), d->world ? d->world : 1u);
    for (size_t k = 0; k < all.size(); k++)
        if (own[k] == d->rank) out.push_back(all[k]);
    return out;
}

std::vector<uint32_t> mrt_internal_local_pixels(const mrt_render_desc* d) {
    if (d->pixels) return std::vector<uint32_t>(d->pixels, d->pixels + d->n_pixels);
    std::vector<uint32_t> px;
    for (const mrt_tile& t : mrt_internal_render_tiles(d))
        for (uint32_t y = t.ymin; y < t.ymax; y++)
            for (uint32_t x = t.xmin; x < t.xmax; x++) px.push_back(x + y * d->width);
    return px;
}

mrt_status mrt_internal_check_pixels(const mrt_render_desc* d) {
    // unknown flag bits fail instead of meaning something else (0x20 was MRT_RF_SPLIT until ABI 5)
    if (d->flags & ~MRT_RF_ALL)
        return mrt_internal_fail(MRT_ERR_INVALID, (d->flags & 0x20u) ? "render desc: flag 0x20 (the removed MRT_RF_SPLIT; MRT_RF_FOLD_ASYNC is 0x40 since ABI 6)"
                                                                      : "render desc: unknown flag bits");
    if (!d->pixels) return MRT_OK;
    if (d->n_pixels == 0) return mrt_internal_fail(MRT_ERR_INVALID, "render desc: empty pixel list");
    const uint64_t wh = (uint64_t)d->width * d->height;
    // pixel indices are 32-bit: a pixel-list render of a larger image cannot address its pixels
    if (wh > (1ull << 32)) return mrt_internal_fail(MRT_ERR_INVALID, "render desc: pixel list on an image above 2^32 pixels");
    for (uint32_t i = 0; i < d->n_pixels; i++)
        if (d->pixels[i] >= wh) return mrt_internal_fail(MRT_ERR_INVALID, "render desc: pixel index outside the image");
    // duplicates: sorted copy of the list (O(n log n) in the list, not the image), no throw across the ABI
    try {
        std::vector<uint32_t> v(d->pixels, d->pixels + d->n_pixels);
        std::sort(v.begin(), v.end());
        if (std::adjacent_find(v.begin(), v.end()) != v.end()) return mrt_internal_fail(MRT_ERR_INVALID, "render desc: pixel listed twice");
    } catch (const std::bad_alloc&) {
        return mrt_internal_fail(MRT_ERR_OOM, "render desc: pixel list check out of memory");
    }
    return MRT_OK;
}

extern "C" mrt_status mrt_local_pixels(const mrt_render_desc* d, uint32_t* n_out, uint32_t* pixels_out) {
    if (!d || !n_out || d->width == 0 || d->height == 0 || (d->world && d->rank >= d->world))
        return mrt_internal_fail(MRT_ERR_INVALID, "mrt_local_pixels: bad desc");
    if (mrt_status st = mrt_internal_check_pixels(d)) return st;
    std::vector<uint32_t> px = mrt_internal_local_pixels(d);
    *n_out = (uint32_t)px.size();
    if (pixels_out) memcpy(pixels_out, px.data(), px.size() * 4);
    return MRT_OK;
}

// ---- Drago adaptive logarithmic tone map + ARGB32 (main.cpp:416-444, vec3.h:275-279, 327-333) ----

// Drago adaptive logarithmic mapping (main.cpp:416-444) on the host; include/mrt_tonemap.h
extern "C" mrt_status mrt_tonemap_argb(const float* rgb, uint32_t W, uint32_t H, uint32_t* argb) {
    if (!rgb || !argb) return mrt_internal_fail(MRT_ERR_INVALID, "tonemap: null");
    size_t n = (size_t)W * H;
    float L_wmax = 0;
    for (size_t i = 0; i < n; i++) {
        float l = mrt_luminance(rgb + i * 4);
        L_wmax = (L_wmax < l) ? l : L_wmax;  // std::max
    }
    mrt_tonemap_params tp;
    mrt_tonemap_setup(L_wmax, &tp);
    for (size_t i = 0; i < n; i++) argb[i] = mrt_tonemap_pixel(&tp, rgb + i * 4);
    return MRT_OK;
}
