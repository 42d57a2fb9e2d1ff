// mrt_cpu.hip -- the CPU backend behind the same C-ABI ("the CPU backend exports
// the same ABI, so main is backend-agnostic", as draw/draw2 are interchangeable at main.cpp:347-354).
//
// One source, two backends: this translation unit is compiled for the HOST only
// (--offload-host-only, MRT_HOST_BACKEND) from the same hot-path headers the gfx950 path kernels
// are built from (mrt_device.h ... mrt_shade.h): the same hit walks (the linear-program
// interpreter or the generic machine), the same materials, pdfs and PCG streams, under the exact
// numerics contract (-ffp-contract=off, IEEE division / sqrt, the shared transcendentals of
// include/mrt_mathfn.h).  Its images are therefore bit-for-bit those of the GPU's exact contract
// and of the reference built exact (tests/test_cpu_backend.py).
//
// Selected explicitly -- mrt_scene_upload(MRT_DEVICE_CPU, ...) -- never as a fallback: the GPU
// entry points fail when no gfx950 device is visible.
//
// Work distribution is the reference's: worker threads pull work_queue tiles in inverted-Hilbert
// order (work_queue.cpp:64-166, one relaxed fetch_add per tile) and render each pixel's samples in
// order (draw(), main.cpp:138-188), folding them as they come (draw2()'s per-pixel running average
// is the same fold with mode 1, main.cpp:205-231).  Path streams are keyed per (pixel, sample) as on
// the GPU, so the image does not depend on the thread count.
//
// MRT_RF_REF_ORDER: the reference's own RNG order instead (its deterministic mode at -threads 1,
// cmdline_parser.h:15): worker i draws every random number from ONE PCG stream seeded with the
// (initstate, initseq) main() gives it (main.cpp:357-366, handed over by mrt_set_worker_seeds),
// mode 0 = draw() over work_queue_seq (tile -> pixel -> sample, main.cpp:138-188,
// work_queue.cpp:133-140), mode 1 = draw2() over work_queue_dynamic (item k -> tile k % n_tiles,
// sample k / n_tiles; every pixel of the tile gets that sample, main.cpp:193-243,
// work_queue.cpp:157-166).  At one thread the image and ray count equal the reference's
// -threads 1 -mode 0|1 (tests/golden/refseq_*.npz); with more threads the result depends on
// scheduling, as the reference's does.
#define MRT_HOST_BACKEND 1
#include <hip/hip_runtime.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <mutex>
#include <cstring>
#include <thread>
#include <vector>

#include "mrt_cpu.h"
#include "mrt_tables.h"

using namespace mrtd;

struct mrt_cpu_scene {
    SceneTables T;
    // the view's arrays, copied: the caller keeps ownership of its blob (mrt.h)
    std::vector<uint32_t> children;
    std::vector<mrt_mesh_node> mnodes;
    std::vector<float4> tri_geo, tri_nrm, ranvec;
    std::vector<mrt_texture> texs;
    std::vector<int32_t> perm;
    std::vector<uint8_t> texels;
    mrt_camera cam;
    DScene S{};
    uint32_t feats = 0;
    // progress of the current render (work_queue::getPercentDone)
    std::atomic<uint64_t> done{0}, total{0};
    double last_ms = 0;
    uint32_t last_threads = 0;
    // the framebuffer the workers fill (G_linearBackBuffer): mrt_preview reads it while they run
    std::vector<float> fb;
    std::vector<uint32_t> fb_px;  // owned pixels, row-major
    uint32_t fb_w = 0, fb_h = 0, fb_ns = 0;
    std::atomic<uint32_t> tiles_done{0};
    uint32_t n_tiles = 0;
    // mrt_set_worker_seeds: (initstate, initseq) of each worker thread (MRT_RF_REF_ORDER renders)
    std::vector<uint64_t> seed_state, seed_seq;
    // MRT_RF_REF_ORDER mode 1: work items published per sample pass (mrt_preview: passes complete)
    std::vector<uint32_t> pass_items;
    uint32_t ref_mode1 = 0;
    // the framebuffer's size, owner list and contents: workers publish a finished work item (a
    // tile's pixels) under it, mrt_preview copies under it
    std::mutex fb_mu;
};

// the two hot-path instantiations of the host backend: any linear hit program through the
// interpreter, any other graph through the generic machine (both bit-identical to the GPU's
// shape-specialised walks, tests/test_gpu_parity.py)
static constexpr uint32_t F_LIN = FT_LIN | FT_ALL | FT_VSUB;
static constexpr uint32_t F_GEN = FT_ALL;

mrt_status mrt_cpu_scene_create(const mrt_scene_view* v, mrt_cpu_scene** out) {
    if (!out) return mrt_internal_fail(MRT_ERR_INVALID, "mrt_cpu_scene_create: null");
    mrt_cpu_scene* c = new mrt_cpu_scene();
    mrt_status st = mrt_internal_scene_tables(v, &c->T);
    if (st) {
        delete c;
        return st;
    }
    c->children.assign(v->children, v->children + v->n_children);
    c->mnodes.assign(v->mesh_nodes, v->mesh_nodes + v->n_mesh_nodes);
    c->tri_geo.assign((const float4*)v->tri_geo, (const float4*)v->tri_geo + (size_t)v->n_tris * 3);
    c->tri_nrm.assign((const float4*)v->tri_nrm, (const float4*)v->tri_nrm + (size_t)v->n_tris * 3);
    c->texs.assign(v->textures, v->textures + v->n_textures);
    c->ranvec.assign((const float4*)v->perlin_ranvec, (const float4*)v->perlin_ranvec + 256);
    c->perm.assign(v->perlin_perm, v->perlin_perm + 768);
    c->texels.assign(v->texels, v->texels + v->n_texels);
    c->cam = v->camera;
    SceneTables& T = c->T;
    DScene& S = c->S;
    S.nodes = T.nodes.data();
    S.children = c->children.data();
    S.mnodes = c->mnodes.data();
    S.mwide = T.wide.data();
    S.mwide_n = (uint32_t)T.wide.size();
    S.bwide = T.bwide.data();
    S.bprims = T.bprims.data();
    S.tri_geo = c->tri_geo.data();
    S.tri_nrm = c->tri_nrm.data();
    S.mats = T.dmats.data();
    S.texs = c->texs.data();
    S.ranvec = c->ranvec.data();
    S.perm = c->perm.data();
    S.texels = c->texels.data();
    S.prog = T.prog.data();
    S.bleaf = T.bleaf.data();
    S.nbleaf = T.nbleaf;
    S.nbleaf_f = (float)T.nbleaf;
    S.inv_nbleaf = 1.0f / S.nbleaf_f;
    S.blist = T.blist;
    S.root = v->root;
    S.biased = v->biased;
    S.sky = v->sky;
    S.cam = v->camera;
    S.camp = &c->cam;
    c->feats = T.features;
    *out = c;
    return MRT_OK;
}

void mrt_cpu_scene_free(mrt_cpu_scene* c) { delete c; }

uint32_t mrt_cpu_scene_features(const mrt_cpu_scene* c) { return c->feats; }

// one worker's stacks: the per-lane LDS stacks of the GPU walk, one lane wide (lane 0, the same
// [slot][word][lane] indexing with a 64-word stride)
struct Stacks {
    std::vector<uint32_t> frames, mesh;
    std::vector<float> rays, save;
    std::vector<v4f> lev;
    Stacks(const SceneTables& T, uint32_t rows)
        : frames((size_t)std::max(T.max_frames, 1) * 128), mesh((size_t)std::max(T.max_mesh, 1) * 64),
          rays((size_t)std::max(T.max_rays, 1) * 11 * 64), save(9 * 64), lev(rows) {}
};

// trace() of one path (main.cpp:66-118) to its end: the same segments the GPU runs one loop
// iteration at a time; returns the radiance after the recursion's fold
template <uint32_t F>
static f3 trace_path(const DScene& S, PathState& ps, uint32_t max_bounces, const LevStore<0>& lev, const LStack& Ls) {
    PhaseClock ph{};
    for (;;) {
        f3 L;
        if (trace_segment<F, 0>(S, ps, max_bounces, lev, Ls, &L, ph)) return end_path(ps, lev, L);
    }
}

template <uint32_t F>
static void render_tiles(mrt_cpu_scene* c, const mrt_render_desc* d, const std::vector<mrt_tile>& tiles,
                         std::atomic<uint32_t>& next, float* rgb_out, std::atomic<uint64_t>& rays_total,
                         const volatile int* cancel, std::atomic<bool>& cancelled) {
    const DScene& S = c->S;
    const uint32_t sq = d->sqrt_samples, ns = sq * sq, W = d->width;
    const uint32_t rows = std::max<uint32_t>(d->max_bounces, 1);
    Stacks st(c->T, rows);
    const LStack Ls{st.frames.data(), st.rays.data(), st.mesh.data(), st.save.data(), 0u, nullptr, 0u};
    const LevStore<0> lev{st.lev.data(), rows, 0u, 0u};
    // the sample grid of main.cpp:319-332, in float like the reference
    std::vector<float2> sd(ns);
    for (uint32_t i = 0; i < sq; i++)
        for (uint32_t j = 0; j < sq; j++) sd[(size_t)i * sq + j] = make_float2(((float)i + 0.5f) / (float)sq, ((float)j + 0.5f) / (float)sq);
    uint64_t my_rays = 0;
    std::vector<float> tb;  // the work item's pixels, published to the framebuffer when done
    for (;;) {
        if (cancel && *cancel) {  // G_isRunning (main.cpp:180)
            cancelled.store(true, std::memory_order_relaxed);
            break;
        }
        const uint32_t k = next.fetch_add(1, std::memory_order_relaxed);  // work_queue::getWork
        if (k >= tiles.size()) break;
        const mrt_tile& t = tiles[k];
        const uint32_t tw = t.xmax - t.xmin;
        tb.assign((size_t)tw * (t.ymax - t.ymin) * 4, 0.0f);
        for (uint32_t y = t.ymin; y < t.ymax; y++)
            for (uint32_t x = t.xmin; x < t.xmax; x++) {
                const uint32_t pix = x + y * W;
                f3 col{0, 0, 0};
                for (uint32_t s = 0; s < ns; s++) {
                    const uint64_t path_id = (uint64_t)pix * ns + s;
                    PathState ps;
                    pcg_seed(ps.rng, splitmix64(d->seed ^ path_id), path_id);
                    const float u = ((float)x + sd[s].x) / (float)d->width, v = ((float)y + sd[s].y) / (float)d->height;
                    ps.r = camera_ray(S, ps.rng, u, v);
                    ps.depth = 0;
                    ps.nlev = 0;
                    const f3 L = trace_path<F>(S, ps, d->max_bounces, lev, Ls);
                    my_rays += ps.rays();
                    col = fold_sample(col, L, s, d->mode, d->max_luminance);
                }
                col = final_pixel(col, ns, d->mode, d->max_luminance);
                float* o = tb.data() + ((size_t)(x - t.xmin) + (size_t)(y - t.ymin) * tw) * 4;
                o[0] = col.x;
                o[1] = col.y;
                o[2] = col.z;
            }
        {
            std::lock_guard<std::mutex> lk(c->fb_mu);
            for (uint32_t y = t.ymin; y < t.ymax; y++)
                memcpy(c->fb.data() + ((size_t)t.xmin + (size_t)y * W) * 4, tb.data() + (size_t)(y - t.ymin) * tw * 4, (size_t)tw * 16);
        }
        c->done.fetch_add((uint64_t)tw * (t.ymax - t.ymin) * ns, std::memory_order_relaxed);
        c->tiles_done.fetch_add(1, std::memory_order_release);
    }
    rays_total.fetch_add(my_rays, std::memory_order_relaxed);
}

// MRT_RF_REF_ORDER: worker `wi` with its own continuing PCG stream (Init_Thread_RNG(initstate,
// initseq), main.cpp:143 / 198), work items from the shared queue in the reference's order.
template <uint32_t F>
static void render_ref_order(mrt_cpu_scene* c, const mrt_render_desc* d, const std::vector<mrt_tile>& tiles, uint32_t wi,
                             std::atomic<uint64_t>& next, std::atomic<uint64_t>& rays_total, const volatile int* cancel,
                             std::atomic<bool>& cancelled) {
    const DScene& S = c->S;
    const uint32_t sq = d->sqrt_samples, ns = sq * sq, W = d->width;
    const uint32_t rows = std::max<uint32_t>(d->max_bounces, 1);
    Stacks st(c->T, rows);
    const LStack Ls{st.frames.data(), st.rays.data(), st.mesh.data(), st.save.data(), 0u, nullptr, 0u};
    const LevStore<0> lev{st.lev.data(), rows, 0u, 0u};
    std::vector<float2> sd(ns);
    for (uint32_t i = 0; i < sq; i++)
        for (uint32_t j = 0; j < sq; j++) sd[(size_t)i * sq + j] = make_float2(((float)i + 0.5f) / (float)sq, ((float)j + 0.5f) / (float)sq);
    Pcg rng;
    pcg_seed(rng, c->seed_state[wi], c->seed_seq[wi]);
    const uint64_t nt = tiles.size();
    const uint64_t items = d->mode == 0 ? nt : nt * ns;  // work_queue_seq: tiles; work_queue_dynamic: (tile, sample)
    uint64_t my_rays = 0;
    // one path of the worker's stream: camera::get_ray then trace() (main.cpp:153-157, 208-210)
    auto path = [&](uint32_t x, uint32_t y, uint32_t s) {
        PathState ps;
        ps.rng = rng;
        const float u = ((float)x + sd[s].x) / (float)d->width, v = ((float)y + sd[s].y) / (float)d->height;
        ps.r = camera_ray(S, ps.rng, u, v);
        ps.depth = 0;
        ps.nlev = 0;
        const f3 L = trace_path<F>(S, ps, d->max_bounces, lev, Ls);
        rng = ps.rng;
        my_rays += ps.rays();
        return L;
    };
    std::vector<float> tb;
    for (;;) {
        if (cancel && *cancel) {  // G_isRunning (main.cpp:180, 235)
            cancelled.store(true, std::memory_order_relaxed);
            break;
        }
        const uint64_t k = next.fetch_add(1, std::memory_order_relaxed);  // work_queue::getWork
        if (k >= items) break;
        const mrt_tile& t = tiles[k % nt];
        const uint32_t s = d->mode == 0 ? 0u : (uint32_t)(k / nt);
        const uint32_t tw = t.xmax - t.xmin, th = t.ymax - t.ymin;
        tb.resize((size_t)tw * th * 4);
        if (d->mode == 1) {  // draw2() folds into the buffer's running average: the tile's current values
            std::lock_guard<std::mutex> lk(c->fb_mu);
            for (uint32_t y = t.ymin; y < t.ymax; y++)
                memcpy(tb.data() + (size_t)(y - t.ymin) * tw * 4, c->fb.data() + ((size_t)t.xmin + (size_t)y * W) * 4, (size_t)tw * 16);
        }
        for (uint32_t y = t.ymin; y < t.ymax; y++)
            for (uint32_t x = t.xmin; x < t.xmax; x++) {
                float* o = tb.data() + ((size_t)(x - t.xmin) + (size_t)(y - t.ymin) * tw) * 4;
                f3 col;
                if (d->mode == 0) {  // draw(): every sample of the pixel in order
                    col = f3{0, 0, 0};
                    for (uint32_t j = 0; j < ns; j++) col = fold_sample(col, path(x, y, j), j, 0u, d->max_luminance);
                    col = final_pixel(col, ns, 0u, d->max_luminance);
                } else {  // draw2(): sample s of the pixel into its running average
                    col = fold_sample(f3{o[0], o[1], o[2]}, path(x, y, s), s, 1u, d->max_luminance);
                }
                o[0] = col.x;
                o[1] = col.y;
                o[2] = col.z;
                o[3] = 0.0f;
            }
        {
            std::lock_guard<std::mutex> lk(c->fb_mu);
            for (uint32_t y = t.ymin; y < t.ymax; y++)
                memcpy(c->fb.data() + ((size_t)t.xmin + (size_t)y * W) * 4, tb.data() + (size_t)(y - t.ymin) * tw * 4, (size_t)tw * 16);
            if (d->mode == 1) c->pass_items[s]++;
        }
        c->done.fetch_add((uint64_t)tw * th * (d->mode == 0 ? ns : 1u), std::memory_order_relaxed);
        if (d->mode == 0) c->tiles_done.fetch_add(1, std::memory_order_release);
    }
    rays_total.fetch_add(my_rays, std::memory_order_relaxed);
}

mrt_status mrt_cpu_set_worker_seeds(mrt_cpu_scene* c, uint32_t n, const uint64_t* initstate, const uint64_t* initseq) {
    if (!c || (n && (!initstate || !initseq))) return mrt_internal_fail(MRT_ERR_INVALID, "mrt_set_worker_seeds: null");
    std::lock_guard<std::mutex> lk(c->fb_mu);
    c->seed_state.assign(initstate, initstate + n);
    c->seed_seq.assign(initseq, initseq + n);
    return MRT_OK;
}

mrt_status mrt_cpu_render(mrt_cpu_scene* c, const mrt_render_desc* d, float* rgb_out, uint64_t* rays_out, const volatile int* cancel) {
    if (!c || !d || !rgb_out || d->width == 0 || d->height == 0 || d->sqrt_samples == 0 || (d->world && d->rank >= d->world))
        return mrt_internal_fail(MRT_ERR_INVALID, "mrt_render (CPU backend): bad desc");
    if (d->flags & MRT_RF_FAST)
        return mrt_internal_fail(MRT_ERR_INVALID, "the CPU backend implements the exact numerics contract only");
    if (d->flags & MRT_RF_PATH_DEBUG) return mrt_internal_fail(MRT_ERR_INVALID, "MRT_RF_PATH_DEBUG is a GPU-backend render flag");
    if (mrt_status st = mrt_internal_check_pixels(d)) return st;
    const bool ref_order = (d->flags & MRT_RF_REF_ORDER) != 0;
    if (ref_order) {
        if (d->world > 1 || d->pixels)
            return mrt_internal_fail(MRT_ERR_INVALID, "MRT_RF_REF_ORDER renders the whole image (the reference has no ranks or pixel lists)");
        if (c->seed_state.empty()) return mrt_internal_fail(MRT_ERR_INVALID, "MRT_RF_REF_ORDER needs mrt_set_worker_seeds first");
        if (d->threads && d->threads != c->seed_state.size())
            return mrt_internal_fail(MRT_ERR_INVALID, "MRT_RF_REF_ORDER: desc.threads must equal the worker seeds given");
    }
    const auto t0 = std::chrono::steady_clock::now();
    const uint32_t ns = d->sqrt_samples * d->sqrt_samples;
    // this rank's tiles in work_queue order (or one 1x1 tile per listed pixel)
    const std::vector<mrt_tile> tiles = mrt_internal_render_tiles(d);
    uint64_t px = 0;
    for (const mrt_tile& t : tiles) px += (uint64_t)(t.xmax - t.xmin) * (t.ymax - t.ymin);
    c->done.store(0, std::memory_order_relaxed);
    c->total.store(px * ns, std::memory_order_relaxed);
    {
        std::lock_guard<std::mutex> lk(c->fb_mu);
        c->fb.assign((size_t)d->width * d->height * 4, 0.0f);
        c->fb_px = mrt_internal_local_pixels(d);
        c->fb_w = d->width;
        c->fb_h = d->height;
        c->fb_ns = ns;
        c->tiles_done.store(0, std::memory_order_relaxed);
        c->n_tiles = (uint32_t)tiles.size();
        c->ref_mode1 = ref_order && d->mode == 1;
        c->pass_items.assign(c->ref_mode1 ? ns : 0u, 0u);
    }
    uint32_t n = ref_order ? (uint32_t)c->seed_state.size() : d->threads ? d->threads : std::max(1u, std::thread::hardware_concurrency());
    if (!ref_order) n = (uint32_t)std::min<size_t>(n, std::max<size_t>(tiles.size(), 1));
    std::atomic<uint32_t> next{0};
    std::atomic<uint64_t> next_item{0};
    std::atomic<uint64_t> rays{0};
    std::atomic<bool> cancelled{false};
    auto work = [&](uint32_t wi) {
        if (ref_order) {
            if (c->feats & FT_LIN) render_ref_order<F_LIN>(c, d, tiles, wi, next_item, rays, cancel, cancelled);
            else render_ref_order<F_GEN>(c, d, tiles, wi, next_item, rays, cancel, cancelled);
        } else {
            if (c->feats & FT_LIN) render_tiles<F_LIN>(c, d, tiles, next, rgb_out, rays, cancel, cancelled);
            else render_tiles<F_GEN>(c, d, tiles, next, rgb_out, rays, cancel, cancelled);
        }
    };
    std::vector<std::thread> pool;
    for (uint32_t i = 1; i < n; i++) pool.emplace_back(work, i);
    work(0u);
    for (std::thread& t : pool) t.join();
    for (uint32_t p : c->fb_px) memcpy(rgb_out + (size_t)p * 4, c->fb.data() + (size_t)p * 4, 16);
    c->last_ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
    c->last_threads = n;
    if (rays_out) *rays_out = rays.load();
    if (cancelled.load()) return mrt_internal_fail(MRT_ERR_CANCELLED, "cancelled (partial image)");
    return MRT_OK;
}

mrt_status mrt_cpu_progress(mrt_cpu_scene* c, float* pct) {
    const uint64_t t = c->total.load(std::memory_order_relaxed), dn = c->done.load(std::memory_order_relaxed);
    *pct = t ? (float)std::min(100.0, 100.0 * (double)dn / (double)t) : 0.0f;
    return MRT_OK;
}

mrt_status mrt_cpu_last_ms(mrt_cpu_scene* c, float* ms, uint32_t* threads) {
    *ms = (float)c->last_ms;
    if (threads) *threads = c->last_threads;
    return MRT_OK;
}

// The framebuffer as the UI thread sees it (main.cpp:387-444), copied under the lock the workers
// publish finished work items with (never a half-written tile).  draw() (mode 0, and every
// stream-keyed render): finished tiles with all their samples, the others black; samples_done = spp
// once every tile is in, 0 before.  draw2() in the reference's order (MRT_RF_REF_ORDER, mode 1):
// the running averages; samples_done = the leading sample passes every tile has published.
mrt_status mrt_cpu_preview(mrt_cpu_scene* c, float* rgb_out, uint32_t* samples_done) {
    std::lock_guard<std::mutex> lk(c->fb_mu);
    *samples_done = 0;
    if (c->fb.empty()) return MRT_OK;
    for (uint32_t p : c->fb_px) memcpy(rgb_out + (size_t)p * 4, c->fb.data() + (size_t)p * 4, 16);
    if (c->ref_mode1) {
        uint32_t s = 0;
        while (s < c->pass_items.size() && c->pass_items[s] == c->n_tiles) s++;
        *samples_done = s;
    } else {
        *samples_done = c->tiles_done.load(std::memory_order_acquire) == c->n_tiles ? c->fb_ns : 0u;
    }
    return MRT_OK;
}

// Test hook (tests/test_host.py): the scene's linear hit program as compiled, or its
// tolerance-contract rewrite (mrt_sig.h lin_rewrite_fast) -- per op its code word and skip.
extern "C" int mrt_debug_lin_program(const mrt_scene_view* v, int rewritten, uint32_t* codes, uint32_t* skips, uint32_t cap,
                                     uint32_t* n) {
    SceneTables T;
    if (mrt_internal_scene_tables(v, &T) != MRT_OK) return 1;
    const std::vector<LinOp>& p = rewritten ? T.prog_fast : T.prog;
    *n = (uint32_t)p.size();
    for (uint32_t i = 0; i < p.size() && i < cap; i++) {
        codes[i] = p[i].code;
        skips[i] = p[i].skip;
    }
    return 0;
}
