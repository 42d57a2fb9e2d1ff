/* mrt.h -- C-ABI of the MI355X render path (libmrt.so).  Plain C types only; return codes, never
 * exceptions; the library owns device memory, the caller owns all host memory.
 *
 * What each entry point replaces in the reference (Maraneshi/MiniRayTracer, no FFI of its own --
 * the seam is the worker-thread spawn in main(), main.cpp:347-382):
 *
 *   mrt_default_params / mrt_parse_argv   MRT_Params defaults + ParseArgv   cmdline_parser.h:5-18, cmdline_parser.cpp:78-107
 *   mrt_select_scene                      select_scene(scenes, aspect)      scene.cpp:25-49 (+ scene 9)
 *   mrt_scene_upload                      (new) scene -> HBM, once, outside the timed region (main.cpp:309 vs 375)
 *   mrt_render / mrt_render_device        std::thread(draw|draw2) x N over work_queue + trace()
 *                                         main.cpp:66-118, 138-243, 347-382; work_queue.cpp:133-175
 *   mrt_render_join                       the worker threads' join()             main.cpp:490-493
 *   mrt_progress                          work_queue::getPercentDone        work_queue.cpp:142-149, 168-175
 *   rays_out                              G_rayCounter                      main.cpp:55, 68, 403-405
 *   cancel                                G_isRunning                       main.cpp:54, 180, 235
 *   mrt_tonemap_argb                      Drago tone map + ARGB32            main.cpp:416-444, vec3.h:327-333
 *   mrt_lum_max_device/mrt_tonemap_device the same, on the device              main.cpp:421-442
 *
 * Threading: one host thread per device; calls on distinct scenes are thread-safe, calls on the
 * same scene handle are not reentrant.
 */
#ifndef MRT_H
#define MRT_H
#include <stdint.h>
#include "mrt_scene.h"

#ifdef __cplusplus
extern "C" {
#endif

typedef enum mrt_status {
    MRT_OK = 0,
    MRT_ERR_INVALID = 1,     /* bad argument / unsupported scene graph */
    MRT_ERR_NO_DEVICE = 2,   /* no gfx950 device visible */
    MRT_ERR_HIP = 3,         /* HIP runtime error */
    MRT_ERR_OOM = 4,
    MRT_ERR_IO = 5,          /* asset (OBJ / texels) not found or unreadable */
    MRT_ERR_CANCELLED = 6
} mrt_status;

/* MRT_Params (cmdline_parser.h:5-18), same defaults and field meaning. */
typedef struct mrt_params {
    uint32_t window_width, window_height;
    uint32_t buffer_width, buffer_height;
    uint32_t samples_per_pixel;
    uint32_t tile_size;
    uint32_t num_threads;     /* CPU worker threads, as in the reference (0 = all); the GPU backend has none */
    uint32_t max_bounces;
    uint32_t scene_select;
    uint32_t threading_mode;  /* 0 = draw() per-pixel mean, 1 = draw2() progressive average */
    float max_luminance;
    uint32_t delay;
    /* additions (not in the reference): */
    uint64_t seed;            /* path stream-key seed, default = the reference main seed */
    uint32_t gpus;            /* -gpus: GPUs to shard the work_queue tiles over (0 = every visible GPU) */
    uint32_t numerics;        /* -numerics: 0 exact contract, 1 tolerance contract (MRT_RF_FAST) */
    uint32_t backend;         /* -backend: 0 GPU (default), 1 CPU (MRT_DEVICE_CPU, -threads workers, exact) */
    uint32_t order;           /* -order: 0 = per-path stream keys (the GPU's; any thread / GPU count gives
                                 the same image), 1 = the reference's RNG order (one PCG stream per worker
                                 thread, work_queue order; CPU backend only, MRT_RF_REF_ORDER).  Default:
                                 1 with -backend cpu, 0 otherwise */
} mrt_params;

void mrt_default_params(mrt_params* p);
/* Same flags, ranges and warnings as ParseArgv; also -seed.  Returns MRT_OK (the reference never
 * fails on bad values: it warns and keeps the default). -help prints help and returns INVALID. */
mrt_status mrt_parse_argv(int argc, char** argv, mrt_params* p);

/* ---- host scene (select_scene) ------------------------------------------------------------ */
typedef struct mrt_scene_blob mrt_scene_blob;
/* asset_dir: directory holding bunny.obj / wt_teapot.obj (or their packed .tri forms) and
 * earthmap.rgb (stb-decoded texels); NULL = $MRT_ASSET_DIR or the package assets/ directory. */
mrt_status mrt_select_scene(uint32_t scene, float aspect, const char* asset_dir, mrt_scene_blob** out);
mrt_status mrt_scene_blob_view(const mrt_scene_blob* blob, mrt_scene_view* out);
/* JSON dump in the schema of oracle/ref/harness.cpp --h-mode scene (parity fixture check). */
mrt_status mrt_scene_blob_dump_json(const mrt_scene_blob* blob, char** json_out);
void mrt_free_string(char* s);
/* Store the parsed records of an OBJ file as a packed <name>.mesh asset (same parser as
 * mrt_select_scene; used when the .obj itself is not shipped). */
mrt_status mrt_pack_obj(const char* obj_path, const char* out_path);
void mrt_scene_blob_free(mrt_scene_blob* blob);
/* The (initstate, initseq) main() hands its worker threads (main.cpp:357-361): drawn from the main
 * thread's PCG after select_scene consumed what it needs.  Only renders in the reference's own RNG
 * order depend on them (the CPU backend's MRT_RF_REF_ORDER renders, via mrt_set_worker_seeds, and
 * the oracle's restatement); the GPU path keys its streams per path instead. */
mrt_status mrt_worker_seeds(const mrt_scene_blob* blob, uint32_t n_threads, uint64_t* initstate, uint64_t* initseq);

/* ---- device -------------------------------------------------------------------------------- */
mrt_status mrt_init(int* device_count);
typedef struct mrt_scene mrt_scene;
/* device: a HIP device index, or MRT_DEVICE_CPU for the CPU backend -- the same hot-path source
 * compiled for the host (exact numerics contract; worker threads over the work_queue tiles like
 * draw()/draw2(), main.cpp:347-382).  It is only ever chosen explicitly: with no gfx950 device the
 * GPU entry points fail (MRT_ERR_NO_DEVICE), they never fall back to the CPU. */
#define MRT_DEVICE_CPU (-1)
mrt_status mrt_scene_upload(int device, const mrt_scene_view* view, mrt_scene** out);
void mrt_scene_free(mrt_scene* scene);
/* CPU backend only: the drawArgs (initstate, initseq) of each worker thread (main.cpp:127-135,
 * 357-366; from mrt_worker_seeds) for renders with MRT_RF_REF_ORDER, which run n_threads workers. */
mrt_status mrt_set_worker_seeds(mrt_scene* s, uint32_t n_threads, const uint64_t* initstate, const uint64_t* initseq);

typedef struct mrt_render_desc {
    uint32_t width, height;
    uint32_t sqrt_samples;   /* spp = sqrt_samples^2, regular grid (main.cpp:319-332) */
    uint32_t max_bounces;
    float max_luminance;
    uint32_t mode;           /* 0 draw() semantics, 1 draw2() semantics */
    uint64_t seed;           /* stream key: path p -> pcg32_srandom(splitmix64(seed ^ p), p) */
    uint32_t tile_size;      /* work_queue tiles (work_queue.cpp:64-128) */
    uint32_t rank, world;    /* this call renders the tiles (inverted-Hilbert order) dealt to `rank`: rounds of
                                `world` consecutive tiles, each round in its own permutation of the ranks */
    uint32_t chunk_samples;  /* samples per launch (0 = auto, bounded by HBM budget) */
    uint32_t flags;          /* MRT_RF_* */
    uint32_t threads;        /* CPU backend: worker threads (0 = every core); the GPU backend ignores it */
    /* Optional pixel list (an addition; the reference always renders the whole buffer): when
     * non-NULL this call renders exactly these n_pixels row-major pixel indices (row 0 = bottom,
     * each < width*height, no repeats), in this order as its local pixels, instead of the tiles
     * dealt to `rank` -- every sample of each, the same per-path streams, so a listed pixel equals
     * the same pixel of a whole-image render bit for bit.  Caller-owned; read during the call. */
    const uint32_t* pixels;
    uint32_t n_pixels;
} mrt_render_desc;
#define MRT_RF_PATH_DEBUG 0x1u /* also keep per-path radiance + ray counts (mrt_render_debug) */
#define MRT_RF_FAST 0x2u       /* tolerance numerics contract: FMA contraction, hardware rcp/sqrt/rsq,
                                  f32 transcendentals; per-pixel RMSE < 1e-3 vs the reference as
                                  shipped (DESIGN.md "Numerics contracts").  Unset: the exact
                                  contract, bit-for-bit the reference built exact. */
#define MRT_RF_PREVIEW 0x4u    /* keep a progressive preview for mrt_preview: after every launch's
                                  fold, the running image (mode 1: the running average, draw2();
                                  mode 0: the mean of the samples so far) is copied to pinned host
                                  memory in stream order (G_linearBackBuffer as the UI thread reads
                                  it every 33 ms, main.cpp:387-444) */
#define MRT_RF_FOLD_BEHIND 0x8u /* mode 0: fold with a kernel lean enough (8 VGPRs) to run beside
                                   another context's persistent path kernel instead of after it --
                                   for callers that pipeline renders on several streams; slower
                                   when nothing else runs (same bits either way) */
#define MRT_RF_FOLD_ASYNC 0x40u /* GPU, no preview / debug / lean fold: each launch's fold runs on
                                   the context's own stream, beside the NEXT launch's (or render's)
                                   path kernel, instead of after its own (two radiance buffers used in
                                   turn).  The output is complete once mrt_render_join has ordered a
                                   stream after it (or the device is synchronised).  Same bits as the
                                   fold in stream order.  Not for stream capture (the fold's stream is
                                   the context's own).  (ABI 6: was 0x20, the bit of the removed
                                   MRT_RF_SPLIT; 0x20 and every other unknown bit are now rejected
                                   with MRT_ERR_INVALID instead of silently changing meaning.) */
#define MRT_RF_REF_ORDER 0x10u  /* CPU backend: the reference's own RNG order -- worker i draws from
                                   one PCG stream seeded by mrt_set_worker_seeds' i-th pair; mode 0 =
                                   draw() over work_queue_seq (tile -> pixel -> sample), mode 1 =
                                   draw2() over work_queue_dynamic ((tile, sample) items,
                                   work_queue.cpp:133-166).  One thread reproduces the reference's
                                   -threads 1 run bit for bit (its deterministic mode,
                                   cmdline_parser.h:15); world must be 1 */
#define MRT_RF_ALL (MRT_RF_PATH_DEBUG | MRT_RF_FAST | MRT_RF_PREVIEW | MRT_RF_FOLD_BEHIND | MRT_RF_REF_ORDER | MRT_RF_FOLD_ASYNC)

/* ABI version of this header: bumped whenever a flag's meaning or a struct layout changes (6: the
 * MRT_RF_FOLD_ASYNC bit moved to 0x40, mrt_kernel_info gained handover_lost, mrt_comm_* added).
 * A binding checks mrt_abi_version() == MRT_ABI_VERSION before its first call. */
#define MRT_ABI_VERSION 6u
uint32_t mrt_abi_version(void);

void mrt_default_render_desc(const mrt_params* p, mrt_render_desc* d);

/* Number of pixels this rank owns and their row-major indices (row 0 = bottom, like
 * G_linearBackBuffer main.cpp:58) in the order mrt_render_device writes them (d->pixels when set). */
mrt_status mrt_local_pixels(const mrt_render_desc* d, uint32_t* n_out, uint32_t* pixels_out /* may be NULL */);

/* Render into a host W*H*4 float buffer (x,y,z,0 per pixel; only owned pixels are written).
 * Both backends; on the CPU backend the call returns when the render is done (cancel is polled
 * per tile, as G_isRunning at main.cpp:180). */
mrt_status mrt_render(mrt_scene* s, const mrt_render_desc* d, float* rgb_out, uint64_t* rays_out,
                      const volatile int* cancel);
/* GPU backend only.  Render into device memory: d_local = n_local*4 floats in mrt_local_pixels order.  Enqueued on
 * `stream` (hipStream_t or NULL); rays are accumulated into the device uint64 *d_rays; nothing is
 * synchronised and nothing is allocated when the scene's workspace already fits (capturable). */
mrt_status mrt_render_device(mrt_scene* s, const mrt_render_desc* d, float* d_local, uint64_t* d_rays, void* stream);
/* GPU backend only.  Enqueue on `stream` a wait for the context's last mrt_render_device (its
 * fold, on the context's own stream under MRT_RF_FOLD_ASYNC): work enqueued on `stream` afterwards
 * sees its output.  (No-op order for renders whose fold ran on their own stream.) */
mrt_status mrt_render_join(mrt_scene* s, void* stream);
/* Allocate/grow the scene's workspace for d (call once before timing mrt_render_device). */
mrt_status mrt_prepare(mrt_scene* s, const mrt_render_desc* d);
/* Per-path radiance (n_local*spp*3 floats, sample-major: [s][local pixel]) and ray counts of the
 * last render made with MRT_RF_PATH_DEBUG (host copies). */
mrt_status mrt_render_debug(mrt_scene* s, float* path_rgb, uint32_t* path_rays, uint64_t n_paths);
mrt_status mrt_progress(mrt_scene* s, float* pct);
/* The newest preview of the running render, callable from another host thread while it runs: the
 * image after *samples_done samples of every pixel (W*H*4 floats, owned pixels only, as rgb_out of
 * mrt_render), never a mix of two passes (the snapshot is sequence-locked).  GPU backend: renders
 * made with MRT_RF_PREVIEW (samples_done = 0 until the first launch is folded); CPU backend: the
 * framebuffer as far as its tiles are done (every sample of a finished pixel; samples_done = spp
 * once the render is over, 0 before). */
mrt_status mrt_preview(mrt_scene* s, float* rgb_out, uint32_t* samples_done);
/* Device time of the path-kernel launches of the last render (HIP events recorded on the render's
 * stream around each mrt_path_kernel launch); waits for the last one. */
mrt_status mrt_kernel_ms(mrt_scene* s, float* path_ms, uint32_t* launches);

/* Which path kernel the scene runs: feature bits of the scene (FT_* of mrt_trace.h; bit 11 =
 * linear hit program, bit 14 = a volume bounded by a sub-program, DESIGN.md "Kernels"), dynamic LDS bytes per workgroup, grid size in
 * workgroups, threads per workgroup, the BVH nodes each workgroup keeps in LDS, and the build of
 * the kernel for the last render's numerics: MRT_BUILD_* (the tolerance contract runs the fast,
 * the denormal-flushing or the path-exact build per kernel variant). */
#define MRT_BUILD_EXACT 0u
#define MRT_BUILD_FAST 1u
#define MRT_BUILD_FAST_FTZ 2u
#define MRT_BUILD_PATH_EXACT 3u
typedef struct mrt_kernel_info {
    uint32_t features, kernel_features, lds_bytes, grid, prog_ops, vgprs, wg, tree_nodes, build;
    /* handed_over: paths the fast-arithmetic kernels listed for the exact arithmetic since the
       scene's upload (rounding-critical light samples); handover_lost: listed
       paths beyond a launch's list capacity (they keep their fast radiance; 0 in every BASELINE
       config).  Reading them waits for the scene's last render (its fold included).  pad: 0 */
    uint32_t pad;
    uint64_t handed_over;
    uint64_t handover_lost;
} mrt_kernel_info;
mrt_status mrt_scene_kernel_info(const mrt_scene* s, mrt_kernel_info* out);

/* Drago adaptive-log tone map of a linear W*H*4 buffer to ARGB32 (main.cpp:416-444, no gamma). */
mrt_status mrt_tonemap_argb(const float* rgb, uint32_t width, uint32_t height, uint32_t* argb_out);
/* The same on the device, in two steps so ranks can combine L_wmax (all_reduce max) in between:
 *   mrt_lum_max_device  *d_lwmax = max(*d_lwmax, max luminance of the n float4 pixels) -- the
 *                       caller zeroes *d_lwmax first (main.cpp:424-429)
 *   mrt_tonemap_device  d_argb[i] = ARGB32(Drago(d_rgb[i]; *d_lwmax)) (main.cpp:430-442)
 * Pixel order is free (e.g. the local-pixel order of mrt_render_device); enqueued on `stream`. */
mrt_status mrt_lum_max_device(const float* d_rgb, uint32_t n, float* d_lwmax, void* stream);
mrt_status mrt_tonemap_device(const float* d_rgb, uint32_t n, const float* d_lwmax, uint32_t* d_argb, void* stream);

/* ---- multi-GPU: the framebuffer gather over RCCL (xGMI) ---------------------------------------
 * The reference's seam is main.cpp:347-382 (the worker threads over one work_queue) writing
 * G_linearBackBuffer (main.cpp:58): here each rank renders the work_queue tiles dealt to it
 * (mrt_render_desc.rank / world) on its own GPU, and ONE RCCL gather of the equal-size padded shards
 * to the root plus one device scatter assembles the W*H framebuffer on the root's GPU; ray counts
 * are summed with one all-reduce.  RCCL is loaded at mrt_comm_init_* (librccl.so.1: the copy already
 * in the process, else the loader's search path, else /opt/rocm/lib; $MRT_RCCL_LIB overrides);
 * without it those calls fail with MRT_ERR_NO_DEVICE.  Collective calls (mrt_gather_frame,
 * mrt_render_gather) are made by every rank of the communicator, one host thread (or process) per
 * rank. */
typedef struct mrt_comm mrt_comm;
#define MRT_COMM_ID_BYTES 128
/* one process per GPU: rank 0 makes the id (ncclGetUniqueId) and hands it to the others out of band */
mrt_status mrt_comm_unique_id(uint8_t id[MRT_COMM_ID_BYTES]);
mrt_status mrt_comm_init_rank(int device, uint32_t world, uint32_t rank, const uint8_t id[MRT_COMM_ID_BYTES], mrt_comm** out);
/* one process driving `world` GPUs (ncclCommInitAll): comms_out[r] is rank r on devices[r] */
mrt_status mrt_comm_init_all(uint32_t world, const int* devices, mrt_comm** comms_out);
void mrt_comm_free(mrt_comm* c);
/* Pixels of the largest rank shard of d's tile deal (the gather's padded shard, in pixels). */
mrt_status mrt_gather_shard_pixels(const mrt_render_desc* d, uint32_t* n_out);
/* Collective, enqueued on `stream` (the caller has ordered it after its render, mrt_render_join):
 * this rank's d_local (mrt_render_device output: n_local float4 in mrt_local_pixels order, d.rank
 * = the communicator's rank, d.world = its size, no pixel list) goes to the root with one
 * ncclGather of the padded shards; on the root the shards are scattered into d_frame (W*H float4,
 * row-major, row 0 = bottom, like G_linearBackBuffer; other ranks pass NULL).  d_rays (device
 * uint64, may be NULL) is summed over the ranks in place (ncclAllReduce), in the same group. */
mrt_status mrt_gather_frame(mrt_comm* c, const mrt_render_desc* d, const float* d_local, float* d_frame, uint64_t* d_rays,
                            void* stream);
/* The drop-in for one worker thread of main.cpp:347-382 on its own GPU: renders this rank's tiles
 * (mrt_render_device into the communicator's buffers), gathers the frame to the root over RCCL and,
 * on the root, copies it to rgb_out (W*H*4 floats, every pixel; other ranks may pass NULL).  The ray
 * total of all ranks goes to *rays_out on every rank (may be NULL).  Returns when this rank's part is
 * done. */
mrt_status mrt_render_gather(mrt_scene* s, mrt_comm* c, const mrt_render_desc* d, float* rgb_out, uint64_t* rays_out);

const char* mrt_strerror(mrt_status s);
const char* mrt_last_error(void);

#ifdef __cplusplus
}
#endif
#endif
