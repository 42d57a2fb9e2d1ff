// mrt_comm.hip -- the framebuffer gather over RCCL behind the C-ABI (include/mrt.h, "multi-GPU").
//
// The reference renders one framebuffer with N worker threads pulling tiles from one work_queue
// (main.cpp:347-382) and writing G_linearBackBuffer (main.cpp:58).  Here each rank (one GPU) renders
// the work_queue tiles dealt to it (mrt_local_pixels order, mrt_common.cpp) into a shard; the frame
// is assembled on the root's GPU by ONE ncclGather of the equal-size padded shards over xGMI and
// one scatter kernel that places every shard pixel at its row-major index.  Ray counts (the
// reference's G_rayCounter) are summed by one ncclAllReduce in the same RCCL group.
//
// RCCL is bound at run time (dlopen): the librccl.so.1 already in the process (torch's, when the
// caller imported it -- one RCCL per process), else the loader's search path, else /opt/rocm/lib;
// $MRT_RCCL_LIB overrides.  Only mrt_comm_* and the two gather entry points need it.
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>
#include <dlfcn.h>

#include <algorithm>
#include <cstring>
#include <mutex>
#include <string>
#include <vector>

#include "mrt_internal.h"

namespace {

struct Rccl {
    decltype(&ncclGetUniqueId) get_unique_id = nullptr;
    decltype(&ncclCommInitRank) init_rank = nullptr;
    decltype(&ncclCommInitAll) init_all = nullptr;
    decltype(&ncclCommDestroy) destroy = nullptr;
    decltype(&ncclGather) gather = nullptr;
    decltype(&ncclAllReduce) all_reduce = nullptr;
    decltype(&ncclGroupStart) group_start = nullptr;
    decltype(&ncclGroupEnd) group_end = nullptr;
    decltype(&ncclGetErrorString) error_string = nullptr;
    std::string why;  // empty once every symbol is bound
};

const Rccl& rccl() {
    static Rccl r;
    static std::once_flag once;
    std::call_once(once, [] {
        void* h = nullptr;
        const char* e = getenv("MRT_RCCL_LIB");
        if (e && *e) {
            h = dlopen(e, RTLD_NOW | RTLD_LOCAL);
        } else {
            for (const char* n : {"librccl.so.1", "librccl.so"})
                if ((h = dlopen(n, RTLD_NOW | RTLD_NOLOAD))) break;
            if (!h) h = dlopen("librccl.so.1", RTLD_NOW | RTLD_LOCAL);
            if (!h) h = dlopen("/opt/rocm/lib/librccl.so.1", RTLD_NOW | RTLD_LOCAL);
        }
        if (!h) {
            const char* d = dlerror();
            r.why = std::string("RCCL not loadable: ") + (d ? d : "librccl.so.1 not found");
            return;
        }
        auto sym = [&](auto& fn, const char* name) {
            fn = reinterpret_cast<std::remove_reference_t<decltype(fn)>>(dlsym(h, name));
            if (!fn && r.why.empty()) r.why = std::string("RCCL lacks ") + name;
        };
        sym(r.get_unique_id, "ncclGetUniqueId");
        sym(r.init_rank, "ncclCommInitRank");
        sym(r.init_all, "ncclCommInitAll");
        sym(r.destroy, "ncclCommDestroy");
        sym(r.gather, "ncclGather");
        sym(r.all_reduce, "ncclAllReduce");
        sym(r.group_start, "ncclGroupStart");
        sym(r.group_end, "ncclGroupEnd");
        sym(r.error_string, "ncclGetErrorString");
    });
    return r;
}

mrt_status need_rccl() {
    const Rccl& r = rccl();
    return r.why.empty() ? MRT_OK : mrt_internal_fail(MRT_ERR_NO_DEVICE, r.why.c_str());
}

mrt_status nccl_fail(const char* what, ncclResult_t e) {
    return mrt_internal_fail(MRT_ERR_HIP, (std::string(what) + ": " + rccl().error_string(e)).c_str());
}

#define NCCLCHK(what, x)                              \
    do {                                              \
        ncclResult_t e_ = (x);                        \
        if (e_ != ncclSuccess) return nccl_fail(what, e_); \
    } while (0)
#define HIPCHK(x)                                                                                                       \
    do {                                                                                                                \
        hipError_t e_ = (x);                                                                                            \
        if (e_ != hipSuccess) return mrt_internal_fail(MRT_ERR_HIP, (std::string(#x) + ": " + hipGetErrorString(e_)).c_str()); \
    } while (0)

// Every rank's pixel count under d's tile deal (world ranks), and the padded shard: the largest.
std::vector<uint32_t> shard_counts(const mrt_render_desc* d) {
    const uint32_t world = d->world ? d->world : 1u;
    std::vector<uint32_t> n(world);
    mrt_render_desc q = *d;
    q.pixels = nullptr;
    q.world = world;
    for (uint32_t r = 0; r < world; r++) {
        q.rank = r;
        n[r] = (uint32_t)mrt_internal_local_pixels(&q).size();
    }
    return n;
}

// Shard slot i = r * maxn + k of the gathered buffer holds pixel k of rank r: frame[map[i]] = it.
__global__ void __launch_bounds__(256) mrt_scatter_kernel(const float4* __restrict__ gathered, const uint32_t* __restrict__ map, uint32_t n,
                                                          float4* __restrict__ frame) {
    for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) {
        const uint32_t p = map[i];
        if (p != 0xFFFFFFFFu) frame[p] = gathered[i];
    }
}

}  // namespace

struct mrt_comm {
    ncclComm_t comm = nullptr;
    int device = 0;
    uint32_t world = 1, rank = 0;
    hipStream_t stream = nullptr;  // mrt_render_gather's
    // the tile deal of the last gather (width, height, tile size): padded shard and, on the root,
    // the shard-slot -> pixel map
    uint32_t w = 0, h = 0, tile = 0;
    bool have_layout = false;
    uint32_t maxn = 0, nlocal = 0;
    uint32_t* d_map = nullptr;
    float4* d_send = nullptr;   // this rank's shard, padded to maxn
    float4* d_recv = nullptr;   // root: world * maxn
    float4* d_local = nullptr;  // mrt_render_gather: the render's output (maxn)
    float4* d_frame = nullptr;  // mrt_render_gather, root: W * H
    uint64_t* d_rays = nullptr;
    size_t frame_cap = 0;
};

static mrt_status comm_setup(mrt_comm* c) {
    HIPCHK(hipSetDevice(c->device));
    HIPCHK(hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking));
    HIPCHK(hipMalloc((void**)&c->d_rays, 64));
    return MRT_OK;
}

extern "C" mrt_status mrt_comm_unique_id(uint8_t id[MRT_COMM_ID_BYTES]) {
    if (!id) return mrt_internal_fail(MRT_ERR_INVALID, "mrt_comm_unique_id: null");
    if (mrt_status st = need_rccl()) return st;
    ncclUniqueId u;
    NCCLCHK("ncclGetUniqueId", rccl().get_unique_id(&u));
    static_assert(sizeof u == MRT_COMM_ID_BYTES, "ncclUniqueId size");
    memcpy(id, &u, sizeof u);
    return MRT_OK;
}

extern "C" mrt_status mrt_comm_init_rank(int device, uint32_t world, uint32_t rank, const uint8_t id[MRT_COMM_ID_BYTES], mrt_comm** out) {
    if (!id || !out || world == 0 || rank >= world || device < 0) return mrt_internal_fail(MRT_ERR_INVALID, "mrt_comm_init_rank: bad argument");
    *out = nullptr;
    if (mrt_status st = need_rccl()) return st;
    HIPCHK(hipSetDevice(device));
    mrt_comm* c = new mrt_comm();
    c->device = device;
    c->world = world;
    c->rank = rank;
    ncclUniqueId u;
    memcpy(&u, id, sizeof u);
    const ncclResult_t e = rccl().init_rank(&c->comm, (int)world, u, (int)rank);
    if (e != ncclSuccess) {
        delete c;
        return nccl_fail("ncclCommInitRank", e);
    }
    if (mrt_status st = comm_setup(c)) {
        mrt_comm_free(c);
        return st;
    }
    *out = c;
    return MRT_OK;
}

extern "C" mrt_status mrt_comm_init_all(uint32_t world, const int* devices, mrt_comm** comms_out) {
    if (!devices || !comms_out || world == 0) return mrt_internal_fail(MRT_ERR_INVALID, "mrt_comm_init_all: bad argument");
    if (mrt_status st = need_rccl()) return st;
    std::vector<ncclComm_t> cs(world, nullptr);
    NCCLCHK("ncclCommInitAll", rccl().init_all(cs.data(), (int)world, devices));
    for (uint32_t r = 0; r < world; r++) {
        mrt_comm* c = new mrt_comm();
        c->comm = cs[r];
        c->device = devices[r];
        c->world = world;
        c->rank = r;
        comms_out[r] = c;
    }
    for (uint32_t r = 0; r < world; r++)
        if (mrt_status st = comm_setup(comms_out[r])) {
            for (uint32_t k = 0; k < world; k++) mrt_comm_free(comms_out[k]), comms_out[k] = nullptr;
            return st;
        }
    return MRT_OK;
}

extern "C" void mrt_comm_free(mrt_comm* c) {
    if (!c) return;
    (void)hipSetDevice(c->device);
    if (c->stream) (void)hipStreamSynchronize(c->stream);
    if (c->comm) (void)rccl().destroy(c->comm);
    for (void* p : {(void*)c->d_map, (void*)c->d_send, (void*)c->d_recv, (void*)c->d_local, (void*)c->d_frame, (void*)c->d_rays})
        if (p) (void)hipFree(p);
    if (c->stream) (void)hipStreamDestroy(c->stream);
    delete c;
}

extern "C" mrt_status mrt_gather_shard_pixels(const mrt_render_desc* d, uint32_t* n_out) {
    if (!d || !n_out || d->width == 0 || d->height == 0 || d->pixels) return mrt_internal_fail(MRT_ERR_INVALID, "mrt_gather_shard_pixels: bad desc");
    const std::vector<uint32_t> n = shard_counts(d);
    *n_out = *std::max_element(n.begin(), n.end());
    return MRT_OK;
}

// the padded shard and the root's slot -> pixel map for d's tile deal (cached per layout)
static mrt_status layout(mrt_comm* c, const mrt_render_desc* d) {
    const uint32_t tile = d->tile_size ? d->tile_size : 32u;
    if (c->have_layout && c->w == d->width && c->h == d->height && c->tile == tile) return MRT_OK;
    HIPCHK(hipSetDevice(c->device));
    if (c->stream) HIPCHK(hipStreamSynchronize(c->stream));  // (a gather in flight reads the old buffers)
    for (void** p : {(void**)&c->d_map, (void**)&c->d_send, (void**)&c->d_recv, (void**)&c->d_local})
        if (*p) (void)hipFree(*p), *p = nullptr;
    c->have_layout = false;
    mrt_render_desc q = *d;
    q.world = c->world;
    const std::vector<uint32_t> cnt = shard_counts(&q);
    c->maxn = std::max(1u, *std::max_element(cnt.begin(), cnt.end()));
    c->nlocal = cnt[c->rank];
    HIPCHK(hipMalloc((void**)&c->d_send, (size_t)c->maxn * 16));
    HIPCHK(hipMemset(c->d_send, 0, (size_t)c->maxn * 16));  // (the padding travels: defined bytes)
    HIPCHK(hipMalloc((void**)&c->d_local, (size_t)c->maxn * 16));
    if (c->rank == 0) {
        std::vector<uint32_t> map((size_t)c->world * c->maxn, 0xFFFFFFFFu);
        for (uint32_t r = 0; r < c->world; r++) {
            q.rank = r;
            const std::vector<uint32_t> px = mrt_internal_local_pixels(&q);
            std::copy(px.begin(), px.end(), map.begin() + (size_t)r * c->maxn);
        }
        HIPCHK(hipMalloc((void**)&c->d_map, map.size() * 4));
        HIPCHK(hipMemcpy(c->d_map, map.data(), map.size() * 4, hipMemcpyHostToDevice));
        HIPCHK(hipMalloc((void**)&c->d_recv, map.size() * 16));
    }
    c->w = d->width;
    c->h = d->height;
    c->tile = tile;
    c->have_layout = true;
    return MRT_OK;
}

extern "C" mrt_status mrt_gather_frame(mrt_comm* c, const mrt_render_desc* d, const float* d_local, float* d_frame, uint64_t* d_rays,
                                       void* stream) {
    if (!c || !d || !d_local) return mrt_internal_fail(MRT_ERR_INVALID, "mrt_gather_frame: null");
    if (d->pixels) return mrt_internal_fail(MRT_ERR_INVALID, "mrt_gather_frame: pixel-list renders are not tile shards");
    if ((d->world ? d->world : 1u) != c->world || d->rank != c->rank)
        return mrt_internal_fail(MRT_ERR_INVALID, "mrt_gather_frame: desc rank / world differ from the communicator's");
    if (c->rank == 0 && !d_frame) return mrt_internal_fail(MRT_ERR_INVALID, "mrt_gather_frame: the root needs d_frame");
    if (mrt_status st = layout(c, d)) return st;
    hipStream_t q = (hipStream_t)stream;
    HIPCHK(hipSetDevice(c->device));
    if (c->nlocal) HIPCHK(hipMemcpyAsync(c->d_send, d_local, (size_t)c->nlocal * 16, hipMemcpyDeviceToDevice, q));
    const Rccl& R = rccl();
    NCCLCHK("ncclGroupStart", R.group_start());
    ncclResult_t e = R.gather(c->d_send, c->rank == 0 ? (void*)c->d_recv : nullptr, (size_t)c->maxn * 4, ncclFloat32, 0, c->comm, q);
    if (e == ncclSuccess && d_rays) e = R.all_reduce(d_rays, d_rays, 1, ncclUint64, ncclSum, c->comm, q);
    const ncclResult_t e2 = R.group_end();
    if (e != ncclSuccess) return nccl_fail("ncclGather / ncclAllReduce", e);
    if (e2 != ncclSuccess) return nccl_fail("ncclGroupEnd", e2);
    if (c->rank == 0) {
        const uint32_t n = c->world * c->maxn;
        const uint32_t blocks = std::min<uint32_t>((n + 255) / 256, 4096);
        hipLaunchKernelGGL(mrt_scatter_kernel, dim3(blocks), dim3(256), 0, q, (const float4*)c->d_recv, (const uint32_t*)c->d_map, n,
                           (float4*)d_frame);
        HIPCHK(hipGetLastError());
    }
    return MRT_OK;
}

extern "C" mrt_status mrt_render_gather(mrt_scene* s, mrt_comm* c, const mrt_render_desc* d, float* rgb_out, uint64_t* rays_out) {
    if (!s || !c || !d) return mrt_internal_fail(MRT_ERR_INVALID, "mrt_render_gather: null");
    if (mrt_internal_scene_device(s) != c->device)
        return mrt_internal_fail(MRT_ERR_INVALID, "mrt_render_gather: the scene is not on the communicator's device");
    if (c->rank == 0 && !rgb_out) return mrt_internal_fail(MRT_ERR_INVALID, "mrt_render_gather: the root needs rgb_out");
    if (mrt_status st = layout(c, d)) return st;
    HIPCHK(hipSetDevice(c->device));
    const size_t frame = (size_t)d->width * d->height;
    if (c->rank == 0 && c->frame_cap < frame) {
        if (c->d_frame) (void)hipFree(c->d_frame);
        c->d_frame = nullptr;
        c->frame_cap = 0;
        HIPCHK(hipMalloc((void**)&c->d_frame, frame * 16));
        c->frame_cap = frame;
    }
    HIPCHK(hipMemsetAsync(c->d_rays, 0, 8, c->stream));
    if (mrt_status st = mrt_render_device(s, d, (float*)c->d_local, c->d_rays, c->stream)) return st;
    if (mrt_status st = mrt_render_join(s, c->stream)) return st;  // (MRT_RF_FOLD_ASYNC: the fold's stream)
    if (mrt_status st = mrt_gather_frame(c, d, (const float*)c->d_local, (float*)c->d_frame, c->d_rays, c->stream)) return st;
    uint64_t rays = 0;  // (every rank holds the all-reduced total)
    if (c->rank == 0) HIPCHK(hipMemcpyAsync(rgb_out, c->d_frame, frame * 16, hipMemcpyDeviceToHost, c->stream));
    HIPCHK(hipMemcpyAsync(&rays, c->d_rays, 8, hipMemcpyDeviceToHost, c->stream));
    HIPCHK(hipStreamSynchronize(c->stream));
    if (rays_out) *rays_out = rays;
    return MRT_OK;
}
