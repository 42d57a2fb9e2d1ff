// mrt_cli.cpp -- headless command-line driver with the reference's flags (cmdline_parser.cpp:78-123)
// in place of the SDL window loop of main() (main.cpp:283-498): builds the scene, renders it on the
// MI355X(s) through the C-ABI, prints the reference's "Trace: ... Mrays/s" line (main.cpp:403-406)
// and writes the image (-o out.pfm: linear; -o out.ppm: Drago tone map, main.cpp:416-444).
//
// -gpus N shards the work_queue tiles over N ranks (one host thread per rank, the tiles dealt in
// permuted rounds of N, mrt_local_pixels); 0 = every visible GPU.  Rank r renders on GPU r % (GPUs
// visible): with fewer GPUs than ranks several ranks share a device (the multi-rank assembly runs
// on one GPU as on eight); with -backend cpu each rank is a CPU-backend context of -threads workers.  -backend cpu renders on the host instead (the CPU backend: the
// same hot-path code compiled for the host, exact contract), with -threads worker threads as the
// reference's -threads (0 = every core).  -numerics exact|fast picks the GPU's arithmetic contract.
// -gather rccl|host: how a multi-GPU frame is assembled.  rccl (the default when every rank has a
// GPU of its own): each rank's mrt_render_gather renders its shard into device memory and one RCCL
// gather over xGMI plus a device scatter assemble the frame on GPU 0 (mrt_comm_init_all: one
// communicator per GPU in this process); host: each rank's mrt_render copies its own pixels into the
// shared host framebuffer (the only choice when ranks share a GPU, or with -backend cpu).
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <thread>
#include <vector>

#include "../../include/mrt.h"

static int fail(const char* what, mrt_status s) {
    fprintf(stderr, "%s: %s (%s)\n", what, mrt_strerror(s), mrt_last_error());
    return 1;
}

int main(int argc, char** argv) {
    mrt_params p;
    if (mrt_parse_argv(argc, argv, &p) != MRT_OK) return 0;  // -help
    const char* out = nullptr;
    const char* gather = nullptr;
    for (int i = 1; i + 1 < argc; i++) {
        if (!strcmp(argv[i], "-o")) out = argv[i + 1];
        if (!strcmp(argv[i], "-gather")) gather = argv[i + 1];
    }
    if (gather && strcmp(gather, "rccl") && strcmp(gather, "host")) {
        fprintf(stderr, "-gather: rccl or host\n");
        return 1;
    }

    auto t_gen = std::chrono::steady_clock::now();
    mrt_scene_blob* blob = nullptr;
    mrt_status st = mrt_select_scene(p.scene_select, float(p.buffer_width) / float(p.buffer_height), nullptr, &blob);
    if (st) return fail("select_scene", st);
    double gen_ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t_gen).count();
    mrt_scene_view view;
    mrt_scene_blob_view(blob, &view);

    const bool cpu = p.backend == 1;
    int ndev = 0, world = p.gpus ? (int)p.gpus : 1;
    if (!cpu) {
        if ((st = mrt_init(&ndev))) return fail("mrt_init", st);
        if (ndev < 1) return fail("mrt_init", MRT_ERR_NO_DEVICE);
        if (!p.gpus) world = ndev;
        if (world > ndev) fprintf(stderr, "-gpus %d: %d rank(s) on %d visible GPU(s)\n", world, world, ndev);
    }

    std::vector<mrt_scene*> scenes(world, nullptr);
    std::vector<mrt_render_desc> descs(world);
    for (int r = 0; r < world; r++) {
        if ((st = mrt_scene_upload(cpu ? MRT_DEVICE_CPU : r % ndev, &view, &scenes[r]))) return fail("scene_upload", st);
        mrt_default_render_desc(&p, &descs[r]);
        descs[r].rank = (uint32_t)r;
        descs[r].world = (uint32_t)world;
        if (!cpu && (st = mrt_prepare(scenes[r], &descs[r]))) return fail("prepare", st);
    }
    if (descs[0].flags & MRT_RF_REF_ORDER) {  // main.cpp:338-366: the workers' (initstate, initseq)
        if (!cpu) {
            fprintf(stderr, "-order ref: the reference's per-thread RNG order runs on the CPU backend only (-backend cpu)\n");
            return 1;
        }
        if (world > 1) {
            fprintf(stderr, "-order ref: the reference's per-thread RNG order is one rank's (use -order path with -gpus)\n");
            return 1;
        }
        const uint32_t n = p.num_threads ? p.num_threads : std::max(1u, std::thread::hardware_concurrency());
        std::vector<uint64_t> is(n), iq(n);
        if ((st = mrt_worker_seeds(blob, n, is.data(), iq.data()))) return fail("worker_seeds", st);
        if ((st = mrt_set_worker_seeds(scenes[0], n, is.data(), iq.data()))) return fail("set_worker_seeds", st);
        descs[0].threads = n;
    }
    // the RCCL gather needs a GPU per rank (RCCL refuses two ranks on one device)
    const bool use_rccl = !cpu && world <= ndev && (gather ? !strcmp(gather, "rccl") : world > 1);
    if (gather && !strcmp(gather, "rccl") && !use_rccl) {
        fprintf(stderr, "-gather rccl: needs the GPU backend and a GPU per rank (%d ranks, %d GPUs)\n", world, ndev);
        return 1;
    }
    std::vector<mrt_comm*> comms(world, nullptr);
    if (use_rccl) {
        std::vector<int> devs(world);
        for (int r = 0; r < world; r++) devs[r] = r;
        if ((st = mrt_comm_init_all((uint32_t)world, devs.data(), comms.data()))) return fail("comm_init_all", st);
    }
    std::vector<float> img((size_t)p.buffer_width * p.buffer_height * 4, 0.0f);
    std::vector<uint64_t> rays(world, 0);
    std::vector<mrt_status> sts(world, MRT_OK);

    auto t0 = std::chrono::steady_clock::now();  // main.cpp:375
    std::vector<std::thread> th;
    for (int r = 0; r < world; r++)
        th.emplace_back([&, r] {
            sts[r] = use_rccl ? mrt_render_gather(scenes[r], comms[r], &descs[r], r == 0 ? img.data() : nullptr, &rays[r])
                              : mrt_render(scenes[r], &descs[r], img.data(), &rays[r], nullptr);
        });
    for (auto& t : th) t.join();
    double secs = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
    for (int r = 0; r < world; r++)
        if (sts[r]) return fail("render", sts[r]);
    uint64_t total = 0;
    if (use_rccl) total = rays[0];  // (all-reduced over the ranks)
    else
        for (uint64_t x : rays) total += x;
    char where[64];
    if (cpu) {
        mrt_kernel_info ki{};
        mrt_scene_kernel_info(scenes[0], &ki);
        snprintf(where, sizeof where, "CPU, %d x %u threads", world, ki.grid);
    } else if (world <= ndev) {
        snprintf(where, sizeof where, use_rccl ? "%d x MI355X, RCCL gather" : "%d x MI355X", world);
    } else {
        snprintf(where, sizeof where, "%d ranks on %d x MI355X", world, ndev);
    }
    printf("MiniRayTracer - Scene: %.0fms - Trace: %.2fs - %.3f Mrays/s | %.3f us/ray  [%s, %u spp, %s numerics]\n", gen_ms,
           secs, (total * 0.000001) / secs, (secs * 1000000.0) / (double)total, where, descs[0].sqrt_samples * descs[0].sqrt_samples,
           p.numerics ? "fast" : "exact");
    printf("rays %llu\n", (unsigned long long)total);

    if (out) {
        std::string o = out;
        FILE* f = fopen(out, "wb");
        if (!f) return fail("open output", MRT_ERR_IO);
        if (o.size() > 4 && o.substr(o.size() - 4) == ".ppm") {
            std::vector<uint32_t> argb((size_t)p.buffer_width * p.buffer_height);
            mrt_tonemap_argb(img.data(), p.buffer_width, p.buffer_height, argb.data());
            fprintf(f, "P6\n%u %u\n255\n", p.buffer_width, p.buffer_height);
            for (int y = (int)p.buffer_height - 1; y >= 0; y--)  // display is flipped (platform_linux.cpp:84)
                for (uint32_t x = 0; x < p.buffer_width; x++) {
                    uint32_t c = argb[(size_t)y * p.buffer_width + x];
                    unsigned char px[3] = {(unsigned char)(c >> 16), (unsigned char)(c >> 8), (unsigned char)c};
                    fwrite(px, 1, 3, f);
                }
        } else {
            fprintf(f, "PF\n%u %u\n-1.0\n", p.buffer_width, p.buffer_height);
            for (size_t i = 0; i < (size_t)p.buffer_width * p.buffer_height; i++) fwrite(&img[i * 4], 4, 3, f);
        }
        fclose(f);
    }
    for (auto* c : comms) mrt_comm_free(c);
    for (auto* s : scenes) mrt_scene_free(s);
    mrt_scene_blob_free(blob);
    return 0;
}
