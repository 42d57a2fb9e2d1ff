// oracle/ref/harness.cpp -- TEST INFRASTRUCTURE ONLY (never shipped, never on the product path).
//
// Headless driver that links the reference's OWN translation units (compiled from
// /root/reference by oracle/ref/build_ref.sh) and exposes them as a command-line oracle:
//
//   --h-mode shipped   run the reference main() as shipped (threads, work_queue, tone map loop),
//                      headless; print rays / trace seconds / Mrays/s from the reference's own
//                      title string (main.cpp:399-406) and dump G_linearBackBuffer as PFM
//                      (--h-out) and the Drago tone-mapped G_backBuffer as raw ARGB32 (--h-argb).
//   --h-mode stream    "stream-matched" render: for every (pixel, sample) path re-seed the
//                      reference PCG with the path key (see path_key below), call the reference
//                      camera::get_ray + trace() unchanged, accumulate with draw() (mode 0,
//                      main.cpp:151-175) or draw2() (mode 1, main.cpp:207-231) rules.
//                      --h-pixels FILE (raw uint32 pixel indices) renders only those pixels and
//                      --h-px-out FILE writes their values (raw float32 n x 3, list order).
//   --h-mode kat       PCG / sampler known-answer vectors (pcg.cpp).
//   --h-mode scene     dump the scene graph select_scene() builds (types, parameters as float
//                      bits, BVH topology incl. node_order) and the camera.
//   --h-mode hits      closest-hit KATs: seeded random rays against scene.objects->hit().
//
// The reference's platform layer (SDL / GDI) is not compiled; the MRT_* entry points declared in
// platform.h:4-19 are implemented below as a headless driver.  With -DMRT_MATHMATCH the float
// libm entry points the reference calls (sinf, cosf, tanf, logf, powf, atan2f, asinf, ...) are
// interposed by the numerics-contract functions of include/mrt_mathfn.h -- the definition the
// product and the C restatement use -- so the oracle can be compared bit-for-bit.

#include <atomic>
#include <algorithm>
#include <cassert>
#include <cinttypes>
#include <cmath>
#include <cstdarg>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <iostream>
#include <limits>
#include <memory>
#include <string>
#include <thread>
#include <type_traits>
#include <utility>
#include <vector>
#include <time.h>
#include <unistd.h>
#include <x86intrin.h>

#ifdef MRT_MATHMATCH
#include "../../include/mrt_mathfn.h"  // the project's numerics contract for transcendentals
extern "C" {
float sinf(float x) { return mrt_sinf(x); }
float cosf(float x) { return mrt_cosf(x); }
void sincosf(float x, float* s, float* c) { *s = mrt_sinf(x); *c = mrt_cosf(x); }
float tanf(float x) { return mrt_tanf(x); }
float logf(float x) { return mrt_logf(x); }
float log10f(float x) { return mrt_log10f(x); }
float expf(float x) { return mrt_expf(x); }
float powf(float x, float y) { return mrt_powf(x, y); }
float atan2f(float y, float x) { return mrt_atan2f(y, x); }
float asinf(float x) { return mrt_asinf(x); }
}
#endif

// read pod_bvh / object internals for topology dumps (layout unchanged by class->struct)
#define class struct
#include "all_scene_objects.h"
#include "scene.h"
#include "cmdline_parser.h"
#include "work_queue.h"
#undef class

scene harness_select_scene(scenes choose, float aspect);
#define select_scene harness_select_scene
#define main mrt_main
#include "main.cpp"
#undef main
#undef select_scene

// ------------------------------------------------------------------------------------------
// headless platform layer (platform.h:4-19)
// ------------------------------------------------------------------------------------------
static std::atomic<bool> H_done{false};
static std::string H_title;

void MRT_PlatformInit() {}
void MRT_PlatformDestroy() {}
void MRT_HandleMessages() {
    if (H_done.load()) MRT::WindowCallback(MRT::MRT_CLOSE);
}
void MRT_CreateWindow(uint32_t, uint32_t, uint32_t, uint32_t) {}
void MRT_SetWindowTitle(const char* str) {
    if (strstr(str, "Mrays/s")) {
        H_title = str;
        H_done.store(true);
    }
}
void MRT_DrawToWindow(const uint32_t*) {}
void MRT_ReportProgress(uint64_t, uint64_t) {}
void MRT_DebugPrint(const char* format, ...) {
    va_list a;
    va_start(a, format);
    vfprintf(stderr, format, a);
    va_end(a);
}
void MRT_Assert(bool cond) {
    if (!cond) abort();
}
void MRT_Assert(bool cond, const char* msg) {
    if (!cond) {
        fprintf(stderr, "assert: %s\n", msg ? msg : "");
        abort();
    }
}
void MRT_Sleep(uint32_t ms) { usleep(ms * 1000u); }
void MRT_LowerThreadPriority() {}
uint64_t MRT_GetTime() {
    struct timespec ts;
    clock_gettime(CLOCK_MONOTONIC_RAW, &ts);
    return (uint64_t)ts.tv_nsec + (uint64_t)ts.tv_sec * 1000000000ull;
}
float MRT_TimeDelta(uint64_t start, uint64_t stop) { return ((stop - start) / 1000000000.0); }

// ------------------------------------------------------------------------------------------
// helpers
// ------------------------------------------------------------------------------------------
static const char* harg(int argc, char** argv, const char* name, const char* def) {
    for (int i = 1; i + 1 < argc; i++)
        if (!strcmp(argv[i], name)) return argv[i + 1];
    return def;
}
static uint32_t fbits(float f) {
    uint32_t u;
    memcpy(&u, &f, 4);
    return u;
}

// Path key of the stream-matched contract (DESIGN.md "Stream key"): every (pixel, sample) path
// owns one PCG32 stream, independent of tiles, threads and GPU count.
static uint64_t splitmix64(uint64_t z) {
    z += 0x9E3779B97F4A7C15ull;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}
static void path_key(uint64_t seed, uint64_t path, uint64_t* st, uint64_t* sq) {
    *st = splitmix64(seed ^ path);
    *sq = path;
}

// minimal .npy writer (little-endian, C order)
static void write_npy(const char* fn, const char* descr, const std::vector<size_t>& shape, const void* data,
                      size_t bytes) {
    std::string sh = "(";
    for (size_t i = 0; i < shape.size(); i++) sh += std::to_string(shape[i]) + (shape.size() == 1 ? "," : (i + 1 < shape.size() ? ", " : ""));
    sh += ")";
    std::string hdr = std::string("{'descr': '") + descr + "', 'fortran_order': False, 'shape': " + sh + ", }";
    size_t total = 10 + hdr.size() + 1;
    size_t pad = (64 - total % 64) % 64;
    hdr += std::string(pad, ' ') + "\n";
    FILE* f = fopen(fn, "wb");
    if (!f) { perror(fn); exit(2); }
    unsigned char magic[8] = {0x93, 'N', 'U', 'M', 'P', 'Y', 1, 0};
    fwrite(magic, 1, 8, f);
    uint16_t hl = (uint16_t)hdr.size();
    fwrite(&hl, 2, 1, f);
    fwrite(hdr.data(), 1, hdr.size(), f);
    fwrite(data, 1, bytes, f);
    fclose(f);
}

static void write_pfm(const char* fn, const Vec3* buf, uint32_t w, uint32_t h) {
    FILE* f = fopen(fn, "wb");
    if (!f) { perror(fn); exit(2); }
    fprintf(f, "PF\n%u %u\n-1.0\n", w, h);
    for (size_t i = 0; i < (size_t)w * h; i++) fwrite(&buf[i].x, 4, 3, f);  // row 0 = bottom (PFM order)
    fclose(f);
}

// ------------------------------------------------------------------------------------------
// custom scenes (config C3: wt_teapot in the Cornell box) built from reference
// classes only; everything else forwards to the reference select_scene.
// ------------------------------------------------------------------------------------------
#undef select_scene
scene select_scene(scenes choose, float aspect);
static const char* H_custom = nullptr;
static const char* H_objdir = "../obj";

scene harness_select_scene(scenes choose, float aspect) {
    if (H_custom && !strcmp(H_custom, "teapot")) {
        Vec3 cam_pos = {278, 278, -800};
        Vec3 lookat = {278, 278, 100};
        Vec3 up = {0, 1, 0};
        float focus_dist = (cam_pos - lookat).length();
        camera* cam = new camera(cam_pos, lookat, up, 40.0f, aspect, 0.0f, focus_dist, 0.0f, 1.0f);
        scene_object** list = new scene_object*[8];
        int i = 0;
        material* red = new lambertian(new color_tex(Vec3(0.65f, 0.055f, 0.06f)));
        material* white = new lambertian(new color_tex(Vec3(0.73f, 0.73f, 0.73f)));
        material* green = new lambertian(new color_tex(Vec3(0.117f, 0.44f, 0.115f)));
        material* light = new diffuse_light(new color_tex(Vec3(15.f)));
        list[i++] = new yz_rect(555, 0, 0, 555, 555, green);
        list[i++] = new yz_rect(0, 555, 0, 555, 0, red);
        xz_rect* l = new xz_rect(343, 213, 227, 332, 554, light);
        list[i++] = l;
        list[i++] = new xz_rect(555, 0, 0, 555, 555, white);
        list[i++] = new xz_rect(0, 555, 0, 555, 0, white);
        list[i++] = new xy_rect(555, 0, 0, 555, 555, white);
        size_t tris = 0;
        std::string p = std::string(H_objdir) + "/wt_teapot.obj";
        std::unique_ptr<triangle[]> tp = readObj(p.c_str(), white, &tris, false, Mat4::Scale(200.0f), Vec3(264.3f, 0, 278));
        if (!tris) { fprintf(stderr, "teapot obj not found: %s\n", p.c_str()); exit(2); }
        list[i++] = new pod_bvh<triangle>(tp.get(), tris, 0.0f, 1.0f);
        scene_object* objects = new object_list<scene_object>(list, i, 0.0f, 1.0f);
        scene_object** b = new scene_object*[1];
        b[0] = l;
        scene_object* biased = new object_list<scene_object>(b, 1, 0.0f, 1.0f);
        return scene{objects, biased, cam};
    }
    return select_scene(choose, aspect);
}

// ------------------------------------------------------------------------------------------
// scene dump (vtable identity; the reference is built without RTTI)
// ------------------------------------------------------------------------------------------
static void* vt(const void* o) { return *(void* const*)o; }

struct VT {
    void *ol_so, *ol_sp, *ol_bx, *bvh_sp, *bvh_box, *pod_tri, *tr, *roty, *sph, *xy, *xz, *yz, *bx, *vol;
    void *lam, *iso, *met, *die, *lig;
    void *ctex, *chk, *per, *img;
};
static VT vts() {
    static VT v;
    static bool init = false;
    if (init) return v;
    init = true;
    material* m = new lambertian(new color_tex(Vec3(1.f)));
    sphere** sl = new sphere*[1];
    sl[0] = new sphere(Vec3(0, 0, 0), 1, m);
    box** bl = new box*[1];
    bl[0] = new box(Vec3(0, 0, 0), Vec3(1, 1, 1), m);
    scene_object** ol = new scene_object*[1];
    ol[0] = sl[0];
    triangle* tri = new triangle(Vec3(0, 0, 0), Vec3(1, 0, 0), Vec3(0, 1, 0), m);
    v.ol_so = vt(new object_list<scene_object>(ol, 1, 0, 0));
    v.ol_sp = vt(new object_list<sphere>(sl, 1, 0, 0));
    v.ol_bx = vt(new object_list<box>(bl, 1, 0, 0));
    v.bvh_sp = vt(new bvh_node<sphere>(sl, 1, 0, 0));
    v.bvh_box = vt(new bvh_node<box>(bl, 1, 0, 0));
    v.pod_tri = vt(new pod_bvh<triangle>(tri, 1, 0, 0));
    v.tr = vt(new translate(sl[0], Vec3(0, 0, 0)));
    v.roty = vt(new rotate_y(sl[0], 10));
    v.sph = vt(sl[0]);
    v.xy = vt(new xy_rect(0, 1, 0, 1, 0, m));
    v.xz = vt(new xz_rect(0, 1, 0, 1, 0, m));
    v.yz = vt(new yz_rect(0, 1, 0, 1, 0, m));
    v.bx = vt(bl[0]);
    v.vol = vt(new constant_volume(sl[0], 1, new color_tex(Vec3(1.f))));
    v.lam = vt(m);
    v.iso = vt(new isotropic(new color_tex(Vec3(1.f))));
    v.met = vt(new metal(new color_tex(Vec3(1.f)), 1));
    v.die = vt(new dielectric(1.5f));
    v.lig = vt(new diffuse_light(new color_tex(Vec3(1.f))));
    v.ctex = vt(new color_tex(Vec3(1.f)));
    v.chk = vt(new checker_tex(nullptr, nullptr, 1));
    v.per = vt(new perlin_tex(1));
    v.img = vt(new image_tex(nullptr, 1, 1));
    return v;
}

static std::string F(float f) { return std::to_string(fbits(f)); }
static std::string V3(const Vec3& v) { return "[" + F(v.x) + "," + F(v.y) + "," + F(v.z) + "]"; }
static std::string BOX(const aabb& b) { return "[" + V3(b.min) + "," + V3(b.max) + "]"; }

static std::string dump_tex(const texture* t) {
    VT v = vts();
    void* p = vt(t);
    if (p == v.ctex) return "{\"t\":\"color\",\"c\":" + V3(((color_tex*)t)->color) + "}";
    if (p == v.chk) {
        const checker_tex* c = (const checker_tex*)t;
        return "{\"t\":\"checker\",\"scale\":" + F(c->scale) + ",\"even\":" + dump_tex(c->even) + ",\"odd\":" + dump_tex(c->odd) + "}";
    }
    if (p == v.per) return "{\"t\":\"perlin\",\"scale\":" + F(((perlin_tex*)t)->scale) + "}";
    if (p == v.img) {
        const image_tex* im = (const image_tex*)t;
        uint64_t h = 1469598103934665603ull;  // FNV-1a of the texels
        for (size_t i = 0; i < (size_t)im->width * im->height * 3; i++) h = (h ^ im->data[i]) * 1099511628211ull;
        return "{\"t\":\"image\",\"w\":" + std::to_string(im->width) + ",\"h\":" + std::to_string(im->height) + ",\"fnv\":\"" + std::to_string(h) + "\"}";
    }
    return "{\"t\":\"?\"}";
}
static std::string dump_mat(const material* m) {
    VT v = vts();
    void* p = vt(m);
    if (p == v.lam) return "{\"m\":\"lambertian\",\"tex\":" + dump_tex(((lambertian*)m)->albedo) + "}";
    if (p == v.iso) return "{\"m\":\"isotropic\",\"tex\":" + dump_tex(((isotropic*)m)->albedo) + "}";
    if (p == v.met) return "{\"m\":\"metal\",\"gloss\":" + F(((metal*)m)->gloss) + ",\"tex\":" + dump_tex(((metal*)m)->albedo) + "}";
    if (p == v.die) return "{\"m\":\"dielectric\",\"ref\":" + F(((dielectric*)m)->ref_index) + "}";
    if (p == v.lig) return "{\"m\":\"light\",\"scale\":" + F(((diffuse_light*)m)->scale) + ",\"tex\":" + dump_tex(((diffuse_light*)m)->emissive) + "}";
    return "{\"m\":\"?\"}";
}

static std::string dump_obj(const scene_object* o);

template <typename T>
static std::string dump_list(const object_list<T>* l) {
    std::string s = "{\"k\":\"list\",\"hasBox\":" + std::to_string((int)l->hasBox) + ",\"box\":" + (l->hasBox ? BOX(l->box) : std::string("null")) + ",\"ch\":[";
    for (size_t i = 0; i < l->count; i++) s += (i ? "," : "") + dump_obj(l->list[i]);
    return s + "]}";
}
template <typename T>
static std::string dump_bvh(const bvh_node<T>* b) {
    return "{\"k\":\"bvh\",\"box\":" + BOX(b->box) + ",\"order\":" + std::to_string((int)b->node_order) + ",\"same\":" +
           std::to_string((int)(b->left == b->right)) + ",\"l\":" + dump_obj(b->left) + ",\"r\":" + dump_obj(b->right) + "}";
}

static std::string dump_obj(const scene_object* o) {
    VT v = vts();
    void* p = vt(o);
    if (p == v.ol_so) return dump_list((const object_list<scene_object>*)o);
    if (p == v.ol_sp) return dump_list((const object_list<sphere>*)o);
    if (p == v.ol_bx) return dump_list((const object_list<box>*)o);
    if (p == v.bvh_sp) return dump_bvh((const bvh_node<sphere>*)o);
    if (p == v.bvh_box) return dump_bvh((const bvh_node<box>*)o);
    if (p == v.tr) {
        const translate* t = (const translate*)o;
        return "{\"k\":\"translate\",\"off\":" + V3(t->offset) + ",\"c\":" + dump_obj(t->obj) + "}";
    }
    if (p == v.roty) {
        const rotate_y* r = (const rotate_y*)o;
        return "{\"k\":\"rotate_y\",\"sin\":" + F(r->sin_theta) + ",\"cos\":" + F(r->cos_theta) + ",\"hasBox\":" +
               std::to_string((int)r->hasBox) + ",\"box\":" + BOX(r->bbox) + ",\"c\":" + dump_obj(r->obj) + "}";
    }
    if (p == v.sph) {
        const sphere* s = (const sphere*)o;
        return "{\"k\":\"sphere\",\"c0\":" + V3(s->center0) + ",\"c1\":" + V3(s->center1) + ",\"t0\":" + F(s->time0) + ",\"t1\":" +
               F(s->time1) + ",\"moving\":" + std::to_string((int)s->isMoving) + ",\"r\":" + F(s->radius) + ",\"mat\":" + dump_mat(s->mat_ptr) + "}";
    }
    if (p == v.xy || p == v.xz || p == v.yz) {
        const char* k = p == v.xy ? "xy_rect" : (p == v.xz ? "xz_rect" : "yz_rect");
        float a0, a1, b0, b1, kk, ns;
        material* m;
        if (p == v.xy) { auto r = (const xy_rect*)o; a0 = r->x0; a1 = r->x1; b0 = r->y0; b1 = r->y1; kk = r->z; ns = r->normal_sign; m = r->mat_ptr; }
        else if (p == v.xz) { auto r = (const xz_rect*)o; a0 = r->x0; a1 = r->x1; b0 = r->z0; b1 = r->z1; kk = r->y; ns = r->normal_sign; m = r->mat_ptr; }
        else { auto r = (const yz_rect*)o; a0 = r->y0; a1 = r->y1; b0 = r->z0; b1 = r->z1; kk = r->x; ns = r->normal_sign; m = r->mat_ptr; }
        return std::string("{\"k\":\"") + k + "\",\"a0\":" + F(a0) + ",\"a1\":" + F(a1) + ",\"b0\":" + F(b0) + ",\"b1\":" + F(b1) +
               ",\"kk\":" + F(kk) + ",\"ns\":" + F(ns) + ",\"mat\":" + dump_mat(m) + "}";
    }
    if (p == v.bx) {
        const box* b = (const box*)o;
        return "{\"k\":\"box\",\"min\":" + V3(b->min) + ",\"max\":" + V3(b->max) + ",\"rects\":" + dump_list(b->rect_list) + "}";
    }
    if (p == v.vol) {
        const constant_volume* c = (const constant_volume*)o;
        return "{\"k\":\"volume\",\"density\":" + F(c->density) + ",\"phase\":" + dump_mat(c->phase_function) + ",\"b\":" + dump_obj(c->boundary) + "}";
    }
    if (p == v.pod_tri) {
        const pod_bvh<triangle>* b = (const pod_bvh<triangle>*)o;
        std::string s = "{\"k\":\"pod_bvh\",\"prim_count\":" + std::to_string(b->prim_count) + ",\"node_count\":" + std::to_string(b->node_count) +
                        ",\"mat\":" + dump_mat(b->prim_count ? b->prims[0].mat_ptr : nullptr) + ",\"nodes\":[";
        for (uint32_t i = 0; i < b->node_count; i++) {
            const pod_bvh_node& n = b->nodes[i];
            s += (i ? "," : "") + std::string("[") + BOX(n.box) + "," + std::to_string(n.left) + "," + std::to_string(n.prim_offset) + "," +
                 std::to_string(n.prim_count) + "," + std::to_string((int)n.node_order) + "]";
        }
        s += "],\"prims\":[";
        for (uint32_t i = 0; i < b->prim_count; i++) {
            const triangle& t = b->prims[i];
            s += (i ? "," : "") + std::string("[") + V3(t.m) + "," + V3(t.u) + "," + V3(t.v) + "," + V3(t.mn) + "," + V3(t.un) + "," + V3(t.vn) + "]";
        }
        return s + "]}";
    }
    return "{\"k\":\"?\"}";
}

// ------------------------------------------------------------------------------------------
// modes
// ------------------------------------------------------------------------------------------
static int mode_kat(int argc, char** argv) {
    uint64_t st = strtoull(harg(argc, argv, "--h-state", "42"), nullptr, 0);
    uint64_t sq = strtoull(harg(argc, argv, "--h-seq", "54"), nullptr, 0);
    int n = atoi(harg(argc, argv, "--h-n", "64"));
    printf("{\"state\":%" PRIu64 ",\"seq\":%" PRIu64 ",", st, sq);
    Init_Thread_RNG(st, sq);
    printf("\"rand32\":[");
    for (int i = 0; i < n; i++) printf("%s%u", i ? "," : "", rand32());
    Init_Thread_RNG(st, sq);
    printf("],\"randf\":[");
    for (int i = 0; i < n; i++) printf("%s%u", i ? "," : "", fbits(randf()));
    auto vec = [&](const char* name, Vec3 (*fn)()) {
        Init_Thread_RNG(st, sq);
        printf("],\"%s\":[", name);
        for (int i = 0; i < n; i++) {
            Vec3 v = fn();
            printf("%s[%u,%u,%u]", i ? "," : "", fbits(v.x), fbits(v.y), fbits(v.z));
        }
        printf("],\"%s_next\":%u", name, rand32());
        printf(",\"%s_dummy\":[", name);
    };
    vec("in_sphere", random_in_sphere);
    vec("in_disk", random_in_disk);
    vec("cosine_dir", random_cosine_direction);
    vec("on_sphere", random_on_sphere_uniform);
    printf("]}\n");
    return 0;
}

// stb-decoded earthmap texels exactly as scene.cpp:139/268/402 load them (stbi_load(..., 3))
extern "C" unsigned char* stbi_load(char const* filename, int* x, int* y, int* comp, int req_comp);
static int mode_texels(int argc, char** argv) {
    const char* in = harg(argc, argv, "--h-in", "../earthmap.jpg");
    const char* out = harg(argc, argv, "--h-out", "earthmap.rgb");
    int w, h, c;
    unsigned char* px = stbi_load(in, &w, &h, &c, 3);
    if (!px) { fprintf(stderr, "stbi_load failed: %s\n", in); return 2; }
    FILE* f = fopen(out, "wb");
    fwrite(px, 1, (size_t)w * h * 3, f);
    fclose(f);
    printf("{\"w\":%d,\"h\":%d,\"channels\":%d}\n", w, h, c);
    return 0;
}

static int mode_scene(int argc, char** argv) {
    MRT_Params* p = getParams();
    Init_Thread_RNG(11350390909718046443uLL, 6305599193148252115uLL);
    scene sc = harness_select_scene((scenes)p->sceneSelect, float(p->bufferWidth) / float(p->bufferHeight));
    const camera* c = sc.camera;
    printf("{\"camera\":{\"origin\":%s,\"u\":%s,\"v\":%s,\"w\":%s,\"llc\":%s,\"horz\":%s,\"vert\":%s,\"lens\":%s,\"t0\":%s,\"t1\":%s},",
           V3(c->origin).c_str(), V3(c->u).c_str(), V3(c->v).c_str(), V3(c->w).c_str(), V3(c->llcorner).c_str(), V3(c->horz).c_str(),
           V3(c->vert).c_str(), F(c->lens_radius).c_str(), F(c->time0).c_str(), F(c->time1).c_str());
    // worker seeds exactly as main.cpp:357-361 for 2 threads (RNG state after scene generation)
    uint64_t s0a = (uint64(rand32()) << 32);
    s0a |= rand32();
    uint64_t s0b = (uint64(rand32()) << 32);
    s0b |= rand32();
    printf("\"worker0\":[\"%" PRIu64 "\",\"%" PRIu64 "\"],", s0a, s0b);
    printf("\"objects\":%s,", dump_obj(sc.objects).c_str());
    printf("\"biased\":%s}\n", sc.biased_objects ? dump_obj(sc.biased_objects).c_str() : "null");
    return 0;
}

static int mode_hits(int argc, char** argv) {
    MRT_Params* p = getParams();
    Init_Thread_RNG(11350390909718046443uLL, 6305599193148252115uLL);
    scene sc = harness_select_scene((scenes)p->sceneSelect, float(p->bufferWidth) / float(p->bufferHeight));
    int n = atoi(harg(argc, argv, "--h-n", "4096"));
    const char* out = harg(argc, argv, "--h-out", "hits.npy");
    // rays: camera rays at random (u,v) then one random continuation from the hit point
    std::vector<float> rec((size_t)n * 16, 0.f);
    for (int i = 0; i < n; i++) {
        Init_Thread_RNG(1234567 + (uint64_t)i, 7654321);  // ray generation stream
        float* r = &rec[(size_t)i * 16];
        Vec3 o, d;
        float tm;
        int ins = 0;
        if (i % 2 == 0) {
            ray cr = sc.camera->get_ray(randf(), randf());
            o = cr.origin; d = cr.dir; tm = cr.time;
        } else {
            o = Vec3(randf() * 555.f, randf() * 555.f, randf() * 555.f);
            d = random_in_sphere();
            tm = randf();
            ins = (i % 6 == 1);
        }
        ray rr(o, d, tm, ins);
        hit_record h;
        Init_Thread_RNG((uint64_t)i, 4242);  // constant_volume::hit draws randf() (volumes.cpp:24)
        bool hit = sc.objects->hit(rr, 0.001f, std::numeric_limits<float>::max(), &h);
        r[0] = rr.origin.x; r[1] = rr.origin.y; r[2] = rr.origin.z;
        r[3] = d.x; r[4] = d.y; r[5] = d.z;  // constructor input (rr.dir = normalize(d))
        r[6] = rr.time; memcpy(&r[7], &ins, 4);
        int hh = hit ? 1 : 0;
        memcpy(&r[8], &hh, 4);
        if (hit) { r[9] = h.t; r[10] = h.p.x; r[11] = h.p.y; r[12] = h.p.z; r[13] = h.n.x; r[14] = h.n.y; r[15] = h.n.z; }
    }
    write_npy(out, "<f4", {(size_t)n, 16}, rec.data(), rec.size() * 4);
    printf("{\"n\":%d}\n", n);
    return 0;
}

static int mode_stream(int argc, char** argv) {
    MRT_Params* p = getParams();
    uint64_t seed = strtoull(harg(argc, argv, "--h-seed", "11350390909718046443"), nullptr, 0);
    int nthreads = atoi(harg(argc, argv, "--h-threads", "1"));
    const char* out = harg(argc, argv, "--h-out", nullptr);
    const char* paths_out = harg(argc, argv, "--h-paths", nullptr);
    int acc_mode = atoi(harg(argc, argv, "--h-acc", "0"));
    const uint32_t W = p->bufferWidth, H = p->bufferHeight;

    Init_Thread_RNG(11350390909718046443uLL, 6305599193148252115uLL);  // main.cpp:302
    scene sc = harness_select_scene((scenes)p->sceneSelect, float(W) / float(H));

    uint32 sqrt_samples = (uint32)MRT::sqrt((float)p->samplesPerPixel);  // main.cpp:319-332
    uint32 ns = sqrt_samples * sqrt_samples;
    std::vector<vec2> dist(ns);
    for (uint32 i = 0; i < sqrt_samples; i++)
        for (uint32 j = 0; j < sqrt_samples; j++) {
            dist[i * sqrt_samples + j].x = (i + 0.5f) / (float)sqrt_samples;
            dist[i * sqrt_samples + j].y = (j + 0.5f) / (float)sqrt_samples;
        }

    std::vector<Vec3> img((size_t)W * H);
    std::vector<float> paths;
    std::vector<uint32_t> pathrays;
    if (paths_out) {
        paths.resize((size_t)W * H * ns * 3);
        pathrays.resize((size_t)W * H * ns);
        nthreads = 1;  // per-path ray counts come from the shared counter
    }
    // --h-pixels: render only the listed pixels (raw little-endian uint32 row-major indices) and
    // write their values to --h-px-out (raw float32, n x 3, list order); rays = the listed pixels'
    std::vector<uint32_t> plist;
    const char* plist_in = harg(argc, argv, "--h-pixels", nullptr);
    const char* plist_out = harg(argc, argv, "--h-px-out", nullptr);
    if (plist_in) {
        FILE* f = fopen(plist_in, "rb");
        if (!f) { fprintf(stderr, "cannot read %s\n", plist_in); return 2; }
        uint32_t v;
        while (fread(&v, 4, 1, f) == 1) {
            if (v >= W * H) { fprintf(stderr, "pixel %u outside the image\n", v); return 2; }
            plist.push_back(v);
        }
        fclose(f);
        if (paths_out) { fprintf(stderr, "--h-pixels and --h-paths are exclusive\n"); return 2; }
    }
    std::atomic<uint32_t> next_row{0};
    uint64_t t0 = MRT_GetTime();
    auto worker = [&]() {
        for (;;) {
            uint32_t y = next_row.fetch_add(1);
            if (plist_in ? y >= plist.size() : y >= H) break;
            const uint32_t x0 = plist_in ? plist[y] % W : 0u, x1 = plist_in ? x0 + 1u : W;
            if (plist_in) y = plist[y] / W;
            for (uint32_t x = x0; x < x1; x++) {
                uint64_t pix = (uint64_t)x + (uint64_t)y * W;
                Vec3 color(0, 0, 0);
                for (uint32_t s = 0; s < ns; s++) {
                    uint64_t st, sq;
                    path_key(seed, pix * ns + s, &st, &sq);
                    Init_Thread_RNG(st, sq);
                    size_t before = G_rayCounter.load();
                    float u = (x + dist[s].x) / (float)W;
                    float v = (y + dist[s].y) / (float)H;
                    ray r = sc.camera->get_ray(u, v);
                    Vec3 sample = trace(r, *sc.objects, sc.biased_objects, 0);
                    if (paths_out) {
                        size_t k = pix * ns + s;
                        paths[k * 3 + 0] = sample.r; paths[k * 3 + 1] = sample.g; paths[k * 3 + 2] = sample.b;
                        pathrays[k] = (uint32_t)(G_rayCounter.load() - before);
                    }
                    if (acc_mode == 0) {  // draw(), main.cpp:161-167
                        if (!isfinite(sample.r) || !isfinite(sample.g) || !isfinite(sample.b)) sample = color;
                        color += sample;
                    } else {  // draw2(), main.cpp:212-229 (sequential in sample order)
                        if (!isfinite(sample.r) || !isfinite(sample.g) || !isfinite(sample.b)) sample = (s > 0) ? color : Vec3(0.0f);
                        if (s > 0) sample = color + (sample - color) * (1.0f / (s + 1.0f));
                        float lum = luminance(sample);
                        if (lum > p->maxLuminance) sample = sample * (p->maxLuminance / lum);
                        color = sample;
                    }
                }
                if (acc_mode == 0) {  // main.cpp:168-173
                    color /= float(ns);
                    float lum = luminance(color);
                    if (lum > p->maxLuminance) color = color * (p->maxLuminance / lum);
                }
                img[pix] = color;
            }
        }
    };
    std::vector<std::thread> th;
    for (int i = 0; i < nthreads; i++) th.emplace_back(worker);
    for (auto& t : th) t.join();
    double secs = MRT_TimeDelta(t0, MRT_GetTime());
    size_t rays = G_rayCounter.load();
    if (out) write_pfm(out, img.data(), W, H);
    if (plist_out) {
        std::vector<float> v(plist.size() * 3);
        for (size_t i = 0; i < plist.size(); i++) {
            v[i * 3 + 0] = img[plist[i]].r;
            v[i * 3 + 1] = img[plist[i]].g;
            v[i * 3 + 2] = img[plist[i]].b;
        }
        FILE* f = fopen(plist_out, "wb");
        if (!f || fwrite(v.data(), 4, v.size(), f) != v.size()) { fprintf(stderr, "cannot write %s\n", plist_out); return 2; }
        fclose(f);
    }
    if (paths_out) {
        std::string a = std::string(paths_out) + ".rgb.npy", b = std::string(paths_out) + ".rays.npy";
        write_npy(a.c_str(), "<f4", {(size_t)W * H * ns, 3}, paths.data(), paths.size() * 4);
        write_npy(b.c_str(), "<u4", {(size_t)W * H * ns}, pathrays.data(), pathrays.size() * 4);
    }
    printf("{\"rays\":%zu,\"seconds\":%.6f,\"mrays_per_s\":%.4f,\"ns\":%u,\"threads\":%d}\n", rays, secs, rays * 1e-6 / secs, ns, nthreads);
    return 0;
}

static int mode_shipped(int argc, char** argv) {
    const char* out = harg(argc, argv, "--h-out", nullptr);
    uint64_t t0 = MRT_GetTime();
    int rc = mrt_main(argc, argv);
    double wall = MRT_TimeDelta(t0, MRT_GetTime());
    MRT_Params* p = getParams();
    if (out) write_pfm(out, G_linearBackBuffer, p->bufferWidth, p->bufferHeight);
    if (const char* argb = harg(argc, argv, "--h-argb", nullptr)) {  // the tone-mapped display buffer
        FILE* f = fopen(argb, "wb");
        if (f) {
            fwrite(G_backBuffer, 4, (size_t)p->bufferWidth * p->bufferHeight, f);
            fclose(f);
        }
    }
    float secs = 0, mrays = 0;
    const char* tr = strstr(H_title.c_str(), "Trace: ");
    if (tr) sscanf(tr, "Trace: %fs - %f Mrays/s", &secs, &mrays);
    printf("{\"rays\":%zu,\"trace_seconds\":%.3f,\"mrays_per_s\":%.3f,\"wall_seconds\":%.3f,\"threads\":%u}\n", (size_t)G_rayCounter.load(), secs,
           mrays, wall, p->numThreads);
    return rc;
}

int main(int argc, char** argv) {
    const char* mode = harg(argc, argv, "--h-mode", "shipped");
    H_custom = harg(argc, argv, "--h-custom", nullptr);
    H_objdir = harg(argc, argv, "--h-objdir", "../obj");
    if (!strcmp(mode, "kat")) return mode_kat(argc, argv);
    if (!strcmp(mode, "texels")) return mode_texels(argc, argv);
    ParseArgv(argc, argv);
    if (!strcmp(mode, "scene")) return mode_scene(argc, argv);
    if (!strcmp(mode, "hits")) return mode_hits(argc, argv);
    if (!strcmp(mode, "stream")) return mode_stream(argc, argv);
    return mode_shipped(argc, argv);
}
