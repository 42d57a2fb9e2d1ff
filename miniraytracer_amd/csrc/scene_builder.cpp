// scene_builder.cpp -- host C++ restatement of the reference scene surface: select_scene and
// its nine builders (scene.cpp:25-528), the object_list / bvh_node / pod_bvh constructors
// (scene_object.h:105-131, 282-319; triangle.h:77-168), rotate_y (scene_object.cpp:33-68), the
// camera (camera.h:16-36), readObj (obj_loader.cpp:14-163) and the Perlin tables
// (texture.cpp:167-203) -- flattened into the mrt_scene_view arrays that the HIP kernel walks.
//
// Everything that feeds the hit semantics is reproduced bit for bit: RNG call order during scene
// generation (left-to-right argument evaluation, as the clang-built reference does), stable
// qsort tie order, the FLT_MIN box seed of pod_bvh::update_node_box, node_order bits, rect
// padding.  tests/test_scene_parity.py compares mrt_scene_blob_dump_json() with the reference's
// own scene dump (tests/golden/scene_*.json.gz).
#include <algorithm>
#include <cfloat>
#include <cinttypes>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <limits>
#include <map>
#include <memory>
#include <string>
#include <vector>

#include "../../include/mrt.h"
#include "host_math.h"
#include "mrt_internal.h"

namespace mrt {

struct Box {
    V3 min, max;
};
static Box surrounding(const Box& a, const Box& b) { return Box{vmin(a.min, b.min), vmax(a.max, b.max)}; }

enum { HK_BOX = 100 };  // host-only kind: box (box.h) -> emitted as the LIST of its rects

struct Tri {
    V3 m, u, v, mn, un, vn;
};

struct ObjFace {
    int32_t with_normals;
    int32_t v[3], n[3];
};
struct ObjData {
    std::vector<V3> verts, norms;
    std::vector<ObjFace> faces;
};

struct HMesh {
    std::vector<Tri> prims;
    std::vector<mrt_mesh_node> nodes;  // relative indices
    std::vector<V3> centroids;
    uint32_t node_count = 0;
};

struct HObj {
    int kind = 0;
    uint32_t mat = MRT_NONE;
    // params
    V3 c0{}, c1{};  // sphere centers / translate offset / box min,max
    float t0 = 0, t1 = 0, radius = 0;
    bool moving = false;
    float a0 = 0, a1 = 0, b0 = 0, b1 = 0, k = 0, nsign = 1;  // rects
    float sin_t = 0, cos_t = 0, density = 0;
    bool has_box = false;
    Box box{};
    uint8_t order = 0;
    std::vector<HObj*> ch;  // LIST children; BVH: l, r; TRANSLATE/ROTY/VOLUME: child; BOX: rect list
    std::unique_ptr<HMesh> mesh;
    uint32_t node_id = MRT_NONE;
};

struct Builder {
    std::vector<std::unique_ptr<HObj>> objs;
    std::vector<mrt_material> mats;
    std::vector<mrt_texture> texs;
    std::vector<uint8_t> texels;
    std::string asset_dir;
    mrt_status err = MRT_OK;
    std::string errmsg;

    HObj* make(int kind) {
        objs.emplace_back(new HObj());
        objs.back()->kind = kind;
        return objs.back().get();
    }
    // ---- textures / materials (texture.h, material.h) ----
    uint32_t color(V3 c) {
        mrt_texture t{};
        t.kind = MRT_T_COLOR;
        t.f[0] = c.x; t.f[1] = c.y; t.f[2] = c.z;
        texs.push_back(t);
        return (uint32_t)texs.size() - 1;
    }
    uint32_t checker(uint32_t even, uint32_t odd, float scale) {
        mrt_texture t{};
        t.kind = MRT_T_CHECKER; t.a = even; t.b = odd; t.f[0] = scale;
        texs.push_back(t);
        return (uint32_t)texs.size() - 1;
    }
    uint32_t perlin(float scale) {
        mrt_texture t{};
        t.kind = MRT_T_PERLIN; t.f[0] = scale;
        texs.push_back(t);
        return (uint32_t)texs.size() - 1;
    }
    uint32_t image() {  // image_tex over the stb-decoded earthmap.jpg (scene.cpp:139, 268, 402)
        static const uint32_t W = 2700, H = 1350;
        if (texels.empty()) {
            std::string p = asset_dir + "/earthmap.rgb";
            FILE* f = fopen(p.c_str(), "rb");
            if (!f) { err = MRT_ERR_IO; errmsg = "missing asset " + p; return 0; }
            texels.resize((size_t)W * H * 3);
            size_t got = fread(texels.data(), 1, texels.size(), f);
            fclose(f);
            if (got != texels.size()) { err = MRT_ERR_IO; errmsg = "short asset " + p; return 0; }
        }
        mrt_texture t{};
        t.kind = MRT_T_IMAGE; t.a = 0; t.b = W; t.c = H;
        texs.push_back(t);
        return (uint32_t)texs.size() - 1;
    }
    uint32_t mat(uint32_t kind, uint32_t tex, float p) {
        mrt_material m{};
        m.kind = kind; m.tex = tex; m.p = p;
        mats.push_back(m);
        return (uint32_t)mats.size() - 1;
    }
    uint32_t lambertian(uint32_t tex) { return mat(MRT_M_LAMBERTIAN, tex, 0); }
    uint32_t metal(uint32_t tex, float gloss) { return mat(MRT_M_METAL, tex, std::min(gloss, 1.0f)); }  // material.h:84-86
    uint32_t dielectric(float ri) { return mat(MRT_M_DIELECTRIC, MRT_NONE, ri); }
    uint32_t light(uint32_t tex, float scale = 1.0f) { return mat(MRT_M_LIGHT, tex, scale); }

    // ---- primitives ----
    HObj* sphere(V3 c0, float r, uint32_t m, V3 c1 = V3{0, 0, 0}, float t0 = 0.0f, float t1 = 0.0f) {  // sphere.h:18-22
        HObj* o = make(MRT_K_SPHERE);
        o->c0 = c0; o->c1 = c1; o->t0 = t0; o->t1 = t1; o->radius = r; o->mat = m;
        o->moving = (t1 - t0) > std::numeric_limits<float>::epsilon();
        return o;
    }
    HObj* rect(int kind, float a0, float a1, float b0, float b1, float k, uint32_t m) {  // rect.cpp:6-22
        HObj* o = make(kind);
        float ns = 1;
        if (a0 > a1) { ns *= -1; std::swap(a0, a1); }
        if (b0 > b1) { ns *= -1; std::swap(b0, b1); }
        o->a0 = a0; o->a1 = a1; o->b0 = b0; o->b1 = b1; o->k = k; o->nsign = ns; o->mat = m;
        return o;
    }
    HObj* xy(float x0, float x1, float y0, float y1, float z, uint32_t m) { return rect(MRT_K_XY, x0, x1, y0, y1, z, m); }
    HObj* xz(float x0, float x1, float z0, float z1, float y, uint32_t m) { return rect(MRT_K_XZ, x0, x1, z0, z1, y, m); }
    HObj* yz(float y0, float y1, float z0, float z1, float x, uint32_t m) { return rect(MRT_K_YZ, y0, y1, z0, z1, x, m); }

    // ---- bounding boxes (each class's bounding_box) ----
    static V3 center(const HObj* s, float time) {  // sphere.h:24-31
        if (s->moving) return s->c0 + ((time - s->t0) / (s->t1 - s->t0)) * (s->c1 - s->c0);
        return s->c0;
    }
    bool bbox(const HObj* o, float t0, float t1, Box* out) const {
        switch (o->kind) {
        case MRT_K_LIST:
            if (!o->has_box) return false;
            *out = o->box;
            return true;
        case MRT_K_BVH:
            *out = o->box;
            return true;
        case MRT_K_MESH: {
            const mrt_mesh_node& n = o->mesh->nodes[0];
            *out = Box{V3{n.bmin[0], n.bmin[1], n.bmin[2]}, V3{n.bmax[0], n.bmax[1], n.bmax[2]}};
            return true;
        }
        case MRT_K_TRANSLATE: {  // scene_object.cpp:20-27
            Box b;
            if (!bbox(o->ch[0], t0, t1, &b)) return false;
            *out = Box{b.min + o->c0, b.max + o->c0};
            return true;
        }
        case MRT_K_ROTY:
            *out = o->box;
            return o->has_box;
        case MRT_K_SPHERE: {  // sphere.cpp:48-61
            float ar = std::fabs(o->radius);
            V3 r{ar, ar, ar};
            V3 a = center(o, t0), b = center(o, t1);
            *out = surrounding(Box{a - r, a + r}, Box{b - r, b + r});
            return true;
        }
        case MRT_K_XY:  // rect.h:18-21 (padding 1e-4 on the plane axis)
            *out = Box{V3{o->a0, o->b0, o->k - 0.0001f}, V3{o->a1, o->b1, o->k + 0.0001f}};
            return true;
        case MRT_K_XZ:
            *out = Box{V3{o->a0, o->k - 0.0001f, o->b0}, V3{o->a1, o->k + 0.0001f, o->b1}};
            return true;
        case MRT_K_YZ:
            *out = Box{V3{o->k - 0.0001f, o->a0, o->b0}, V3{o->k + 0.0001f, o->a1, o->b1}};
            return true;
        case MRT_K_VOLUME:
            return bbox(o->ch[0], t0, t1, out);
        case HK_BOX:
            *out = Box{o->c0, o->c1};
            return true;
        }
        return false;
    }

    // object_list ctor (scene_object.h:105-131)
    HObj* list(const std::vector<HObj*>& l, float time0, float time1) {
        HObj* o = make(MRT_K_LIST);
        o->ch = l;
        const float mx = std::numeric_limits<float>::max(), lo = std::numeric_limits<float>::lowest();
        V3 minbb{mx, mx, mx}, maxbb{lo, lo, lo};
        for (HObj* c : l) {
            Box b;
            if (bbox(c, time0, time1, &b)) {
                minbb = vmin(minbb, b.min);
                maxbb = vmax(maxbb, b.max);
            } else {
                o->has_box = false;
                return o;
            }
        }
        o->box = Box{minbb, maxbb};
        o->has_box = true;
        return o;
    }

    // box (box.h:12-21)
    HObj* box(V3 mn, V3 mx, uint32_t m) {
        HObj* o = make(HK_BOX);
        o->c0 = mn; o->c1 = mx;
        std::vector<HObj*> r(6);
        r[0] = xy(mn.x, mx.x, mn.y, mx.y, mx.z, m);
        r[1] = xy(mx.x, mn.x, mn.y, mx.y, mn.z, m);
        r[2] = xz(mn.x, mx.x, mn.z, mx.z, mx.y, m);
        r[3] = xz(mx.x, mn.x, mn.z, mx.z, mn.y, m);
        r[4] = yz(mn.y, mx.y, mn.z, mx.z, mx.x, m);
        r[5] = yz(mx.y, mn.y, mn.z, mx.z, mn.x, m);
        o->ch.push_back(list(r, 0, 0));
        return o;
    }

    HObj* translate(HObj* c, V3 off) {
        HObj* o = make(MRT_K_TRANSLATE);
        o->ch.push_back(c);
        o->c0 = off;
        return o;
    }
    // rotate_y ctor (scene_object.cpp:33-68)
    HObj* rotate_y(HObj* c, float angle) {
        HObj* o = make(MRT_K_ROTY);
        o->ch.push_back(c);
        float radians = rad(angle);
        o->sin_t = sin_(radians);
        o->cos_t = cos_(radians);
        Box bb;
        o->has_box = bbox(c, 0, 1, &bb);
        if (!o->has_box) {
            o->box = Box{V3{1, 1, 1}, V3{-1, -1, -1}};
            return o;
        }
        const float mx = std::numeric_limits<float>::max(), lo = std::numeric_limits<float>::lowest();
        V3 minbb{mx, mx, mx}, maxbb{lo, lo, lo};
        for (int i = 0; i < 2; i++)
            for (int j = 0; j < 2; j++)
                for (int k2 = 0; k2 < 2; k2++) {
                    // one scalar expression each, fused as shipped (x86 FMA, scene_object.cpp:54-59)
                    float x = std::fma((float)i, bb.max.x, (float)(1 - i) * bb.min.x);
                    float y = std::fma((float)j, bb.max.y, (float)(1 - j) * bb.min.y);
                    float z = std::fma((float)k2, bb.max.z, (float)(1 - k2) * bb.min.z);
                    float newx = std::fma(o->cos_t, x, o->sin_t * z);
                    float newz = std::fma(o->cos_t, z, -(o->sin_t * x));
                    V3 t{newx, y, newz};
                    minbb = vmin(minbb, t);
                    maxbb = vmax(maxbb, t);
                }
        o->box = Box{minbb, maxbb};
        return o;
    }
    HObj* volume(HObj* boundary, float density, uint32_t albedo) {  // volumes.h:14-16
        HObj* o = make(MRT_K_VOLUME);
        o->ch.push_back(boundary);
        o->density = density;
        o->mat = mat(MRT_M_ISOTROPIC, albedo, 0);
        return o;
    }

    // node_order (scene_object.h:154-205, triangle.h:282-322): bit (7-o) set iff !(dot(C0-C1, D_o) < 0)
    static uint8_t node_order(const Box& l, const Box& r) {
        V3 C0 = (l.max + l.min) * 0.5f, C1 = (r.max + r.min) * 0.5f;
        V3 d = C0 - C1;
        static const float S[8][3] = {{1, 1, 1}, {1, 1, -1}, {1, -1, 1}, {1, -1, -1}, {-1, 1, 1}, {-1, 1, -1}, {-1, -1, 1}, {-1, -1, -1}};
        uint8_t code = 0;
        for (int o = 0; o < 8; o++) {
            V3 D = normalize(V3{S[o][0], S[o][1], S[o][2]});
            bool neg = dot(d, D) < 0.0f;
            if (!neg) code |= (uint8_t)(1u << (7 - o));
        }
        return code;
    }

    // bvh_node<T> ctor (scene_object.h:282-319).  glibc 2.35 qsort is a stable merge sort for
    // these sizes; box_compare (scene_object.h:246-267) is a strict "<" on box.min[axis] (t=0,0).
    HObj* bvh(std::vector<HObj*> l, float time0, float time1) {
        HObj* tmp = list(l, time0, time1);
        HObj* o = make(MRT_K_BVH);
        o->box = tmp->box;  // ol.bounding_box(&box, ...)
        V3 dim = o->box.max - o->box.min;
        int axis = max_dim(dim);
        std::stable_sort(l.begin(), l.end(), [&](HObj* a, HObj* b) {
            Box ba, bb;
            bbox(a, 0, 0, &ba);
            bbox(b, 0, 0, &bb);
            return get(ba.min, axis) - get(bb.min, axis) < 0.0f;
        });
        size_t n = l.size();
        HObj *L, *R;
        if (n == 1) {
            L = R = l[0];
        } else if (n == 2) {
            L = l[0]; R = l[1];
        } else if (n < 11) {
            L = list(std::vector<HObj*>(l.begin(), l.begin() + n / 2), time0, time1);
            R = list(std::vector<HObj*>(l.begin() + n / 2, l.end()), time0, time1);
        } else {
            L = bvh(std::vector<HObj*>(l.begin(), l.begin() + n / 2), time0, time1);
            R = bvh(std::vector<HObj*>(l.begin() + n / 2, l.end()), time0, time1);
        }
        o->ch = {L, R};
        Box lb, rb;
        bbox(L, 0, 1, &lb);
        bbox(R, 0, 1, &rb);
        o->order = node_order(lb, rb);
        return o;
    }

    // ---- pod_bvh<triangle> (triangle.h:77-168) ----
    static void add_to_box(const Tri& t, V3* mn, V3* mx) {  // triangle.h:34-41
        V3 b = t.m + t.u, c = t.m + t.v;
        *mn = vmin(*mn, t.m); *mn = vmin(*mn, b); *mn = vmin(*mn, c);
        *mx = vmax(*mx, t.m); *mx = vmax(*mx, b); *mx = vmax(*mx, c);
    }
    static void update_node_box(HMesh& M, uint32_t ni) {
        mrt_mesh_node& n = M.nodes[ni];
        const float maxf = std::numeric_limits<float>::max();
        const float minf = std::numeric_limits<float>::min();  // sic: FLT_MIN, triangle.h:160
        V3 mn{maxf, maxf, maxf}, mx{minf, minf, minf};
        uint32_t cnt = n.count_order & 0xFFFFFFu;
        for (uint32_t i = 0; i < cnt; i++) add_to_box(M.prims[n.left_or_first + i], &mn, &mx);
        n.bmin[0] = mn.x; n.bmin[1] = mn.y; n.bmin[2] = mn.z;
        n.bmax[0] = mx.x; n.bmax[1] = mx.y; n.bmax[2] = mx.z;
    }
    static Box nbox(const mrt_mesh_node& n) {
        return Box{V3{n.bmin[0], n.bmin[1], n.bmin[2]}, V3{n.bmax[0], n.bmax[1], n.bmax[2]}};
    }
    static void subdivide(HMesh& M, uint32_t ni) {
        uint32_t cnt = M.nodes[ni].count_order & 0xFFFFFFu;
        if (cnt <= 2) return;
        Box nb = nbox(M.nodes[ni]);
        V3 e = nb.max - nb.min;
        int axis = 0;
        if (e.y > e.x) axis = 1;
        if (e.z > get(e, axis)) axis = 2;
        float split = get(nb.min, axis) + get(e, axis) * 0.5f;
        int off = (int)M.nodes[ni].left_or_first;
        int i = off, j = i + (int)cnt - 1;
        while (i <= j) {
            if (get(M.centroids[i], axis) < split) i++;
            else {
                std::swap(M.prims[i], M.prims[j]);
                std::swap(M.centroids[i], M.centroids[j]);
                j--;
            }
        }
        int left_count = i - off;
        if (left_count == 0 || left_count == (int)cnt) return;
        uint32_t lc = M.node_count++, rc = M.node_count++;
        M.nodes[lc].left_or_first = (uint32_t)off;
        M.nodes[lc].count_order = (uint32_t)left_count;
        M.nodes[rc].left_or_first = (uint32_t)i;
        M.nodes[rc].count_order = cnt - (uint32_t)left_count;
        update_node_box(M, lc);
        update_node_box(M, rc);
        M.nodes[ni].left_or_first = lc;
        M.nodes[ni].count_order = (uint32_t)node_order(nbox(M.nodes[lc]), nbox(M.nodes[rc])) << 24;
        subdivide(M, lc);
        subdivide(M, rc);
    }
    HObj* pod_bvh(const std::vector<Tri>& tris, uint32_t m) {
        HObj* o = make(MRT_K_MESH);
        o->mat = m;
        o->mesh.reset(new HMesh());
        HMesh& M = *o->mesh;
        M.prims = tris;
        size_t n = tris.size();
        M.nodes.assign(n * 2 - 1, mrt_mesh_node{});
        M.centroids.resize(n);
        for (size_t i = 0; i < n; i++)  // get_centroid (triangle.h:31-33)
            M.centroids[i] = ((tris[i].m + (tris[i].m + tris[i].u)) + (tris[i].m + tris[i].v)) * (1.0f / 3.0f);
        M.node_count = 1;
        M.nodes[0].left_or_first = 0;
        M.nodes[0].count_order = (uint32_t)n;
        update_node_box(M, 0);
        subdivide(M, 0);
        M.nodes.resize(M.node_count);
        return o;
    }

    // ---- Mat4 pieces used by readObj (mat4.h:44-102) ----
    struct M4 {
        float c[4][4];  // column-major, c[col][row]
    };
    static M4 scale4(float s) {
        M4 m{};
        m.c[0][0] = s; m.c[1][1] = s; m.c[2][2] = s; m.c[3][3] = 1;
        return m;
    }
    static M4 ident() { return scale4(1.0f); }
    static V3 mul(const M4& m, V3 v) {  // (vx*c0 + vy*c1) + vz*c2 per lane
        V3 r;
        float* rp = &r.x;
        for (int i = 0; i < 3; i++) rp[i] = (v.x * m.c[0][i] + v.y * m.c[1][i]) + v.z * m.c[2][i];
        return r;
    }
    // readObj (obj_loader.cpp:14-163) split in two: parse the records (v, vn, "f a b c",
    // "f a//n b//n c//n", %i integers; whether a face takes the normals branch is decided by
    // norms.empty() at the time the face is read), then build triangles from them.  The parsed
    // records can be stored as a packed .mesh asset (mrt_pack_obj) for hosts without the .obj.
    bool read_obj(const std::string& fn, ObjData* out) {
        FILE* f = fopen(fn.c_str(), "r");
        if (!f) return false;
        char line[4096];
        while (fgets(line, sizeof line, f)) {
            char* s = line;
            while (*s == ' ' || *s == '\t' || *s == '\n' || *s == '\r') s++;
            if (s[0] == 'v' && (s[1] == ' ' || s[1] == '\t')) {
                float x, y, z;
                if (sscanf(s + 2, " %f %f %f", &x, &y, &z) == 3) out->verts.push_back(V3{x, y, z});
            } else if (s[0] == 'v' && s[1] == 'n') {
                float x, y, z;
                if (sscanf(s + 2, " %f %f %f", &x, &y, &z) == 3) out->norms.push_back(V3{x, y, z});
            } else if (s[0] == 'f') {
                ObjFace fc{};
                if (out->norms.empty()) {
                    if (sscanf(s + 1, " %i %i %i", &fc.v[0], &fc.v[1], &fc.v[2]) != 3) continue;
                    fc.with_normals = 0;
                } else {
                    if (sscanf(s + 1, " %i//%i %i//%i %i//%i", &fc.v[0], &fc.n[0], &fc.v[1], &fc.n[1], &fc.v[2], &fc.n[2]) != 6) continue;
                    fc.with_normals = 1;
                }
                out->faces.push_back(fc);
            }
        }
        fclose(f);
        return true;
    }
    static bool read_packed(const std::string& fn, ObjData* out) {
        FILE* f = fopen(fn.c_str(), "rb");
        if (!f) return false;
        char magic[8];
        uint32_t hdr[3];
        bool ok = fread(magic, 1, 8, f) == 8 && memcmp(magic, "MRTMESH1", 8) == 0 && fread(hdr, 4, 3, f) == 3;
        if (ok) {
            out->verts.resize(hdr[0]);
            out->norms.resize(hdr[1]);
            out->faces.resize(hdr[2]);
            ok = fread(out->verts.data(), 12, hdr[0], f) == hdr[0] && fread(out->norms.data(), 12, hdr[1], f) == hdr[1] &&
                 fread(out->faces.data(), sizeof(ObjFace), hdr[2], f) == hdr[2];
        }
        fclose(f);
        return ok;
    }
    bool build_tris(const ObjData& o, bool flip, float scale, V3 translate, std::vector<Tri>* out) {
        M4 S = scale4(scale), R = ident();
        int nv = (int)o.verts.size(), nn = (int)o.norms.size();
        for (const ObjFace& fc : o.faces) {
            int ai = fc.v[0], bi = fc.v[1], ci = fc.v[2], an = fc.n[0], bn = fc.n[1], cn = fc.n[2];
            if (flip) { std::swap(ai, ci); std::swap(an, cn); }
            if (ai < 1 || bi < 1 || ci < 1 || ai > nv || bi > nv || ci > nv) { err = MRT_ERR_IO; errmsg = "OBJ face index out of range"; return false; }
            V3 a = mul(R, mul(S, o.verts[ai - 1])) + translate;
            V3 b = mul(R, mul(S, o.verts[bi - 1])) + translate;
            V3 c = mul(R, mul(S, o.verts[ci - 1])) + translate;
            Tri t;  // triangle ctors (triangle.cpp:178-208)
            t.m = a; t.u = b - a; t.v = c - a;
            if (!fc.with_normals) {
                t.mn = t.un = t.vn = normalize(cross(t.u, t.v));
            } else {
                if (an < 1 || bn < 1 || cn < 1 || an > nn || bn > nn || cn > nn) { err = MRT_ERR_IO; errmsg = "OBJ normal index out of range"; return false; }
                // n * Invert(Identity) (row-vector product) leaves the normals' non-zero values unchanged
                t.mn = o.norms[an - 1]; t.un = o.norms[bn - 1]; t.vn = o.norms[cn - 1];
            }
            out->push_back(t);
        }
        return true;
    }
    // OBJ asset: raw <name>.obj if present, else the packed <name>.mesh (same parsed records)
    bool load_mesh(const char* name, bool flip, float scale, V3 tr, std::vector<Tri>* out) {
        ObjData o;
        std::string obj = asset_dir + "/" + name + ".obj", packed = asset_dir + "/" + name + ".mesh";
        if (!read_obj(obj, &o) && !read_packed(packed, &o)) {
            err = MRT_ERR_IO;
            errmsg = "missing asset " + obj + " (or " + packed + ")";
            return false;
        }
        return build_tris(o, flip, scale, tr, out);
    }
};

// camera ctor (camera.h:16-36)
static mrt_camera make_camera(V3 pos, V3 lookat, V3 up, float vfov, float aspect, float aperture, float focus_dist, float t0, float t1) {
    mrt_camera c{};
    c.time0 = t0;
    c.time1 = t1;
    float theta = rad(vfov);
    float height = 2.0f * tan_(theta / 2);
    float width = aspect * height;
    V3 w = normalize(pos - lookat);
    V3 u = normalize(cross(up, w));
    V3 v = cross(w, u);
    c.lens_radius = aperture / 2.0f;
    V3 horz = (focus_dist * width) * u;
    V3 vert = (focus_dist * height) * v;
    V3 llc = ((pos - 0.5f * horz) - 0.5f * vert) - focus_dist * w;
    auto put = [](float* d, V3 s) { d[0] = s.x; d[1] = s.y; d[2] = s.z; d[3] = 0; };
    put(c.origin, pos); put(c.u, u); put(c.v, v); put(c.w, w);
    put(c.llcorner, llc); put(c.horz, horz); put(c.vert, vert);
    return c;
}

struct BuiltScene {
    HObj* objects = nullptr;
    HObj* biased = nullptr;
    mrt_camera cam{};
};

static const V3 SPHERE_CAM_POS{11, 2.2f, 2.5f}, SPHERE_LOOKAT{2.8f, 0.5f, 1.2f}, UP{0, 1, 0};
static mrt_camera sphere_cam(float aspect) {
    return make_camera(SPHERE_CAM_POS, SPHERE_LOOKAT, UP, 27.0f, aspect, 0.09f, length(SPHERE_CAM_POS - SPHERE_LOOKAT), 0.0f, 1.0f);
}

// random_scene (scene.cpp:51-119) and random_scene_2 (scene.cpp:121-198)
static BuiltScene random_scene(Builder& B, Pcg& rng, int n, float aspect, bool v2) {
    BuiltScene S;
    S.cam = sphere_cam(aspect);
    std::vector<HObj*> l;
    uint32_t earth = 0, checker = 0, perlin = 0, perlin_small = 0;
    if (!v2) {
        uint32_t chk = B.checker(B.color(V3{0.2f, 0.3f, 0.1f}), B.color(V3{0.9f, 0.9f, 0.9f}), 10.0f);
        l.push_back(B.sphere(V3{0, -1000, 0}, 1000, B.lambertian(chk)));
    } else {
        earth = B.lambertian(B.image());
        checker = B.lambertian(B.checker(B.color(V3{0.2f, 0.3f, 0.1f}), B.color(V3{0.9f, 0.9f, 0.9f}), 10.0f));
        perlin = B.lambertian(B.perlin(1.0f));
        perlin_small = B.lambertian(B.perlin(4.0f));
        l.push_back(B.sphere(V3{0, -1000, 0}, 1000, perlin));
    }
    int half = int(std::sqrt(float(n)) * 0.5f);
    for (int a = -half; a < half; a++) {
        for (int b = -half; b < half; b++) {
            float choose = randf(rng);
            float r1 = randf(rng);
            float cx = std::fma(0.9f, r1, (float)a);  // scene.cpp:78, fused as shipped
            float r2 = randf(rng);
            float cz = std::fma(0.9f, r2, (float)b);
            V3 center{cx, 0.2f, cz};
            if (length(center - V3{4, 0.2f, 0}) > 0.9f) {
                HObj* s;
                if (choose < (v2 ? 0.3f : 0.5f)) {
                    float q[6];
                    for (int k = 0; k < 6; k++) q[k] = randf(rng);
                    uint32_t m = B.lambertian(B.color(V3{q[0] * q[1], q[2] * q[3], q[4] * q[5]}));
                    float r3 = randf(rng);
                    s = B.sphere(center, 0.2f, m, center + V3{0, 0.5f * r3, 0}, 0.0f, 1.0f);
                } else {
                    uint32_t m;
                    if (!v2 ? (choose < 0.9f) : (choose < 0.6f)) {
                        float q0 = randf(rng), q1 = randf(rng), q2 = randf(rng);
                        uint32_t t = B.color(0.5f * V3{1 + q0, 1 + q1, 1 + q2});
                        float g = randf(rng);
                        m = B.metal(t, g);
                    } else if (!v2 || choose < 0.7f) {
                        m = B.dielectric(1.4f + randf(rng));
                    } else if (choose < 0.75f) {
                        m = earth;
                    } else {
                        m = perlin_small;
                    }
                    s = B.sphere(center, 0.2f, m);
                }
                l.push_back(s);
            }
        }
    }
    l.push_back(B.sphere(V3{0, 1, 0}, 1.0f, B.dielectric(1.5f)));
    if (!v2) l.push_back(B.sphere(V3{-4, 1, 0}, 1.0f, B.lambertian(B.color(V3{0.4f, 0.2f, 0.1f}))));
    else l.push_back(B.sphere(V3{-4, 1, 0}, 1.0f, checker));
    l.push_back(B.sphere(V3{4, 1, 0}, 1.0f, B.metal(B.color(V3{0.7f, 0.6f, 0.5f}), 1.0f)));
    l.push_back(B.sphere(V3{4, 1, 3}, 1.0f, B.dielectric(2.4f)));
    l.push_back(B.sphere(V3{4, 1, 3}, -0.95f, B.dielectric(2.4f)));
    S.objects = B.bvh(l, 0.0f, 1.0f);
    return S;
}

static BuiltScene two_spheres(Builder& B, float aspect) {  // scene.cpp:201-225
    BuiltScene S;
    S.cam = sphere_cam(aspect);
    uint32_t chk = B.checker(B.color(V3{0.2f, 0.3f, 0.1f}), B.color(V3{0.9f, 0.9f, 0.9f}), 10.0f);
    uint32_t m0 = B.lambertian(chk), m1 = B.lambertian(chk);
    S.objects = B.list({B.sphere(V3{0, -10, 0}, 10, m0), B.sphere(V3{0, 10, 0}, 10, m1)}, 0.0f, 1.0f);
    return S;
}

static BuiltScene spheres_perlin(Builder& B, float aspect, bool earth) {  // scene.cpp:227-281
    BuiltScene S;
    S.cam = sphere_cam(aspect);
    HObj* s0 = B.sphere(V3{0, -1001, 0}, 1000, B.lambertian(B.perlin(1.0f)));
    HObj *s1, *s2;
    if (!earth) {
        s1 = B.sphere(V3{0, 1, 0}, 2, B.lambertian(B.perlin(4.0f)));
        s2 = B.sphere(V3{0.5f, -0.5f, 2}, 0.5f, B.lambertian(B.perlin(16.0f)));
    } else {
        uint32_t m = B.lambertian(B.image());
        s1 = B.sphere(V3{0, 1, 0}, 2, m);
        s2 = B.sphere(V3{0.5f, -0.5f, 2}, 0.5f, m);
    }
    S.objects = B.list({s0, s1, s2}, 0.0f, 1.0f);
    return S;
}

static const V3 CORNELL_POS{278, 278, -800}, CORNELL_LOOK{278, 278, 100};

static BuiltScene cornell_box(Builder& B, float aspect) {  // scene.cpp:283-332
    BuiltScene S;
    S.cam = make_camera(CORNELL_POS, CORNELL_LOOK, UP, 40.0f, aspect, 0.0f, length(CORNELL_POS - CORNELL_LOOK), 0.0f, 1.0f);
    uint32_t red = B.lambertian(B.color(V3{0.65f, 0.055f, 0.06f}));
    uint32_t white = B.lambertian(B.color(V3{0.73f, 0.73f, 0.73f}));
    uint32_t green = B.lambertian(B.color(V3{0.117f, 0.44f, 0.115f}));
    uint32_t light = B.light(B.color(V3{15.f, 15.f, 15.f}));
    uint32_t glass = B.dielectric(1.5f);
    std::vector<HObj*> l;
    l.push_back(B.yz(555, 0, 0, 555, 555, green));
    l.push_back(B.yz(0, 555, 0, 555, 0, red));
    HObj* lt = B.xz(343, 213, 227, 332, 554, light);
    l.push_back(lt);
    l.push_back(B.xz(555, 0, 0, 555, 555, white));
    l.push_back(B.xz(0, 555, 0, 555, 0, white));
    l.push_back(B.xy(555, 0, 0, 555, 555, white));
    l.push_back(B.translate(B.rotate_y(B.box(V3{0, 0, 0}, V3{165, 330, 165}, white), 15), V3{265, 0, 295}));
    l.push_back(B.sphere(V3{190, 90, 190}, 90, glass));
    S.objects = B.list(l, 0.0f, 1.0f);
    S.biased = B.list({lt}, 0.0f, 1.0f);  // b[1] = sphere is allocated but count == 1 (scene.cpp:326-329)
    return S;
}

static BuiltScene cornell_smoke(Builder& B, float aspect) {  // scene.cpp:334-378
    BuiltScene S;
    S.cam = make_camera(CORNELL_POS, CORNELL_LOOK, UP, 40.0f, aspect, 0.0f, length(CORNELL_POS - CORNELL_LOOK), 0.0f, 1.0f);
    uint32_t red = B.lambertian(B.color(V3{0.65f, 0.05f, 0.05f}));
    uint32_t white = B.lambertian(B.color(V3{0.73f, 0.73f, 0.73f}));
    uint32_t green = B.lambertian(B.color(V3{0.12f, 0.45f, 0.15f}));
    uint32_t light = B.light(B.color(V3{7.0f, 7.0f, 7.0f}));
    std::vector<HObj*> l;
    l.push_back(B.yz(555, 0, 0, 555, 555, green));
    l.push_back(B.yz(0, 555, 0, 555, 0, red));
    HObj* lt = B.xz(443, 113, 127, 432, 554, light);
    l.push_back(lt);
    l.push_back(B.xz(555, 0, 0, 555, 555, white));
    l.push_back(B.xz(0, 555, 0, 555, 0, white));
    l.push_back(B.xy(555, 0, 0, 555, 555, white));
    HObj* b1 = B.translate(B.rotate_y(B.box(V3{0, 0, 0}, V3{165, 165, 165}, white), -18), V3{130, 0, 65});
    HObj* b2 = B.translate(B.rotate_y(B.box(V3{0, 0, 0}, V3{165, 330, 165}, white), 15), V3{265, 0, 295});
    l.push_back(B.volume(b1, 0.01f, B.color(V3{1.0f, 1.0f, 1.0f})));
    l.push_back(B.volume(b2, 0.01f, B.color(V3{0.0f, 0.0f, 0.0f})));
    S.objects = B.list(l, 0.0f, 1.0f);
    S.biased = B.list({lt}, 0.0f, 1.0f);
    return S;
}

static BuiltScene book2_final(Builder& B, Pcg& rng, float aspect) {  // scene.cpp:380-462
    BuiltScene S;
    V3 pos{450, 278, -560}, look{200, 278, 300};
    S.cam = make_camera(pos, look, UP, 40.0f, aspect, 0.0f, length(pos - look), 0.0f, 1.0f);
    const int nb = 20, ns = 1000;
    uint32_t earth = B.lambertian(B.image());
    uint32_t white = B.lambertian(B.color(V3{0.73f, 0.73f, 0.73f}));
    uint32_t green = B.lambertian(B.color(V3{0.48f, 0.83f, 0.53f}));
    uint32_t light = B.light(B.color(V3{7.0f, 7.0f, 7.0f}));
    uint32_t orange = B.lambertian(B.color(V3{0.7f, 0.3f, 0.1f}));
    uint32_t perlin = B.lambertian(B.perlin(0.05f));
    std::vector<HObj*> boxes;
    for (int i = 0; i < nb; i++)
        for (int j = 0; j < nb; j++) {
            float w = 100;
            float x0 = std::fma((float)i, w, -1000.0f), z0 = std::fma((float)j, w, -1000.0f), y0 = 0;  // scene.cpp:418-419
            float x1 = x0 + w, y1 = 100 * (randf(rng) + 0.01f), z1 = z0 + w;
            boxes.push_back(B.box(V3{x0, y0, z0}, V3{x1, y1, z1}, green));
        }
    std::vector<HObj*> l;
    l.push_back(B.bvh(boxes, 0.0f, 1.0f));
    HObj* lo = B.xz(423, 123, 147, 412, 554, light);
    l.push_back(lo);
    V3 center{400, 400, 200};
    l.push_back(B.sphere(center, 50, orange, center + V3{30, 0, 0}, 0, 1));
    HObj* gs = B.sphere(V3{260, 150, 45}, 50, B.dielectric(1.5f));
    l.push_back(gs);
    l.push_back(B.sphere(V3{0, 150, 145}, 50, B.metal(B.color(V3{0.8f, 0.8f, 0.9f}), 0.1f)));
    l.push_back(B.sphere(V3{400, 200, 400}, 100, earth));
    l.push_back(B.sphere(V3{220, 280, 300}, 80, perlin));
    HObj* vb = B.sphere(V3{360, 150, 145}, 70, B.dielectric(1.5f));
    l.push_back(vb);
    l.push_back(B.volume(vb, 0.2f, B.color(V3{0.2f, 0.4f, 0.9f})));
    HObj* fogb = B.sphere(V3{0, 0, 0}, 5000, B.dielectric(1.5f));
    l.push_back(B.volume(fogb, 0.0001f, B.color(V3{1.0f, 1.0f, 1.0f})));
    std::vector<HObj*> sl;
    for (int i = 0; i < ns; i++) {
        float a = randf(rng), b = randf(rng), c = randf(rng);
        sl.push_back(B.sphere(V3{165 * a, 165 * b, 165 * c}, 10, white));
    }
    l.push_back(B.translate(B.rotate_y(B.bvh(sl, 0.0f, 1.0f), 15), V3{-100, 270, 395}));
    S.objects = B.list(l, 0.0f, 1.0f);
    S.biased = B.list({lo}, 0.0f, 1.0f);
    return S;
}

static BuiltScene triangles(Builder& B, float aspect) {  // scene.cpp:464-529
    BuiltScene S;
    S.cam = make_camera(CORNELL_POS, CORNELL_LOOK, UP, 40.0f, aspect, 20.0f, length(CORNELL_POS - CORNELL_LOOK), 0.0f, 1.0f);
    uint32_t red = B.lambertian(B.color(V3{0.65f, 0.05f, 0.05f}));
    uint32_t white = B.lambertian(B.color(V3{0.73f, 0.73f, 0.73f}));
    uint32_t green = B.lambertian(B.color(V3{0.12f, 0.45f, 0.15f}));
    uint32_t light = B.light(B.color(V3{4.0f, 4.0f, 4.0f}));
    uint32_t silver = B.metal(B.color(V3{0.8f, 0.8f, 0.9f}), 0.9f);
    uint32_t dia = B.dielectric(2.4f);
    std::vector<HObj*> l;
    l.push_back(B.yz(555, 0, 0, 555, 555, green));
    l.push_back(B.yz(0, 555, 0, 555, 0, red));
    HObj* lt = B.xz(443, 113, 127, 432, 554, light);
    l.push_back(lt);
    l.push_back(B.xz(555, 0, 0, 555, 555, white));
    l.push_back(B.xz(0, 555, 0, 555, 0, white));
    l.push_back(B.xy(555, 0, 0, 555, 555, silver));
    std::vector<Tri> bunny;
    if (!B.load_mesh("bunny", true, 2000.0f, V3{195, -20, 280}, &bunny)) return S;
    if (!bunny.empty()) l.push_back(B.pod_bvh(bunny, dia));
    // the reference also reads "../obj/teapot3_no_vt.obj" (scene.cpp:509); on a case-sensitive
    // file system that path does not exist (the file is Teapot3_no_vt.obj), so no teapot.
    S.objects = B.list(l, 0.0f, 1.0f);
    S.biased = B.list({lt}, 0.0f, 1.0f);
    return S;
}

// scene 9 (config C3): wt_teapot in the Cornell box, built by the oracle harness
// from reference classes (oracle/ref/harness.cpp harness_select_scene).
static BuiltScene teapot_cornell(Builder& B, float aspect) {
    BuiltScene S;
    S.cam = make_camera(CORNELL_POS, CORNELL_LOOK, UP, 40.0f, aspect, 0.0f, length(CORNELL_POS - CORNELL_LOOK), 0.0f, 1.0f);
    uint32_t red = B.lambertian(B.color(V3{0.65f, 0.055f, 0.06f}));
    uint32_t white = B.lambertian(B.color(V3{0.73f, 0.73f, 0.73f}));
    uint32_t green = B.lambertian(B.color(V3{0.117f, 0.44f, 0.115f}));
    uint32_t light = B.light(B.color(V3{15.f, 15.f, 15.f}));
    std::vector<HObj*> l;
    l.push_back(B.yz(555, 0, 0, 555, 555, green));
    l.push_back(B.yz(0, 555, 0, 555, 0, red));
    HObj* lt = B.xz(343, 213, 227, 332, 554, light);
    l.push_back(lt);
    l.push_back(B.xz(555, 0, 0, 555, 555, white));
    l.push_back(B.xz(0, 555, 0, 555, 0, white));
    l.push_back(B.xy(555, 0, 0, 555, 555, white));
    std::vector<Tri> tp;
    if (!B.load_mesh("wt_teapot", false, 200.0f, V3{264.3f, 0, 278}, &tp)) return S;
    l.push_back(B.pod_bvh(tp, white));
    S.objects = B.list(l, 0.0f, 1.0f);
    S.biased = B.list({lt}, 0.0f, 1.0f);
    return S;
}

// Perlin tables from the pre-seeded global RNG (pcg.cpp:40; texture.cpp:167-203)
static void perlin_tables(float* ranvec, int32_t* perm) {
    Pcg g{11350390909718046443uLL, 6305599193148252115uLL};
    for (int i = 0; i < 256; i++) {
        V3 p = random_in_sphere(g);
        ranvec[i * 4 + 0] = p.x; ranvec[i * 4 + 1] = p.y; ranvec[i * 4 + 2] = p.z; ranvec[i * 4 + 3] = 0;
    }
    for (int s = 0; s < 3; s++) {
        int32_t* p = perm + s * 256;
        for (int i = 0; i < 256; i++) p[i] = i;
        for (int i = 255; i > 0; i--) {
            int target = int(randf(g) * (i + 1));
            std::swap(p[i], p[target]);
        }
    }
}

// ---- flatten ----
struct Flat {
    std::vector<mrt_node> nodes;
    std::vector<uint32_t> children;
    std::vector<mrt_mesh_node> mesh_nodes;
    std::vector<float> tri_geo, tri_nrm;
};

static void put_box(float* f, const Box& b) {
    f[0] = b.min.x; f[1] = b.min.y; f[2] = b.min.z; f[3] = b.max.x; f[4] = b.max.y; f[5] = b.max.z;
}

static uint32_t emit(Flat& F, HObj* o) {
    if (o->node_id != MRT_NONE) return o->node_id;
    if (o->kind == HK_BOX) return o->node_id = emit(F, o->ch[0]);
    uint32_t id = (uint32_t)F.nodes.size();
    o->node_id = id;
    F.nodes.push_back(mrt_node{});
    mrt_node n{};
    n.kind = (uint32_t)o->kind;
    n.mat = o->mat;
    n.a = n.b = MRT_NONE;
    switch (o->kind) {
    case MRT_K_LIST: {
        std::vector<uint32_t> ids;
        for (HObj* c : o->ch) ids.push_back(emit(F, c));
        n.a = (uint32_t)F.children.size();
        n.b = (uint32_t)ids.size();
        F.children.insert(F.children.end(), ids.begin(), ids.end());
        if (o->has_box) { n.kind |= MRT_F_HASBOX << 16; put_box(n.f, o->box); }
        break;
    }
    case MRT_K_BVH:
        n.a = emit(F, o->ch[0]);
        n.b = emit(F, o->ch[1]);
        n.kind |= (uint32_t)o->order << 8;
        put_box(n.f, o->box);
        break;
    case MRT_K_MESH: {
        HMesh& M = *o->mesh;
        uint32_t nb = (uint32_t)F.mesh_nodes.size(), pb = (uint32_t)(F.tri_geo.size() / 12);
        for (const mrt_mesh_node& mn : M.nodes) {
            mrt_mesh_node x = mn;
            if ((x.count_order & 0xFFFFFFu) == 0) x.left_or_first += nb;
            else x.left_or_first += pb;
            F.mesh_nodes.push_back(x);
        }
        for (const Tri& t : M.prims) {
            const V3* g[3] = {&t.m, &t.u, &t.v};
            const V3* q[3] = {&t.mn, &t.un, &t.vn};
            for (int i = 0; i < 3; i++) {
                F.tri_geo.insert(F.tri_geo.end(), {g[i]->x, g[i]->y, g[i]->z, 0.0f});
                F.tri_nrm.insert(F.tri_nrm.end(), {q[i]->x, q[i]->y, q[i]->z, 0.0f});
            }
        }
        n.a = nb;
        n.b = (uint32_t)M.nodes.size();
        n.f[6] = (float)M.prims.size();
        put_box(n.f, Builder::nbox(M.nodes[0]));
        break;
    }
    case MRT_K_TRANSLATE:
        n.a = emit(F, o->ch[0]);
        n.f[0] = o->c0.x; n.f[1] = o->c0.y; n.f[2] = o->c0.z;
        break;
    case MRT_K_ROTY:
        n.a = emit(F, o->ch[0]);
        if (o->has_box) n.kind |= MRT_F_HASBOX << 16;
        put_box(n.f, o->box);
        n.f[6] = o->sin_t;
        n.f[7] = o->cos_t;
        break;
    case MRT_K_SPHERE:
        if (o->moving) n.kind |= MRT_F_MOVING << 16;
        n.f[0] = o->c0.x; n.f[1] = o->c0.y; n.f[2] = o->c0.z;
        n.f[3] = o->c1.x; n.f[4] = o->c1.y; n.f[5] = o->c1.z;
        n.f[6] = o->t0; n.f[7] = o->t1; n.f[8] = o->radius;
        break;
    case MRT_K_XY: case MRT_K_XZ: case MRT_K_YZ:
        n.f[0] = o->a0; n.f[1] = o->a1; n.f[2] = o->b0; n.f[3] = o->b1; n.f[4] = o->k; n.f[5] = o->nsign;
        break;
    case MRT_K_VOLUME:
        n.a = emit(F, o->ch[0]);
        n.f[0] = o->density;
        break;
    }
    F.nodes[id] = n;
    return id;
}

}  // namespace mrt

using namespace mrt;

struct mrt_scene_blob {
    mrt_scene_view view;
    Flat flat;
    std::vector<mrt_material> mats;
    std::vector<mrt_texture> texs;
    std::vector<uint8_t> texels;
    float ranvec[256 * 4];
    int32_t perm[3 * 256];
    Pcg main_rng;  // main()'s T_rng after select_scene: the worker seeds come from it (main.cpp:357-361)
};

static std::string default_asset_dir() {
    const char* e = getenv("MRT_ASSET_DIR");
    if (e && *e) return e;
    return mrt_internal_package_dir() + "/../assets";
}

extern "C" mrt_status mrt_select_scene(uint32_t scene, float aspect, const char* asset_dir, mrt_scene_blob** out) {
    if (!out || scene > 9 || !(aspect > 0.0f)) return mrt_internal_fail(MRT_ERR_INVALID, "mrt_select_scene: bad argument");
    Builder B;
    B.asset_dir = asset_dir ? asset_dir : default_asset_dir();
    Pcg rng;
    pcg_seed(rng, 11350390909718046443uLL, 6305599193148252115uLL);  // main.cpp:302
    BuiltScene S;
    switch (scene) {
    case 0: S = random_scene(B, rng, 500, aspect, false); break;
    case 1: S = random_scene(B, rng, 500, aspect, true); break;
    case 2: S = two_spheres(B, aspect); break;
    case 3: S = spheres_perlin(B, aspect, false); break;
    case 4: S = spheres_perlin(B, aspect, true); break;
    case 5: S = cornell_box(B, aspect); break;
    case 6: S = cornell_smoke(B, aspect); break;
    case 7: S = book2_final(B, rng, aspect); break;
    case 8: S = triangles(B, aspect); break;
    case 9: S = teapot_cornell(B, aspect); break;
    }
    if (B.err != MRT_OK) return mrt_internal_fail(B.err, B.errmsg.c_str());
    mrt_scene_blob* b = new mrt_scene_blob();
    b->main_rng = rng;
    uint32_t root = emit(b->flat, S.objects);
    uint32_t biased = S.biased ? emit(b->flat, S.biased) : MRT_NONE;
    b->mats = std::move(B.mats);
    b->texs = std::move(B.texs);
    b->texels = std::move(B.texels);
    perlin_tables(b->ranvec, b->perm);
    mrt_scene_view& v = b->view;
    memset(&v, 0, sizeof v);
    v.scene_id = scene;
    v.root = root;
    v.biased = biased;
    v.sky = scene < 5 ? 1u : 0u;  // main.cpp:110 (scene 9 renders as a Cornell scene)
    v.camera = S.cam;
    v.nodes = b->flat.nodes.data(); v.n_nodes = (uint32_t)b->flat.nodes.size();
    v.children = b->flat.children.data(); v.n_children = (uint32_t)b->flat.children.size();
    v.mesh_nodes = b->flat.mesh_nodes.data(); v.n_mesh_nodes = (uint32_t)b->flat.mesh_nodes.size();
    v.tri_geo = b->flat.tri_geo.data(); v.tri_nrm = b->flat.tri_nrm.data();
    v.n_tris = (uint32_t)(b->flat.tri_geo.size() / 12);
    v.materials = b->mats.data(); v.n_materials = (uint32_t)b->mats.size();
    v.textures = b->texs.data(); v.n_textures = (uint32_t)b->texs.size();
    v.perlin_ranvec = b->ranvec;
    v.perlin_perm = b->perm;
    v.texels = b->texels.data(); v.n_texels = b->texels.size();
    *out = b;
    return MRT_OK;
}

extern "C" mrt_status mrt_scene_blob_view(const mrt_scene_blob* blob, mrt_scene_view* out) {
    if (!blob || !out) return mrt_internal_fail(MRT_ERR_INVALID, "mrt_scene_blob_view: null");
    *out = blob->view;
    return MRT_OK;
}

extern "C" void mrt_scene_blob_free(mrt_scene_blob* blob) { delete blob; }

// main.cpp:357-361: for each worker, initstate = rand32() << 32 | rand32(), then initseq the same
// way, drawn from main()'s T_rng after scene generation (operands of | left to right, as clang
// evaluates the reference's expression)
extern "C" mrt_status mrt_worker_seeds(const mrt_scene_blob* blob, uint32_t n_threads, uint64_t* initstate, uint64_t* initseq) {
    if (!blob || (n_threads && (!initstate || !initseq))) return mrt_internal_fail(MRT_ERR_INVALID, "mrt_worker_seeds: null");
    Pcg r = blob->main_rng;
    for (uint32_t i = 0; i < n_threads; i++) {
        uint64_t hi = pcg_next(r);
        initstate[i] = (hi << 32) | pcg_next(r);
        hi = pcg_next(r);
        initseq[i] = (hi << 32) | pcg_next(r);
    }
    return MRT_OK;
}

// ---- JSON dump in the schema of oracle/ref/harness.cpp (--h-mode scene) ----
static std::string Fb(float f) {
    uint32_t u;
    memcpy(&u, &f, 4);
    return std::to_string(u);
}
static std::string V3s(const float* p) { return "[" + Fb(p[0]) + "," + Fb(p[1]) + "," + Fb(p[2]) + "]"; }
static std::string BOXs(const float* f) { return "[" + V3s(f) + "," + V3s(f + 3) + "]"; }

static std::string jtex(const mrt_scene_view& v, uint32_t t) {
    const mrt_texture& x = v.textures[t];
    switch (x.kind) {
    case MRT_T_COLOR: return "{\"t\":\"color\",\"c\":" + V3s(x.f) + "}";
    case MRT_T_CHECKER: return "{\"t\":\"checker\",\"scale\":" + Fb(x.f[0]) + ",\"even\":" + jtex(v, x.a) + ",\"odd\":" + jtex(v, x.b) + "}";
    case MRT_T_PERLIN: return "{\"t\":\"perlin\",\"scale\":" + Fb(x.f[0]) + "}";
    case MRT_T_IMAGE: {
        uint64_t h = 1469598103934665603ull;
        for (size_t i = 0; i < (size_t)x.b * x.c * 3; i++) h = (h ^ v.texels[x.a + i]) * 1099511628211ull;
        return "{\"t\":\"image\",\"w\":" + std::to_string(x.b) + ",\"h\":" + std::to_string(x.c) + ",\"fnv\":\"" + std::to_string(h) + "\"}";
    }
    }
    return "{\"t\":\"?\"}";
}
static std::string jmat(const mrt_scene_view& v, uint32_t m) {
    if (m == MRT_NONE) return "{\"m\":\"?\"}";
    const mrt_material& x = v.materials[m];
    switch (x.kind) {
    case MRT_M_LAMBERTIAN: return "{\"m\":\"lambertian\",\"tex\":" + jtex(v, x.tex) + "}";
    case MRT_M_ISOTROPIC: return "{\"m\":\"isotropic\",\"tex\":" + jtex(v, x.tex) + "}";
    case MRT_M_METAL: return "{\"m\":\"metal\",\"gloss\":" + Fb(x.p) + ",\"tex\":" + jtex(v, x.tex) + "}";
    case MRT_M_DIELECTRIC: return "{\"m\":\"dielectric\",\"ref\":" + Fb(x.p) + "}";
    case MRT_M_LIGHT: return "{\"m\":\"light\",\"scale\":" + Fb(x.p) + ",\"tex\":" + jtex(v, x.tex) + "}";
    }
    return "{\"m\":\"?\"}";
}
static std::string jnode(const mrt_scene_view& v, uint32_t id) {
    const mrt_node& n = v.nodes[id];
    uint32_t kind = n.kind & 0xFF, order = (n.kind >> 8) & 0xFF, fl = (n.kind >> 16) & 0xFF;
    switch (kind) {
    case MRT_K_LIST: {
        std::string s = "{\"k\":\"list\",\"hasBox\":" + std::to_string(fl & MRT_F_HASBOX ? 1 : 0) + ",\"box\":" +
                        ((fl & MRT_F_HASBOX) ? BOXs(n.f) : std::string("null")) + ",\"ch\":[";
        for (uint32_t i = 0; i < n.b; i++) s += (i ? "," : "") + jnode(v, v.children[n.a + i]);
        return s + "]}";
    }
    case MRT_K_BVH:
        return "{\"k\":\"bvh\",\"box\":" + BOXs(n.f) + ",\"order\":" + std::to_string(order) + ",\"same\":" + std::to_string(n.a == n.b ? 1 : 0) +
               ",\"l\":" + jnode(v, n.a) + ",\"r\":" + jnode(v, n.b) + "}";
    case MRT_K_TRANSLATE:
        return "{\"k\":\"translate\",\"off\":" + V3s(n.f) + ",\"c\":" + jnode(v, n.a) + "}";
    case MRT_K_ROTY:
        return "{\"k\":\"rotate_y\",\"sin\":" + Fb(n.f[6]) + ",\"cos\":" + Fb(n.f[7]) + ",\"hasBox\":" + std::to_string(fl & MRT_F_HASBOX ? 1 : 0) +
               ",\"box\":" + BOXs(n.f) + ",\"c\":" + jnode(v, n.a) + "}";
    case MRT_K_SPHERE:
        return "{\"k\":\"sphere\",\"c0\":" + V3s(n.f) + ",\"c1\":" + V3s(n.f + 3) + ",\"t0\":" + Fb(n.f[6]) + ",\"t1\":" + Fb(n.f[7]) +
               ",\"moving\":" + std::to_string(fl & MRT_F_MOVING ? 1 : 0) + ",\"r\":" + Fb(n.f[8]) + ",\"mat\":" + jmat(v, n.mat) + "}";
    case MRT_K_XY: case MRT_K_XZ: case MRT_K_YZ: {
        const char* k = kind == MRT_K_XY ? "xy_rect" : (kind == MRT_K_XZ ? "xz_rect" : "yz_rect");
        return std::string("{\"k\":\"") + k + "\",\"a0\":" + Fb(n.f[0]) + ",\"a1\":" + Fb(n.f[1]) + ",\"b0\":" + Fb(n.f[2]) + ",\"b1\":" +
               Fb(n.f[3]) + ",\"kk\":" + Fb(n.f[4]) + ",\"ns\":" + Fb(n.f[5]) + ",\"mat\":" + jmat(v, n.mat) + "}";
    }
    case MRT_K_VOLUME:
        return "{\"k\":\"volume\",\"density\":" + Fb(n.f[0]) + ",\"phase\":" + jmat(v, n.mat) + ",\"b\":" + jnode(v, n.a) + "}";
    case MRT_K_MESH: {
        uint32_t nb = n.a, cnt = n.b;
        uint32_t pb = v.mesh_nodes[nb].count_order & 0xFFFFFFu ? v.mesh_nodes[nb].left_or_first : MRT_NONE;
        // first triangle index of this mesh = smallest leaf offset
        uint32_t tmin = MRT_NONE;
        for (uint32_t i = 0; i < cnt; i++) {
            const mrt_mesh_node& m = v.mesh_nodes[nb + i];
            if (m.count_order & 0xFFFFFFu) tmin = std::min(tmin, m.left_or_first);
        }
        (void)pb;
        uint32_t ntri = (uint32_t)n.f[6];
        std::string s = "{\"k\":\"pod_bvh\",\"prim_count\":" + std::to_string(ntri) + ",\"node_count\":" + std::to_string(cnt) + ",\"mat\":" +
                        jmat(v, n.mat) + ",\"nodes\":[";
        for (uint32_t i = 0; i < cnt; i++) {
            const mrt_mesh_node& m = v.mesh_nodes[nb + i];
            uint32_t c = m.count_order & 0xFFFFFFu;
            uint32_t left = c ? 0 : m.left_or_first - nb, off = c ? m.left_or_first - tmin : 0;
            s += (i ? "," : "") + std::string("[[") + V3s(m.bmin) + "," + V3s(m.bmax) + "]," + std::to_string(left) + "," + std::to_string(off) + "," +
                 std::to_string(c) + "," + std::to_string(m.count_order >> 24) + "]";
        }
        s += "],\"prims\":[";
        for (uint32_t i = 0; i < ntri; i++) {
            const float* g = v.tri_geo + (size_t)(tmin + i) * 12;
            const float* q = v.tri_nrm + (size_t)(tmin + i) * 12;
            s += (i ? "," : "") + std::string("[") + V3s(g) + "," + V3s(g + 4) + "," + V3s(g + 8) + "," + V3s(q) + "," + V3s(q + 4) + "," + V3s(q + 8) + "]";
        }
        return s + "]}";
    }
    }
    return "{\"k\":\"?\"}";
}

extern "C" mrt_status mrt_scene_blob_dump_json(const mrt_scene_blob* blob, char** json_out) {
    if (!blob || !json_out) return mrt_internal_fail(MRT_ERR_INVALID, "dump: null");
    const mrt_scene_view& v = blob->view;
    const mrt_camera& c = v.camera;
    std::string s = "{\"camera\":{\"origin\":" + V3s(c.origin) + ",\"u\":" + V3s(c.u) + ",\"v\":" + V3s(c.v) + ",\"w\":" + V3s(c.w) +
                    ",\"llc\":" + V3s(c.llcorner) + ",\"horz\":" + V3s(c.horz) + ",\"vert\":" + V3s(c.vert) + ",\"lens\":" + Fb(c.lens_radius) +
                    ",\"t0\":" + Fb(c.time0) + ",\"t1\":" + Fb(c.time1) + "},";
    s += "\"objects\":" + jnode(v, v.root) + ",";
    s += "\"biased\":" + (v.biased != MRT_NONE ? jnode(v, v.biased) : std::string("null")) + ",";
    s += "\"perlin_ranvec\":[";
    for (int i = 0; i < 256; i++) s += (i ? "," : "") + V3s(v.perlin_ranvec + i * 4);
    s += "],\"perlin_perm\":[";
    for (int i = 0; i < 768; i++) s += (i ? "," : "") + std::to_string(v.perlin_perm[i]);
    s += "]}";
    char* r = (char*)malloc(s.size() + 1);
    memcpy(r, s.c_str(), s.size() + 1);
    *json_out = r;
    return MRT_OK;
}

extern "C" void mrt_free_string(char* s) { free(s); }

// Pack the parsed records of an OBJ file (tools/pack_assets.py) -- same parser as mrt_select_scene.
extern "C" mrt_status mrt_pack_obj(const char* obj_path, const char* out_path) {
    Builder B;
    ObjData o;
    if (!obj_path || !out_path || !B.read_obj(obj_path, &o)) return mrt_internal_fail(MRT_ERR_IO, "mrt_pack_obj: cannot read OBJ");
    FILE* f = fopen(out_path, "wb");
    if (!f) return mrt_internal_fail(MRT_ERR_IO, "mrt_pack_obj: cannot write");
    uint32_t hdr[3] = {(uint32_t)o.verts.size(), (uint32_t)o.norms.size(), (uint32_t)o.faces.size()};
    fwrite("MRTMESH1", 1, 8, f);
    fwrite(hdr, 4, 3, f);
    fwrite(o.verts.data(), 12, o.verts.size(), f);
    fwrite(o.norms.data(), 12, o.norms.size(), f);
    fwrite(o.faces.data(), sizeof(ObjFace), o.faces.size(), f);
    fclose(f);
    return MRT_OK;
}
