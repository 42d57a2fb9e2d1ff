/* mrt_scene.h -- flattened scene format ("scene blob") shared by the host scene builder, the HIP
 * trace kernel and the C restatement in oracle/.  Plain C, no torch / HIP types.
 *
 * The reference keeps its scene as a tree of heap objects with virtual hit()/bounding_box()
 * (scene_object.h:20-31) built by select_scene() (scene.cpp:25-49).  Here every scene_object
 * becomes one 64-byte mrt_node record in one array (children referenced by index), materials and
 * textures become small tagged records, pod_bvh<triangle> meshes (triangle.h:46-322) become a
 * flat node array plus triangle arrays split by use: intersection data (m,u,v) apart from shading
 * normals (mn,un,vn), so a BVH walk touches only 48 B per triangle test.
 *
 * Node semantics (each restates one reference class; see DESIGN.md "Scene blob"):
 *   MRT_K_LIST      object_list<T>          scene_object.h:37-131   a=first slot in children[], b=count,
 *                                                                    flags&MRT_F_HASBOX, f[0..5]=box
 *   MRT_K_BVH       bvh_node<T>             scene_object.h:138-319  a=left node, b=right node,
 *                                                                    flags>>8 = node_order, f[0..5]=box
 *   MRT_K_MESH      pod_bvh<triangle>       triangle.h:58-322       a=root index in mesh_nodes[],
 *                                                                    b=node count, mat, f[0..5]=root box
 *   MRT_K_TRANSLATE translate               scene_object.cpp:9-27   a=child, f[0..2]=offset
 *   MRT_K_ROTY      rotate_y                scene_object.cpp:33-98  a=child, flags&MRT_F_HASBOX,
 *                                                                    f[0..5]=bbox, f[6]=sin, f[7]=cos
 *   MRT_K_SPHERE    sphere                  sphere.cpp:13-78        mat, flags&MRT_F_MOVING, f[0..2]=center0,
 *                                                                    f[3..5]=center1, f[6]=time0, f[7]=time1, f[8]=radius
 *   MRT_K_XY/XZ/YZ  xy_rect/xz_rect/yz_rect rect.cpp:6-152          mat, f[0]=a0 f[1]=a1 f[2]=b0 f[3]=b1
 *                                                                    f[4]=k (plane) f[5]=normal_sign
 *   MRT_K_VOLUME    constant_volume         volumes.cpp:5-35        a=boundary node, mat=phase material,
 *                                                                    f[0]=density
 * (box, box.h:6-30, is emitted as the MRT_K_LIST of its six rects.)
 */
#ifndef MRT_SCENE_H
#define MRT_SCENE_H
#include <stdint.h>
#include <stddef.h>

#ifdef __cplusplus
extern "C" {
#endif

enum mrt_node_kind {
    MRT_K_LIST = 1,
    MRT_K_BVH = 2,
    MRT_K_MESH = 3,
    MRT_K_TRANSLATE = 4,
    MRT_K_ROTY = 5,
    MRT_K_SPHERE = 6,
    MRT_K_XY = 7,
    MRT_K_XZ = 8,
    MRT_K_YZ = 9,
    MRT_K_VOLUME = 10
};
#define MRT_F_HASBOX 0x1u
#define MRT_F_MOVING 0x2u
#define MRT_NONE 0xFFFFFFFFu

typedef struct mrt_node {
    uint32_t kind;  /* low 8 bits: mrt_node_kind; bits 8..15: bvh node_order; bits 16..23: MRT_F_* */
    uint32_t a, b;
    uint32_t mat;
    float f[12];
} mrt_node; /* 64 bytes */

/* pod_bvh_node (triangle.h:46-56) with left/prim_offset made absolute into the blob arrays.
 * inner: count_order&0xFFFFFF == 0, left_or_first = left child (right = left+1)
 * leaf : count = count_order&0xFFFFFF, left_or_first = first triangle            */
typedef struct mrt_mesh_node {
    float bmin[3];
    uint32_t left_or_first;
    float bmax[3];
    uint32_t count_order; /* count | node_order << 24 */
} mrt_mesh_node; /* 32 bytes */

enum mrt_material_kind { MRT_M_LAMBERTIAN = 1, MRT_M_ISOTROPIC = 2, MRT_M_METAL = 3, MRT_M_DIELECTRIC = 4, MRT_M_LIGHT = 5 };
/* material.h:34-200: lambertian(tex), isotropic(tex), metal(tex, p=gloss), dielectric(p=ref_index),
 * diffuse_light(tex, p=scale) */
typedef struct mrt_material {
    uint32_t kind;
    uint32_t tex;
    float p;
    float pad;
} mrt_material;

enum mrt_texture_kind { MRT_T_COLOR = 1, MRT_T_CHECKER = 2, MRT_T_PERLIN = 3, MRT_T_IMAGE = 4 };
/* texture.h:11-75: color(f[0..2]), checker(a=even, b=odd, f[0]=scale), perlin(f[0]=scale),
 * image(a=texel byte offset, b=width, c=height) */
typedef struct mrt_texture {
    uint32_t kind;
    uint32_t a, b, c;
    float f[4];
} mrt_texture;

/* camera.h:6-46 (derived vectors precomputed exactly as the constructor does) */
typedef struct mrt_camera {
    float origin[4], u[4], v[4], w[4], llcorner[4], horz[4], vert[4];
    float lens_radius, time0, time1, pad;
} mrt_camera;

/* A read-only view of a built scene: the arrays the HIP backend uploads to HBM. */
typedef struct mrt_scene_view {
    uint32_t scene_id;      /* reference scenes enum (scene.h:6-17); 9 = teapot-in-Cornell (C3) */
    uint32_t root;          /* node index of scene.objects */
    uint32_t biased;        /* node index of scene.biased_objects or MRT_NONE */
    uint32_t sky;           /* 1: miss returns the sky gradient (main.cpp:110-116 sceneSelect<5) */
    mrt_camera camera;
    const mrt_node* nodes;  uint32_t n_nodes;
    const uint32_t* children; uint32_t n_children;
    const mrt_mesh_node* mesh_nodes; uint32_t n_mesh_nodes;
    const float* tri_geo;   /* 12 floats per triangle: m.xyz,0, u.xyz,0, v.xyz,0 */
    const float* tri_nrm;   /* 12 floats per triangle: mn, un, vn (xyz,0 each) */
    uint32_t n_tris;
    const mrt_material* materials; uint32_t n_materials;
    const mrt_texture* textures; uint32_t n_textures;
    const float* perlin_ranvec; /* 256 x (x,y,z,0) -- texture.cpp:167-172 */
    const int32_t* perlin_perm; /* 3 x 256 -- texture.cpp:174-203 */
    const uint8_t* texels; uint64_t n_texels;
} mrt_scene_view;

#ifdef __cplusplus
}
#endif
#endif
