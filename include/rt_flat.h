/* rt_flat.h — the flattened, pointer-free scene that crosses the C ABI into the HIP kernel.
 *
 * Camera_render (reference src/raytracing.c:86) receives a pointer graph of vtable-polymorphic
 * objects.  GPUs want flat arrays, so rt_flatten() (ray-tracing-c_amd/host/rt_flatten.c) converts
 * the World once per render into the typed arrays below.  Every array is plain-old-data, 16-byte
 * aligned, and copied verbatim to HBM (one allocation, see rt_hip.hip: rt_scene_upload).
 *
 * Object references ("refs") are int32: (kind << RT_REF_SHIFT) | index into that kind's array,
 * or RT_REF_NONE.  Traversal visits refs in exactly the reference's order (BVH: left then right;
 * lists: insertion order) so closest-hit ties, t_max shrinking and rng draws inside constant
 * media happen as in the CPU render.
 *
 * Everything numeric is the value the reference computes at the same point (e.g. sphere r*r and
 * 1/r are pre-evaluated exactly as src/hittable.c:126 and src/vec3.c:19 would), so the kernel
 * never re-derives a scene constant with different rounding.
 */
#ifndef RT_FLAT_H
#define RT_FLAT_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define RT_REF_SHIFT 28
#define RT_REF_INDEX_MASK ((1 << RT_REF_SHIFT) - 1)
#define RT_REF_NONE (-1)

enum rt_kind {
  RT_KIND_BVH = 0,       /* rt_bvh_node           (reference BVHNode)          */
  RT_KIND_SPHERE = 1,    /* rt_sphere             (reference Sphere)           */
  RT_KIND_QUAD = 2,      /* rt_quad               (reference Quad)             */
  RT_KIND_LIST = 3,      /* rt_list + item pool   (reference HittableList)     */
  RT_KIND_TRANSLATE = 4, /* rt_translate          (reference Translate)        */
  RT_KIND_ROTATE_Y = 5,  /* rt_rotate_y           (reference RotateY)          */
  RT_KIND_MEDIUM = 6,    /* rt_medium             (reference ConstantMedium)   */
  RT_KIND_COUNT = 7
};

/* macros rather than inline functions so host C and gfx950 device code share them */
#define rt_ref(kind, index) ((int32_t)(((uint32_t)(kind) << RT_REF_SHIFT) | (uint32_t)(index)))
#define rt_ref_kind(ref) ((int)((uint32_t)(ref) >> RT_REF_SHIFT))
#define rt_ref_index(ref) ((int32_t)((ref) & RT_REF_INDEX_MASK))

/* 32 B: bounds then child refs.  right == RT_REF_NONE encodes the reference's n == 1 leaf whose
 * left and right are the same object (src/hittable.c:294-296): the second visit can never change
 * the closest hit of an rng-free child, so it is dropped.  Children that consume rng keep both. */
typedef struct rt_bvh_node {
  float lo[3];
  float hi[3];
  int32_t left;
  int32_t right;
} rt_bvh_node;

typedef struct rt_sphere { /* 32 B */
  float center[3];
  float radius;
  float radius_sq;  /* radius * radius              (src/hittable.c:126) */
  float inv_radius; /* 1.0f / radius                 (src/hittable.c:143 via src/vec3.c:19) */
  int32_t material;
  int32_t pad;
} rt_sphere;

typedef struct rt_quad { /* 80 B */
  float Q[3];
  float D;
  float u[3];
  float area;
  float v[3];
  int32_t material;
  float normal[3];
  float pad0;
  float w[3];
  float pad1;
} rt_quad;

typedef struct rt_list { /* items are list_items[first .. first+count) */
  int32_t first;
  int32_t count;
} rt_list;

typedef struct rt_translate {
  float offset[3];
  int32_t child;
  int32_t parent_xform; /* enclosing transform ref or RT_REF_NONE (world frame) */
  int32_t pad[3];
} rt_translate;

typedef struct rt_rotate_y {
  float sin_theta;
  float cos_theta;
  int32_t child;
  int32_t parent_xform;
} rt_rotate_y;

typedef struct rt_medium {
  int32_t boundary;       /* ref of a sphere or quad */
  float neg_inv_density;  /* -1.0f / density (src/hittable.c:429) */
  int32_t phase_material; /* an ISOTROPIC material */
  int32_t parent_xform;
} rt_medium;

enum rt_material_tag { /* same numbering as the reference MaterialType (include/material.h:20-27) */
  RT_MAT_SURFACE_NORMAL = 0,
  RT_MAT_LAMBERTIAN = 1,
  RT_MAT_METAL = 2,
  RT_MAT_DIELECTRIC = 3,
  RT_MAT_DIFFUSE_LIGHT = 4,
  RT_MAT_ISOTROPIC = 5
};

typedef struct rt_material {
  int32_t tag;
  int32_t texture; /* index into textures, -1 for DIELECTRIC / SURFACE_NORMAL */
  float param;     /* fuzz (METAL) or eta (DIELECTRIC) */
  int32_t pad;
} rt_material;

enum rt_texture_kind { RT_TEX_SOLID = 0, RT_TEX_CHECKER = 1, RT_TEX_IMAGE = 2, RT_TEX_PERLIN = 3 };

typedef struct rt_texture { /* 32 B */
  int32_t kind;
  int32_t a;     /* CHECKER: even texture; IMAGE: image index; PERLIN: perlin index */
  int32_t b;     /* CHECKER: odd texture */
  float scale;   /* CHECKER / PERLIN */
  float color[3];/* SOLID */
  int32_t pad;
} rt_texture;

typedef struct rt_image {
  int32_t width;
  int32_t height;
  int64_t offset; /* byte offset into image_bytes (RGB8, row-major) */
} rt_image;

typedef struct rt_perlin { /* reference Perlin (include/texture.h:40-48), minus the vtable */
  float grad[256][4];    /* xyz + pad */
  int32_t perm_x[256];
  int32_t perm_y[256];
  int32_t perm_z[256];
  int32_t depth;
  int32_t pad[3];
} rt_perlin;

/* Camera_init's derived values (reference src/raytracing.c:13-37), consumed verbatim. */
typedef struct rt_camera {
  int32_t width, height, spp, max_depth;
  float pixel00[3];
  float dof_angle;
  float delta_u[3];
  float light_prob;
  float delta_v[3];
  float pad0;
  float origin[3];
  float pad1;
  float disc_u[3];
  float pad2;
  float disc_v[3];
  float pad3;
  float background[3];
  float pad4;
} rt_camera;

enum rt_feature_bits { /* which code paths a scene needs (kernel specialisation + validation) */
  RT_FEAT_BVH = 1 << 0,
  RT_FEAT_QUAD = 1 << 1,
  RT_FEAT_XFORM = 1 << 2,
  RT_FEAT_MEDIUM = 1 << 3,
  RT_FEAT_LIGHTS = 1 << 4,     /* mixture-pdf light sampling active (lights non-empty, p != 0) */
  RT_FEAT_TEX_UV = 1 << 5,     /* checker / image textures: sphere u,v needed */
  RT_FEAT_TEX_PERLIN = 1 << 6,
  RT_FEAT_EMISSIVE = 1 << 7,   /* DIFFUSE_LIGHT or SURFACE_NORMAL materials present */
  RT_FEAT_DOF = 1 << 8
};

typedef struct rt_flat_scene {
  rt_camera camera;
  int32_t root;          /* ref of World.objects (always a list) */
  int32_t lights;        /* list index of World.lights in `lists` */
  int32_t features;      /* rt_feature_bits */
  int32_t stack_needed;  /* deepest traversal stack the DFS needs (checked against the kernel) */

  int32_t n_bvh, n_spheres, n_quads, n_lists, n_list_items;
  int32_t n_translates, n_rotates, n_media, n_materials, n_textures, n_images, n_perlins;
  int64_t n_image_bytes;

  rt_bvh_node *bvh;
  rt_sphere *spheres;
  rt_quad *quads;
  rt_list *lists;
  int32_t *list_items;
  rt_translate *translates;
  rt_rotate_y *rotates;
  rt_medium *media;
  rt_material *materials;
  rt_texture *textures;
  rt_image *images;
  rt_perlin *perlins;
  uint8_t *image_bytes;
} rt_flat_scene;

#ifdef __cplusplus
}
#endif

#endif /* RT_FLAT_H */
