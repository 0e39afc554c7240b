/* hittable.h — drop-in for ray-tracing-c include/hittable.h (reference include/hittable.h:1-115).
 *
 * The scene graph keeps the reference's layout: every object starts with a `Hittable` header
 * (vtable pointer + padded AABB) and owns child pointers, so reference-style scene builders link
 * against this library unchanged.
 *
 * What differs from the reference is where the per-ray methods run.  Camera_render flattens the
 * graph (ray-tracing-c_amd/host/flatten.c: object kind is identified by vtable identity) and
 * traces every ray on the GPU.  The host-side `hit`/`pdf`/`rand` entries stored in the vtables are
 * identity tokens: calling one aborts with a message, because per-object CPU evaluation is not
 * part of this library (INTEGRATION.md §"Per-object methods").  Which entries are NULL matches the
 * reference exactly (BVHNode/Translate/RotateY/ConstantMedium have no pdf/rand), because light
 * sampling semantics depend on it (reference src/hittable.c:94, :104).
 */
#ifndef RT_HITTABLE_H
#define RT_HITTABLE_H
#ifndef HITTABLE_H
#define HITTABLE_H
#endif

#include "vec3.h"
#include <stdbool.h>
#include <stddef.h>

typedef struct Texture Texture;
typedef struct Material Material;
typedef struct HitRecord HitRecord;

typedef struct Ray {
  Vec3 origin;
  Vec3 direction; /* not normalised by the camera (reference src/raytracing.c:121) */
} Ray;

/* origin + direction * t (reference src/hittable.c:7) */
Vec3 ray_at(const Ray *ray, float t);

/* axis-aligned box: values[axis][0] = low, values[axis][1] = high */
typedef union AABB {
  struct {
    float x[2];
    float y[2];
    float z[2];
  };
  float values[3][2];
} AABB;

typedef struct Hittable Hittable;
typedef struct HittableVTable {
  bool (*hit)(const Hittable *self, const Ray *ray, float t_min, float t_max, HitRecord *rec, PCG32 *rng);
  float (*pdf)(const Hittable *self, const Ray *ray, PCG32 *rng);
  Vec3 (*rand)(const Hittable *self, Vec3 origin, PCG32 *rng);
} HittableVTable;

struct Hittable {
  HittableVTable *vtable;
  AABB bbox;
};

/* ordered container; closest hit over items in insertion order (reference src/hittable.c:74-88) */
typedef struct HittableList {
  Hittable hittable;
  size_t max_size;
  size_t size;
  Hittable **items;
} HittableList;

void HittableList_init(HittableList *self, size_t max_size);
Hittable *HittableList_new(size_t max_size);
void HittableList_append(HittableList *self, Hittable *item);

typedef struct Sphere {
  Hittable hittable;
  Vec3 center;
  float radius;
  Material *material;
} Sphere;

void Sphere_init(Sphere *self, Vec3 center, float radius, Material *mat);
Hittable *Sphere_new(Vec3 center, float radius, Material *mat);

/* parallelogram Q + a*u + b*v, a,b in [0,1] (reference src/hittable.c:186-243) */
typedef struct Quad {
  Hittable hittable;
  Vec3 Q;
  Vec3 u;
  Vec3 v;
  Vec3 normal;
  float D;
  Vec3 w;
  Material *material;
  float area;
} Quad;

void Quad_init(Quad *self, Vec3 Q, Vec3 u, Vec3 v, Material *mat);
Hittable *Quad_new(Vec3 Q, Vec3 u, Vec3 v, Material *mat);
/* six quads in a HittableList, fixed face order (reference src/hittable.c:246-264) */
Hittable *Box_new(Vec3 a, Vec3 b, Material *mat);

/* random-axis median-split BVH built with the caller's rng (reference src/hittable.c:280-323) */
typedef struct BVHNode {
  Hittable hittable;
  Hittable *left;
  Hittable *right;
} BVHNode;

void BVHNode_init(BVHNode *self, const HittableList *list, PCG32 *rng);
Hittable *BVHNode_new(const HittableList *list, PCG32 *rng);

typedef struct Translate {
  Hittable hittable;
  Hittable *object;
  Vec3 offset;
} Translate;

void Translate_init(Translate *self, Hittable *object, Vec3 offset);
Hittable *Translate_new(Hittable *object, Vec3 offset);

typedef struct RotateY {
  Hittable hittable;
  Hittable *object;
  float sin_theta;
  float cos_theta;
} RotateY;

/* angle in degrees */
void RotateY_init(RotateY *self, Hittable *object, float angle);
Hittable *RotateY_new(Hittable *object, float angle);

/* homogeneous participating medium bounded by `boundary`, Isotropic phase function */
typedef struct ConstantMedium {
  Hittable hittable;
  Hittable *boundary;
  float neg_inv_density;
  Material *phase_fn;
} ConstantMedium;

void ConstantMedium_init(ConstantMedium *self, Hittable *boundary, float density, Texture *albedo);
Hittable *ConstantMedium_new(Hittable *boundary, float density, Texture *albedo);

#endif /* RT_HITTABLE_H */
