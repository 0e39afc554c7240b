/* material.h — drop-in for ray-tracing-c include/material.h (reference include/material.h:1-68).
 *
 * Materials are a tagged union (MaterialType + albedo texture + fuzz/eta).  Scattering itself is
 * evaluated on the GPU (ray-tracing-c_amd/csrc/rt_device.h, rt_scatter); the host entry points
 * Material_scatter / Material_scatter_pdf / Material_emit exist for link compatibility and abort
 * when called (INTEGRATION.md §"Per-object methods").  ONB helpers are plain vector math and are
 * implemented on the host.
 */
#ifndef RT_MATERIAL_H
#define RT_MATERIAL_H
#ifndef MATERIAL_H
#define MATERIAL_H
#endif

#include "vec3.h"
#include <stdbool.h>

typedef struct Texture Texture;
typedef struct Material Material;

typedef struct HitRecord {
  Vec3 p;
  Vec3 normal; /* faces against the incoming ray */
  Material *material;
  float t;
  float u;
  float v;
  bool front_face;
} HitRecord;

typedef enum MaterialType {
  SURFACE_NORMAL, /* debug: emits (n+1)/2, never scatters */
  LAMBERTIAN,     /* cosine-weighted scattering in the normal's ONB */
  METAL,          /* mirror reflection + fuzz * random unit vector */
  DIELECTRIC,     /* Schlick-weighted reflect / refract, rng-gated */
  DIFFUSE_LIGHT,  /* emits albedo on the front face, never scatters */
  ISOTROPIC,      /* uniform-sphere phase function (volumes) */
} MaterialType;

struct Material {
  MaterialType tag;
  Texture *albedo; /* NULL for DIELECTRIC */
  union {
    float fuzz; /* METAL */
    float eta;  /* DIELECTRIC */
  };
};

bool Material_scatter(const HitRecord *rec, Vec3 r_in, Vec3 *r_out, Vec3 *color, bool *skip_pdf, PCG32 *rng);
float Material_scatter_pdf(const Material *mat, Vec3 normal, Vec3 r_in, Vec3 r_out);
Vec3 Material_emit(const HitRecord *rec);

void SurfaceNormal_init(Material *self);
Material *SurfaceNormal_new();

void Lambertian_init(Material *self, Texture *albedo);
Material *Lambertian_new(Texture *albedo);

void Metal_init(Material *self, Texture *albedo, float fuzz);
Material *Metal_new(Texture *albedo, float fuzz);

void Dielectric_init(Material *self, float eta);
Material *Dielectric_new(float eta);

void DiffuseLight_init(Material *self, Texture *albedo);
Material *DiffuseLight_new(Texture *albedo);

void Isotropic_init(Material *self, Texture *albedo);
Material *Isotropic_new(Texture *albedo);

/* orthonormal basis around w (reference src/material.c:144-152) */
typedef struct ONB {
  Vec3 u;
  Vec3 v;
  Vec3 w;
} ONB;
Vec3 ONB_local(const ONB *self, Vec3 a);
void ONB_from_w(ONB *self, Vec3 w);

#endif /* RT_MATERIAL_H */
