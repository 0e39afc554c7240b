/* raytracing.h — drop-in for ray-tracing-c include/raytracing.h (reference include/raytracing.h:1-43).
 *
 * Camera_render is THE boundary this library replaces (reference src/raytracing.c:86-135, called
 * once from src/main.c:336).  Same signature, same output contract: `buffer` is caller-owned,
 * width*height*3 bytes, row-major top to bottom, RGB, gamma-2 encoded, byte-identical to the
 * reference CPU render.  Internally it flattens `world` and hands it through the C ABI in
 * rt_hip.h to the gfx950 kernel, split row-interleaved over the visible GPUs
 * (RT_NUM_GPUS=<n> to restrict).  It aborts with a message on any GPU/runtime error instead of
 * returning a partial image; there is no CPU fallback.
 */
#ifndef RT_RAYTRACING_H
#define RT_RAYTRACING_H
#ifndef RAYTRACING_H
#define RAYTRACING_H
#endif

#include "hittable.h"
#include "material.h"
#include "vec3.h"
#include <stddef.h>
#include <stdint.h>

typedef struct World {
  HittableList objects; /* root: traced with t in [1e-3, inf) */
  HittableList lights;  /* importance-sampled emitters (may be empty) */
} World;

void World_init(World *world, size_t max_objects);

typedef struct Camera {
  /* user inputs */
  float aspect_ratio;
  int img_width;
  int img_height; /* derived by Camera_init */
  int samples_per_pixel;
  int max_depth;
  Vec3 background;
  float vfov; /* degrees */
  Vec3 look_from;
  Vec3 look_to;
  Vec3 vup;
  float dof_angle; /* degrees; > 0 enables the thin-lens disc */
  float focal_length;
  /* derived by Camera_init (reference src/raytracing.c:13-37) */
  Vec3 pixel00_loc;
  Vec3 pixel_delta_u;
  Vec3 pixel_delta_v;
  Vec3 u; /* camera basis */
  Vec3 v;
  Vec3 w;
  Vec3 dof_disc_u;
  Vec3 dof_disc_v;
  /* user input */
  float lights_sampling_prob;
} Camera;

void Camera_init(Camera *camera);
void Camera_render(const Camera *camera, const World *world, uint8_t *buffer);

#endif /* RT_RAYTRACING_H */
