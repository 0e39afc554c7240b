/* rt_camera.c — World/Camera setup and the Camera_render boundary.
 *
 * Camera_init is host-side precompute (reference src/raytracing.c:13-37) and stays bit-exact
 * with the reference (same glibc tanf, same operation order).  Camera_render
 * (reference src/raytracing.c:86-135) is the drop-in boundary: flatten the World, render on the
 * GPU(s) through rt_hip.h, abort on failure.  No CPU rendering path exists in this library.
 */
#include "rt_internal.h"

#include <math.h>
#include <stdarg.h>
#include <stdio.h>
#include <stdlib.h>

void World_init(World *world, size_t max_objects) {
  HittableList_init(&world->objects, max_objects);
  HittableList_init(&world->lights, max_objects);
}

void Camera_init(Camera *cam) {
  cam->img_height = (int)((float)cam->img_width / cam->aspect_ratio);

  const float half_fov = cam->vfov * (float)M_PI / 360.0f;
  const float vp_h = 2.0f * tanf(half_fov) * cam->focal_length;
  const float vp_w = vp_h * (float)cam->img_width / (float)cam->img_height;

  cam->w = vec3_normalize(vec3_sub_vec3(cam->look_from, cam->look_to));
  cam->u = vec3_cross(cam->vup, cam->w);
  cam->v = vec3_cross(cam->w, cam->u);

  const Vec3 span_u = vec3_mul_float(cam->u, vp_w);   /* left -> right */
  const Vec3 span_v = vec3_mul_float(cam->v, -vp_h);  /* top -> bottom */
  cam->pixel_delta_u = vec3_div_float(span_u, (float)cam->img_width);
  cam->pixel_delta_v = vec3_div_float(span_v, (float)cam->img_height);

  Vec3 corner = vec3_add_vec3(cam->look_from, vec3_mul_float(cam->w, -cam->focal_length));
  corner = vec3_add_vec3(corner, vec3_mul_float(span_u, -0.5f));
  corner = vec3_add_vec3(corner, vec3_mul_float(span_v, -0.5f));
  Vec3 p00 = vec3_add_vec3(corner, vec3_mul_float(cam->pixel_delta_u, 0.5f));
  cam->pixel00_loc = vec3_add_vec3(p00, vec3_mul_float(cam->pixel_delta_v, 0.5f));

  const float lens_r = cam->focal_length * tanf(cam->dof_angle * (float)M_PI / 360.0f);
  cam->dof_disc_u = vec3_mul_float(cam->u, lens_r);
  cam->dof_disc_v = vec3_mul_float(cam->v, lens_r);
}

static int gpus_requested(void) {
  const char *e = getenv("RT_NUM_GPUS");
  return (e && *e) ? atoi(e) : 0;
}

void Camera_render(const Camera *camera, const World *world, uint8_t *buffer) {
  rt_flat_scene *flat = rt_flatten(camera, world);
  if (flat == NULL) {
    fprintf(stderr, "rt: Camera_render: cannot flatten the scene: %s\n", rt_last_error());
    abort();
  }
  fprintf(stderr, "rt: rendering %dx%d, %d spp, depth %d on the GPU\n", flat->camera.width, flat->camera.height,
          flat->camera.spp, flat->camera.max_depth);
  const int rc = rt_render(flat, gpus_requested(), buffer);
  rt_flat_free(flat);
  if (rc != 0) {
    fprintf(stderr, "rt: Camera_render: GPU render failed: %s\n", rt_last_error());
    abort();
  }
  fprintf(stderr, "Done\n");
}
