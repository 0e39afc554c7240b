/* rt_internal.h — private glue of the host library (not installed). */
#ifndef RT_INTERNAL_H
#define RT_INTERNAL_H

#include "hittable.h"
#include "material.h"
#include "raytracing.h"
#include "rt_flat.h"
#include "rt_hip.h"
#include "texture.h"
#include "tiff.h"
#include "utils.h"
#include "vec3.h"

#define RT_HIDDEN __attribute__((visibility("hidden")))

/* vtables: their addresses are the object-kind identity used by the flattener */
extern RT_HIDDEN HittableVTable rt_vt_list;
extern RT_HIDDEN HittableVTable rt_vt_sphere;
extern RT_HIDDEN HittableVTable rt_vt_quad;
extern RT_HIDDEN HittableVTable rt_vt_bvh;
extern RT_HIDDEN HittableVTable rt_vt_translate;
extern RT_HIDDEN HittableVTable rt_vt_rotate_y;
extern RT_HIDDEN HittableVTable rt_vt_medium;

/* texture value entry points: identity tokens for the flattener */
RT_HIDDEN Vec3 rt_tex_solid_value(const Texture *self, float u, float v, Vec3 p);
RT_HIDDEN Vec3 rt_tex_checker_value(const Texture *self, float u, float v, Vec3 p);
RT_HIDDEN Vec3 rt_tex_image_value(const Texture *self, float u, float v, Vec3 p);
RT_HIDDEN Vec3 rt_tex_perlin_value(const Texture *self, float u, float v, Vec3 p);


/* reference driver scenes (src/main.c:9-273); defined in rt_scenes.c */
void scene_metal_and_lambertian(World *world, Camera *camera);
void scene_book1_final(World *world, Camera *camera);
void scene_checker(World *world, Camera *camera);
void scene_earth(World *world, Camera *camera);
void scene_perlin(World *world, Camera *camera);
void scene_simple_light(World *world, Camera *camera);
void scene_cornell_box(World *world, Camera *camera);
void scene_book2_final(World *world, Camera *camera, bool enable_bvh);
/* reference main()'s camera defaults (src/main.c:278-287) */
void rt_camera_defaults(Camera *camera);
/* scene switch of src/main.c:294-329; returns the scene title */
const char *rt_build_scene(int scene_id, World *world, Camera *camera);

/* error channel shared with the HIP side */
void rt_set_error(const char *fmt, ...);

/* baseline JPEG -> RGB (rt_jpeg.c); NULL on failure with the reason in err */
RT_HIDDEN uint8_t *rt_jpeg_decode(const uint8_t *buf, size_t len, int *width, int *height, char *err, size_t err_len);
/* Image_new failures: the reference aborts (src/texture.c:41); rt_scene_preset instead records the
 * failure (rt_image_soft_begin/end) and returns NULL with the message in rt_last_error().  dir: where
 * relative image file names are looked up (NULL: the working directory, as the reference does) */
RT_HIDDEN void rt_image_soft_begin(const char *dir);
RT_HIDDEN int rt_image_soft_end(void);  /* 0: every image loaded */

#endif /* RT_INTERNAL_H */
