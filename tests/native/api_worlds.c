/* api_worlds.c — TEST INFRASTRUCTURE.  Worlds that none of the reference driver's presets builds,
 * made only through the reference's public C API (include/{raytracing,hittable,material,texture,
 * vec3,pcg32}.h) and rendered with Camera_render.  The same source is linked twice:
 *   oracle/_ref/api_worlds_ref      against the reference's own src/*.c (oracle/Makefile), run here
 *                                   to make the fixtures tests/golden/api_*.rgb.gz;
 *   tests/native/bin/api_worlds_gpu against librtc_amd.so (the drop-in), run by the -m gpu tests.
 * The paths it covers (VERDICT r01 "parity on API paths outside the presets"):
 *   0 SurfaceNormal material (src/material.c:19-20, :105, :135)
 *   1 hollow glass: a negative-radius sphere inside a glass sphere (src/hittable.c:120-151)
 *   2 Metal with fuzz > 1 and fuzz 0, thin-lens DOF on a sphere world (src/material.c:48-58)
 *   3 quads, Box under RotateY + Translate, a constant medium, Checker texture, a light with
 *     importance sampling, DOF (src/hittable.c:186-432, src/raytracing.c:56-71)
 *   4 max_depth 100 inside a mirror sphere: most paths run to the depth limit
 *   5 a 1-pixel-wide image (48 rows) of a BVH world
 *   6 a flat list of 120 spheres (no BVH), Book-1 materials, 64 spp
 *   7 max_depth 100 on a BVH world of Book-1 materials (the fast path's depth limit)
 * and, for the product library's size-driven fallbacks (VERDICT r04 "what's weak" 6: reached with the
 * product build and natural inputs, no diagnostic switch):
 *   8 a 1100-sphere BVH at 64 spp: 2200 preorder items (70 KiB) exceed the 64 KiB a Book-1 workgroup
 *     stages in LDS, so the chain kernel reads the items from global memory, and with more than 512
 *     leaves its whole-wave items take the exact scan (coop_trace9) instead of the candidate trace
 *   9 the same world at 16 spp: the lane kernel on global-memory items
 *  10 1000 boxes (6000 quads) in a BVH under a sampled light: ~7000 preorder entries (220 KiB) exceed
 *     one workgroup's 160 KiB of LDS, so the general path runs its 256-thread kernel with the first
 *     entries in LDS and the rest in global memory
 * usage: see main()     prints "width height" on stdout per frame */
#include "hittable.h"
#include "material.h"
#include "pcg32.h"
#include "raytracing.h"
#include "texture.h"
#include "vec3.h"

#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

/* The drop-in library's C ABI (include/rt_hip.h), when this source is linked to it: weak, so the
 * reference build (which has none of it) links too.  API_WORLDS_KERNEL=1 prints on stderr the frame
 * kernel the library picks for the world -- the tests check that worlds 8-10 reach their fallbacks. */
typedef struct rt_flat_scene rt_flat_scene;
typedef struct rt_device_scene rt_device_scene;
extern rt_flat_scene *rt_flatten(const Camera *camera, const World *world) __attribute__((weak));
extern void rt_flat_free(rt_flat_scene *scene) __attribute__((weak));
extern rt_device_scene *rt_scene_upload(const rt_flat_scene *scene, int device) __attribute__((weak));
extern void rt_scene_release(rt_device_scene *dscene) __attribute__((weak));
extern const char *rt_scene_kernel(const rt_device_scene *dscene) __attribute__((weak));

static void report_kernel(const Camera *c, const World *w) {
  if (!getenv("API_WORLDS_KERNEL") || !rt_flatten || !rt_scene_upload || !rt_scene_kernel) return;
  rt_flat_scene *flat = rt_flatten(c, w);
  rt_device_scene *d = flat ? rt_scene_upload(flat, 0) : NULL;
  fprintf(stderr, "kernel: %s\n", d ? rt_scene_kernel(d) : "(upload failed)");
  if (d) rt_scene_release(d);
  if (flat) rt_flat_free(flat);
}

static void camera_defaults(Camera *c, int width, float aspect, int spp, int depth) {
  c->aspect_ratio = aspect;
  c->img_width = width;
  c->samples_per_pixel = spp;
  c->max_depth = depth;
  c->vup = vec3(0.0f, 1.0f, 0.0f);
  c->dof_angle = 0.0f;
  c->focal_length = 1.0f;
  c->lights_sampling_prob = 0.5f;
  c->background = vec3(0.70f, 0.80f, 1.00f);
  c->vfov = 50.0f;
  c->look_from = vec3(0.0f, 0.4f, 1.5f);
  c->look_to = vec3(0.0f, 0.0f, -1.0f);
}

static void add(World *w, Hittable *h) { HittableList_append(&w->objects, h); }

static Material *lamb(float r, float g, float b) { return Lambertian_new(Solid_new(vec3(r, g, b))); }

static void ground(World *w) { add(w, Sphere_new(vec3(0.0f, -1000.5f, -1.0f), 1000.0f, lamb(0.45f, 0.5f, 0.4f))); }

static void world_surface_normal(World *w, Camera *c) {
  camera_defaults(c, 96, 16.0f / 9.0f, 40, 20);
  ground(w);
  add(w, Sphere_new(vec3(0.0f, 0.0f, -1.0f), 0.5f, SurfaceNormal_new()));
  add(w, Sphere_new(vec3(-1.05f, 0.0f, -1.2f), 0.45f, lamb(0.8f, 0.3f, 0.3f)));
  add(w, Sphere_new(vec3(1.05f, 0.0f, -1.2f), 0.45f, SurfaceNormal_new()));
}

static void world_hollow_glass(World *w, Camera *c) {
  camera_defaults(c, 96, 16.0f / 9.0f, 64, 50);
  ground(w);
  add(w, Sphere_new(vec3(0.0f, 0.0f, -1.0f), 0.5f, Dielectric_new(1.5f)));
  add(w, Sphere_new(vec3(0.0f, 0.0f, -1.0f), -0.42f, Dielectric_new(1.5f)));  // the hollow inside
  add(w, Sphere_new(vec3(-1.0f, 0.0f, -1.4f), 0.5f, lamb(0.1f, 0.2f, 0.5f)));
  add(w, Sphere_new(vec3(1.0f, 0.0f, -1.4f), 0.5f, Metal_new(Solid_new(vec3(0.8f, 0.6f, 0.2f)), 0.05f)));
  add(w, Sphere_new(vec3(0.3f, -0.35f, -0.3f), 0.15f, Dielectric_new(1.0f / 1.33f)));
}

static void world_metal_fuzz(World *w, Camera *c) {
  camera_defaults(c, 96, 16.0f / 9.0f, 48, 50);
  c->dof_angle = 2.0f;
  c->focal_length = 2.4f;
  ground(w);
  add(w, Sphere_new(vec3(-1.1f, 0.0f, -1.0f), 0.5f, Metal_new(Solid_new(vec3(0.8f, 0.8f, 0.8f)), 1.5f)));
  add(w, Sphere_new(vec3(0.0f, 0.0f, -1.0f), 0.5f, Metal_new(Solid_new(vec3(0.7f, 0.6f, 0.5f)), 0.0f)));
  add(w, Sphere_new(vec3(1.1f, 0.0f, -1.0f), 0.5f, Metal_new(Solid_new(vec3(0.2f, 0.5f, 0.8f)), 3.0f)));
  add(w, Sphere_new(vec3(0.0f, -0.3f, -0.2f), 0.2f, lamb(0.9f, 0.1f, 0.1f)));
}

static void world_quads_xform(World *w, Camera *c) {
  camera_defaults(c, 96, 1.0f, 24, 30);
  c->background = vec3(0.02f, 0.02f, 0.03f);
  c->dof_angle = 1.5f;
  c->focal_length = 6.0f;
  c->vfov = 40.0f;
  c->look_from = vec3(2.0f, 2.5f, 6.0f);
  c->look_to = vec3(0.0f, 0.8f, 0.0f);
  Texture *chk = Checker_new(0.6f, Solid_new(vec3(0.2f, 0.3f, 0.1f)), Solid_new(vec3(0.9f, 0.9f, 0.9f)));
  add(w, Quad_new(vec3(-4.0f, 0.0f, -4.0f), vec3(8.0f, 0.0f, 0.0f), vec3(0.0f, 0.0f, 8.0f), Lambertian_new(chk)));
  add(w, Quad_new(vec3(-4.0f, 0.0f, -3.0f), vec3(8.0f, 0.0f, 0.0f), vec3(0.0f, 5.0f, 0.0f), lamb(0.6f, 0.3f, 0.3f)));
  Hittable *box = Box_new(vec3(0.0f, 0.0f, 0.0f), vec3(1.2f, 1.6f, 1.0f), lamb(0.73f, 0.73f, 0.73f));
  box = RotateY_new(box, 25.0f);
  box = Translate_new(box, vec3(-1.6f, 0.0f, -0.6f));
  add(w, box);
  Hittable *fog = Sphere_new(vec3(1.3f, 0.8f, 0.2f), 0.8f, Dielectric_new(1.5f));
  add(w, ConstantMedium_new(fog, 0.9f, Solid_new(vec3(0.2f, 0.4f, 0.9f))));
  add(w, Sphere_new(vec3(0.4f, 0.45f, 1.2f), 0.45f, Metal_new(Solid_new(vec3(0.9f, 0.9f, 0.9f)), 0.2f)));
  Material *light = DiffuseLight_new(Solid_new(vec3(6.0f, 6.0f, 6.0f)));
  Hittable *panel = Quad_new(vec3(-1.0f, 4.0f, -1.0f), vec3(2.0f, 0.0f, 0.0f), vec3(0.0f, 0.0f, 2.0f), light);
  add(w, panel);
  HittableList_append(&w->lights, panel);
}

static void world_deep_mirror(World *w, Camera *c) {
  camera_defaults(c, 64, 16.0f / 9.0f, 8, 100);
  c->background = vec3(0.0f, 0.0f, 0.0f);
  c->look_from = vec3(0.0f, 0.0f, 0.0f);
  c->look_to = vec3(0.0f, 0.0f, -1.0f);
  c->vfov = 80.0f;
  // inside a near-perfect mirror: a path leaves only through the small light
  add(w, Sphere_new(vec3(0.0f, 0.0f, 0.0f), 4.0f, Metal_new(Solid_new(vec3(0.97f, 0.96f, 0.95f)), 0.01f)));
  add(w, Sphere_new(vec3(1.5f, 1.0f, -2.0f), 0.3f, DiffuseLight_new(Solid_new(vec3(4.0f, 3.0f, 2.0f)))));
  add(w, Sphere_new(vec3(-1.0f, -0.8f, -2.5f), 0.6f, lamb(0.5f, 0.7f, 0.4f)));
}

static Hittable *random_bvh(int n, uint64_t seed, float spread) {
  PCG32 rng;
  pcg32_seed(&rng, seed, 7u);
  Hittable *list = HittableList_new((size_t)n);
  for (int k = 0; k < n; k++) {
    const float x = pcg32_f32_between(&rng, -spread, spread);
    const float z = pcg32_f32_between(&rng, -spread - 2.0f, spread - 2.0f);
    const float r = pcg32_f32_between(&rng, 0.08f, 0.25f);
    const float pick = pcg32_f32(&rng);
    Material *m;
    if (pick < 0.6f) {
      const float g = pcg32_f32(&rng);
      m = lamb(0.2f + 0.6f * g, 0.5f, 0.9f - 0.6f * g);
    } else if (pick < 0.85f) {
      m = Metal_new(Solid_new(vec3(0.8f, 0.8f, 0.7f)), pcg32_f32(&rng));
    } else {
      m = Dielectric_new(1.5f);
    }
    HittableList_append((HittableList *)list, Sphere_new(vec3(x, r - 0.5f, z), r, m));
  }
  return BVHNode_new((HittableList *)list, &rng);
}

static void world_one_px_wide(World *w, Camera *c) {
  camera_defaults(c, 1, 1.0f / 48.0f, 64, 50);
  c->vfov = 60.0f;
  ground(w);
  add(w, random_bvh(40, 11u, 1.5f));
}

static void world_flat_list(World *w, Camera *c) {
  camera_defaults(c, 96, 16.0f / 9.0f, 64, 50);
  ground(w);
  PCG32 rng;
  pcg32_seed(&rng, 5u, 3u);
  for (int k = 0; k < 120; k++) {
    const float x = pcg32_f32_between(&rng, -2.5f, 2.5f);
    const float z = pcg32_f32_between(&rng, -4.0f, -0.5f);
    const float r = pcg32_f32_between(&rng, 0.05f, 0.2f);
    const float pick = pcg32_f32(&rng);
    Material *m = pick < 0.5f ? lamb(0.3f, 0.6f, 0.3f)
                  : pick < 0.8f ? Metal_new(Solid_new(vec3(0.9f, 0.8f, 0.8f)), 0.3f * pick)
                                : Dielectric_new(1.5f);
    add(w, Sphere_new(vec3(x, r - 0.5f, z), r, m));
  }
}

static void world_bvh_depth100(World *w, Camera *c) {
  camera_defaults(c, 96, 16.0f / 9.0f, 32, 100);
  ground(w);
  add(w, random_bvh(60, 23u, 2.0f));
  add(w, Sphere_new(vec3(0.0f, 0.1f, -1.5f), 0.6f, Dielectric_new(1.5f)));
}

static void world_big_bvh(World *w, Camera *c, int spp) {
  camera_defaults(c, 96, 16.0f / 9.0f, spp, 50);
  c->look_from = vec3(0.0f, 1.2f, 3.0f);
  c->look_to = vec3(0.0f, 0.0f, -2.0f);
  ground(w);
  add(w, random_bvh(1100, 31u, 5.0f));
}

static void world_many_boxes(World *w, Camera *c) {
  camera_defaults(c, 64, 1.0f, 64, 20);
  c->background = vec3(0.05f, 0.05f, 0.08f);
  c->vfov = 45.0f;
  c->look_from = vec3(0.0f, 7.0f, 9.0f);
  c->look_to = vec3(0.0f, 0.0f, 0.0f);
  PCG32 rng;
  pcg32_seed(&rng, 41u, 9u);
  Hittable *boxes = HittableList_new(1000);
  Material *grey = lamb(0.6f, 0.6f, 0.55f), *blue = lamb(0.2f, 0.3f, 0.7f);
  for (int k = 0; k < 1000; k++) {
    const float x = pcg32_f32_between(&rng, -6.0f, 6.0f);
    const float z = pcg32_f32_between(&rng, -6.0f, 6.0f);
    const float s = pcg32_f32_between(&rng, 0.1f, 0.35f);
    const float h = pcg32_f32_between(&rng, 0.1f, 1.2f);
    HittableList_append((HittableList *)boxes, Box_new(vec3(x, 0.0f, z), vec3(x + s, h, z + s), k % 3 ? grey : blue));
  }
  add(w, BVHNode_new((HittableList *)boxes, &rng));
  add(w, Quad_new(vec3(-8.0f, 0.0f, -8.0f), vec3(16.0f, 0.0f, 0.0f), vec3(0.0f, 0.0f, 16.0f), lamb(0.4f, 0.45f, 0.3f)));
  Material *light = DiffuseLight_new(Solid_new(vec3(8.0f, 8.0f, 7.0f)));
  Hittable *panel = Quad_new(vec3(-1.5f, 5.0f, -1.5f), vec3(3.0f, 0.0f, 0.0f), vec3(0.0f, 0.0f, 3.0f), light);
  add(w, panel);
  HittableList_append(&w->lights, panel);
}

static int render_world(int id, const char *path) {
  World world;
  World_init(&world, 256);
  Camera camera;
  switch (id) {
    case 0: world_surface_normal(&world, &camera); break;
    case 1: world_hollow_glass(&world, &camera); break;
    case 2: world_metal_fuzz(&world, &camera); break;
    case 3: world_quads_xform(&world, &camera); break;
    case 4: world_deep_mirror(&world, &camera); break;
    case 5: world_one_px_wide(&world, &camera); break;
    case 6: world_flat_list(&world, &camera); break;
    case 7: world_bvh_depth100(&world, &camera); break;
    case 8: world_big_bvh(&world, &camera, 64); break;
    case 9: world_big_bvh(&world, &camera, 16); break;
    case 10: world_many_boxes(&world, &camera); break;
    default: fprintf(stderr, "unknown world\n"); return 2;
  }
  Camera_init(&camera);
  const size_t n = (size_t)camera.img_width * camera.img_height * 3;
  uint8_t *img = malloc(n);
  Camera_render(&camera, &world, img);
  report_kernel(&camera, &world);
  FILE *f = fopen(path, "wb");
  if (!f || fwrite(img, 1, n, f) != n) {
    fprintf(stderr, "cannot write %s\n", path);
    return 1;
  }
  fclose(f);
  free(img);
  printf("%d %d\n", camera.img_width, camera.img_height);
  return 0;
}

/* usage: api_worlds <id> <out.rgb>
 *        api_worlds seq <out_prefix> <id> <id> ...   several worlds, each built afresh and rendered by
 *        Camera_render in this one process, into <out_prefix>_<k>.rgb (k = position in the list): a
 *        repeated world reuses the drop-in library's cached device scene, a different one replaces it */
int main(int argc, char **argv) {
  if (argc < 3) {
    fprintf(stderr, "usage: %s <world 0-10> <out.rgb> | seq <out_prefix> <world> ...\n", argv[0]);
    return 2;
  }
  if (argv[1][0] == 's') {
    char path[4096];
    for (int k = 3; k < argc; k++) {
      snprintf(path, sizeof path, "%s_%d.rgb", argv[2], k - 3);
      const int rc = render_world(atoi(argv[k]), path);
      if (rc) return rc;
    }
    return 0;
  }
  return render_world(atoi(argv[1]), argv[2]);
}
