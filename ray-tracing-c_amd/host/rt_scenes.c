/* rt_scenes.c — the reference driver's eight scenes (reference src/main.c:9-273) and its camera
 * defaults (src/main.c:278-287), built through the drop-in API.
 *
 * Where a reference expression makes several rng draws inside one argument list, the draws are
 * sequenced here in the order gcc evaluates them (right-to-left), so these scenes equal the ones a
 * gcc-built reference renders.  Component-wise products of two vec3_rand() results
 * are order-independent and need no sequencing.
 */
#include "rt_internal.h"

#include <stdio.h>

void rt_camera_defaults(Camera *camera) {
  camera->aspect_ratio = 16.0f / 9.0f;
  camera->img_width = 500;
  camera->samples_per_pixel = 100;
  camera->max_depth = 50;
  camera->vup = vec3(0, 1, 0);
  camera->dof_angle = 0.0f;
  camera->focal_length = 10.0f;
  camera->lights_sampling_prob = 0.5f;
}

static void look(Camera *c, float vfov, Vec3 background, Vec3 from, Vec3 to) {
  c->vfov = vfov;
  c->background = background;
  c->look_from = from;
  c->look_to = to;
}

/* scene 0 — src/main.c:9-30 */
void scene_metal_and_lambertian(World *world, Camera *camera) {
  World_init(world, 4);
  HittableList *objs = &world->objects;
  HittableList_append(objs, Sphere_new(vec3(0, -100.5, -1), 100, Lambertian_new(Solid_new(vec3(0.8, 0.8, 0.0)))));
  HittableList_append(objs, Sphere_new(vec3(0, 0, -1), 0.5, Lambertian_new(Solid_new(vec3(0.7, 0.3, 0.3)))));
  HittableList_append(objs, Sphere_new(vec3(-1, 0, -1), 0.5, Metal_new(Solid_new(vec3(0.8, 0.8, 0.8)), 0.3)));
  HittableList_append(objs, Sphere_new(vec3(1, 0, -1), 0.5, Metal_new(Solid_new(vec3(0.8, 0.6, 0.2)), 1.0)));
  look(camera, 90.0f, vec3(0.7, 0.8, 1), VEC3_ZERO, vec3(0, 0, -1));
}

/* scene 1 — src/main.c:32-85: 4 large spheres + up to 22x22 random small ones, one BVH */
void scene_book1_final(World *world, Camera *camera) {
  World_init(world, 4 + 22 * 22);
  HittableList *objs = &world->objects;
  HittableList_append(objs, Sphere_new(vec3(0, -1000, -1), 1000, Lambertian_new(Solid_new(vec3(0.5, 0.5, 0.5)))));
  HittableList_append(objs, Sphere_new(vec3(0, 1, 0), 1, Dielectric_new(1.5)));
  HittableList_append(objs, Sphere_new(vec3(-4, 1, 0), 1, Lambertian_new(Solid_new(vec3(0.4, 0.2, 0.1)))));
  HittableList_append(objs, Sphere_new(vec3(4, 1, 0), 1, Metal_new(Solid_new(vec3(0.7, 0.6, 0.5)), 0)));

  PCG32 rng;
  pcg32_seed(&rng, 19, 29);
  const Vec3 keep_clear = vec3(4, 0.2, 0);
  const float r = 0.2f;
  for (int a = -11; a < 11; a++) {
    for (int b = -11; b < 11; b++) {
      const float pick = pcg32_f32(&rng);
      const float jitter_z = pcg32_f32(&rng); /* gcc evaluates the z argument first */
      const float jitter_x = pcg32_f32(&rng);
      const Vec3 c = vec3((float)a + 0.9f * jitter_x, r, (float)b + 0.9f * jitter_z);
      if (!(vec3_length(vec3_sub_vec3(c, keep_clear)) > 0.9f)) continue;
      Material *m;
      if (pick < 0.8f) {
        const Vec3 k1 = vec3_rand(&rng);
        const Vec3 k2 = vec3_rand(&rng);
        m = Lambertian_new(Solid_new(vec3_mul_vec3(k2, k1)));
      } else if (pick < 0.95f) {
        const Vec3 albedo = vec3_rand_between(&rng, 0.5f, 1);
        m = Metal_new(Solid_new(albedo), pcg32_f32(&rng) * 0.5f);
      } else {
        m = Dielectric_new(1.5f);
      }
      HittableList_append(objs, Sphere_new(c, r, m));
    }
  }

  Hittable *bvh = BVHNode_new(objs, &rng);
  free(objs->items);
  HittableList_init(objs, 1);
  HittableList_append(objs, bvh);

  look(camera, 20.0f, vec3(0.7, 0.8, 1), vec3(13, 2, 3), VEC3_ZERO);
  camera->dof_angle = 0.6f;
}

/* scene 2 — src/main.c:87-99 */
void scene_checker(World *world, Camera *camera) {
  World_init(world, 2);
  Texture *chk = Checker_new(0.01f, Solid_new(vec3(0.2, 0.3, 0.1)), Solid_new(vec3(0.9, 0.9, 0.9)));
  Material *m = Lambertian_new(chk);
  HittableList_append(&world->objects, Sphere_new(vec3(0, -10, 0), 10, m));
  HittableList_append(&world->objects, Sphere_new(vec3(0, 10, 0), 10, m));
  look(camera, 20.0f, vec3(0.7, 0.8, 1), vec3(13, 2, 3), VEC3_ZERO);
}

/* scene 3 — src/main.c:101-111 */
void scene_earth(World *world, Camera *camera) {
  World_init(world, 1);
  HittableList_append(&world->objects, Sphere_new(VEC3_ZERO, 2, Lambertian_new(Image_new("earthmap.jpg"))));
  look(camera, 20.0f, vec3(0.7, 0.8, 1), vec3(13, 2, 3), VEC3_ZERO);
}

/* scene 4 — src/main.c:113-129 */
void scene_perlin(World *world, Camera *camera) {
  World_init(world, 2);
  PCG32 rng;
  pcg32_seed(&rng, 19, 29);
  Material *m = Lambertian_new(Perlin_new(4.0f, 7, &rng));
  HittableList_append(&world->objects, Sphere_new(vec3(0, -1000, 0), 1000, m));
  HittableList_append(&world->objects, Sphere_new(vec3(0, 2, 0), 2, m));
  look(camera, 20.0f, vec3(0.7, 0.8, 1), vec3(13, 2, 3), VEC3_ZERO);
  camera->dof_angle = 0.0f;
  camera->focal_length = 10.0f;
}

/* scene 5 — src/main.c:131-155 */
void scene_simple_light(World *world, Camera *camera) {
  World_init(world, 4);
  PCG32 rng;
  pcg32_seed(&rng, 19, 29);
  Material *marble = Lambertian_new(Perlin_new(4.0f, 7, &rng));
  Material *lamp = DiffuseLight_new(Solid_new(vec3(4, 4, 4)));
  HittableList_append(&world->objects, Sphere_new(vec3(0, -1000, 0), 1000, marble));
  HittableList_append(&world->objects, Sphere_new(vec3(0, 2, 0), 2, marble));
  Hittable *panel = Quad_new(vec3(3, 1, -2), vec3(2, 0, 0), vec3(0, 2, 0), lamp);
  HittableList_append(&world->objects, panel);
  HittableList_append(&world->lights, panel);
  Hittable *bulb = Sphere_new(vec3(0, 7, 0), 2, lamp);
  HittableList_append(&world->objects, bulb);
  HittableList_append(&world->lights, bulb);
  look(camera, 20.0f, VEC3_ZERO, vec3(26, 3, 6), vec3(0, 2, 0));
}

/* scene 6 — src/main.c:157-190 */
void scene_cornell_box(World *world, Camera *camera) {
  World_init(world, 6 + 2);
  Material *red = Lambertian_new(Solid_new(vec3(0.65, 0.05, 0.05)));
  Material *white = Lambertian_new(Solid_new(vec3(0.73, 0.73, 0.73)));
  Material *green = Lambertian_new(Solid_new(vec3(0.12, 0.45, 0.15)));
  Material *lamp = DiffuseLight_new(Solid_new(vec3(15, 15, 15)));
  HittableList *objs = &world->objects;
  HittableList_append(objs, Quad_new(vec3(555, 0, 0), vec3(0, 555, 0), vec3(0, 0, 555), green));
  HittableList_append(objs, Quad_new(vec3(0, 0, 0), vec3(0, 555, 0), vec3(0, 0, 555), red));
  HittableList_append(objs, Quad_new(vec3(0, 0, 0), vec3(555, 0, 0), vec3(0, 0, 555), white));
  HittableList_append(objs, Quad_new(vec3(555, 555, 555), vec3(-555, 0, 0), vec3(0, 0, -555), white));
  HittableList_append(objs, Quad_new(vec3(0, 0, 555), vec3(555, 0, 0), vec3(0, 555, 0), white));
  Hittable *panel = Quad_new(vec3(343, 554, 332), vec3(-130, 0, 0), vec3(0, 0, -105), lamp);
  HittableList_append(objs, panel);
  HittableList_append(&world->lights, panel);
  Hittable *tall = Translate_new(RotateY_new(Box_new(vec3(0, 0, 0), vec3(165, 330, 165), white), 15),
                                 vec3(265, 0, 295));
  HittableList_append(objs, tall);
  Hittable *shorty = Translate_new(RotateY_new(Box_new(vec3(0, 0, 0), vec3(165, 165, 165), white), -18),
                                   vec3(130, 0, 65));
  HittableList_append(objs, shorty);
  camera->aspect_ratio = 1.0f;
  look(camera, 40.0f, vec3(0, 0, 0), vec3(278, 278, -800), vec3(278, 278, 0));
}

/* scene 7 — src/main.c:192-273 */
void scene_book2_final(World *world, Camera *camera, bool enable_bvh) {
  World_init(world, 11);
  PCG32 rng;
  pcg32_seed(&rng, 19, 29);

  const int per_side = 20;
  Material *ground = Lambertian_new(Solid_new(vec3(0.48, 0.83, 0.53)));
  HittableList *floor_boxes = (HittableList *)HittableList_new(per_side * per_side);
  for (int i = 0; i < per_side; i++)
    for (int j = 0; j < per_side; j++) {
      const float w = 100.0f;
      const Vec3 p0 = vec3(-1000.0f + i * w, 0.0f, -1000.0f + j * w);
      const Vec3 p1 = vec3(-1000.0f + (i + 1) * w, pcg32_f32_between(&rng, 1, 101), -1000.0f + (j + 1) * w);
      HittableList_append(floor_boxes, Box_new(p0, p1, ground));
    }
  Hittable *floor_root = &floor_boxes->hittable;
  if (enable_bvh) {
    floor_root = BVHNode_new(floor_boxes, &rng);
    free(floor_boxes->items);
    free(floor_boxes);
  }
  HittableList_append(&world->objects, floor_root);

  Material *lamp = DiffuseLight_new(Solid_new(vec3(7, 7, 7)));
  Hittable *panel = Quad_new(vec3(123, 554, 147), vec3(300, 0, 0), vec3(0, 0, 265), lamp);
  HittableList_append(&world->objects, panel);
  HittableList_append(&world->lights, panel);

  HittableList_append(&world->objects, Sphere_new(vec3(400, 400, 200), 50, Lambertian_new(Solid_new(vec3(0.7, 0.3, 0.1)))));
  Material *glass = Dielectric_new(1.5);
  HittableList_append(&world->objects, Sphere_new(vec3(260, 150, 45), 50, glass));
  HittableList_append(&world->objects, Sphere_new(vec3(0, 150, 145), 50, Metal_new(Solid_new(vec3(0.8, 0.8, 0.9)), 1.0)));

  Hittable *bubble = Sphere_new(vec3(360, 150, 145), 70, glass); /* subsurface: glass shell + medium */
  HittableList_append(&world->objects, bubble);
  HittableList_append(&world->objects, ConstantMedium_new(bubble, 0.2, Solid_new(vec3(0.2, 0.4, 0.9))));
  Hittable *haze = Sphere_new(vec3(0, 0, 0), 5000, glass); /* mist */
  HittableList_append(&world->objects, ConstantMedium_new(haze, 0.0001, Solid_new(vec3(1, 1, 1))));

  HittableList_append(&world->objects, Sphere_new(vec3(400, 200, 400), 100, Lambertian_new(Image_new("earthmap.jpg"))));
  HittableList_append(&world->objects, Sphere_new(vec3(220, 280, 300), 80, Lambertian_new(Perlin_new(0.1, 7, &rng))));

  const int ns = 1000;
  Material *white = Lambertian_new(Solid_new(vec3(0.73, 0.73, 0.73)));
  HittableList *cluster = (HittableList *)HittableList_new(ns);
  for (int i = 0; i < ns; i++) HittableList_append(cluster, Sphere_new(vec3_rand_between(&rng, 0, 165), 10, white));
  Hittable *cluster_root = &cluster->hittable;
  if (enable_bvh) {
    cluster_root = BVHNode_new(cluster, &rng);
    free(cluster->items);
    free(cluster);
  }
  cluster_root = Translate_new(RotateY_new(cluster_root, 15.0f), vec3(-100, 270, 395));
  HittableList_append(&world->objects, cluster_root);

  camera->aspect_ratio = 1.0f;
  look(camera, 40.0f, VEC3_ZERO, vec3(478, 278, -600), vec3(278, 278, 0));
}

const char *rt_build_scene(int scene_id, World *world, Camera *camera) {
  switch (scene_id) {
  case 1: scene_book1_final(world, camera); return "Book 1: Final scene";
  case 2: scene_checker(world, camera); return "Book 2: Checker";
  case 3: scene_earth(world, camera); return "Book 2: Earth";
  case 4: scene_perlin(world, camera); return "Book 2: Perlin noise";
  case 5: scene_simple_light(world, camera); return "Book 2: Simple light";
  case 6: scene_cornell_box(world, camera); return "Book 2: Cornell box";
  case 7: scene_book2_final(world, camera, true); return "Book 2: Final scene";
  case 0: scene_metal_and_lambertian(world, camera); return "Book 1: Metal and Lambertian";
  default:
    fprintf(stderr, "Unsupported option. Default to 0\n");
    scene_metal_and_lambertian(world, camera);
    return "Book 1: Metal and Lambertian";
  }
}

rt_flat_scene *rt_scene_preset_in(int scene_id, int width, int spp, int max_depth, const char *image_dir) {
  World world = {0};
  Camera camera = {0};
  rt_camera_defaults(&camera);
  if (width > 0) camera.img_width = width;
  if (spp > 0) camera.samples_per_pixel = spp;
  rt_image_soft_begin(image_dir);
  (void)rt_build_scene(scene_id, &world, &camera);
  if (rt_image_soft_end()) return NULL; /* (rt_last_error() names the image) */
  if (max_depth > 0) camera.max_depth = max_depth;
  Camera_init(&camera);
  return rt_flatten(&camera, &world); /* the scene graph is leaked, as in the reference driver */
}

rt_flat_scene *rt_scene_preset(int scene_id, int width, int spp, int max_depth) {
  return rt_scene_preset_in(scene_id, width, spp, max_depth, NULL);
}
