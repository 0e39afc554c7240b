/* ref_harness.c — TEST INFRASTRUCTURE (oracle).  Never linked into the product.
 *
 * Driver for the reference build in oracle/_ref/: links the reference's own sources (compiled
 * where they lie under /root/reference, src/main.c with -Dmain=ref_main so its scene builders are
 * callable) and exposes what main() cannot: width/spp/depth control, raw RGB output, the pcg32
 * known answers and a canonical dump of the scene graph the reference builds.
 *
 *   ref_render render <scene> <width> <spp> <depth> <out.rgb>   (prints "W H" on stdout)
 *   ref_render kat
 *   ref_render dump <scene>
 * Camera defaults replicate reference src/main.c:278-287.  Scenes 3 and 7 read earthmap.jpg from the
 * current directory, as the reference does (run from a directory holding rtc/earth.py's picture).
 */
#define _POSIX_C_SOURCE 200809L /* access() under -std=c11 */
#include "hittable.h"
#include "material.h"
#include "raytracing.h"
#include "texture.h"
#include "tiff.h"
#include "utils.h"

#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <unistd.h>

void scene_metal_and_lambertian(World *world, Camera *camera);
void scene_book1_final(World *world, Camera *camera);
void scene_checker(World *world, Camera *camera);
void scene_earth(World *world, Camera *camera);
void scene_perlin(World *world, Camera *camera);
void scene_simple_light(World *world, Camera *camera);
void scene_cornell_box(World *world, Camera *camera);
void scene_book2_final(World *world, Camera *camera, bool enable_bvh);

static void defaults(Camera *c) {
  memset(c, 0, sizeof *c);
  c->aspect_ratio = 16.0f / 9.0f;
  c->img_width = 500;
  c->samples_per_pixel = 100;
  c->max_depth = 50;
  c->vup = vec3(0, 1, 0);
  c->dof_angle = 0.0f;
  c->focal_length = 10.0f;
  c->lights_sampling_prob = 0.5f;
}

static void build(int id, World *w, Camera *c) {
  switch (id) {
  case 1: scene_book1_final(w, c); break;
  case 2: scene_checker(w, c); break;
  case 3: scene_earth(w, c); break;
  case 4: scene_perlin(w, c); break;
  case 5: scene_simple_light(w, c); break;
  case 6: scene_cornell_box(w, c); break;
  case 7: scene_book2_final(w, c, true); break;
  default: scene_metal_and_lambertian(w, c); break;
  }
}

/* ---------------------------------------------------------------- canonical scene dump */
static HittableVTable *VT_LIST, *VT_SPHERE, *VT_QUAD, *VT_BVH, *VT_TRANSLATE, *VT_ROTATE, *VT_MEDIUM;
static void *TX_SOLID, *TX_CHECKER, *TX_IMAGE, *TX_PERLIN;

static void learn_kinds(void) {
  Material *m = Lambertian_new(Solid_new(vec3(0, 0, 0)));
  Hittable *s = Sphere_new(vec3(0, 0, 0), 1, m);
  HittableList *l = (HittableList *)HittableList_new(1);
  HittableList_append(l, s);
  PCG32 g;
  pcg32_seed(&g, 1, 1);
  VT_LIST = l->hittable.vtable;
  VT_SPHERE = s->vtable;
  VT_QUAD = Quad_new(vec3(0, 0, 0), vec3(1, 0, 0), vec3(0, 1, 0), m)->vtable;
  VT_BVH = BVHNode_new(l, &g)->vtable;
  VT_TRANSLATE = Translate_new(s, vec3(0, 0, 0))->vtable;
  VT_ROTATE = RotateY_new(s, 0)->vtable;
  VT_MEDIUM = ConstantMedium_new(s, 1, Solid_new(vec3(0, 0, 0)))->vtable;
  TX_SOLID = (void *)Solid_new(vec3(0, 0, 0))->value;
  TX_CHECKER = (void *)Checker_new(1, m->albedo, m->albedo)->value;
  /* the reference's Image_init asserts on an unreadable file (src/texture.c:38-42): learn the image
   * kind only when the scene's picture is present (scenes 3 and 7 need it anyway) */
  TX_IMAGE = access("earthmap.jpg", R_OK) == 0 ? (void *)Image_new("earthmap.jpg")->value : NULL;
  PCG32 g2;
  pcg32_seed(&g2, 1, 1);
  TX_PERLIN = (void *)Perlin_new(1, 1, &g2)->value;
}

static void dump_texture(const Texture *t) {
  if (!t) {
    printf(" tex=none");
    return;
  }
  if ((void *)t->value == TX_SOLID) {
    const Solid *s = (const Solid *)t;
    printf(" solid(%a %a %a)", s->color.x, s->color.y, s->color.z);
  } else if ((void *)t->value == TX_CHECKER) {
    const Checker *c = (const Checker *)t;
    printf(" checker(%a", c->scale);
    dump_texture(c->even);
    dump_texture(c->odd);
    printf(")");
  } else if ((void *)t->value == TX_IMAGE) {
    const Image *im = (const Image *)t;
    unsigned long long h = 1469598103934665603ULL;
    for (long i = 0; i < (long)im->width * im->height * 3; i++) h = (h ^ im->buffer[i]) * 1099511628211ULL;
    printf(" image(%d %d %016llx)", im->width, im->height, h);
  } else if ((void *)t->value == TX_PERLIN) {
    const Perlin *p = (const Perlin *)t;
    unsigned long long h = 1469598103934665603ULL;
    for (int i = 0; i < N_PERLIN; i++) {
      unsigned int v[6];
      memcpy(v, &p->grad_field[i], 12);
      v[3] = (unsigned)p->perm_x[i];
      v[4] = (unsigned)p->perm_y[i];
      v[5] = (unsigned)p->perm_z[i];
      for (int k = 0; k < 6; k++) h = (h ^ v[k]) * 1099511628211ULL;
    }
    printf(" perlin(%a %d %016llx)", p->scale, p->depth, h);
  } else {
    printf(" tex=?");
  }
}

static void dump_material(const Material *m) {
  printf(" mat(%d %a", (int)m->tag, m->fuzz);
  if (m->tag != DIELECTRIC && m->tag != SURFACE_NORMAL) dump_texture(m->albedo);
  printf(")");
}

static void dump(const Hittable *h, int depth) {
  printf("%*s", depth, "");
  const AABB *b = &h->bbox;
  if (h->vtable == VT_LIST) {
    const HittableList *l = (const HittableList *)h;
    printf("LIST %zu\n", l->size);
    for (size_t i = 0; i < l->size; i++) dump(l->items[i], depth + 1);
  } else if (h->vtable == VT_BVH) {
    const BVHNode *n = (const BVHNode *)h;
    printf("BVH %a %a %a %a %a %a%s\n", b->x[0], b->y[0], b->z[0], b->x[1], b->y[1], b->z[1],
           n->left == n->right ? " dup" : "");
    dump(n->left, depth + 1);
    if (n->right != n->left) dump(n->right, depth + 1);
  } else if (h->vtable == VT_SPHERE) {
    const Sphere *s = (const Sphere *)h;
    printf("SPHERE %a %a %a %a", s->center.x, s->center.y, s->center.z, s->radius);
    dump_material(s->material);
    printf("\n");
  } else if (h->vtable == VT_QUAD) {
    const Quad *q = (const Quad *)h;
    printf("QUAD %a %a %a %a %a %a %a %a %a %a %a %a %a %a %a %a %a", q->Q.x, q->Q.y, q->Q.z, q->u.x, q->u.y, q->u.z,
           q->v.x, q->v.y, q->v.z, q->normal.x, q->normal.y, q->normal.z, q->D, q->w.x, q->w.y, q->w.z, q->area);
    dump_material(q->material);
    printf("\n");
  } else if (h->vtable == VT_TRANSLATE) {
    const Translate *t = (const Translate *)h;
    printf("TRANSLATE %a %a %a\n", t->offset.x, t->offset.y, t->offset.z);
    dump(t->object, depth + 1);
  } else if (h->vtable == VT_ROTATE) {
    const RotateY *r = (const RotateY *)h;
    printf("ROTATE %a %a\n", r->sin_theta, r->cos_theta);
    dump(r->object, depth + 1);
  } else if (h->vtable == VT_MEDIUM) {
    const ConstantMedium *m = (const ConstantMedium *)h;
    printf("MEDIUM %a", m->neg_inv_density);
    dump_material(m->phase_fn);
    printf("\n");
    dump(m->boundary, depth + 1);
  } else {
    printf("UNKNOWN\n");
  }
}

int main(int argc, char **argv) {
  if (argc >= 2 && strcmp(argv[1], "kat") == 0) {
    const unsigned long long seeds[3][2] = {{17, 23}, {691, 1222}, {19, 29}};
    for (int s = 0; s < 3; s++) {
      PCG32 g;
      pcg32_seed(&g, seeds[s][0], seeds[s][1]);
      printf("seed %llu %llu state %016llx inc %016llx u32", seeds[s][0], seeds[s][1],
             (unsigned long long)g.state, (unsigned long long)g.inc);
      for (int k = 0; k < 8; k++) printf(" %08x", pcg32_u32(&g));
      printf("\n");
    }
    PCG32 g;
    pcg32_seed(&g, 19, 29);
    Vec3 r = vec3_rand(&g);
    printf("vec3_rand(seed 19 29) %a %a %a\n", r.x, r.y, r.z);
    Vec3 u = vec3_rand_unit_vector(&g);
    printf("vec3_rand_unit_vector(next) %a %a %a\n", u.x, u.y, u.z);
    printf("f32_between(next,-1,1) %a\n", pcg32_f32_between(&g, -1.0f, 1.0f));
    printf("u32_between(next,0,3) %u\n", pcg32_u32_between(&g, 0, 3));
    return 0;
  }
  if (argc >= 3 && strcmp(argv[1], "dump") == 0) {
    learn_kinds();
    World w = {0};
    Camera c;
    defaults(&c);
    build(atoi(argv[2]), &w, &c);
    Camera_init(&c);
    printf("CAMERA %d %d %a %a %a | %a %a %a | %a %a %a | %a %a %a | %a %a %a | %a %a %a | %a %a %a %a\n",
           c.img_width, c.img_height, c.pixel00_loc.x, c.pixel00_loc.y, c.pixel00_loc.z, c.pixel_delta_u.x,
           c.pixel_delta_u.y, c.pixel_delta_u.z, c.pixel_delta_v.x, c.pixel_delta_v.y, c.pixel_delta_v.z,
           c.look_from.x, c.look_from.y, c.look_from.z, c.dof_disc_u.x, c.dof_disc_u.y, c.dof_disc_u.z,
           c.dof_disc_v.x, c.dof_disc_v.y, c.dof_disc_v.z, c.background.x, c.background.y, c.background.z,
           c.dof_angle);
    dump(&w.objects.hittable, 0);
    printf("LIGHTS %zu\n", w.lights.size);
    for (size_t i = 0; i < w.lights.size; i++) dump(w.lights.items[i], 1);
    return 0;
  }
  if (argc >= 7 && strcmp(argv[1], "render") == 0) {
    World w = {0};
    Camera c;
    defaults(&c);
    c.img_width = atoi(argv[3]);
    c.samples_per_pixel = atoi(argv[4]);
    build(atoi(argv[2]), &w, &c);
    c.max_depth = atoi(argv[5]);
    Camera_init(&c);
    uint8_t *img = my_malloc((size_t)c.img_width * c.img_height * 3);
    Camera_render(&c, &w, img);
    FILE *f = strcmp(argv[6], "-") ? fopen(argv[6], "wb") : stdout;
    if (!f) return 2;
    if (strstr(argv[6], ".tiff"))
      write_tiff(f, c.img_width, c.img_height, 3, img);
    else
      fwrite(img, 1, (size_t)c.img_width * c.img_height * 3, f);
    if (f != stdout) fclose(f);
    fprintf(stdout == f ? stderr : stdout, "%d %d\n", c.img_width, c.img_height);
    return 0;
  }
  fprintf(stderr, "usage: ref_render render <scene> <width> <spp> <depth> <out> | kat | dump <scene>\n");
  return 1;
}
