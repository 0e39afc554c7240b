/* rt_flatten.c — World pointer graph -> rt_flat_scene (include/rt_flat.h).
 *
 * Walks the reference-layout object graph once per render.  Object kinds are recognised by the
 * identity of this library's vtables / texture entry points, shared objects are emitted once
 * (pointer memo), and every derived constant is evaluated the way the reference evaluates it at
 * its point of use so the GPU never re-derives one with different rounding.
 *
 * Validation is strict: anything the GPU path does not implement exactly (objects from another
 * library, a medium whose boundary is not a primitive, a light list item that is itself a list,
 * non-solid volume albedo) is reported through rt_last_error() and rt_flatten returns NULL.
 */
#define _POSIX_C_SOURCE 200809L
#include "rt_internal.h"

#include <math.h>
#include <stdarg.h>
#include <stdio.h>
#include <string.h>

/* ------------------------------------------------------------------ growable arrays */
typedef struct {
  void *data;
  int32_t count, cap;
  size_t elem;
} vec_t;

static int32_t vec_push(vec_t *v, const void *elem) {
  if (v->count == v->cap) {
    v->cap = v->cap ? 2 * v->cap : 16;
    void *p = realloc(v->data, (size_t)v->cap * v->elem);
    if (!p) abort();
    v->data = p;
  }
  memcpy((char *)v->data + (size_t)v->count * v->elem, elem, v->elem);
  return v->count++;
}
static void *vec_at(vec_t *v, int32_t i) { return (char *)v->data + (size_t)i * v->elem; }

/* ------------------------------------------------------------------ pointer memo */
typedef struct {
  const void **keys;
  int32_t *vals;
  size_t cap, used;
} memo_t;

static size_t memo_hash(const void *p, size_t cap) {
  uint64_t x = (uint64_t)(uintptr_t)p;
  x ^= x >> 33;
  x *= 0xff51afd7ed558ccdULL;
  x ^= x >> 33;
  return (size_t)(x & (cap - 1));
}
static int32_t *memo_slot(memo_t *m, const void *key, int create) {
  if (create && 2 * (m->used + 1) > m->cap) {
    memo_t n = {0};
    n.cap = m->cap ? 2 * m->cap : 1024;
    n.keys = calloc(n.cap, sizeof *n.keys);
    n.vals = calloc(n.cap, sizeof *n.vals);
    for (size_t i = 0; i < m->cap; i++)
      if (m->keys[i]) {
        size_t h = memo_hash(m->keys[i], n.cap);
        while (n.keys[h]) h = (h + 1) & (n.cap - 1);
        n.keys[h] = m->keys[i];
        n.vals[h] = m->vals[i];
        n.used++;
      }
    free(m->keys);
    free(m->vals);
    *m = n;
  }
  if (!m->cap) return NULL;
  size_t h = memo_hash(key, m->cap);
  while (m->keys[h] && m->keys[h] != key) h = (h + 1) & (m->cap - 1);
  if (m->keys[h]) return &m->vals[h];
  if (!create) return NULL;
  m->keys[h] = key;
  m->used++;
  return &m->vals[h];
}

/* ------------------------------------------------------------------ state */
typedef struct {
  vec_t bvh, spheres, quads, lists, items, translates, rotates, media, materials, textures, images, perlins, bytes;
  memo_t obj_memo, mat_memo, tex_memo;
  int32_t features;
  int failed;
} flat_ctx;

static void fail(flat_ctx *c, const char *fmt, ...) {
  char msg[512];
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(msg, sizeof msg, fmt, ap);
  va_end(ap);
  if (!c->failed) rt_set_error("rt_flatten: %s", msg);
  c->failed = 1;
}

static void v3(float dst[3], Vec3 s) {
  dst[0] = s.x;
  dst[1] = s.y;
  dst[2] = s.z;
}

/* ------------------------------------------------------------------ textures and materials */
static int32_t flat_texture(flat_ctx *c, const Texture *t) {
  if (t == NULL) {
    fail(c, "material without albedo texture");
    return -1;
  }
  int32_t *slot = memo_slot(&c->tex_memo, t, 0);
  if (slot) return *slot;
  rt_texture rec;
  memset(&rec, 0, sizeof rec);
  if (t->value == rt_tex_solid_value) {
    rec.kind = RT_TEX_SOLID;
    v3(rec.color, ((const Solid *)t)->color);
  } else if (t->value == rt_tex_checker_value) {
    const Checker *k = (const Checker *)t;
    rec.kind = RT_TEX_CHECKER;
    rec.scale = k->scale;
    rec.a = flat_texture(c, k->even);
    rec.b = flat_texture(c, k->odd);
    c->features |= RT_FEAT_TEX_UV;
  } else if (t->value == rt_tex_image_value) {
    const Image *im = (const Image *)t;
    if (!im->buffer || im->width <= 0 || im->height <= 0) {
      fail(c, "image texture without pixels");
      return -1;
    }
    rt_image desc = {im->width, im->height, c->bytes.count};
    const size_t n = (size_t)im->width * im->height * 3;
    for (size_t i = 0; i < n; i++) vec_push(&c->bytes, &im->buffer[i]);
    rec.kind = RT_TEX_IMAGE;
    rec.a = vec_push(&c->images, &desc);
    c->features |= RT_FEAT_TEX_UV;
  } else if (t->value == rt_tex_perlin_value) {
    const Perlin *p = (const Perlin *)t;
    rt_perlin pd;
    memset(&pd, 0, sizeof pd);
    for (int i = 0; i < N_PERLIN; i++) {
      v3(pd.grad[i], p->grad_field[i]);
      pd.perm_x[i] = p->perm_x[i];
      pd.perm_y[i] = p->perm_y[i];
      pd.perm_z[i] = p->perm_z[i];
    }
    pd.depth = p->depth;
    rec.kind = RT_TEX_PERLIN;
    rec.scale = p->scale;
    rec.a = vec_push(&c->perlins, &pd);
    c->features |= RT_FEAT_TEX_PERLIN;
  } else {
    fail(c, "texture %p has an unknown value() function (not created by this library)", (const void *)t);
    return -1;
  }
  const int32_t id = vec_push(&c->textures, &rec);
  *memo_slot(&c->tex_memo, t, 1) = id;
  return id;
}

static int32_t flat_material(flat_ctx *c, const Material *m) {
  if (m == NULL) {
    fail(c, "primitive without material");
    return -1;
  }
  int32_t *slot = memo_slot(&c->mat_memo, m, 0);
  if (slot) return *slot;
  rt_material rec;
  memset(&rec, 0, sizeof rec);
  rec.tag = (int32_t)m->tag;
  rec.texture = -1;
  switch (m->tag) {
  case LAMBERTIAN:
  case DIFFUSE_LIGHT:
  case ISOTROPIC:
    rec.texture = flat_texture(c, m->albedo);
    break;
  case METAL:
    rec.texture = flat_texture(c, m->albedo);
    rec.param = m->fuzz;
    break;
  case DIELECTRIC:
    rec.param = m->eta;
    break;
  case SURFACE_NORMAL:
    break;
  default:
    fail(c, "unknown material tag %d", (int)m->tag);
    return -1;
  }
  if (m->tag == DIFFUSE_LIGHT || m->tag == SURFACE_NORMAL) c->features |= RT_FEAT_EMISSIVE;
  const int32_t id = vec_push(&c->materials, &rec);
  *memo_slot(&c->mat_memo, m, 1) = id;
  return id;
}

/* ------------------------------------------------------------------ hittables */
static int rng_free(flat_ctx *c, int32_t ref);

static int32_t flat_object(flat_ctx *c, const Hittable *h, int32_t parent_xform);

static int32_t flat_list_items(flat_ctx *c, Hittable *const *items, size_t n, int32_t parent_xform) {
  int32_t *tmp = my_malloc(sizeof(int32_t) * (n ? n : 1));
  for (size_t i = 0; i < n; i++) tmp[i] = flat_object(c, items[i], parent_xform);
  rt_list l = {c->items.count, (int32_t)n};
  for (size_t i = 0; i < n; i++) vec_push(&c->items, &tmp[i]);
  free(tmp);
  return vec_push(&c->lists, &l);
}

static int32_t flat_object(flat_ctx *c, const Hittable *h, int32_t parent_xform) {
  if (c->failed) return RT_REF_NONE;
  if (h == NULL || h->vtable == NULL) {
    fail(c, "NULL object in the scene graph");
    return RT_REF_NONE;
  }
  int32_t *slot = memo_slot(&c->obj_memo, h, 0);
  if (slot) {
    const int k = rt_ref_kind(*slot);
    if ((k == RT_KIND_TRANSLATE || k == RT_KIND_ROTATE_Y || k == RT_KIND_MEDIUM) && parent_xform != RT_REF_NONE)
      fail(c, "a transform/medium object is shared under a transform (unsupported)");
    return *slot;
  }
  const HittableVTable *vt = h->vtable;
  int32_t ref = RT_REF_NONE;
  if (vt == &rt_vt_sphere) {
    const Sphere *s = (const Sphere *)h;
    rt_sphere rec;
    memset(&rec, 0, sizeof rec);
    v3(rec.center, s->center);
    rec.radius = s->radius;
    rec.radius_sq = s->radius * s->radius;
    rec.inv_radius = 1.0f / s->radius;
    rec.material = flat_material(c, s->material);
    ref = rt_ref(RT_KIND_SPHERE, vec_push(&c->spheres, &rec));
  } else if (vt == &rt_vt_quad) {
    const Quad *q = (const Quad *)h;
    rt_quad rec;
    memset(&rec, 0, sizeof rec);
    v3(rec.Q, q->Q);
    v3(rec.u, q->u);
    v3(rec.v, q->v);
    v3(rec.normal, q->normal);
    v3(rec.w, q->w);
    rec.D = q->D;
    rec.area = q->area;
    rec.material = flat_material(c, q->material);
    c->features |= RT_FEAT_QUAD;
    ref = rt_ref(RT_KIND_QUAD, vec_push(&c->quads, &rec));
  } else if (vt == &rt_vt_list) {
    const HittableList *l = (const HittableList *)h;
    ref = rt_ref(RT_KIND_LIST, flat_list_items(c, l->items, l->size, parent_xform));
  } else if (vt == &rt_vt_bvh) {
    const BVHNode *b = (const BVHNode *)h;
    rt_bvh_node rec;
    memset(&rec, 0, sizeof rec);
    for (int a = 0; a < 3; a++) {
      rec.lo[a] = b->hittable.bbox.values[a][0];
      rec.hi[a] = b->hittable.bbox.values[a][1];
    }
    const int32_t idx = vec_push(&c->bvh, &rec);
    const int32_t l = flat_object(c, b->left, parent_xform);
    int32_t r = (b->right == b->left) ? RT_REF_NONE : flat_object(c, b->right, parent_xform);
    /* the reference visits a duplicated n==1 leaf twice; only an rng-consuming child can notice */
    if (b->right == b->left && !rng_free(c, l)) r = l;
    rt_bvh_node *dst = vec_at(&c->bvh, idx);
    dst->left = l;
    dst->right = r;
    c->features |= RT_FEAT_BVH;
    ref = rt_ref(RT_KIND_BVH, idx);
  } else if (vt == &rt_vt_translate) {
    const Translate *t = (const Translate *)h;
    rt_translate rec;
    memset(&rec, 0, sizeof rec);
    v3(rec.offset, t->offset);
    rec.parent_xform = parent_xform;
    const int32_t idx = vec_push(&c->translates, &rec);
    ref = rt_ref(RT_KIND_TRANSLATE, idx);
    const int32_t child = flat_object(c, t->object, ref);
    ((rt_translate *)vec_at(&c->translates, idx))->child = child;
    c->features |= RT_FEAT_XFORM;
  } else if (vt == &rt_vt_rotate_y) {
    const RotateY *rot = (const RotateY *)h;
    rt_rotate_y rec;
    memset(&rec, 0, sizeof rec);
    rec.sin_theta = rot->sin_theta;
    rec.cos_theta = rot->cos_theta;
    rec.parent_xform = parent_xform;
    const int32_t idx = vec_push(&c->rotates, &rec);
    ref = rt_ref(RT_KIND_ROTATE_Y, idx);
    const int32_t child = flat_object(c, rot->object, ref);
    ((rt_rotate_y *)vec_at(&c->rotates, idx))->child = child;
    c->features |= RT_FEAT_XFORM;
  } else if (vt == &rt_vt_medium) {
    const ConstantMedium *m = (const ConstantMedium *)h;
    rt_medium rec;
    memset(&rec, 0, sizeof rec);
    rec.boundary = flat_object(c, m->boundary, parent_xform);
    const int bk = rt_ref_kind(rec.boundary);
    if (!c->failed && bk != RT_KIND_SPHERE && bk != RT_KIND_QUAD)
      fail(c, "ConstantMedium boundary must be a Sphere or Quad on the GPU path");
    rec.neg_inv_density = m->neg_inv_density;
    rec.phase_material = flat_material(c, m->phase_fn);
    rec.parent_xform = parent_xform;
    if (!c->failed) {
      const rt_material *pm = vec_at(&c->materials, rec.phase_material);
      const rt_texture *pt = pm->texture >= 0 ? vec_at(&c->textures, pm->texture) : NULL;
      /* the reference leaves normal/front_face/u/v of a medium hit stale (src/hittable.c:418);
       * only an Isotropic phase with a solid albedo is independent of them */
      if (pm->tag != RT_MAT_ISOTROPIC || pt == NULL || pt->kind != RT_TEX_SOLID)
        fail(c, "ConstantMedium phase function must be Isotropic with a Solid albedo");
    }
    c->features |= RT_FEAT_MEDIUM;
    ref = rt_ref(RT_KIND_MEDIUM, vec_push(&c->media, &rec));
  } else {
    fail(c, "object %p has an unknown vtable (not created by this library)", (const void *)h);
    return RT_REF_NONE;
  }
  *memo_slot(&c->obj_memo, h, 1) = ref;
  return ref;
}

/* does traversing `ref` ever draw from the rng? (only constant media do) */
static int rng_free(flat_ctx *c, int32_t ref) {
  if (ref == RT_REF_NONE) return 1;
  const int32_t i = rt_ref_index(ref);
  switch (rt_ref_kind(ref)) {
  case RT_KIND_MEDIUM: return 0;
  case RT_KIND_SPHERE:
  case RT_KIND_QUAD: return 1;
  case RT_KIND_BVH: {
    const rt_bvh_node *b = vec_at(&c->bvh, i);
    return rng_free(c, b->left) && rng_free(c, b->right);
  }
  case RT_KIND_LIST: {
    const rt_list *l = vec_at(&c->lists, i);
    for (int32_t k = 0; k < l->count; k++)
      if (!rng_free(c, *(int32_t *)vec_at(&c->items, l->first + k))) return 0;
    return 1;
  }
  case RT_KIND_TRANSLATE: return rng_free(c, ((rt_translate *)vec_at(&c->translates, i))->child);
  case RT_KIND_ROTATE_Y: return rng_free(c, ((rt_rotate_y *)vec_at(&c->rotates, i))->child);
  }
  return 0;
}

/* Stack slots the device DFS needs for `ref` (mirrors rt_kernel.hip: rt_trace's push order). */
static int stack_need(flat_ctx *c, int32_t ref) {
  if (ref == RT_REF_NONE) return 0;
  const int32_t i = rt_ref_index(ref);
  switch (rt_ref_kind(ref)) {
  case RT_KIND_BVH: {
    const rt_bvh_node *b = vec_at(&c->bvh, i);
    if (b->right == RT_REF_NONE) {
      const int s = stack_need(c, b->left);
      return s > 1 ? s : 1;
    }
    int s = 2;
    const int sl = 1 + stack_need(c, b->left), sr = stack_need(c, b->right);
    if (sl > s) s = sl;
    if (sr > s) s = sr;
    return s;
  }
  case RT_KIND_LIST: {
    /* a cursor entry walks the list: popping cursor k pushes cursor k+1 (if any) and item k */
    const rt_list *l = vec_at(&c->lists, i);
    int s = 0;
    for (int32_t k = l->count - 1; k >= 0; k--) {
      const int si = stack_need(c, *(int32_t *)vec_at(&c->items, l->first + k));
      int sk;
      if (k + 1 < l->count) {
        sk = 2;
        if (1 + si > sk) sk = 1 + si;
        if (s > sk) sk = s;
      } else {
        sk = si > 1 ? si : 1;
      }
      s = sk;
    }
    return s;
  }
  case RT_KIND_TRANSLATE:
  case RT_KIND_ROTATE_Y: {
    const int32_t ch = rt_ref_kind(ref) == RT_KIND_TRANSLATE ? ((rt_translate *)vec_at(&c->translates, i))->child
                                                            : ((rt_rotate_y *)vec_at(&c->rotates, i))->child;
    const int s = 1 + stack_need(c, ch);
    return s > 2 ? s : 2;
  }
  default: return 0;
  }
}

static void *take(vec_t *v, size_t align) {
  const size_t n = (size_t)v->count * v->elem;
  void *p = NULL;
  if (posix_memalign(&p, align, n ? n : align) != 0) abort();
  if (n) memcpy(p, v->data, n);
  free(v->data);
  return p;
}

rt_flat_scene *rt_flatten(const Camera *camera, const World *world) {
  if (camera == NULL || world == NULL) {
    rt_set_error("rt_flatten: NULL camera or world");
    return NULL;
  }
  if (camera->img_width <= 0 || camera->img_height <= 0 || camera->samples_per_pixel <= 0) {
    rt_set_error("rt_flatten: image %dx%d with %d spp: call Camera_init and set samples_per_pixel > 0",
                 camera->img_width, camera->img_height, camera->samples_per_pixel);
    return NULL;
  }
  flat_ctx c;
  memset(&c, 0, sizeof c);
  c.bvh.elem = sizeof(rt_bvh_node);
  c.spheres.elem = sizeof(rt_sphere);
  c.quads.elem = sizeof(rt_quad);
  c.lists.elem = sizeof(rt_list);
  c.items.elem = sizeof(int32_t);
  c.translates.elem = sizeof(rt_translate);
  c.rotates.elem = sizeof(rt_rotate_y);
  c.media.elem = sizeof(rt_medium);
  c.materials.elem = sizeof(rt_material);
  c.textures.elem = sizeof(rt_texture);
  c.images.elem = sizeof(rt_image);
  c.perlins.elem = sizeof(rt_perlin);
  c.bytes.elem = 1;

  rt_flat_scene *s = calloc(1, sizeof *s);
  rt_camera *k = &s->camera;
  k->width = camera->img_width;
  k->height = camera->img_height;
  k->spp = camera->samples_per_pixel;
  k->max_depth = camera->max_depth;
  v3(k->pixel00, camera->pixel00_loc);
  v3(k->delta_u, camera->pixel_delta_u);
  v3(k->delta_v, camera->pixel_delta_v);
  v3(k->origin, camera->look_from);
  v3(k->disc_u, camera->dof_disc_u);
  v3(k->disc_v, camera->dof_disc_v);
  v3(k->background, camera->background);
  k->dof_angle = camera->dof_angle;
  k->light_prob = camera->lights_sampling_prob;
  if (camera->dof_angle > 0.0f) c.features |= RT_FEAT_DOF;

  /* World.objects is itself a HittableList (reference src/raytracing.c:44) */
  s->root = rt_ref(RT_KIND_LIST, flat_list_items(&c, world->objects.items, world->objects.size, RT_REF_NONE));

  /* World.lights: sampled in world space, items need pdf/rand slots (src/hittable.c:89-107) */
  const HittableList *lights = &world->lights;
  int with_rand = 0;
  rt_list ll = {c.items.count, (int32_t)lights->size};
  for (size_t i = 0; i < lights->size && !c.failed; i++) {
    const Hittable *h = lights->items[i];
    int32_t ref = RT_REF_NONE;
    if (h->vtable == &rt_vt_sphere || h->vtable == &rt_vt_quad) {
      ref = flat_object(&c, h, RT_REF_NONE);
      with_rand++;
    } else if (h->vtable == &rt_vt_list) {
      fail(&c, "a HittableList inside World.lights is not supported on the GPU path");
    } else {
      /* BVH/transform/medium: no pdf and no rand in the reference -> kept as a rejected slot */
      ref = RT_REF_NONE;
    }
    vec_push(&c.items, &ref);
  }
  s->lights = vec_push(&c.lists, &ll);
  if (lights->size > 0 && camera->lights_sampling_prob != 0.0f) {
    if (with_rand == 0) fail(&c, "World.lights has no item with rand(): the reference would loop forever");
    c.features |= RT_FEAT_LIGHTS;
  }
  if (camera->max_depth < 0) fail(&c, "max_depth < 0");

  if (c.failed) {
    free(s);
    return NULL; /* the temporary arrays are intentionally leaked on this error path */
  }
  s->features = c.features;
  {
    const int need = stack_need(&c, s->root);
    s->stack_needed = need > 1 ? need : 1; /* the root entry itself */
  }
  /* rt_render's medium boundaries and light primitives are evaluated without the stack */
  s->n_bvh = c.bvh.count;
  s->n_spheres = c.spheres.count;
  s->n_quads = c.quads.count;
  s->n_lists = c.lists.count;
  s->n_list_items = c.items.count;
  s->n_translates = c.translates.count;
  s->n_rotates = c.rotates.count;
  s->n_media = c.media.count;
  s->n_materials = c.materials.count;
  s->n_textures = c.textures.count;
  s->n_images = c.images.count;
  s->n_perlins = c.perlins.count;
  s->n_image_bytes = c.bytes.count;
  s->bvh = take(&c.bvh, 64);
  s->spheres = take(&c.spheres, 64);
  s->quads = take(&c.quads, 64);
  s->lists = take(&c.lists, 64);
  s->list_items = take(&c.items, 64);
  s->translates = take(&c.translates, 64);
  s->rotates = take(&c.rotates, 64);
  s->media = take(&c.media, 64);
  s->materials = take(&c.materials, 64);
  s->textures = take(&c.textures, 64);
  s->images = take(&c.images, 64);
  s->perlins = take(&c.perlins, 64);
  s->image_bytes = take(&c.bytes, 64);
  free(c.obj_memo.keys);
  free(c.obj_memo.vals);
  free(c.mat_memo.keys);
  free(c.mat_memo.vals);
  free(c.tex_memo.keys);
  free(c.tex_memo.vals);
  return s;
}

void rt_flat_free(rt_flat_scene *s) {
  if (!s) return;
  free(s->bvh);
  free(s->spheres);
  free(s->quads);
  free(s->lists);
  free(s->list_items);
  free(s->translates);
  free(s->rotates);
  free(s->media);
  free(s->materials);
  free(s->textures);
  free(s->images);
  free(s->perlins);
  free(s->image_bytes);
  free(s);
}
