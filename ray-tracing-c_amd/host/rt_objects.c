/* rt_objects.c — scene-graph constructors of the drop-in API: hittables, BVH build, materials,
 * textures.  Everything that runs once per scene lives here and reproduces the reference's
 * construction arithmetic exactly (bounding boxes, BVH topology, Perlin tables), because the GPU
 * traversal order and culling depend on it.  Per-ray methods run on the GPU; the host-side
 * method slots are identity tokens that abort if called (see include/hittable.h).
 */
#include "rt_internal.h"

#include <math.h>
#include <stdio.h>
#include <string.h>

/* ------------------------------------------------------------------ per-ray method tokens */
static void rt_host_method_called(const char *what) {
  fprintf(stderr,
          "rt: %s is evaluated on the GPU inside Camera_render; this library has no host "
          "implementation of per-ray methods (see INTEGRATION.md)\n",
          what);
  abort();
}

static bool tok_hit_list(const Hittable *s, const Ray *r, float a, float b, HitRecord *h, PCG32 *g) {
  (void)s, (void)r, (void)a, (void)b, (void)h, (void)g;
  rt_host_method_called("HittableList hit()");
  return false;
}
static float tok_pdf_list(const Hittable *s, const Ray *r, PCG32 *g) {
  (void)s, (void)r, (void)g;
  rt_host_method_called("HittableList pdf()");
  return 0.0f;
}
static Vec3 tok_rand_list(const Hittable *s, Vec3 o, PCG32 *g) {
  (void)s, (void)o, (void)g;
  rt_host_method_called("HittableList rand()");
  return VEC3_ZERO;
}
static bool tok_hit_sphere(const Hittable *s, const Ray *r, float a, float b, HitRecord *h, PCG32 *g) {
  (void)s, (void)r, (void)a, (void)b, (void)h, (void)g;
  rt_host_method_called("Sphere hit()");
  return false;
}
static float tok_pdf_sphere(const Hittable *s, const Ray *r, PCG32 *g) {
  (void)s, (void)r, (void)g;
  rt_host_method_called("Sphere pdf()");
  return 0.0f;
}
static Vec3 tok_rand_sphere(const Hittable *s, Vec3 o, PCG32 *g) {
  (void)s, (void)o, (void)g;
  rt_host_method_called("Sphere rand()");
  return VEC3_ZERO;
}
static bool tok_hit_quad(const Hittable *s, const Ray *r, float a, float b, HitRecord *h, PCG32 *g) {
  (void)s, (void)r, (void)a, (void)b, (void)h, (void)g;
  rt_host_method_called("Quad hit()");
  return false;
}
static float tok_pdf_quad(const Hittable *s, const Ray *r, PCG32 *g) {
  (void)s, (void)r, (void)g;
  rt_host_method_called("Quad pdf()");
  return 0.0f;
}
static Vec3 tok_rand_quad(const Hittable *s, Vec3 o, PCG32 *g) {
  (void)s, (void)o, (void)g;
  rt_host_method_called("Quad rand()");
  return VEC3_ZERO;
}
static bool tok_hit_bvh(const Hittable *s, const Ray *r, float a, float b, HitRecord *h, PCG32 *g) {
  (void)s, (void)r, (void)a, (void)b, (void)h, (void)g;
  rt_host_method_called("BVHNode hit()");
  return false;
}
static bool tok_hit_translate(const Hittable *s, const Ray *r, float a, float b, HitRecord *h, PCG32 *g) {
  (void)s, (void)r, (void)a, (void)b, (void)h, (void)g;
  rt_host_method_called("Translate hit()");
  return false;
}
static bool tok_hit_rotate(const Hittable *s, const Ray *r, float a, float b, HitRecord *h, PCG32 *g) {
  (void)s, (void)r, (void)a, (void)b, (void)h, (void)g;
  rt_host_method_called("RotateY hit()");
  return false;
}
static bool tok_hit_medium(const Hittable *s, const Ray *r, float a, float b, HitRecord *h, PCG32 *g) {
  (void)s, (void)r, (void)a, (void)b, (void)h, (void)g;
  rt_host_method_called("ConstantMedium hit()");
  return false;
}

/* NULL slots exactly where the reference has them (src/hittable.c:278, :335, :368, :424) */
HittableVTable rt_vt_list = {tok_hit_list, tok_pdf_list, tok_rand_list};
HittableVTable rt_vt_sphere = {tok_hit_sphere, tok_pdf_sphere, tok_rand_sphere};
HittableVTable rt_vt_quad = {tok_hit_quad, tok_pdf_quad, tok_rand_quad};
HittableVTable rt_vt_bvh = {tok_hit_bvh, NULL, NULL};
HittableVTable rt_vt_translate = {tok_hit_translate, NULL, NULL};
HittableVTable rt_vt_rotate_y = {tok_hit_rotate, NULL, NULL};
HittableVTable rt_vt_medium = {tok_hit_medium, NULL, NULL};

/* ------------------------------------------------------------------ bounding boxes */
static AABB box_empty(void) {
  AABB b;
  for (int a = 0; a < 3; a++) {
    b.values[a][0] = INFINITY;
    b.values[a][1] = -INFINITY;
  }
  return b;
}

static AABB box_of_points(Vec3 p, Vec3 q) {
  AABB b;
  for (int a = 0; a < 3; a++) {
    b.values[a][0] = fminf(p.values[a], q.values[a]);
    b.values[a][1] = fmaxf(p.values[a], q.values[a]);
  }
  return b;
}

static AABB box_union(AABB p, AABB q) {
  AABB b;
  for (int a = 0; a < 3; a++) {
    b.values[a][0] = fminf(p.values[a][0], q.values[a][0]);
    b.values[a][1] = fmaxf(p.values[a][1], q.values[a][1]);
  }
  return b;
}

/* widen degenerate slabs to 2e-4 (reference src/hittable.c:24-37) */
static AABB box_padded(AABB b) {
  const float delta = 1e-4f;
  for (int a = 0; a < 3; a++) {
    if (b.values[a][1] - b.values[a][0] < delta) {
      b.values[a][0] = b.values[a][0] - delta;
      b.values[a][1] = b.values[a][1] + delta;
    }
  }
  return b;
}

/* ------------------------------------------------------------------ HittableList */
void HittableList_init(HittableList *self, size_t max_size) {
  self->hittable.vtable = &rt_vt_list;
  self->hittable.bbox = box_empty();
  self->max_size = max_size;
  self->size = 0;
  self->items = my_malloc(sizeof(Hittable *) * max_size);
}

Hittable *HittableList_new(size_t max_size) {
  HittableList *l = my_malloc(sizeof *l);
  HittableList_init(l, max_size);
  return &l->hittable;
}

void HittableList_append(HittableList *self, Hittable *item) {
  if (self->size >= self->max_size) {
    fprintf(stderr, "rt: HittableList_append: list is full (max_size %zu)\n", self->max_size);
    abort();
  }
  self->items[self->size] = item;
  self->size += 1;
  self->hittable.bbox = box_union(self->hittable.bbox, item->bbox);
}

/* ------------------------------------------------------------------ Sphere */
void Sphere_init(Sphere *self, Vec3 center, float radius, Material *mat) {
  self->hittable.vtable = &rt_vt_sphere;
  self->hittable.bbox = box_of_points(vec3_sub_float(center, radius), vec3_add_float(center, radius));
  self->center = center;
  self->radius = radius;
  self->material = mat;
}

Hittable *Sphere_new(Vec3 center, float radius, Material *mat) {
  Sphere *s = my_malloc(sizeof *s);
  Sphere_init(s, center, radius, mat);
  return &s->hittable;
}

/* ------------------------------------------------------------------ Quad and Box */
void Quad_init(Quad *self, Vec3 Q, Vec3 u, Vec3 v, Material *mat) {
  self->hittable.vtable = &rt_vt_quad;
  /* the reference boxes only the Q and Q+u+v corners (src/hittable.c:232) */
  self->hittable.bbox = box_padded(box_of_points(Q, vec3_add_vec3(vec3_add_vec3(Q, u), v)));
  self->Q = Q;
  self->u = u;
  self->v = v;
  self->material = mat;
  const Vec3 n = vec3_cross(u, v);
  self->normal = vec3_normalize(n);
  self->D = vec3_dot(self->normal, Q);
  self->w = vec3_div_float(n, vec3_length2(n));
  self->area = vec3_length(n);
}

Hittable *Quad_new(Vec3 Q, Vec3 u, Vec3 v, Material *mat) {
  Quad *q = my_malloc(sizeof *q);
  Quad_init(q, Q, u, v, mat);
  return &q->hittable;
}

Hittable *Box_new(Vec3 a, Vec3 b, Material *mat) {
  HittableList *faces = (HittableList *)HittableList_new(6);
  const Vec3 lo = vec3_min(a, b), hi = vec3_max(a, b);
  const Vec3 ex = vec3(hi.x - lo.x, 0, 0);
  const Vec3 ey = vec3(0, hi.y - lo.y, 0);
  const Vec3 ez = vec3(0, 0, hi.z - lo.z);
  /* face order is part of the contract: equal-t quad hits resolve to the later face */
  HittableList_append(faces, Quad_new(vec3(lo.x, lo.y, hi.z), ex, ey, mat));            /* front */
  HittableList_append(faces, Quad_new(vec3(hi.x, lo.y, hi.z), vec3_neg(ez), ey, mat));  /* right */
  HittableList_append(faces, Quad_new(vec3(hi.x, lo.y, lo.z), vec3_neg(ex), ey, mat));  /* back */
  HittableList_append(faces, Quad_new(vec3(lo.x, lo.y, lo.z), ez, ey, mat));            /* left */
  HittableList_append(faces, Quad_new(vec3(lo.x, hi.y, hi.z), ex, vec3_neg(ez), mat));  /* top */
  HittableList_append(faces, Quad_new(vec3(lo.x, lo.y, lo.z), ex, ez, mat));            /* bottom */
  return &faces->hittable;
}

/* ------------------------------------------------------------------ BVH
 * Median split on a random axis; children sorted by their box minimum along that axis with a
 * STABLE sort, which is what glibc's merge-sort qsort does for the reference's comparator
 * (src/hittable.c:59-63, :309).  Topology therefore matches the gcc/glibc reference exactly. */
static int key_before(const Hittable *a, const Hittable *b, int axis) {
  const float ka = a->bbox.values[axis][0], kb = b->bbox.values[axis][0];
  return (ka < kb) ? -1 : (ka > kb) ? 1 : 0;
}

static void stable_sort_by_axis(Hittable **v, Hittable **tmp, size_t n, int axis) {
  if (n < 2) return;
  const size_t h = n / 2;
  stable_sort_by_axis(v, tmp, h, axis);
  stable_sort_by_axis(v + h, tmp, n - h, axis);
  size_t i = 0, j = h, k = 0;
  while (i < h && j < n) tmp[k++] = (key_before(v[i], v[j], axis) <= 0) ? v[i++] : v[j++];
  while (i < h) tmp[k++] = v[i++];
  while (j < n) tmp[k++] = v[j++];
  memcpy(v, tmp, n * sizeof *v);
}

static void bvh_build(BVHNode *node, Hittable *const *items, size_t n, PCG32 *rng) {
  node->hittable.vtable = &rt_vt_bvh;
  Hittable **work = my_malloc(sizeof(Hittable *) * n);
  memcpy(work, items, n * sizeof *work);
  const int axis = (int)pcg32_u32_between(rng, 0, 3); /* drawn at every node, leaves included */
  if (n == 1) {
    node->left = node->right = work[0];
  } else if (n == 2) {
    const int first_smaller = key_before(work[0], work[1], axis) < 0;
    node->left = first_smaller ? work[0] : work[1];
    node->right = first_smaller ? work[1] : work[0];
  } else {
    Hittable **tmp = my_malloc(sizeof(Hittable *) * n);
    stable_sort_by_axis(work, tmp, n, axis);
    free(tmp);
    const size_t half = n / 2;
    BVHNode *l = my_malloc(sizeof *l);
    bvh_build(l, work, half, rng);
    BVHNode *r = my_malloc(sizeof *r);
    bvh_build(r, work + half, n - half, rng);
    node->left = &l->hittable;
    node->right = &r->hittable;
  }
  free(work);
  node->hittable.bbox = box_union(node->left->bbox, node->right->bbox);
}

void BVHNode_init(BVHNode *self, const HittableList *list, PCG32 *rng) {
  bvh_build(self, list->items, list->size, rng);
}

Hittable *BVHNode_new(const HittableList *list, PCG32 *rng) {
  BVHNode *b = my_malloc(sizeof *b);
  BVHNode_init(b, list, rng);
  return &b->hittable;
}

/* ------------------------------------------------------------------ instancing */
void Translate_init(Translate *self, Hittable *object, Vec3 offset) {
  AABB b = object->bbox;
  for (int k = 0; k < 2; k++) {
    b.x[k] += offset.x;
    b.y[k] += offset.y;
    b.z[k] += offset.z;
  }
  self->hittable.vtable = &rt_vt_translate;
  self->hittable.bbox = b;
  self->object = object;
  self->offset = offset;
}

Hittable *Translate_new(Hittable *object, Vec3 offset) {
  Translate *t = my_malloc(sizeof *t);
  Translate_init(t, object, offset);
  return &t->hittable;
}

void RotateY_init(RotateY *self, Hittable *object, float angle) {
  const float rad = angle * (float)M_PI / 180.f;
  const float s = sinf(rad), c = cosf(rad);
  const AABB b = object->bbox;
  Vec3 lo = vec3(INFINITY, INFINITY, INFINITY);
  Vec3 hi = vec3(-INFINITY, -INFINITY, -INFINITY);
  /* rotate the 8 corners back into world space (reference src/hittable.c:377-386) */
  for (int i = 0; i < 2; i++)
    for (int j = 0; j < 2; j++)
      for (int k = 0; k < 2; k++) {
        const float cx = (float)i * b.x[1] + (float)(1 - i) * b.x[0];
        const float cy = (float)j * b.y[1] + (float)(1 - j) * b.y[0];
        const float cz = (float)k * b.z[1] + (float)(1 - k) * b.z[0];
        const Vec3 corner = vec3(c * cx + s * cz, cy, -s * cx + c * cz);
        lo = vec3_min(lo, corner);
        hi = vec3_max(hi, corner);
      }
  self->hittable.vtable = &rt_vt_rotate_y;
  self->hittable.bbox = box_of_points(lo, hi);
  self->object = object;
  self->sin_theta = s;
  self->cos_theta = c;
}

Hittable *RotateY_new(Hittable *object, float angle) {
  RotateY *r = my_malloc(sizeof *r);
  RotateY_init(r, object, angle);
  return &r->hittable;
}

void ConstantMedium_init(ConstantMedium *self, Hittable *boundary, float density, Texture *albedo) {
  self->hittable.vtable = &rt_vt_medium;
  self->hittable.bbox = boundary->bbox;
  self->boundary = boundary;
  self->neg_inv_density = -1.0f / density;
  self->phase_fn = Isotropic_new(albedo);
}

Hittable *ConstantMedium_new(Hittable *boundary, float density, Texture *albedo) {
  ConstantMedium *m = my_malloc(sizeof *m);
  ConstantMedium_init(m, boundary, density, albedo);
  return &m->hittable;
}

/* ------------------------------------------------------------------ materials */
static Material *material_alloc(void) { return my_malloc(sizeof(Material)); }

static void material_set(Material *m, MaterialType tag, Texture *albedo, float param) {
  memset(m, 0, sizeof *m);
  m->tag = tag;
  m->albedo = albedo;
  m->fuzz = param; /* shares storage with eta */
}

void SurfaceNormal_init(Material *self) { material_set(self, SURFACE_NORMAL, NULL, 0.0f); }
Material *SurfaceNormal_new() {
  Material *m = material_alloc();
  SurfaceNormal_init(m);
  return m;
}
void Lambertian_init(Material *self, Texture *albedo) { material_set(self, LAMBERTIAN, albedo, 0.0f); }
Material *Lambertian_new(Texture *albedo) {
  Material *m = material_alloc();
  Lambertian_init(m, albedo);
  return m;
}
void Metal_init(Material *self, Texture *albedo, float fuzz) { material_set(self, METAL, albedo, fuzz); }
Material *Metal_new(Texture *albedo, float fuzz) {
  Material *m = material_alloc();
  Metal_init(m, albedo, fuzz);
  return m;
}
void Dielectric_init(Material *self, float eta) { material_set(self, DIELECTRIC, NULL, eta); }
Material *Dielectric_new(float eta) {
  Material *m = material_alloc();
  Dielectric_init(m, eta);
  return m;
}
void DiffuseLight_init(Material *self, Texture *albedo) { material_set(self, DIFFUSE_LIGHT, albedo, 0.0f); }
Material *DiffuseLight_new(Texture *albedo) {
  Material *m = material_alloc();
  DiffuseLight_init(m, albedo);
  return m;
}
void Isotropic_init(Material *self, Texture *albedo) { material_set(self, ISOTROPIC, albedo, 0.0f); }
Material *Isotropic_new(Texture *albedo) {
  Material *m = material_alloc();
  Isotropic_init(m, albedo);
  return m;
}

bool Material_scatter(const HitRecord *rec, Vec3 r_in, Vec3 *r_out, Vec3 *color, bool *skip_pdf, PCG32 *rng) {
  (void)rec, (void)r_in, (void)r_out, (void)color, (void)skip_pdf, (void)rng;
  rt_host_method_called("Material_scatter()");
  return false;
}
float Material_scatter_pdf(const Material *mat, Vec3 normal, Vec3 r_in, Vec3 r_out) {
  (void)mat, (void)normal, (void)r_in, (void)r_out;
  rt_host_method_called("Material_scatter_pdf()");
  return 0.0f;
}
Vec3 Material_emit(const HitRecord *rec) {
  (void)rec;
  rt_host_method_called("Material_emit()");
  return VEC3_ZERO;
}

Vec3 ONB_local(const ONB *self, Vec3 a) {
  const Vec3 pu = vec3_mul_float(self->u, a.x);
  const Vec3 pv = vec3_mul_float(self->v, a.y);
  const Vec3 pw = vec3_mul_float(self->w, a.z);
  return vec3_add_vec3(vec3_add_vec3(pu, pv), pw);
}

void ONB_from_w(ONB *self, Vec3 w) {
  self->w = vec3_normalize(w);
  const Vec3 helper = (fabsf(self->w.x) > 0.9f) ? vec3(0, 1, 0) : vec3(1, 0, 0);
  self->v = vec3_normalize(vec3_cross(self->w, helper));
  self->u = vec3_cross(self->w, self->v);
}

/* ------------------------------------------------------------------ textures */
Vec3 rt_tex_solid_value(const Texture *self, float u, float v, Vec3 p) {
  (void)self, (void)u, (void)v, (void)p;
  rt_host_method_called("Solid texture value()");
  return VEC3_ZERO;
}
Vec3 rt_tex_checker_value(const Texture *self, float u, float v, Vec3 p) {
  (void)self, (void)u, (void)v, (void)p;
  rt_host_method_called("Checker texture value()");
  return VEC3_ZERO;
}
Vec3 rt_tex_image_value(const Texture *self, float u, float v, Vec3 p) {
  (void)self, (void)u, (void)v, (void)p;
  rt_host_method_called("Image texture value()");
  return VEC3_ZERO;
}
Vec3 rt_tex_perlin_value(const Texture *self, float u, float v, Vec3 p) {
  (void)self, (void)u, (void)v, (void)p;
  rt_host_method_called("Perlin texture value()");
  return VEC3_ZERO;
}

void Solid_init(Solid *self, Vec3 color) {
  self->texture.value = rt_tex_solid_value;
  self->color = color;
}
Texture *Solid_new(Vec3 color) {
  Solid *t = my_malloc(sizeof *t);
  Solid_init(t, color);
  return &t->texture;
}

void Checker_init(Checker *self, float scale, Texture *even, Texture *odd) {
  self->texture.value = rt_tex_checker_value;
  self->scale = scale;
  self->even = even;
  self->odd = odd;
}
Texture *Checker_new(float scale, Texture *even, Texture *odd) {
  Checker *t = my_malloc(sizeof *t);
  Checker_init(t, scale, even, odd);
  return &t->texture;
}

/* Binary PPM (P6, maxval 255) from memory; NULL if it is not one. */
static uint8_t *decode_ppm(const uint8_t *buf, size_t len, int *width, int *height) {
  int w = 0, h = 0, maxval = 0, at = 0;
  char magic[3] = {0};
  char head[64] = {0};
  memcpy(head, buf, len < sizeof head - 1 ? len : sizeof head - 1);
  if (sscanf(head, "%2s %d %d %d%n", magic, &w, &h, &maxval, &at) != 4 || strcmp(magic, "P6") != 0 || w <= 0 ||
      h <= 0 || maxval != 255)
    return NULL;
  const size_t n = (size_t)w * h * 3, off = (size_t)at + 1;  /* one whitespace byte after maxval */
  if (off + n > len) return NULL;
  uint8_t *px = my_malloc(n);
  memcpy(px, buf + off, n);
  *width = w;
  *height = h;
  return px;
}

static _Thread_local int g_image_soft = 0, g_image_failed = 0;
static _Thread_local const char *g_image_dir = NULL;
void rt_image_soft_begin(const char *dir) { g_image_soft = 1, g_image_failed = 0, g_image_dir = dir; }
int rt_image_soft_end(void) {
  g_image_soft = 0;
  g_image_dir = NULL;
  return g_image_failed;
}

/* Image_init (src/texture.c:38-42): the file's content decides the format -- baseline JPEG (as the
 * reference's stb_image decodes it: rt_jpeg.c) or binary PPM (the documented substitute picture) */
void Image_init(Image *self, char *filename) {
  self->texture.value = rt_tex_image_value;
  self->buffer = NULL;
  char why[160] = "cannot open the file";
  char path[4096];
  if (g_image_dir && filename[0] != '/' && snprintf(path, sizeof path, "%s/%s", g_image_dir, filename) < (int)sizeof path)
    filename = path;
  FILE *f = fopen(filename, "rb");
  if (f) {
    uint8_t *buf = NULL;
    size_t len = 0, cap = 0;
    for (;;) {
      if (len == cap) {
        cap = cap ? 2 * cap : 1 << 20;
        uint8_t *grown = realloc(buf, cap);
        if (!grown) {  /* (the block read so far is freed, the failure named) */
          free(buf);
          buf = NULL;
          snprintf(why, sizeof why, "out of memory reading the file");
          break;
        }
        buf = grown;
      }
      const size_t got = fread(buf + len, 1, cap - len, f);
      len += got;
      if (got == 0) break;
    }
    fclose(f);
    if (buf && len >= 2 && buf[0] == 0xff && buf[1] == 0xd8) {
      self->buffer = rt_jpeg_decode(buf, len, &self->width, &self->height, why, sizeof why);
    } else if (buf) {
      self->buffer = decode_ppm(buf, len, &self->width, &self->height);
      snprintf(why, sizeof why, "neither a baseline JPEG nor a binary PPM");
    }
    free(buf);
  }
  if (self->buffer == NULL) {  /* the reference asserts here (src/texture.c:41) */
    if (g_image_soft) {  /* (rt_scene_preset: reported, not fatal) */
      rt_set_error("Image_new(\"%s\"): unable to read image: %s", filename, why);
      g_image_failed = 1;
      self->width = self->height = 1;
      self->buffer = my_malloc(3);
      memset(self->buffer, 0, 3);
      return;
    }
    fprintf(stderr, "rt: Image_new(\"%s\"): Unable to read image: %s\n", filename, why);
    abort();
  }
}
Texture *Image_new(char *filename) {
  Image *t = my_malloc(sizeof *t);
  Image_init(t, filename);
  return &t->texture;
}

/* Fisher-Yates with the modulo draw of the reference (src/texture.c:65-74) */
static void perlin_shuffle(int perm[N_PERLIN], PCG32 *rng) {
  for (int i = 0; i < N_PERLIN; i++) perm[i] = i;
  for (int i = N_PERLIN - 1; i > 0; i--) {
    const uint32_t j = pcg32_u32_between(rng, 0, (uint32_t)i + 1);
    const int t = perm[i];
    perm[i] = perm[j];
    perm[j] = t;
  }
}

void Perlin_init(Perlin *self, float scale, int depth, PCG32 *rng) {
  self->texture.value = rt_tex_perlin_value;
  self->scale = scale;
  self->depth = depth;
  for (int i = 0; i < N_PERLIN; i++) self->grad_field[i] = vec3_rand_unit_vector(rng);
  perlin_shuffle(self->perm_x, rng);
  perlin_shuffle(self->perm_y, rng);
  perlin_shuffle(self->perm_z, rng);
}
Texture *Perlin_new(float scale, int depth, PCG32 *rng) {
  Perlin *t = my_malloc(sizeof *t);
  Perlin_init(t, scale, depth, rng);
  return &t->texture;
}
