/* oracle.c — TEST INFRASTRUCTURE: CPU restatement of the reference hot path.
 *
 * This file is the checker the GPU path is compared against (tests/, __graft_entry__.smoke(),
 * bench.py's cpu_baseline leg).  It is never linked into the product library, and the product
 * never calls it.  It consumes the same flattened scene the kernel receives (include/rt_flat.h)
 * and re-derives every pixel with the reference's structure: recursive ray colour, recursive
 * hit() over lists / BVH nodes / transforms / media, per-pixel pcg32, glibc libm.
 *
 * Pinning: tests/test_oracle_golden.py checks this restatement against golden renders produced by the
 * reference's own sources (oracle/_ref, built by oracle/Makefile; fixtures in tests/golden/).
 *
 * Reference citations (ray-tracing-c @ v2):
 *   pcg32           src/pcg32.c:3-22         vec3 ops        src/vec3.c:5-47
 *   AABB_hit        src/hittable.c:38-55     HittableList    src/hittable.c:74-107
 *   Sphere          src/hittable.c:120-178   Quad            src/hittable.c:186-228
 *   BVHNode_hit     src/hittable.c:266-277   Translate/Rot   src/hittable.c:325-367
 *   ConstantMedium  src/hittable.c:392-423   materials       src/material.c:7-152
 *   textures        src/texture.c:8-114      ray colour      src/raytracing.c:39-84
 *   pixel loop      src/raytracing.c:86-135
 * Build: gcc -std=c11 -O2 (IEEE single precision, no contraction), like the reference oracle.
 */
#include "rt_flat.h"

#include <math.h>
#include <stdbool.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#define PI_F ((float)3.14159265358979323846264338327950288)
#define INV_PI_F ((float)0.318309886183790671537767526745028724)

/* ------------------------------------------------------------------ small vector kit */
typedef struct {
  float x, y, z;
} V;
static V v(float x, float y, float z) {
  V r = {x, y, z};
  return r;
}
static V vl(const float *p) { return v(p[0], p[1], p[2]); }
static V vadd(V a, V b) { return v(a.x + b.x, a.y + b.y, a.z + b.z); }
static V vneg(V a) { return v(-a.x, -a.y, -a.z); }
static V vsub(V a, V b) { return vadd(a, vneg(b)); }
static V vmul(V a, V b) { return v(a.x * b.x, a.y * b.y, a.z * b.z); }
static V vscale(V a, float s) { return v(a.x * s, a.y * s, a.z * s); }
static V vdivs(V a, float s) { return vscale(a, 1.0f / s); }
static float vdot(V a, V b) { return a.x * b.x + a.y * b.y + a.z * b.z; }
static float vlen(V a) { return sqrtf(vdot(a, a)); }
static V vcross(V a, V b) { return v(a.y * b.z - b.y * a.z, a.z * b.x - b.z * a.x, a.x * b.y - b.x * a.y); }
static V vunit(V a) { return vdivs(a, vlen(a)); }

/* ------------------------------------------------------------------ pcg32 */
/* ORACLE_COUNT (scripts/cost_model.c only): per-thread event counters for the cost analysis */
#ifdef ORACLE_COUNT
static __thread long cnt_draw, cnt_ray, cnt_aabb, cnt_sphere;
#define COUNT(x) ((x)++)
#else
#define COUNT(x) ((void)0)
#endif

typedef struct {
  uint64_t state, inc;
} Rng;
static uint32_t rng_u32(Rng *g) {
  COUNT(cnt_draw);
  uint64_t old = g->state;
  g->state = old * 6364136223846793005ULL + g->inc;
  uint32_t xs = (uint32_t)(((old >> 18u) ^ old) >> 27u);
  uint32_t rot = (uint32_t)(old >> 59u);
  return (xs >> rot) | (xs << ((-rot) & 31));
}
static void rng_seed(Rng *g, uint64_t s, uint64_t q) {
  g->state = 0u;
  g->inc = (q << 1u) | 1u;
  rng_u32(g);
  g->state += s;
  rng_u32(g);
}
static float rng_f32(Rng *g) { return (float)(rng_u32(g) >> 8) / (float)(1 << 24); }
static float rng_between(Rng *g, float lo, float hi) { return lo + rng_f32(g) * (hi - lo); }
/* gcc evaluates vec3(f(),f(),f()) right to left: z first */
static V rng_vec_between(Rng *g, float lo, float hi) {
  float z = rng_between(g, lo, hi);
  float y = rng_between(g, lo, hi);
  float x = rng_between(g, lo, hi);
  return v(x, y, z);
}
static V rng_unit(Rng *g) {
  for (;;) {
    V c = rng_vec_between(g, -1.0f, 1.0f);
    float l2 = vdot(c, c);
    if (l2 < 1.0f) return vdivs(c, sqrtf(l2));
  }
}

/* ------------------------------------------------------------------ hit records */
typedef struct {
  V p, normal;
  int32_t material;
  float t, u, w; /* w = the reference's `v` texture coordinate */
  bool front;
} Rec;

typedef struct {
  V o, d;
} Ray;

static V ray_at(const Ray *r, float t) { return vadd(r->o, vscale(r->d, t)); }

static bool aabb_hit(const rt_bvh_node *n, const Ray *r, float tmin, float tmax) {
  COUNT(cnt_aabb);
  const float o[3] = {r->o.x, r->o.y, r->o.z}, d[3] = {r->d.x, r->d.y, r->d.z};
  for (int i = 0; i < 3; i++) {
    float inv = 1.0f / d[i];
    float t0 = (n->lo[i] - o[i]) * inv;
    float t1 = (n->hi[i] - o[i]) * inv;
    if (inv < 0) {
      float s = t0;
      t0 = t1;
      t1 = s;
    }
    tmin = fmaxf(tmin, t0);
    tmax = fminf(tmax, t1);
    if (tmax <= tmin) return false;
  }
  return true;
}

static bool sphere_hit(const rt_sphere *s, const Ray *r, float tmin, float tmax, Rec *rec) {
  COUNT(cnt_sphere);
  V c = vl(s->center);
  V oc = vsub(r->o, c);
  float a = vdot(r->d, r->d);
  float b = vdot(oc, r->d);
  float cc = vdot(oc, oc) - s->radius * s->radius;
  float disc = b * b - a * cc;
  if (disc < 0) return false;
  float sq = sqrtf(disc);
  float root = (-b - sq) / a;
  if (root <= tmin || root >= tmax) {
    root = (-b + sq) / a;
    if (root <= tmin || root >= tmax) return false;
  }
  rec->t = root;
  rec->p = ray_at(r, root);
  V out = vdivs(vsub(rec->p, c), s->radius);
  rec->front = vdot(r->d, out) < 0.0f;
  rec->normal = rec->front ? out : vneg(out);
  rec->u = (atan2f(-out.z, out.x) + PI_F) * INV_PI_F * 0.5f;
  rec->w = acosf(-out.y) * INV_PI_F;
  rec->material = s->material;
  return true;
}

static bool quad_hit(const rt_quad *q, const Ray *r, float tmin, float tmax, Rec *rec) {
  V n = vl(q->normal);
  float den = vdot(n, r->d);
  if (fabsf(den) < 1e-8f) return false;
  float t = (q->D - vdot(n, r->o)) / den;
  if ((t < tmin) || (t > tmax)) return false;
  V p = ray_at(r, t);
  V rel = vsub(p, vl(q->Q));
  float al = vdot(vl(q->w), vcross(rel, vl(q->v)));
  float be = vdot(vl(q->w), vcross(vl(q->u), rel));
  if ((al < 0) || (al > 1) || (be < 0) || (be > 1)) return false;
  rec->u = al;
  rec->w = be;
  rec->t = t;
  rec->p = p;
  rec->material = q->material;
  rec->front = vdot(r->d, n) < 0.0f;
  rec->normal = rec->front ? n : vneg(n);
  return true;
}

static V roty(V a, float c, float s) { return v(c * a.x - s * a.z, a.y, s * a.x + c * a.z); }
static V roty_inv(V a, float c, float s) { return v(c * a.x + s * a.z, a.y, -s * a.x + c * a.z); }

static bool hit(const rt_flat_scene *S, int32_t ref, const Ray *r, float tmin, float tmax, Rec *rec, Rng *g) {
  const int32_t i = rt_ref_index(ref);
  switch (rt_ref_kind(ref)) {
  case RT_KIND_SPHERE: return sphere_hit(&S->spheres[i], r, tmin, tmax, rec);
  case RT_KIND_QUAD: return quad_hit(&S->quads[i], r, tmin, tmax, rec);
  case RT_KIND_LIST: {
    const rt_list *l = &S->lists[i];
    bool any = false;
    for (int k = 0; k < l->count; k++)
      if (hit(S, S->list_items[l->first + k], r, tmin, tmax, rec, g)) {
        tmax = rec->t;
        any = true;
      }
    return any;
  }
  case RT_KIND_BVH: {
    const rt_bvh_node *n = &S->bvh[i];
    if (!aabb_hit(n, r, tmin, tmax)) return false;
    bool hl = hit(S, n->left, r, tmin, tmax, rec, g);
    if (hl) tmax = rec->t;
    /* RT_REF_NONE marks the reference's duplicated n==1 leaf of an rng-free child: revisiting it
     * cannot change rec (see rt_flat.h), so it is skipped here too */
    bool hr = n->right != RT_REF_NONE && hit(S, n->right, r, tmin, tmax, rec, g);
    return hl || hr;
  }
  case RT_KIND_TRANSLATE: {
    const rt_translate *t = &S->translates[i];
    Ray moved = {vsub(r->o, vl(t->offset)), r->d};
    if (!hit(S, t->child, &moved, tmin, tmax, rec, g)) return false;
    rec->p = vadd(rec->p, vl(t->offset));
    return true;
  }
  case RT_KIND_ROTATE_Y: {
    const rt_rotate_y *q = &S->rotates[i];
    Ray turned = {roty(r->o, q->cos_theta, q->sin_theta), roty(r->d, q->cos_theta, q->sin_theta)};
    if (!hit(S, q->child, &turned, tmin, tmax, rec, g)) return false;
    rec->p = roty_inv(rec->p, q->cos_theta, q->sin_theta);
    rec->normal = roty_inv(rec->normal, q->cos_theta, q->sin_theta);
    return true;
  }
  case RT_KIND_MEDIUM: {
    const rt_medium *m = &S->media[i];
    Rec r1, r2;
    if (!hit(S, m->boundary, r, -INFINITY, INFINITY, &r1, g)) return false;
    if (!hit(S, m->boundary, r, r1.t + 0.0001f, INFINITY, &r2, g)) return false;
    r1.t = fmaxf(r1.t, tmin);
    r2.t = fminf(r2.t, tmax);
    if (r1.t >= r2.t) return false;
    r1.t = r1.t > 0.0f ? r1.t : 0.0f;
    float len = vlen(r->d);
    float inside = (r2.t - r1.t) * len;
    float dist = m->neg_inv_density * logf(rng_f32(g));
    if (dist > inside) return false;
    rec->t = r1.t + dist / len;
    rec->p = ray_at(r, rec->t);
    rec->material = m->phase_material;
    return true;
  }
  }
  return false;
}

/* ------------------------------------------------------------------ textures */
static float perlin_noise(const rt_perlin *P, V p) {
  int i = (int)floorf(p.x), j = (int)floorf(p.y), k = (int)floorf(p.z);
  float a = p.x - (float)i, b = p.y - (float)j, c = p.z - (float)k;
  float sa = a * a * (3.0f - 2.0f * a), sb = b * b * (3.0f - 2.0f * b), sc = c * c * (3.0f - 2.0f * c);
  float acc = 0;
  for (int di = 0; di < 2; di++)
    for (int dj = 0; dj < 2; dj++)
      for (int dk = 0; dk < 2; dk++) {
        int gi = P->perm_x[(i + di) & 255] ^ P->perm_y[(j + dj) & 255] ^ P->perm_z[(k + dk) & 255];
        V gr = v(P->grad[gi][0], P->grad[gi][1], P->grad[gi][2]);
        acc += vdot(gr, v(a - di, b - dj, c - dk)) * (di * sa + (1 - di) * (1.0f - sa)) *
               (dj * sb + (1 - dj) * (1.0f - sb)) * (dk * sc + (1 - dk) * (1.0f - sc));
      }
  return acc;
}

static V texture(const rt_flat_scene *S, int32_t id, float u, float w, V p) {
  const rt_texture *t = &S->textures[id];
  switch (t->kind) {
  case RT_TEX_SOLID: return vl(t->color);
  case RT_TEX_CHECKER: {
    int iu = (int)floorf(u / t->scale), iw = (int)floorf(w / t->scale);
    return texture(S, ((iu + iw) % 2) ? t->b : t->a, u, w, p);
  }
  case RT_TEX_IMAGE: {
    const rt_image *im = &S->images[t->a];
    int x = (int)roundf(u * (float)(im->width - 1));
    int y = (int)roundf((1.0f - w) * (float)(im->height - 1));
    const uint8_t *px = S->image_bytes + im->offset + ((int64_t)y * im->width + x) * 3;
    return v((float)px[0] / 255.0f, (float)px[1] / 255.0f, (float)px[2] / 255.0f);
  }
  default: {
    const rt_perlin *P = &S->perlins[t->a];
    p = vscale(p, t->scale);
    float acc = 0.0f, wt = 1.0f;
    V q = p;
    for (int o = 0; o < P->depth; o++) {
      acc += wt * perlin_noise(P, q);
      wt *= 0.5f;
      q = vscale(q, 2.0f);
    }
    float m = 0.5f * (1.0f + sinf(p.z + 10.0f * fabsf(acc)));
    return v(m, m, m);
  }
  }
}

/* ------------------------------------------------------------------ materials */
typedef struct {
  V u, v, w;
} Onb;
static Onb onb(V n) {
  Onb b;
  b.w = vunit(n);
  V a = fabsf(b.w.x) > 0.9f ? v(0, 1, 0) : v(1, 0, 0);
  b.v = vunit(vcross(b.w, a));
  b.u = vcross(b.w, b.v);
  return b;
}
static V onb_local(const Onb *b, V a) { return vadd(vadd(vscale(b->u, a.x), vscale(b->v, a.y)), vscale(b->w, a.z)); }
static V reflect(V d, V n) { return vsub(d, vscale(n, 2.0f * vdot(d, n))); }

static bool scatter(const rt_flat_scene *S, const Rec *rec, V in, V *out, V *albedo, bool *skip, Rng *g) {
  const rt_material *m = &S->materials[rec->material];
  switch (m->tag) {
  case RT_MAT_LAMBERTIAN: {
    Onb b = onb(rec->normal);
    float r1 = rng_f32(g);
    float r2 = rng_f32(g);
    float phi = 2.0f * PI_F * r1;
    *out = onb_local(&b, v(cosf(phi) * sqrtf(r2), sinf(phi) * sqrtf(r2), sqrtf(1.0f - r2)));
    *albedo = texture(S, m->texture, rec->u, rec->w, rec->p);
    *skip = false;
    return true;
  }
  case RT_MAT_METAL: {
    V refl = reflect(vunit(in), rec->normal);
    *out = vadd(refl, vscale(rng_unit(g), m->param));
    *albedo = texture(S, m->texture, rec->u, rec->w, rec->p);
    *skip = true;
    if (vdot(*out, rec->normal) < 0.0f) *out = refl;
    return true;
  }
  case RT_MAT_DIELECTRIC: {
    float eta = m->param;
    if (rec->front) eta = 1.0f / eta;
    in = vunit(in);
    float ct = fminf(-vdot(in, rec->normal), 1.0f);
    float st = sqrtf(1.0f - ct * ct);
    float r0 = (1.0f - eta) / (1.0f + eta);
    r0 *= r0;
    r0 += (1 - r0) * powf(1.0f - ct, 5.0f);
    if (eta * st > 1.0f || r0 > rng_f32(g)) {
      *out = reflect(in, rec->normal);
    } else {
      V perp = vscale(vadd(in, vscale(rec->normal, ct)), eta);
      V para = vscale(rec->normal, -sqrtf(fabsf(1.0f - vdot(perp, perp))));
      *out = vadd(perp, para);
    }
    *albedo = v(1, 1, 1);
    *skip = true;
    return true;
  }
  case RT_MAT_ISOTROPIC:
    *out = rng_unit(g);
    *albedo = texture(S, m->texture, rec->u, rec->w, rec->p);
    *skip = false;
    return true;
  default:
    *skip = true;
    return false;
  }
}

static float scatter_pdf(const rt_flat_scene *S, int32_t mat, V n, V out) {
  switch (S->materials[mat].tag) {
  case RT_MAT_LAMBERTIAN: {
    float c = vdot(n, vunit(out));
    return c < 0.0f ? 0.0f : c / PI_F;
  }
  case RT_MAT_ISOTROPIC: return 1.0f / (4.0f * PI_F);
  default: return 0.0f;
  }
}

static V emit(const rt_flat_scene *S, const Rec *rec) {
  const rt_material *m = &S->materials[rec->material];
  if (m->tag == RT_MAT_SURFACE_NORMAL) return vscale(vadd(rec->normal, v(1.0f, 1.0f, 1.0f)), 0.5f);
  if (m->tag == RT_MAT_DIFFUSE_LIGHT) return rec->front ? texture(S, m->texture, rec->u, rec->w, rec->p) : v(0, 0, 0);
  return v(0, 0, 0);
}

/* ------------------------------------------------------------------ lights (World.lights) */
static float light_pdf(const rt_flat_scene *S, const Ray *r, Rng *g) {
  const rt_list *L = &S->lists[S->lights];
  float pdf = 0.0f, count = 0.0f;
  for (int k = 0; k < L->count; k++) {
    int32_t ref = S->list_items[L->first + k];
    if (ref == RT_REF_NONE) continue;
    Rec rec;
    float val = 0.0f;
    if (rt_ref_kind(ref) == RT_KIND_SPHERE) {
      const rt_sphere *s = &S->spheres[rt_ref_index(ref)];
      if (hit(S, ref, r, 0.001f, INFINITY, &rec, g)) {
        V oc = vsub(vl(s->center), r->o);
        float ctm = sqrtf(1.0f - s->radius * s->radius / vdot(oc, oc));
        val = 1.0f / (2.0f * PI_F * (1.0f - ctm));
      }
    } else {
      const rt_quad *q = &S->quads[rt_ref_index(ref)];
      if (hit(S, ref, r, 0.001f, INFINITY, &rec, g)) {
        float d2 = rec.t * rec.t * vdot(r->d, r->d);
        float c = fabsf(vdot(rec.normal, vunit(r->d)));
        val = d2 / (c * q->area);
      }
    }
    pdf += val;
    count += 1.0f;
  }
  return pdf / fmaxf(count, 1.0f);
}

static V light_rand(const rt_flat_scene *S, V origin, Rng *g) {
  const rt_list *L = &S->lists[S->lights];
  for (;;) {
    int32_t ref = S->list_items[L->first + (int)(0 + rng_u32(g) % (uint32_t)L->count)];
    if (ref == RT_REF_NONE) continue;
    if (rt_ref_kind(ref) == RT_KIND_QUAD) {
      const rt_quad *q = &S->quads[rt_ref_index(ref)];
      float second = rng_f32(g); /* gcc: the v term's draw is evaluated first */
      float first = rng_f32(g);
      return vadd(vadd(vadd(vl(q->Q), vscale(vl(q->u), first)), vscale(vl(q->v), second)), vneg(origin));
    }
    const rt_sphere *s = &S->spheres[rt_ref_index(ref)];
    V oc = vsub(vl(s->center), origin);
    float r1 = rng_f32(g);
    float r2 = rng_f32(g);
    float z = 1.0f + r2 * (sqrtf(1.0f - s->radius * s->radius / vdot(oc, oc)) - 1);
    float phi = 2.0f * PI_F * r1;
    float x = cosf(phi) * sqrtf(1.0f - z * z);
    float y = sinf(phi) * sqrtf(1.0f - z * z);
    Onb b = onb(oc);
    return onb_local(&b, v(x, y, z));
  }
}

/* ------------------------------------------------------------------ ray colour (recursive) */
static V ray_color(const rt_flat_scene *S, const Ray *r, int depth, Rng *g) {
  if (depth <= 0) return v(0, 0, 0);
  COUNT(cnt_ray);
  Rec rec;
  if (!hit(S, S->root, r, 1e-3f, INFINITY, &rec, g)) return vl(S->camera.background);
  Ray next = {rec.p, v(0, 0, 0)};
  V albedo;
  bool skip;
  V e = emit(S, &rec);
  if (!scatter(S, &rec, r->d, &next.d, &albedo, &skip, g)) return e;
  float p = S->camera.light_prob;
  if (skip || p == 0.0f || S->lists[S->lights].count == 0)
    return vadd(e, vmul(albedo, ray_color(S, &next, depth - 1, g)));
  if (rng_f32(g) < p) next.d = light_rand(S, rec.p, g);
  float sp = scatter_pdf(S, rec.material, rec.normal, next.d);
  float spdf = (1.0f - p) * sp + p * light_pdf(S, &next, g);
  return vadd(e, vscale(vmul(albedo, ray_color(S, &next, depth - 1, g)), sp / spdf));
}

#ifdef ORACLE_COUNT
static __thread long *cnt_trace; /* cumulative (draws incl. the 2 of the seed, rays, boxes, spheres) per sample */
#endif
static void pixel(const rt_flat_scene *S, int i, int j, uint8_t *dst) {
  const rt_camera *c = &S->camera;
  Rng g;
  rng_seed(&g, 17 + j, 23 + i);
  V du = vl(c->delta_u), dv = vl(c->delta_v), lf = vl(c->origin);
  V pos = vadd(vadd(vl(c->pixel00), vscale(du, (float)i)), vscale(dv, (float)j));
  V acc = v(0, 0, 0);
  for (int s = 0; s < c->spp; s++) {
    float px = rng_between(&g, -0.5f, 0.5f);
    float py = rng_between(&g, -0.5f, 0.5f);
    Ray r;
    if (c->dof_angle > 0.0f) {
      float a, b;
      for (;;) {
        a = rng_between(&g, -1.0f, 1.0f);
        b = rng_between(&g, -1.0f, 1.0f);
        if (a * a + b * b < 1.0f) break;
      }
      r.o = vadd(vadd(lf, vscale(vl(c->disc_u), a)), vscale(vl(c->disc_v), b));
    } else {
      r.o = lf;
    }
    r.d = vadd(vadd(vadd(pos, vscale(du, px)), vscale(dv, py)), vneg(r.o));
    acc = vadd(acc, ray_color(S, &r, c->max_depth, &g));
#ifdef ORACLE_COUNT
    if (cnt_trace) {
      long *q = cnt_trace + 4L * s;
      q[0] = cnt_draw, q[1] = cnt_ray, q[2] = cnt_aabb, q[3] = cnt_sphere;
    }
#endif
  }
  const float ch[3] = {acc.x, acc.y, acc.z};
  for (int k = 0; k < 3; k++) {
    float val = sqrtf(ch[k] / c->spp);
    val = val > 0.0f ? val : 0.0f;
    val = val < 0.999f ? val : 0.999f;
    dst[k] = (uint8_t)(int)(256.0f * val);
  }
}

/* Render rows row0 + k*row_stride (k < n_rows) into `out` (compact, n_rows*W*3 bytes). */
int oracle_render_rows(const rt_flat_scene *S, int row0, int row_stride, int n_rows, uint8_t *out) {
  const int W = S->camera.width;
  const long total = (long)n_rows * W;
#pragma omp parallel for schedule(dynamic, 64)
  for (long p = 0; p < total; p++) {
    int k = (int)(p / W), i = (int)(p % W);
    pixel(S, i, row0 + k * row_stride, out + p * 3);
  }
  return 0;
}

/* Render an arbitrary pixel list (xs[k], ys[k]) into out[3k..3k+2]. */
int oracle_render_pixels(const rt_flat_scene *S, const int32_t *xs, const int32_t *ys, int n, uint8_t *out) {
#pragma omp parallel for schedule(dynamic, 16)
  for (int k = 0; k < n; k++) pixel(S, xs[k], ys[k], out + 3 * (long)k);
  return 0;
}

/* ------------------------------------------------------------------ canonical dump
 * Same text format as oracle/ref_harness.c `dump`, produced from the flattened scene, so a test
 * can diff the scene this library builds against the scene the reference builds. */
#include <stdio.h>
static void dump_tex(FILE *f, const rt_flat_scene *S, int32_t id) {
  if (id < 0) { fprintf(f, " tex=none"); return; }
  const rt_texture *t = &S->textures[id];
  if (t->kind == RT_TEX_SOLID) fprintf(f, " solid(%a %a %a)", t->color[0], t->color[1], t->color[2]);
  else if (t->kind == RT_TEX_CHECKER) { fprintf(f, " checker(%a", t->scale); dump_tex(f, S, t->a); dump_tex(f, S, t->b); fprintf(f, ")"); }
  else if (t->kind == RT_TEX_IMAGE) {
    const rt_image *im = &S->images[t->a];
    unsigned long long h = 1469598103934665603ULL;
    for (long i = 0; i < (long)im->width * im->height * 3; i++) h = (h ^ S->image_bytes[im->offset + i]) * 1099511628211ULL;
    fprintf(f, " image(%d %d %016llx)", im->width, im->height, h);
  } else {
    const rt_perlin *P = &S->perlins[t->a];
    unsigned long long h = 1469598103934665603ULL;
    for (int i = 0; i < 256; i++) {
      unsigned int vv[6];
      memcpy(vv, P->grad[i], 12);
      vv[3] = (unsigned)P->perm_x[i]; vv[4] = (unsigned)P->perm_y[i]; vv[5] = (unsigned)P->perm_z[i];
      for (int k = 0; k < 6; k++) h = (h ^ vv[k]) * 1099511628211ULL;
    }
    fprintf(f, " perlin(%a %d %016llx)", t->scale, P->depth, h);
  }
}
static void dump_mat(FILE *f, const rt_flat_scene *S, int32_t id) {
  const rt_material *m = &S->materials[id];
  fprintf(f, " mat(%d %a", m->tag, m->param);
  if (m->tag != RT_MAT_DIELECTRIC && m->tag != RT_MAT_SURFACE_NORMAL) dump_tex(f, S, m->texture);
  fprintf(f, ")");
}
static void dump_ref(FILE *f, const rt_flat_scene *S, int32_t ref, int depth) {
  fprintf(f, "%*s", depth, "");
  if (ref == RT_REF_NONE) { fprintf(f, "NONE\n"); return; }
  const int32_t i = rt_ref_index(ref);
  switch (rt_ref_kind(ref)) {
  case RT_KIND_LIST: {
    const rt_list *l = &S->lists[i];
    fprintf(f, "LIST %d\n", l->count);
    for (int k = 0; k < l->count; k++) dump_ref(f, S, S->list_items[l->first + k], depth + 1);
    break;
  }
  case RT_KIND_BVH: {
    const rt_bvh_node *n = &S->bvh[i];
    int dup = n->right == RT_REF_NONE || n->right == n->left;
    fprintf(f, "BVH %a %a %a %a %a %a%s\n", n->lo[0], n->lo[1], n->lo[2], n->hi[0], n->hi[1], n->hi[2], dup ? " dup" : "");
    dump_ref(f, S, n->left, depth + 1);
    if (!dup) dump_ref(f, S, n->right, depth + 1);
    break;
  }
  case RT_KIND_SPHERE: {
    const rt_sphere *s = &S->spheres[i];
    fprintf(f, "SPHERE %a %a %a %a", s->center[0], s->center[1], s->center[2], s->radius);
    dump_mat(f, S, s->material);
    fprintf(f, "\n");
    break;
  }
  case RT_KIND_QUAD: {
    const rt_quad *q = &S->quads[i];
    fprintf(f, "QUAD %a %a %a %a %a %a %a %a %a %a %a %a %a %a %a %a %a", q->Q[0], q->Q[1], q->Q[2], q->u[0], q->u[1],
            q->u[2], q->v[0], q->v[1], q->v[2], q->normal[0], q->normal[1], q->normal[2], q->D, q->w[0], q->w[1],
            q->w[2], q->area);
    dump_mat(f, S, q->material);
    fprintf(f, "\n");
    break;
  }
  case RT_KIND_TRANSLATE: {
    const rt_translate *t = &S->translates[i];
    fprintf(f, "TRANSLATE %a %a %a\n", t->offset[0], t->offset[1], t->offset[2]);
    dump_ref(f, S, t->child, depth + 1);
    break;
  }
  case RT_KIND_ROTATE_Y: {
    const rt_rotate_y *r = &S->rotates[i];
    fprintf(f, "ROTATE %a %a\n", r->sin_theta, r->cos_theta);
    dump_ref(f, S, r->child, depth + 1);
    break;
  }
  case RT_KIND_MEDIUM: {
    const rt_medium *m = &S->media[i];
    fprintf(f, "MEDIUM %a", m->neg_inv_density);
    dump_mat(f, S, m->phase_material);
    fprintf(f, "\n");
    dump_ref(f, S, m->boundary, depth + 1);
    break;
  }
  }
}
int oracle_dump_flat(const rt_flat_scene *S, const char *path) {
  FILE *f = fopen(path, "w");
  if (!f) return -1;
  const rt_camera *c = &S->camera;
  fprintf(f, "CAMERA %d %d %a %a %a | %a %a %a | %a %a %a | %a %a %a | %a %a %a | %a %a %a | %a %a %a %a\n", c->width,
          c->height, c->pixel00[0], c->pixel00[1], c->pixel00[2], c->delta_u[0], c->delta_u[1], c->delta_u[2],
          c->delta_v[0], c->delta_v[1], c->delta_v[2], c->origin[0], c->origin[1], c->origin[2], c->disc_u[0],
          c->disc_u[1], c->disc_u[2], c->disc_v[0], c->disc_v[1], c->disc_v[2], c->background[0], c->background[1],
          c->background[2], c->dof_angle);
  dump_ref(f, S, S->root, 0);
  const rt_list *L = &S->lists[S->lights];
  fprintf(f, "LIGHTS %d\n", L->count);
  for (int k = 0; k < L->count; k++) dump_ref(f, S, S->list_items[L->first + k], 1);
  fclose(f);
  return 0;
}

#ifdef ORACLE_COUNT
/* Event counts of pixel (i, j), cumulative after each sample: trace[4*s + {0,1,2,3}] = pcg32 draws
 * (including the seed's 2), rays, box tests, sphere tests.  Cost analysis only (scripts/cost_model.c). */
void oracle_count_pixel(const rt_flat_scene *S, int i, int j, long *trace) {
  uint8_t px[3];
  cnt_draw = cnt_ray = cnt_aabb = cnt_sphere = 0;
  cnt_trace = trace;
  pixel(S, i, j, px);
  cnt_trace = NULL;
}
#endif
