/* rt_vector.c — Vec3 algebra, PCG32 and allocation for the host library.
 *
 * Semantics follow the reference bit for bit (reference src/vec3.c, src/pcg32.c, src/utils.c),
 * because scene construction (sphere placement, BVH axis draws, Perlin tables) runs here on the
 * host and must produce exactly the scene the reference builds.  Build flags: -std=c11 -O2
 * -ffp-contract=off (no fused multiply-add, no fast-math).
 *
 * Multi-draw expressions are sequenced explicitly in the order gcc evaluates the reference's
 * argument lists (right to left), so this library yields the gcc-built reference's scenes no
 * matter which compiler builds it.
 */
#include "rt_internal.h"

#include <math.h>
#include <stdio.h>

/* ------------------------------------------------------------------ allocation */
void *my_malloc(size_t size) {
  void *p = malloc(size);
  if (p == NULL) {
    fprintf(stderr, "rt: out of host memory (%zu bytes)\n", size);
    abort();
  }
  return p;
}

/* ------------------------------------------------------------------ PCG32 (pcg-c-basic) */
#define RT_PCG_MULT 6364136223846793005ULL

uint32_t pcg32_u32(PCG32 *g) {
  const uint64_t s = g->state;
  g->state = s * RT_PCG_MULT + g->inc;
  const uint32_t mixed = (uint32_t)(((s >> 18u) ^ s) >> 27u);
  const uint32_t r = (uint32_t)(s >> 59u);
  return (mixed >> r) | (mixed << ((32u - r) & 31u));
}

void pcg32_seed(PCG32 *g, uint64_t initstate, uint64_t initseq) {
  g->state = 0u;
  g->inc = (initseq << 1u) | 1u;
  (void)pcg32_u32(g);
  g->state += initstate;
  (void)pcg32_u32(g);
}

uint32_t pcg32_u32_between(PCG32 *g, uint32_t lo, uint32_t hi) { return lo + pcg32_u32(g) % (hi - lo); }

/* 24 high bits scaled by 2^-24: exact, identical to (float)(u>>8) / (float)(1<<24) */
float pcg32_f32(PCG32 *g) { return (float)(pcg32_u32(g) >> 8) / 16777216.0f; }

float pcg32_f32_between(PCG32 *g, float lo, float hi) {
  const float span = hi - lo;
  return lo + pcg32_f32(g) * span;
}

/* ------------------------------------------------------------------ Vec3 */
const Vec3 VEC3_ZERO = {{0.0f, 0.0f, 0.0f}};

Vec3 vec3(float x, float y, float z) {
  Vec3 r;
  r.x = x;
  r.y = y;
  r.z = z;
  return r;
}

Vec3 *Vec3_new(float x, float y, float z) {
  Vec3 *p = my_malloc(sizeof *p);
  *p = vec3(x, y, z);
  return p;
}

Vec3 vec3_neg(Vec3 a) { return vec3(-a.x, -a.y, -a.z); }
Vec3 vec3_inv(Vec3 a) { return vec3(1.0f / a.x, 1.0f / a.y, 1.0f / a.z); }

Vec3 vec3_add_vec3(Vec3 a, Vec3 b) { return vec3(a.x + b.x, a.y + b.y, a.z + b.z); }
Vec3 vec3_mul_vec3(Vec3 a, Vec3 b) { return vec3(a.x * b.x, a.y * b.y, a.z * b.z); }
/* a + (-b) is exactly a - b in IEEE arithmetic */
Vec3 vec3_sub_vec3(Vec3 a, Vec3 b) { return vec3(a.x - b.x, a.y - b.y, a.z - b.z); }
/* division is multiplication by the reciprocal (reference src/vec3.c:14) */
Vec3 vec3_div_vec3(Vec3 a, Vec3 b) { return vec3_mul_vec3(a, vec3_inv(b)); }

Vec3 vec3_add_float(Vec3 a, float s) { return vec3(a.x + s, a.y + s, a.z + s); }
Vec3 vec3_mul_float(Vec3 a, float s) { return vec3(a.x * s, a.y * s, a.z * s); }
Vec3 vec3_sub_float(Vec3 a, float s) { return vec3(a.x - s, a.y - s, a.z - s); }
Vec3 vec3_div_float(Vec3 a, float s) { return vec3_mul_float(a, 1.0f / s); }

Vec3 vec3_lerp(Vec3 a, Vec3 b, float w) {
  const Vec3 pa = vec3_mul_float(a, 1.0f - w);
  const Vec3 pb = vec3_mul_float(b, w);
  return vec3_add_vec3(pa, pb);
}
Vec3 vec3_min(Vec3 a, Vec3 b) { return vec3(fminf(a.x, b.x), fminf(a.y, b.y), fminf(a.z, b.z)); }
Vec3 vec3_max(Vec3 a, Vec3 b) { return vec3(fmaxf(a.x, b.x), fmaxf(a.y, b.y), fmaxf(a.z, b.z)); }

float vec3_dot(Vec3 a, Vec3 b) {
  float acc = a.x * b.x;
  acc = acc + a.y * b.y;
  return acc + a.z * b.z;
}
float vec3_length2(Vec3 a) { return vec3_dot(a, a); }
float vec3_length(Vec3 a) { return sqrtf(vec3_length2(a)); }
Vec3 vec3_cross(Vec3 a, Vec3 b) {
  return vec3(a.y * b.z - b.y * a.z, a.z * b.x - b.z * a.x, a.x * b.y - b.x * a.y);
}
Vec3 vec3_normalize(Vec3 a) { return vec3_div_float(a, vec3_length(a)); }
bool vec3_near_zero(Vec3 a) {
  const float eps = 1e-8f;
  return fabsf(a.x) < eps && fabsf(a.y) < eps && fabsf(a.z) < eps;
}

/* gcc order: the z component's draw happens first, x's last */
Vec3 vec3_rand(PCG32 *g) {
  const float z = pcg32_f32(g);
  const float y = pcg32_f32(g);
  const float x = pcg32_f32(g);
  return vec3(x, y, z);
}

Vec3 vec3_rand_between(PCG32 *g, float lo, float hi) {
  const float z = pcg32_f32_between(g, lo, hi);
  const float y = pcg32_f32_between(g, lo, hi);
  const float x = pcg32_f32_between(g, lo, hi);
  return vec3(x, y, z);
}

/* rejection sampling inside the unit ball, then scale onto the sphere (reference src/vec3.c:36-43) */
Vec3 vec3_rand_unit_vector(PCG32 *g) {
  for (;;) {
    const Vec3 c = vec3_rand_between(g, -1.0f, 1.0f);
    const float l2 = vec3_length2(c);
    if (l2 < 1.0f) return vec3_div_float(c, sqrtf(l2));
  }
}

Vec3 vec3_rand_hemisphere(Vec3 normal, PCG32 *g) {
  const Vec3 d = vec3_rand_unit_vector(g);
  return vec3_dot(d, normal) > 0.0f ? d : vec3_neg(d);
}

Vec3 ray_at(const Ray *ray, float t) { return vec3_add_vec3(ray->origin, vec3_mul_float(ray->direction, t)); }
