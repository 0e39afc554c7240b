/* vec3.h — drop-in for ray-tracing-c include/vec3.h (reference include/vec3.h:1-63).
 *
 * Vec3 is a 12-byte union (x/y/z or values[3]) passed by value.  The arithmetic contract the GPU
 * kernel mirrors op for op:
 *   vec3_add(a,b,c,d) == ((a+b)+c)+d          vec3_mul(a,b,w) == (a*b)*w
 *   vec3_div(u,s)     == u * (1/s)            vec3_normalize(u) == u * (1/sqrtf(|u|^2))
 *   vec3_dot(u,v)     == (ux*vx + uy*vy) + uz*vz   (no contraction)
 * The variadic, type-generic front ends below dispatch on the static type of the second operand
 * (Vec3 or float) exactly like the reference macros, so reference-style call sites compile
 * unchanged.
 */
#ifndef RT_VEC3_H
#define RT_VEC3_H
#ifndef VEC3_H
#define VEC3_H
#endif

#include "pcg32.h"
#include <stdbool.h>

typedef union Vec3 {
  struct {
    float x;
    float y;
    float z;
  };
  float values[3];
} Vec3;

/* ---- type-generic front ends (reference include/vec3.h:7-20) ---------------------------- */
#define RT_V3_SELECT4(a1, a2, a3, a4, chosen, ...) chosen
#define RT_V3_ADD_2(p, q) _Generic((q), Vec3: vec3_add_vec3, float: vec3_add_float)(p, q)
#define RT_V3_ADD_3(p, q, r) RT_V3_ADD_2(RT_V3_ADD_2(p, q), r)
#define RT_V3_ADD_4(p, q, r, s) RT_V3_ADD_2(RT_V3_ADD_3(p, q, r), s)
#define RT_V3_MUL_2(p, q) _Generic((q), Vec3: vec3_mul_vec3, float: vec3_mul_float)(p, q)
#define RT_V3_MUL_3(p, q, r) RT_V3_MUL_2(RT_V3_MUL_2(p, q), r)
#define RT_V3_MUL_4(p, q, r, s) RT_V3_MUL_2(RT_V3_MUL_3(p, q, r), s)

/* vec3_add(u, v[, w[, t]]): left-nested sum; each operand after the first is Vec3 or float */
#define vec3_add(...) RT_V3_SELECT4(__VA_ARGS__, RT_V3_ADD_4, RT_V3_ADD_3, RT_V3_ADD_2, _)(__VA_ARGS__)
/* vec3_mul(u, v[, w[, t]]): left-nested component-wise / scalar product */
#define vec3_mul(...) RT_V3_SELECT4(__VA_ARGS__, RT_V3_MUL_4, RT_V3_MUL_3, RT_V3_MUL_2, _)(__VA_ARGS__)
#define vec3_sub(p, q) _Generic((q), Vec3: vec3_sub_vec3, float: vec3_sub_float)(p, q)
#define vec3_div(p, q) _Generic((q), Vec3: vec3_div_vec3, float: vec3_div_float)(p, q)

/* ---- constructors and element-wise ops (reference src/vec3.c:5-30) ----------------------- */
extern const Vec3 VEC3_ZERO;
Vec3 vec3(float x, float y, float z);
Vec3 *Vec3_new(float x, float y, float z);
Vec3 vec3_neg(Vec3 u);
Vec3 vec3_inv(Vec3 u);

Vec3 vec3_add_vec3(Vec3 u, Vec3 v);
Vec3 vec3_mul_vec3(Vec3 u, Vec3 v);
Vec3 vec3_sub_vec3(Vec3 u, Vec3 v);
Vec3 vec3_div_vec3(Vec3 u, Vec3 v);

Vec3 vec3_add_float(Vec3 u, float v);
Vec3 vec3_sub_float(Vec3 u, float v);
Vec3 vec3_mul_float(Vec3 u, float v);
Vec3 vec3_div_float(Vec3 u, float v);

Vec3 vec3_lerp(Vec3 a, Vec3 b, float w);
Vec3 vec3_min(Vec3 u, Vec3 v);
Vec3 vec3_max(Vec3 u, Vec3 v);

float vec3_length2(Vec3 u);
float vec3_length(Vec3 u);
float vec3_dot(Vec3 u, Vec3 v);
Vec3 vec3_cross(Vec3 u, Vec3 v);
Vec3 vec3_normalize(Vec3 u);
bool vec3_near_zero(Vec3 u);

/* ---- random vectors (reference src/vec3.c:32-47) -----------------------------------------
 * Component draw order is pinned to what gcc emits for the reference (z drawn first, then y,
 * then x: SURVEY §0.3), independent of the compiler that builds this library. */
Vec3 vec3_rand(PCG32 *rng);
Vec3 vec3_rand_between(PCG32 *rng, float lo, float hi);
Vec3 vec3_rand_unit_vector(PCG32 *rng);
Vec3 vec3_rand_hemisphere(Vec3 normal, PCG32 *rng);

#endif /* RT_VEC3_H */
