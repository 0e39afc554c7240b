// rt_device.h — gfx950 device code of the hot path: one ray-colour loop per pixel lane.
//
// Reference hot path (ray-tracing-c @ v2), re-expressed for a 64-wide wavefront:
//   Camera_render       src/raytracing.c:86-135  -> rt_render_pixel   (rt_kernel.hip)
//   Camera_ray_color    src/raytracing.c:39-84   -> rt_path           (iterative, explicit fold)
//   HittableList/BVH/Sphere/Quad/Translate/RotateY/ConstantMedium hit
//                       src/hittable.c:38-423    -> rt_trace          (explicit-stack DFS)
//   Material_*          src/material.c:23-152    -> rt_scatter / rt_emit / rt_scatter_pdf
//   Texture value       src/texture.c:8-114      -> rt_texture_value
//   pcg32               src/pcg32.c:3-22         -> Pcg32
//   vec3                src/vec3.c               -> f3 helpers below (same operation order)
//
// Bit-exactness rules:
//  * build with -ffp-contract=off, IEEE div/sqrt (hipcc default correctly-rounded f32 div/sqrt),
//    denormals on;  every expression below keeps the reference's association order;
//  * rng draws happen in the gcc-built reference's order (right-to-left argument evaluation);
//  * traversal visits objects in the reference's order with the same shrinking t_max;
//  * the recursive colour `e + a * color(next) [* w]` is folded innermost-first from a per-lane
//    record of (e, a, w) so rounding equals the recursion's;
//  * glibc transcendentals come from rt_libm.h (bit-exact ports).
#pragma once
#include <vector>
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <string.h>

#include "../../include/rt_flat.h"
#include "rt_libm.h"

// Device code is also compiled for the host by the test-only harness tests/native/kernel_host_check.cpp
// (AddressSanitizer + comparison with the oracle before anything runs on a GPU).
#define RT_D __host__ __device__ __forceinline__

namespace rt {

constexpr float kPi = 3.14159265358979323846f;      // (float)M_PI
constexpr float kInvPi = 0.318309886183790671538f;  // (float)M_1_PI
constexpr int kStackMax = 48;                       // DFS stack slots (flattener checks need <= this)
constexpr int kMaxDepth = 64;                       // path record slots (host checks max_depth)
constexpr int kMaxDepthDeep = 1 << 16;              // beyond kMaxDepth: rt_render_deep_kernel

// ------------------------------------------------------------------------------ vectors
struct f3 {
  float x, y, z;
};
RT_D f3 mk(float x, float y, float z) { return f3{x, y, z}; }
RT_D f3 ld3(const float *p) { return f3{p[0], p[1], p[2]}; }
RT_D f3 add(f3 a, f3 b) { return mk(a.x + b.x, a.y + b.y, a.z + b.z); }
RT_D f3 sub(f3 a, f3 b) { return mk(a.x - b.x, a.y - b.y, a.z - b.z); }
RT_D f3 mul(f3 a, f3 b) { return mk(a.x * b.x, a.y * b.y, a.z * b.z); }
RT_D f3 scale(f3 a, float s) { return mk(a.x * s, a.y * s, a.z * s); }
RT_D f3 neg(f3 a) { return mk(-a.x, -a.y, -a.z); }
RT_D float dot(f3 a, f3 b) { return (a.x * b.x + a.y * b.y) + a.z * b.z; }
RT_D f3 cross(f3 a, f3 b) { return mk(a.y * b.z - b.y * a.z, a.z * b.x - b.z * a.x, a.x * b.y - b.x * a.y); }
RT_D f3 normalize(f3 a) { return scale(a, 1.0f / sqrtf(dot(a, a))); }  // vec3_div(u, |u|)
RT_D f3 ray_at(f3 o, f3 d, float t) { return add(o, scale(d, t)); }

// ------------------------------------------------------------------------------ pcg32
struct Pcg32 {
  // inc = (initseq << 1) | 1 kept in 32 bits: every seed's initseq is 23 + a pixel column (< 2^30,
  // host-checked image sizes), so the upper half is zero -- one register less per lane
  uint64_t state;
  uint32_t inc;
  uint32_t n;  // draws since seed(): the stream offset (split render, rt_book1.h); dead code elsewhere
  RT_D uint32_t next() {
    const uint64_t s = state;
    state = s * 6364136223846793005ULL + (uint64_t)inc;
    n++;
    const uint32_t x = (uint32_t)(((s >> 18u) ^ s) >> 27u);
    return __builtin_rotateright32(x, (uint32_t)(s >> 59u));
  }
  RT_D void seed(uint64_t initstate, uint64_t initseq) {
    state = 0u;
    inc = (uint32_t)((initseq << 1u) | 1u);
    (void)next();
    state += initstate;
    (void)next();
    n = 0;
  }
  // advance by k draws without generating them: the LCG's k-step map (a^k, c*(a^k-1)/(a-1)) by
  // squaring, O(log k) 64-bit multiplies (pcg32_advance semantics)
  RT_D void skip(uint32_t k) {
    uint64_t am = 6364136223846793005ULL, ac = (uint64_t)inc, mul = 1u, add = 0u;
    for (uint32_t r = k; r != 0u; r >>= 1) {
      if (r & 1u) mul *= am, add = add * am + ac;
      ac = (am + 1u) * ac;
      am *= am;
    }
    state = mul * state + add;
    n += k;
  }
  RT_D float f32() { return (float)(next() >> 8) * 0x1p-24f; }  // == (float)(u>>8) / 2^24
  RT_D float between(float lo, float hi) { return lo + f32() * (hi - lo); }
};

// A cost pre-pass's position of a pixel (rt_book1.h pre_resume, rt_general.h): its first s samples, from
// stream offset 0, in order, by the same code, end at stream offset o.  0: nothing to resume (an offset
// past 24 bits, or more than 255 samples).
RT_D uint32_t pre_word(uint32_t o, uint32_t s) { return o < (1u << 24) && s < 256u ? o | (s << 24) : 0u; }

// vec3_rand_between in gcc order: z first, then y, then x (src/vec3.c:33-35)
RT_D f3 rand_between(Pcg32 &g, float lo, float hi) {
  const float z = g.between(lo, hi);
  const float y = g.between(lo, hi);
  const float x = g.between(lo, hi);
  return mk(x, y, z);
}
RT_D f3 rand_unit_vector(Pcg32 &g) {  // src/vec3.c:36-43
  for (;;) {
    const f3 c = rand_between(g, -1.0f, 1.0f);
    const float l2 = dot(c, c);
    if (l2 < 1.0f) return scale(c, 1.0f / sqrtf(l2));
  }
}

// ------------------------------------------------------------------------------ scene view
struct DScene {
  rt_camera cam;
  int32_t root, lights, features, pad;
  const rt_bvh_node *bvh;
  const rt_sphere *spheres;
  const rt_quad *quads;
  const rt_list *lists;
  const int32_t *items;
  const rt_translate *translates;
  const rt_rotate_y *rotates;
  const rt_medium *media;
  const rt_material *materials;
  const rt_texture *textures;
  const rt_image *images;
  const rt_perlin *perlins;
  const uint8_t *image_bytes;
  int32_t n_textures, n_images;
  const float4 *pre;  // the world in traversal preorder (build_preorder), or null: the stack trace
  int32_t n_pre, pad2;
};

// Kernel variants compiled per feature set; a scene runs on the smallest variant covering it.
constexpr int kFeatBook1 = RT_FEAT_BVH | RT_FEAT_DOF;  // spheres, lists, BVH: scenes 0 and 1
constexpr int kFeatAll = 0x1ff;

// A DScene whose arrays are the given (host or device) copies of the flat scene's arrays.
inline DScene make_view(const rt_flat_scene &s, const void *const arrays[13]) {
  DScene v;
  memset(&v, 0, sizeof v);
  v.cam = s.camera;
  v.root = s.root;
  v.lights = s.lights;
  v.features = s.features;
  v.bvh = (const rt_bvh_node *)arrays[0];
  v.spheres = (const rt_sphere *)arrays[1];
  v.quads = (const rt_quad *)arrays[2];
  v.lists = (const rt_list *)arrays[3];
  v.items = (const int32_t *)arrays[4];
  v.translates = (const rt_translate *)arrays[5];
  v.rotates = (const rt_rotate_y *)arrays[6];
  v.media = (const rt_medium *)arrays[7];
  v.materials = (const rt_material *)arrays[8];
  v.textures = (const rt_texture *)arrays[9];
  v.images = (const rt_image *)arrays[10];
  v.perlins = (const rt_perlin *)arrays[11];
  v.image_bytes = (const uint8_t *)arrays[12];
  v.n_textures = s.n_textures;
  v.n_images = s.n_images;
  return v;
}

// ------------------------------------------------------------------------------ exact fast arithmetic
// What sqrtf() and '/' compile to for f32 on gfx950 (denormals on, correctly rounded): a hardware
// estimate plus a Newton / one-ulp correction core, wrapped in operand scaling for extreme exponents
// and a special-value fix-up (v_div_scale / v_div_fmas / v_div_fixup, and the 2^-96 rescale + class
// test of the sqrt).  On the operand ranges below the wrappers are identities, so the bare cores
// return the same bits; the division's reciprocal refinement depends on the divisor only and is
// hoisted per ray.  Bitwise equality is checked on the device by rt_diag_arith (all floats for the
// sqrt, random pairs for the division: tests/test_libm_port.py).
constexpr float kDivLo = 0x1p-20f, kDivHi = 0x1p20f;  // divisor range (|d|^2 of a ray)
constexpr float kNumHi = 0x1p40f;                     // numerator magnitude bound
constexpr float kSqrtLo = 0x1p-96f;                   // below it the compiler rescales

// (Host passes -- host-side checkers that include this header -- use the libm operations, which
// the cores equal on their domains.)
RT_D float sqrt_core(float x) {  // == sqrtf(x) for x == 0 or kSqrtLo <= x < inf
#if !defined(__HIP_DEVICE_COMPILE__)
  return sqrtf(x);
#else
  const float r = __builtin_amdgcn_sqrtf(x);
  const float rm = __int_as_float(__float_as_int(r) - 1), rp = __int_as_float(__float_as_int(r) + 1);
  float out = fmaf(-rm, r, x) <= 0.0f ? rm : r;
  out = fmaf(-rp, r, x) > 0.0f ? rp : out;
  return out;
#endif
}
RT_D float recip_core(float a) {  // the divisor half of the '/' sequence
#if !defined(__HIP_DEVICE_COMPILE__)
  return 1.0f / a;
#else
  const float y = __builtin_amdgcn_rcpf(a);
  return fmaf(fmaf(-a, y, 1.0f), y, y);
#endif
}
RT_D float div_core(float x, float a, float ra) {  // == x / a for a in [kDivLo, kDivHi], |x| <= kNumHi
  const float q0 = x * ra;
  const float q1 = fmaf(fmaf(-a, q0, x), ra, q0);
  return fmaf(fmaf(-a, q1, x), ra, q1);
}
// For |x| < 2^-40 (zero and denormals included) div_core is not bit-exact, but both it and x / a
// are below 2^-18 < t_min in magnitude, so the Sphere_hit root test rejects both: the decision and
// the recorded root (none) are the same.  Only |x| > kNumHi needs the real division.

// ------------------------------------------------------------------------------ primitives
// Sphere_hit up to the accepted root (src/hittable.c:120-138); a = |d|^2 hoisted per ray.
RT_D bool sphere_t(const rt_sphere &s, f3 o, f3 d, float a, float tmin, float tmax, float &t) {
  const f3 oc = sub(o, ld3(s.center));
  const float b = dot(oc, d);
  const float c = dot(oc, oc) - s.radius_sq;
  const float disc = b * b - a * c;
  if (disc < 0) return false;
  const float sq = sqrtf(disc);
  float root = (-b - sq) / a;
  if (root <= tmin || root >= tmax) {
    root = (-b + sq) / a;
    if (root <= tmin || root >= tmax) return false;
  }
  t = root;
  return true;
}

// Quad_hit up to acceptance (src/hittable.c:186-203); note the INCLUSIVE t range.
RT_D bool quad_t(const rt_quad &q, f3 o, f3 d, float tmin, float tmax, float &t) {
  const f3 n = ld3(q.normal);
  const float denom = dot(n, d);
  if (fabsf(denom) < 1e-8f) return false;
  const float tt = (q.D - dot(n, o)) / denom;
  if ((tt < tmin) || (tt > tmax)) return false;
  const f3 hp = sub(ray_at(o, d, tt), ld3(q.Q));
  const f3 w = ld3(q.w);
  const float alpha = dot(w, cross(hp, ld3(q.v)));
  const float beta = dot(w, cross(ld3(q.u), hp));
  if ((alpha < 0) || (alpha > 1) || (beta < 0) || (beta > 1)) return false;
  t = tt;
  return true;
}

RT_D bool prim_t(const DScene &S, int32_t ref, f3 o, f3 d, float tmin, float tmax, float &t) {
  const int32_t i = rt_ref_index(ref);
  if (rt_ref_kind(ref) == RT_KIND_SPHERE) return sphere_t(S.spheres[i], o, d, dot(d, d), tmin, tmax, t);
  return quad_t(S.quads[i], o, d, tmin, tmax, t);
}

// AABB_hit (src/hittable.c:38-55) with 1/d hoisted per ray (same division, same value).
RT_D bool aabb_hit(const rt_bvh_node &n, f3 o, f3 inv, float tmin, float tmax) {
  const float lo[3] = {n.lo[0], n.lo[1], n.lo[2]};
  const float hi[3] = {n.hi[0], n.hi[1], n.hi[2]};
  const float oo[3] = {o.x, o.y, o.z};
  const float iv[3] = {inv.x, inv.y, inv.z};
#pragma unroll
  for (int a = 0; a < 3; a++) {
    float t0 = (lo[a] - oo[a]) * iv[a];
    float t1 = (hi[a] - oo[a]) * iv[a];
    if (iv[a] < 0) {
      const float s = t0;
      t0 = t1;
      t1 = s;
    }
    tmin = fmaxf(tmin, t0);
    tmax = fminf(tmax, t1);
    if (tmax <= tmin) return false;
  }
  return true;
}

// ------------------------------------------------------------------------------ transforms
RT_D f3 rot_y(f3 u, float c, float s) { return mk(c * u.x - s * u.z, u.y, s * u.x + c * u.z); }
RT_D f3 rot_y_inv(f3 u, float c, float s) { return mk(c * u.x + s * u.z, u.y, -s * u.x + c * u.z); }

// Ray in the frame of transform `xf` (a TRANSLATE / ROTATE_Y ref, or NONE = world):
// apply the chain outermost first, exactly as nested Translate_hit / RotateY_hit do.
RT_D void local_ray(const DScene &S, int32_t xf, f3 wo, f3 wd, f3 &o, f3 &d) {
  int32_t chain[8];
  int n = 0;
  while (xf != RT_REF_NONE && n < 8) {
    chain[n++] = xf;
    xf = rt_ref_kind(xf) == RT_KIND_TRANSLATE ? S.translates[rt_ref_index(xf)].parent_xform
                                               : S.rotates[rt_ref_index(xf)].parent_xform;
  }
  o = wo;
  d = wd;
  for (int k = n - 1; k >= 0; k--) {
    const int32_t r = chain[k];
    if (rt_ref_kind(r) == RT_KIND_TRANSLATE) {
      o = sub(o, ld3(S.translates[rt_ref_index(r)].offset));
    } else {
      const rt_rotate_y &ry = S.rotates[rt_ref_index(r)];
      o = rot_y(o, ry.cos_theta, ry.sin_theta);
      d = rot_y(d, ry.cos_theta, ry.sin_theta);
    }
  }
}

RT_D int32_t parent_of(const DScene &S, int32_t xf) {
  return rt_ref_kind(xf) == RT_KIND_TRANSLATE ? S.translates[rt_ref_index(xf)].parent_xform
                                               : S.rotates[rt_ref_index(xf)].parent_xform;
}

// ------------------------------------------------------------------------------ traversal
struct Hit {
  float t;
  int32_t prim;   // winning SPHERE / QUAD / MEDIUM ref
  int32_t xform;  // transform frame the winner was hit in (NONE = world)
};

// Closest hit over World.objects in [tmin, inf): the reference's recursive visit order
// (lists in order, BVH node box -> left -> right with t_max = closest so far) as an explicit DFS.
// Exit markers restore the parent frame after a transform's subtree.
constexpr int32_t kExitTag = 7;

template <int F>
RT_D bool trace(const DScene &S, f3 wo, f3 wd, float tmin, Pcg32 &g, Hit &h) {
  // entry = ref | (list cursor position << 32); lists are walked through a cursor entry so a list
  // of any length costs one stack slot (need computed by rt_flatten.c: stack_need)
  uint64_t stack[kStackMax];
  int sp = 0;
  // pushes are bounds-checked for memory safety only: rt_scene_upload rejects scenes whose
  // computed stack need exceeds kStackMax, so the guard never fires on a validated scene
#define RT_PUSH(x)                                                                                 \
  do {                                                                                             \
    if (sp < kStackMax) stack[sp++] = (x);                                                         \
  } while (0)
  // the entry processed next is held in `cur` (the last push of the reference order, popped at once)
  // instead of taking a stack round trip: the same visit order, half the stack traffic, and the
  // descent's next node load does not wait on a stack load
  constexpr uint64_t kNoEntry = ~0ull;
  uint64_t cur = (uint32_t)S.root;
  float tmax = __builtin_inff();
  bool found = false;
  int32_t frame = RT_REF_NONE;
  f3 o = wo, d = wd;
  f3 inv = mk(1.0f / d.x, 1.0f / d.y, 1.0f / d.z);
  float dd = dot(d, d);
  for (;;) {
    if (cur == kNoEntry) {
      if (sp == 0) break;
      cur = stack[--sp];
    }
    const uint64_t e = cur;
    cur = kNoEntry;
    const int32_t ref = (int32_t)(uint32_t)e;
    const int kind = rt_ref_kind(ref);
    const int32_t idx = rt_ref_index(ref);
    if ((F & RT_FEAT_BVH) && kind == RT_KIND_BVH) {
      const rt_bvh_node &n = S.bvh[idx];
      if (aabb_hit(n, o, inv, tmin, tmax)) {
        if (n.right != RT_REF_NONE) RT_PUSH((uint32_t)n.right);
        cur = (uint32_t)n.left;
      }
    } else if (kind == RT_KIND_SPHERE) {
      float t;
      if (sphere_t(S.spheres[idx], o, d, dd, tmin, tmax, t)) {
        tmax = t;
        h.t = t;
        h.prim = ref;
        h.xform = frame;
        found = true;
      }
    } else if (kind == RT_KIND_LIST) {
      const rt_list l = S.lists[idx];
      const int32_t pos = (int32_t)(e >> 32);
      if (pos < l.count) {
        if (pos + 1 < l.count) RT_PUSH((uint32_t)ref | ((uint64_t)(pos + 1) << 32));
        cur = (uint32_t)S.items[l.first + pos];
      }
    } else if ((F & RT_FEAT_QUAD) && kind == RT_KIND_QUAD) {
      float t;
      if (quad_t(S.quads[idx], o, d, tmin, tmax, t)) {
        tmax = t;
        h.t = t;
        h.prim = ref;
        h.xform = frame;
        found = true;
      }
    } else if ((F & RT_FEAT_XFORM) && (kind == RT_KIND_TRANSLATE || kind == RT_KIND_ROTATE_Y)) {
      RT_PUSH((uint32_t)rt_ref(kExitTag, 0) | ((uint64_t)(uint32_t)ref << 32));
      cur = (uint32_t)(kind == RT_KIND_TRANSLATE ? S.translates[idx].child : S.rotates[idx].child);
      frame = ref;
      local_ray(S, frame, wo, wd, o, d);
      inv = mk(1.0f / d.x, 1.0f / d.y, 1.0f / d.z);
      dd = dot(d, d);
    } else if ((F & RT_FEAT_XFORM) && kind == kExitTag) {
      frame = parent_of(S, (int32_t)(uint32_t)(e >> 32));
      local_ray(S, frame, wo, wd, o, d);
      inv = mk(1.0f / d.x, 1.0f / d.y, 1.0f / d.z);
      dd = dot(d, d);
    } else if ((F & RT_FEAT_MEDIUM) && kind == RT_KIND_MEDIUM) {
      // ConstantMedium_hit (src/hittable.c:392-423): two boundary hits, clamp, one rng draw
      const rt_medium m = S.media[idx];
      float t1, t2;
      if (prim_t(S, m.boundary, o, d, -__builtin_inff(), __builtin_inff(), t1) &&
          prim_t(S, m.boundary, o, d, t1 + 0.0001f, __builtin_inff(), t2)) {
        t1 = fmaxf(t1, tmin);
        t2 = fminf(t2, tmax);
        if (!(t1 >= t2)) {
          t1 = t1 > 0.0f ? t1 : 0.0f;
          const float len = sqrtf(dd);
          const float inside = (t2 - t1) * len;
          const float dist = m.neg_inv_density * rtm::logf(g.f32());
          if (!(dist > inside)) {
            const float t = t1 + dist / len;
            tmax = t;
            h.t = t;
            h.prim = ref;
            h.xform = frame;
            found = true;
          }
        }
      }
    }
  }
#undef RT_PUSH
  return found;
}

// ------------------------------------------------------------------------------ preorder traversal
// The stack machine above visits the world graph in preorder -- a node's box, then its left
// subtree, then its right; a list's items in order; a transform's child, then the parent frame
// again -- and skips a subtree whose box misses.  build_preorder lays that order out as entries of
// 2 float4, so trace_pre is a scan with skips, without a stack:
//   BVH node:   q0 = (lo.x, lo.y, lo.z, hi.x)  q1 = (hi.y, hi.z, skip, ref)  next = hit ? p+1 : skip
//   transform:  q0 = (end, a0, enclosing transform's position or ~0, a1)  q1 = (a2, -, end, ref)
//               (translate: (a0, a1, a2) = offset; rotate_y: (a0, a1) = (cos, sin))
//   sphere:     q0 = (center, r^2); quad: q0 = (normal, D); q1.w = ref                 next = p+1
//   medium:     sphere boundary: q0 = its (center, r^2), q1 = (-1/density, 1 (bits), -, ref); else -
// (skip / end = the position after the subtree; integers stored as float bits).  Lists need no
// entry.  Visit order, frames, t_max and rng draws (media) are the stack machine's.
// The scan's state, so that a caller can run it a few entries at a time (rt_general.h).
struct PreTrace {
  f3 o, d, inv;            // the ray in the current frame
  float dd, tmax;
  float ra;                // recip_core(dd): the divisor half of '/' by dd, hoisted per frame
  bool fast;               // dd in [kDivLo, kDivHi] (div_core by dd is exact)
  int32_t frame;
  uint32_t p, fend, fpos;  // next entry; the current frame's subtree end and entry position
  bool found;
  Hit h;
};
RT_D void pre_begin(PreTrace &T, f3 wo, f3 wd) {
  T.o = wo, T.d = wd;
  T.inv = mk(1.0f / wd.x, 1.0f / wd.y, 1.0f / wd.z);
  T.dd = dot(wd, wd);
  T.ra = recip_core(T.dd);
  T.fast = T.dd >= kDivLo && T.dd <= kDivHi;
  T.tmax = __builtin_inff();
  T.frame = RT_REF_NONE;
  T.p = 0u, T.fend = 0xffffffffu, T.fpos = 0u;
  T.found = false;
}
// One entry of the scan; returns true once the scan is past the last entry.
// lds / n_lds: the first n_lds entries staged in LDS by the caller (0: none)
template <int F>
RT_D bool pre_step(const DScene &S, PreTrace &T, f3 wo, f3 wd, float tmin, Pcg32 &g, const float4 *lds = nullptr,
                   uint32_t n_lds = 0u) {
  const uint32_t n = (uint32_t)S.n_pre;
  if (T.p >= n) return true;
  if (F & RT_FEAT_XFORM) {
    while (T.p >= T.fend) {  // leaving a transform's subtree: the enclosing frame again
      const uint32_t pp = __builtin_bit_cast(uint32_t, S.pre[2 * T.fpos].z);
      T.frame = parent_of(S, T.frame);
      T.fend = pp == 0xffffffffu ? 0xffffffffu : __builtin_bit_cast(uint32_t, S.pre[2 * pp].x);
      T.fpos = pp == 0xffffffffu ? 0u : pp;
      local_ray(S, T.frame, wo, wd, T.o, T.d);
      T.inv = mk(1.0f / T.d.x, 1.0f / T.d.y, 1.0f / T.d.z);
      T.dd = dot(T.d, T.d);
    }
  }
  float4 q0, q1;
  if (T.p < n_lds) {
    q0 = lds[2 * T.p], q1 = lds[2 * T.p + 1];
  } else {
    q0 = S.pre[2 * T.p], q1 = S.pre[2 * T.p + 1];
  }
  const int32_t ref = (int32_t)__builtin_bit_cast(uint32_t, q1.w);
  const int kind = rt_ref_kind(ref);
  const int32_t idx = rt_ref_index(ref);
  const f3 o = T.o, d = T.d;
  uint32_t next = T.p + 1;
  float t = 0.0f;
  bool hit = false;
  if ((F & RT_FEAT_BVH) && kind == RT_KIND_BVH) {
    rt_bvh_node nd;
    nd.lo[0] = q0.x, nd.lo[1] = q0.y, nd.lo[2] = q0.z;
    nd.hi[0] = q0.w, nd.hi[1] = q1.x, nd.hi[2] = q1.y;
    if (!aabb_hit(nd, o, T.inv, tmin, T.tmax)) next = __builtin_bit_cast(uint32_t, q1.z);
  } else if (kind == RT_KIND_SPHERE) {  // center and r^2 inline: no dependent load
    rt_sphere sp;
    sp.center[0] = q0.x, sp.center[1] = q0.y, sp.center[2] = q0.z, sp.radius_sq = q0.w;
    hit = sphere_t(sp, o, d, T.dd, tmin, T.tmax, t);
  } else if ((F & RT_FEAT_QUAD) && kind == RT_KIND_QUAD) {
    // quad_t with the plane (normal, D) inline: the quad record is read only past the plane test
    const f3 nq = mk(q0.x, q0.y, q0.z);
    const float denom = dot(nq, d);
    const float tt = (q0.w - dot(nq, o)) / denom;
    hit = !(fabsf(denom) < 1e-8f) && !((tt < tmin) || (tt > T.tmax));
    if (hit) {
      const rt_quad &qd = S.quads[idx];
      const f3 hp = sub(ray_at(o, d, tt), ld3(qd.Q));
      const f3 w = ld3(qd.w);
      const float alpha = dot(w, cross(hp, ld3(qd.v)));
      const float beta = dot(w, cross(ld3(qd.u), hp));
      hit = !((alpha < 0) || (alpha > 1) || (beta < 0) || (beta > 1));
      t = tt;
    }
  } else if ((F & RT_FEAT_XFORM) && (kind == RT_KIND_TRANSLATE || kind == RT_KIND_ROTATE_Y)) {
    T.frame = ref;
    T.fend = __builtin_bit_cast(uint32_t, q0.x);
    T.fpos = T.p;
    local_ray(S, T.frame, wo, wd, T.o, T.d);
    T.inv = mk(1.0f / T.d.x, 1.0f / T.d.y, 1.0f / T.d.z);
    T.dd = dot(T.d, T.d);
  } else if ((F & RT_FEAT_MEDIUM) && kind == RT_KIND_MEDIUM) {
    // ConstantMedium_hit (src/hittable.c:392-423): two boundary hits, clamp, one rng draw.  A
    // sphere boundary's centre / r^2 and the density sit in the entry (no dependent loads).
    const bool inl = __builtin_bit_cast(uint32_t, q1.y) == 1u;
    float t1, t2, nid;
    bool both;
    if (inl) {
      rt_sphere sp;
      sp.center[0] = q0.x, sp.center[1] = q0.y, sp.center[2] = q0.z, sp.radius_sq = q0.w;
      const float a = dot(d, d);
      both = sphere_t(sp, o, d, a, -__builtin_inff(), __builtin_inff(), t1) &&
             sphere_t(sp, o, d, a, t1 + 0.0001f, __builtin_inff(), t2);
      nid = q1.x;
    } else {
      const rt_medium m = S.media[idx];
      both = prim_t(S, m.boundary, o, d, -__builtin_inff(), __builtin_inff(), t1) &&
             prim_t(S, m.boundary, o, d, t1 + 0.0001f, __builtin_inff(), t2);
      nid = m.neg_inv_density;
    }
    if (both) {
      t1 = fmaxf(t1, tmin);
      t2 = fminf(t2, T.tmax);
      if (!(t1 >= t2)) {
        t1 = t1 > 0.0f ? t1 : 0.0f;
        const float len = sqrtf(T.dd);
        const float inside = (t2 - t1) * len;
        const float dist = nid * rtm::logf(g.f32());
        if (!(dist > inside)) {
          t = t1 + dist / len;
          hit = true;
        }
      }
    }
  }
  if (hit) {
    T.tmax = t;
    T.h.t = t;
    T.h.prim = ref;
    T.h.xform = T.frame;
    T.found = true;
  }
  T.p = next;
  return next >= n;
}

template <int F>
RT_D bool trace_pre(const DScene &S, f3 wo, f3 wd, float tmin, Pcg32 &g, Hit &h) {
  PreTrace T;
  pre_begin(T, wo, wd);
  while (!pre_step<F>(S, T, wo, wd, tmin, g)) {
  }
  h = T.h;
  return T.found;
}

// Host: the preorder entries of trace_pre for a flattened scene (2 float4 per entry).
struct PreorderBuilder {
  const rt_flat_scene &s;
  std::vector<float4> &out;
  static float b(uint32_t x) {
    float f;
    memcpy(&f, &x, 4);
    return f;
  }
  uint32_t size() const { return (uint32_t)(out.size() / 2); }
  void emit(int32_t ref, uint32_t enclosing) {
    if (ref == RT_REF_NONE) return;
    const int kind = rt_ref_kind(ref);
    const int32_t idx = rt_ref_index(ref);
    const uint32_t p = size();
    if (kind == RT_KIND_LIST) {
      const rt_list &l = s.lists[idx];
      for (int k = 0; k < l.count; k++) emit(s.list_items[l.first + k], enclosing);
      return;
    }
    float4 q0 = make_float4(0.0f, 0.0f, 0.0f, 0.0f);
    if (kind == RT_KIND_SPHERE) {
      const rt_sphere &sp = s.spheres[idx];
      q0 = make_float4(sp.center[0], sp.center[1], sp.center[2], sp.radius_sq);
    } else if (kind == RT_KIND_QUAD) {
      const rt_quad &qd = s.quads[idx];
      q0 = make_float4(qd.normal[0], qd.normal[1], qd.normal[2], qd.D);
    }
    float4 q1 = make_float4(0.0f, 0.0f, 0.0f, b((uint32_t)ref));
    if (kind == RT_KIND_MEDIUM && rt_ref_kind(s.media[idx].boundary) == RT_KIND_SPHERE) {  // boundary inline
      const rt_sphere &sp = s.spheres[rt_ref_index(s.media[idx].boundary)];
      q0 = make_float4(sp.center[0], sp.center[1], sp.center[2], sp.radius_sq);
      q1.x = s.media[idx].neg_inv_density;
      q1.y = b(1u);
    }
    out.push_back(q0);
    out.push_back(q1);
    if (kind == RT_KIND_BVH) {
      const rt_bvh_node &nd = s.bvh[idx];
      emit(nd.left, enclosing);
      if (nd.right != RT_REF_NONE) emit(nd.right, enclosing);
      out[2 * p] = make_float4(nd.lo[0], nd.lo[1], nd.lo[2], nd.hi[0]);
      out[2 * p + 1] = make_float4(nd.hi[1], nd.hi[2], b(size()), b((uint32_t)ref));
    } else if (kind == RT_KIND_TRANSLATE || kind == RT_KIND_ROTATE_Y) {
      emit(kind == RT_KIND_TRANSLATE ? s.translates[idx].child : s.rotates[idx].child, p);
      // the transform itself rides in the free words: translate (q0.y, q0.w, q1.x) = offset,
      // rotate (q0.y, q0.w) = (cos, sin), so the scan changes frames without global loads
      const bool tr = kind == RT_KIND_TRANSLATE;
      const float a0 = tr ? s.translates[idx].offset[0] : s.rotates[idx].cos_theta;
      const float a1 = tr ? s.translates[idx].offset[1] : s.rotates[idx].sin_theta;
      const float a2 = tr ? s.translates[idx].offset[2] : 0.0f;
      out[2 * p] = make_float4(b(size()), a0, b(enclosing), a1);
      out[2 * p + 1] = make_float4(a2, 0.0f, b(size()), b((uint32_t)ref));
    }
  }
};
inline void build_preorder(const rt_flat_scene &s, std::vector<float4> &out) {
  out.clear();
  PreorderBuilder B{s, out};
  B.emit(s.root, 0xffffffffu);
}

// ------------------------------------------------------------------------------ hit record
struct Rec {
  f3 p, normal;
  float u, v;
  int32_t material;
  bool front;
};

// Whether a hit on material `mat` reads the record's u, v: texture_value reads them only for image
// and checker textures (src/texture.c:12-37), and only textured materials call it.
RT_D bool mat_uses_uv(const DScene &S, int32_t mat) {
  const rt_material &m = S.materials[mat];
  if (m.tag != RT_MAT_LAMBERTIAN && m.tag != RT_MAT_METAL && m.tag != RT_MAT_ISOTROPIC &&
      m.tag != RT_MAT_DIFFUSE_LIGHT)
    return false;
  if (m.texture < 0) return true;  // (not built by the flattener; keep the reference's work)
  const int k = S.textures[m.texture].kind;
  return k == RT_TEX_IMAGE || k == RT_TEX_CHECKER;
}

// Rebuild the winner's HitRecord exactly as its hit() wrote it, then apply the enclosing
// transforms' fix-ups innermost-first (RotateY_hit / Translate_hit post-processing).
template <int F>
RT_D void make_record(const DScene &S, f3 wo, f3 wd, const Hit &h, Rec &r) {
  f3 o = wo, d = wd;
  if ((F & RT_FEAT_XFORM) && h.xform != RT_REF_NONE) local_ray(S, h.xform, wo, wd, o, d);
  const int kind = rt_ref_kind(h.prim);
  const int32_t idx = rt_ref_index(h.prim);
  r.p = ray_at(o, d, h.t);
  r.u = r.v = 0.0f;
  r.front = true;
  r.normal = mk(0.0f, 0.0f, 0.0f);
  if (kind == RT_KIND_SPHERE) {
    const rt_sphere &s = S.spheres[idx];
    const f3 outward = scale(sub(r.p, ld3(s.center)), s.inv_radius);
    r.front = dot(d, outward) < 0.0f;
    r.normal = r.front ? outward : neg(outward);
    // u, v (glibc-exact atan2f / acosf ports) only where the material's texture reads them (image,
    // checker): every other texture ignores u, v, so skipping them changes no output
    if ((F & RT_FEAT_TEX_UV) && mat_uses_uv(S, s.material)) {
      r.u = (rtm::atan2f(-outward.z, outward.x) + kPi) * kInvPi * 0.5f;
      r.v = rtm::acosf(-outward.y) * kInvPi;
    }
    r.material = s.material;
  } else if ((F & RT_FEAT_QUAD) && kind == RT_KIND_QUAD) {
    const rt_quad &q = S.quads[idx];
    const f3 hp = sub(r.p, ld3(q.Q));
    const f3 w = ld3(q.w);
    r.u = dot(w, cross(hp, ld3(q.v)));
    r.v = dot(w, cross(ld3(q.u), hp));
    const f3 n = ld3(q.normal);
    r.front = dot(d, n) < 0.0f;
    r.normal = r.front ? n : neg(n);
    r.material = q.material;
  } else {  // medium: normal / front / u / v are stale in the reference and unused by Isotropic
    r.material = S.media[idx].phase_material;
  }
  if ((F & RT_FEAT_XFORM) && h.xform != RT_REF_NONE) {
    for (int32_t xf = h.xform; xf != RT_REF_NONE; xf = parent_of(S, xf)) {
      if (rt_ref_kind(xf) == RT_KIND_ROTATE_Y) {
        const rt_rotate_y &ry = S.rotates[rt_ref_index(xf)];
        r.p = rot_y_inv(r.p, ry.cos_theta, ry.sin_theta);
        r.normal = rot_y_inv(r.normal, ry.cos_theta, ry.sin_theta);
      } else {
        r.p = add(r.p, ld3(S.translates[rt_ref_index(xf)].offset));
      }
    }
  }
}

// ------------------------------------------------------------------------------ textures
RT_D float perlin_noise(const rt_perlin &P, f3 p) {  // src/texture.c:78-103
  const int i = (int)floorf(p.x), j = (int)floorf(p.y), k = (int)floorf(p.z);
  const float t1 = p.x - (float)i, t2 = p.y - (float)j, t3 = p.z - (float)k;
  const float s1 = t1 * t1 * (3.0f - 2.0f * t1);
  const float s2 = t2 * t2 * (3.0f - 2.0f * t2);
  const float s3 = t3 * t3 * (3.0f - 2.0f * t3);
  float value = 0;
  for (int di = 0; di < 2; di++)
    for (int dj = 0; dj < 2; dj++)
      for (int dk = 0; dk < 2; dk++) {
        const int gi = P.perm_x[(i + di) & 255] ^ P.perm_y[(j + dj) & 255] ^ P.perm_z[(k + dk) & 255];
        const f3 grad = mk(P.grad[gi][0], P.grad[gi][1], P.grad[gi][2]);
        const f3 wgt = mk(t1 - (float)di, t2 - (float)dj, t3 - (float)dk);
        value += dot(grad, wgt) * ((float)di * s1 + (float)(1 - di) * (1.0f - s1)) *
                 ((float)dj * s2 + (float)(1 - dj) * (1.0f - s2)) * ((float)dk * s3 + (float)(1 - dk) * (1.0f - s3));
      }
  return value;
}

// The general kernel's copy of a scene's single Perlin texture in LDS (rt_general.h): the permutations
// as bytes (x | y | z, 256 each; host-checked < 256) and the gradients as float4, so the 7 octaves x 8
// corners of table reads per texture value are LDS reads, not scattered global loads.  Same values,
// same arithmetic as perlin_noise.
struct PerlinLds {
  const uint8_t *perm;
  const float4 *grad;
};
constexpr size_t kPerlinLdsBytes = 3 * 256 + 256 * sizeof(float4);
RT_D float perlin_noise_lds(const PerlinLds &P, f3 p) {  // src/texture.c:78-103
  const int i = (int)floorf(p.x), j = (int)floorf(p.y), k = (int)floorf(p.z);
  const float t1 = p.x - (float)i, t2 = p.y - (float)j, t3 = p.z - (float)k;
  const float s1 = t1 * t1 * (3.0f - 2.0f * t1);
  const float s2 = t2 * t2 * (3.0f - 2.0f * t2);
  const float s3 = t3 * t3 * (3.0f - 2.0f * t3);
  float value = 0;
  for (int di = 0; di < 2; di++)
    for (int dj = 0; dj < 2; dj++)
      for (int dk = 0; dk < 2; dk++) {
        const int gi = P.perm[(i + di) & 255] ^ P.perm[256 + ((j + dj) & 255)] ^ P.perm[512 + ((k + dk) & 255)];
        const float4 gq = P.grad[gi];
        const f3 grad = mk(gq.x, gq.y, gq.z);
        const f3 wgt = mk(t1 - (float)di, t2 - (float)dj, t3 - (float)dk);
        value += dot(grad, wgt) * ((float)di * s1 + (float)(1 - di) * (1.0f - s1)) *
                 ((float)dj * s2 + (float)(1 - dj) * (1.0f - s2)) * ((float)dk * s3 + (float)(1 - dk) * (1.0f - s3));
      }
  return value;
}

// pl: perlins[0]'s LDS copy (pl.perm null: none).  solid (optional): the solid texture the value
// came from (its colour, as is), -1 otherwise.
RT_D f3 texture_value(const DScene &S, int32_t tex, float u, float v, f3 p, PerlinLds pl = PerlinLds{nullptr, nullptr},
                      int32_t *solid = nullptr) {
  if (solid) *solid = -1;
  for (int hops = 0; hops < 16; hops++) {
    const rt_texture &t = S.textures[tex];
    if (t.kind == RT_TEX_SOLID) {
      if (solid) *solid = tex;
      return ld3(t.color);
    }
    if (t.kind == RT_TEX_CHECKER) {  // src/texture.c:12-22
      const int iu = (int)floorf(u / t.scale);
      const int iv = (int)floorf(v / t.scale);
      tex = ((iu + iv) % 2) ? t.b : t.a;
      continue;
    }
    if (t.kind == RT_TEX_IMAGE) {  // src/texture.c:28-37
      const rt_image im = S.images[t.a];
      int i = (int)roundf(u * (float)(im.width - 1));
      int j = (int)roundf((1.0f - v) * (float)(im.height - 1));
      i = i < 0 ? 0 : (i > im.width - 1 ? im.width - 1 : i);  // memory safety only: in range for
      j = j < 0 ? 0 : (j > im.height - 1 ? im.height - 1 : j);  // u,v in [0,1]
      const uint8_t *px = S.image_bytes + im.offset + ((int64_t)j * im.width + i) * 3;
      return mk((float)px[0] / 255.0f, (float)px[1] / 255.0f, (float)px[2] / 255.0f);
    }
    // PERLIN: marble (src/texture.c:47-52, :105-114)
    const rt_perlin &P = S.perlins[t.a];
    f3 q = scale(p, t.scale);
    const f3 q0 = q;
    float acc = 0.0f, weight = 1.0f;
    const bool in_lds = pl.perm != nullptr && t.a == 0;
    for (int o = 0; o < P.depth; o++) {
      acc += weight * (in_lds ? perlin_noise_lds(pl, q) : perlin_noise(P, q));
      weight *= 0.5f;
      q = scale(q, 2.0f);
    }
    const float value = 0.5f * (1.0f + rtm::sinf(q0.z + 10.0f * fabsf(acc)));
    return mk(value, value, value);
  }
  return mk(0.0f, 0.0f, 0.0f);
}

// ------------------------------------------------------------------------------ materials
struct Onb {
  f3 u, v, w;
};
RT_D Onb onb_from_w(f3 n) {  // src/material.c:147-152
  Onb b;
  b.w = normalize(n);
  const f3 a = fabsf(b.w.x) > 0.9f ? mk(0, 1, 0) : mk(1, 0, 0);
  b.v = normalize(cross(b.w, a));
  b.u = cross(b.w, b.v);
  return b;
}
RT_D f3 onb_local(const Onb &b, f3 a) { return add(add(scale(b.u, a.x), scale(b.v, a.y)), scale(b.w, a.z)); }
RT_D f3 reflect(f3 v, f3 n) { return sub(v, scale(n, 2.0f * dot(v, n))); }

template <int F>
RT_D f3 emit(const DScene &S, const Rec &r, PerlinLds pl = PerlinLds{nullptr, nullptr}) {  // Material_emit, src/material.c:133-142
  if (F & RT_FEAT_EMISSIVE) {
    const rt_material &m = S.materials[r.material];
    if (m.tag == RT_MAT_SURFACE_NORMAL) return scale(add(r.normal, mk(1.0f, 1.0f, 1.0f)), 0.5f);
    if (m.tag == RT_MAT_DIFFUSE_LIGHT && r.front) return texture_value(S, m.texture, r.u, r.v, r.p, pl);
  }
  return mk(0.0f, 0.0f, 0.0f);
}

// Material_scatter (src/material.c:103-120).  Returns false when the path ends at this hit.
// solid (optional): the solid texture the albedo is the colour of, kUnitAlbedo for (1, 1, 1), else -1.
constexpr int32_t kUnitAlbedo = -2;
template <int F>
RT_D bool scatter(const DScene &S, const Rec &r, f3 r_in, Pcg32 &g, f3 &out, f3 &albedo, bool &skip_pdf,
                  PerlinLds pl = PerlinLds{nullptr, nullptr}, int32_t *solid = nullptr) {
  const rt_material &m = S.materials[r.material];
  switch (m.tag) {
  case RT_MAT_LAMBERTIAN: {  // src/material.c:23-37
    const Onb b = onb_from_w(r.normal);
    const float r1 = g.f32();
    const float r2 = g.f32();
    const float phi = (2.0f * kPi) * r1;
    float sphi, cphi;
    rtm::sincosf(phi, &sphi, &cphi);
    const float sq = sqrtf(r2);
    out = onb_local(b, mk(cphi * sq, sphi * sq, sqrtf(1.0f - r2)));
    albedo = texture_value(S, m.texture, r.u, r.v, r.p, pl, solid);
    skip_pdf = false;
    return true;
  }
  case RT_MAT_METAL: {  // src/material.c:48-58
    const f3 refl = reflect(normalize(r_in), r.normal);
    out = add(refl, scale(rand_unit_vector(g), m.param));
    albedo = texture_value(S, m.texture, r.u, r.v, r.p, pl, solid);
    skip_pdf = true;
    if (dot(out, r.normal) < 0.0f) out = refl;
    return true;
  }
  case RT_MAT_DIELECTRIC: {  // src/material.c:62-86
    float eta = m.param;
    if (r.front) eta = 1.0f / eta;
    const f3 v = normalize(r_in);
    const float cos_t = fminf(-dot(v, r.normal), 1.0f);
    const float sin_t = sqrtf(1.0f - cos_t * cos_t);
    float sch = (1.0f - eta) / (1.0f + eta);
    sch *= sch;
    sch += (1 - sch) * rtm::powf(1.0f - cos_t, 5.0f);
    if (eta * sin_t > 1.0f || sch > g.f32()) {  // rng drawn only when not totally reflected
      out = reflect(v, r.normal);
    } else {
      const f3 perp = scale(add(v, scale(r.normal, cos_t)), eta);
      const f3 para = scale(r.normal, -sqrtf(fabsf(1.0f - dot(perp, perp))));
      out = add(perp, para);
    }
    albedo = mk(1.0f, 1.0f, 1.0f);
    if (solid) *solid = kUnitAlbedo;
    skip_pdf = true;
    return true;
  }
  case RT_MAT_ISOTROPIC: {  // src/material.c:93-98
    out = rand_unit_vector(g);
    albedo = texture_value(S, m.texture, r.u, r.v, r.p, pl, solid);
    skip_pdf = false;
    return true;
  }
  default:  // SURFACE_NORMAL, DIFFUSE_LIGHT
    skip_pdf = true;
    return false;
  }
}

RT_D float scatter_pdf(const DScene &S, int32_t mat, f3 normal, f3 r_out) {  // src/material.c:122-131
  const int tag = S.materials[mat].tag;
  if (tag == RT_MAT_LAMBERTIAN) {
    const float c = dot(normal, normalize(r_out));
    return c < 0.0f ? 0.0f : c / kPi;
  }
  if (tag == RT_MAT_ISOTROPIC) return 1.0f / (4.0f * kPi);
  return 0.0f;
}

// ------------------------------------------------------------------------------ light sampling
// HittableList_rand over World.lights (src/hittable.c:101-107) + Sphere_rand / Quad_rand.
RT_D f3 lights_rand(const DScene &S, f3 origin, Pcg32 &g) {
  const rt_list L = S.lists[S.lights];
  for (;;) {
    const int32_t ref = S.items[L.first + (int32_t)(g.next() % (uint32_t)L.count)];
    if (ref == RT_REF_NONE) continue;  // no rand(): rejection, as the reference recursion does
    const int32_t i = rt_ref_index(ref);
    if (rt_ref_kind(ref) == RT_KIND_QUAD) {  // src/hittable.c:225-228, gcc order: v gets draw 1
      const rt_quad &q = S.quads[i];
      const float fv = g.f32();
      const float fu = g.f32();
      return add(add(add(ld3(q.Q), scale(ld3(q.u), fu)), scale(ld3(q.v), fv)), neg(origin));
    }
    const rt_sphere &s = S.spheres[i];  // src/hittable.c:163-178
    const f3 oc = sub(ld3(s.center), origin);
    const float r1 = g.f32();
    const float r2 = g.f32();
    const float z = 1.0f + r2 * (sqrtf(1.0f - s.radius_sq / dot(oc, oc)) - 1);
    const float phi = (2.0f * kPi) * r1;
    float sphi, cphi;
    rtm::sincosf(phi, &sphi, &cphi);
    const float x = cphi * sqrtf(1.0f - z * z);
    const float y = sphi * sqrtf(1.0f - z * z);
    return onb_local(onb_from_w(oc), mk(x, y, z));
  }
}

// HittableList_pdf over World.lights (src/hittable.c:89-100) + Sphere_pdf / Quad_pdf.
RT_D float lights_pdf(const DScene &S, f3 o, f3 d) {
  const rt_list L = S.lists[S.lights];
  float pdf = 0.0f, count = 0.0f;
  for (int k = 0; k < L.count; k++) {
    const int32_t ref = S.items[L.first + k];
    if (ref == RT_REF_NONE) continue;
    const int32_t i = rt_ref_index(ref);
    float val = 0.0f, t;
    if (rt_ref_kind(ref) == RT_KIND_QUAD) {
      const rt_quad &q = S.quads[i];
      if (quad_t(q, o, d, 0.001f, __builtin_inff(), t)) {
        const float d2 = t * t * dot(d, d);
        const float c = fabsf(dot(ld3(q.normal), normalize(d)));
        val = d2 / (c * q.area);
      }
    } else {
      const rt_sphere &s = S.spheres[i];
      if (sphere_t(s, o, d, dot(d, d), 0.001f, __builtin_inff(), t)) {
        const f3 oc = sub(ld3(s.center), o);
        const float ctm = sqrtf(1.0f - s.radius_sq / dot(oc, oc));
        const float solid_angle = (2.0f * kPi) * (1.0f - ctm);
        val = 1.0f / solid_angle;
      }
    }
    pdf += val;
    count += 1.0f;
  }
  return pdf / fmaxf(count, 1.0f);
}

// ------------------------------------------------------------------------------ one sample path
// Camera_ray_color (src/raytracing.c:39-84) unrolled into a loop.  Each scattering bounce k
// records (e_k, a_k, w_k); when the path ends with tail value c, the colour is folded
// innermost-first: c = e_k + (a_k * c) [* w_k], which is the recursion's evaluation order.
// Paths longer than kMaxDepth (kDeep): the record lives in a caller-provided global-memory slot of
// max_depth entries instead of registers / scratch (rt_render_deep_kernel).
struct DeepRec {
  f3 a;
  float w;
  uint32_t weighted;
};

template <int F, bool kDeep = false>
RT_D f3 path_color(const DScene &S, f3 o, f3 d, Pcg32 &g, DeepRec *deep = nullptr) {
  constexpr bool kFull = (F & (RT_FEAT_EMISSIVE | RT_FEAT_LIGHTS)) != 0;
  // a recorded (scattering) bounce's emission is always +0: only SurfaceNormal and DiffuseLight emit
  // and neither scatters (src/material.c:103-142); the fold adds that +0 as the reference does
  f3 rec_a[kDeep ? 1 : kMaxDepth];
  float rec_w[kFull && !kDeep ? kMaxDepth : 1];
  uint64_t weighted = 0;
  int n = 0;
  f3 tail;
  const float prob = S.cam.light_prob;
  for (int depth = S.cam.max_depth;; depth--) {
    if (depth <= 0) {
      tail = mk(0.0f, 0.0f, 0.0f);
      break;
    }
    Hit h;
    if (!(S.pre ? trace_pre<F>(S, o, d, 1e-3f, g, h) : trace<F>(S, o, d, 1e-3f, g, h))) {
      tail = ld3(S.cam.background);
      break;
    }
    Rec r;
    make_record<F>(S, o, d, h, r);
    const f3 e = emit<F>(S, r);
    f3 out, albedo;
    bool skip_pdf;
    if (!scatter<F>(S, r, d, g, out, albedo, skip_pdf)) {
      tail = e;
      break;
    }
    if (kDeep) deep[n].a = albedo, deep[n].weighted = 0u;
    else rec_a[n] = albedo;
    if (kFull) {
      // mixture pdf (src/raytracing.c:56-71): only when the scene has lights and p != 0 (runtime bit:
      // a kernel variant compiled with the LIGHTS path may run a scene without lights)
      if ((F & RT_FEAT_LIGHTS) && (S.features & RT_FEAT_LIGHTS) && !skip_pdf) {
        if (g.f32() < prob) out = lights_rand(S, r.p, g);
        const float sp = scatter_pdf(S, r.material, r.normal, out);
        const float spdf = (1.0f - prob) * sp + prob * lights_pdf(S, r.p, out);
        if (kDeep) {
          deep[n].w = sp / spdf;
          deep[n].weighted = 1u;
        } else {
          rec_w[n] = sp / spdf;
          weighted |= 1ull << n;
        }
      }
    }
    n++;
    o = r.p;
    d = out;
  }
  f3 c = tail;
  for (int k = n - 1; k >= 0; k--) {
    f3 x = mul(kDeep ? deep[k].a : rec_a[k], c);
    if (kFull && (kDeep ? deep[k].weighted != 0u : ((weighted >> k) & 1) != 0))
      x = scale(x, kDeep ? deep[k].w : rec_w[k]);
    c = add(mk(0.0f, 0.0f, 0.0f), x);
  }
  return c;
}

// ------------------------------------------------------------------------------ one pixel
// Camera_render's per-pixel body (src/raytracing.c:93-131): seed, spp samples (jitter, thin-lens
// disc, primary ray, path colour), mean, gamma 2, clamp-macro semantics (NaN -> 0), truncation.
template <int F, bool kDeep = false>
RT_D void render_pixel(const DScene &S, int i, int j, uint8_t *dst, DeepRec *deep = nullptr) {
  Pcg32 g;
  g.seed((uint64_t)(17 + j), (uint64_t)(23 + i));
  const f3 du = ld3(S.cam.delta_u), dv = ld3(S.cam.delta_v), lf = ld3(S.cam.origin);
  const f3 pixel_pos = add(add(ld3(S.cam.pixel00), scale(du, (float)i)), scale(dv, (float)j));
  const bool dof = S.cam.dof_angle > 0.0f;
  f3 acc = mk(0.0f, 0.0f, 0.0f);
  for (int s = 0; s < S.cam.spp; s++) {
    const float px = g.between(-0.5f, 0.5f);
    const float py = g.between(-0.5f, 0.5f);
    f3 o = lf;
    if (dof) {  // thin-lens disc by rejection (src/raytracing.c:108-117)
      float a, b;
      for (;;) {
        a = g.between(-1.0f, 1.0f);
        b = g.between(-1.0f, 1.0f);
        if (a * a + b * b < 1.0f) break;
      }
      o = add(add(lf, scale(ld3(S.cam.disc_u), a)), scale(ld3(S.cam.disc_v), b));
    }
    const f3 d = add(add(add(pixel_pos, scale(du, px)), scale(dv, py)), neg(o));
    acc = add(acc, path_color<F, kDeep>(S, o, d, g, deep));
  }
  const float spp_f = (float)S.cam.spp;
  const float ch[3] = {acc.x, acc.y, acc.z};
  for (int c = 0; c < 3; c++) {
    float v = sqrtf(ch[c] / spp_f);
    v = v > 0.0f ? v : 0.0f;
    v = v < 0.999f ? v : 0.999f;
    dst[c] = (uint8_t)(int)(256.0f * v);
  }
}

}  // namespace rt
