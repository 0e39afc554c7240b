// rt_general.h — persistent, lane-refilling render loop for every scene (Book-2 features: quads,
// transforms, constant media, light sampling, textures).  Same arithmetic and call order as
// rt_device.h's render_pixel / path_color (bit-exact with the reference); different execution
// structure: the per-pixel sample loop and the per-sample bounce loop are flattened into one
// per-lane state machine, one bounce per iteration, and a lane that finishes its pixel takes the
// next one (wave ballot + one atomic), optionally in the longest-first order of a cost pre-pass.
// The one-lane-per-pixel kernel (rt_render_rows_kernel) keeps every lane of a wave waiting for the
// wave's slowest pixel; here a wave only waits for its slowest ray of the current bounce.
#pragma once
#include "rt_device.h"

namespace rt {
namespace gen {

constexpr int kBlock = 256;

struct GeneralView {
  DScene S;
  int32_t row0, row_stride, n_rows;
  int32_t *work_counter;     // zeroed before each launch
  const int32_t *order;      // work item order (longest-first), or null
  uint32_t *cost_out;        // cost pass: rays traced per work item, or null
  float4 *pre_out;           // cost pass: each pixel's colour sum and position (pre_word), or null
  const float4 *pre_in;      // the launch after it: pixels go on from there instead of sample 0, or null
  int32_t batch;             // kBatch: shade once this many lanes of a wave wait (RT_GEN_BATCH)
  int32_t steps;             // kBatch: preorder entries per lane per traversal iteration (RT_GEN_STEPS)
  int32_t n_lds;             // kBatch: the first n_lds preorder entries are staged in LDS (RT_GEN_LDS)
  int32_t rare_min;          // kBatch: run rare scan actions once this many lanes wait at one (RT_GEN_RARE)
  int32_t flat;              // kBatch: common entries as one straight-line block (pre_common) plus up to
                             // flat - 1 box entries in the same step (RT_GEN_FLAT, >= 1)
  unsigned long long *stats;  // diagnostic builds (-DRT_GEN_STATS): kGs* counters, summed over waves
  int32_t perlin_lds;        // kAllLds: byte offset of perlins[0]'s LDS copy (PerlinLds) behind the preorder; -1: none
  float4 *xrec;              // explicit albedos of path records beyond the register stack (XStack): kMaxDepth
                             // per thread of the grid, thread-contiguous
  float *xw;                 // pdf weights beyond the register stack (RegStack): kMaxDepth per thread
  int32_t code_bits;         // 4 (scenes of <= 13 textures) or 8: width of a path record's albedo code
};

// Path records as runs of codes in one u64 register pair (PathRuns).  A record's code is its albedo
// in b bits (b = code_bits) -- 1..2^b - 3 = the colour of solid texture code - 1, 2^b - 2 = (1, 1, 1),
// 2^b - 1 = explicit: the albedo is on the lane's explicit-albedo stack (XStack: image / noise textures,
// textures past the code range) -- and bit b: weighted, the pdf weight is on its weight stack.  Consecutive
// bounces of one code (a random walk in a medium: scene 7's subsurface sphere runs every such path
// to max_depth) are one run of (code, length - 1: 6 bits); bits 60..63 count the runs, 15 = full:
// the bounces past the runs are explicit and weighted (weight 1 when the bounce had none:
// x * 1.0f == x).  The fold reads back the same floats.
struct PathRuns {
  uint64_t w;
  int cb, code_bits, run_bits, max_runs;
  uint32_t code_mask;
};
RT_D PathRuns runs_init(int albedo_bits) {
  PathRuns R;
  R.w = 0;
  R.cb = albedo_bits;
  R.code_bits = albedo_bits + 1;
  R.run_bits = R.code_bits + 6;
  R.max_runs = 60 / R.run_bits;
  R.code_mask = (1u << R.code_bits) - 1u;
  return R;
}
// Record a bounce of this code; false when it is past the runs (store it explicitly, weighted).
RT_D bool runs_push(PathRuns &R, uint32_t code) {
  const uint32_t cnt = (uint32_t)(R.w >> 60);
  if (cnt == 15u) return false;
  if (cnt > 0u) {
    const int at = R.run_bits * (int)(cnt - 1u);
    const uint32_t last = (uint32_t)(R.w >> at) & R.code_mask;
    if (last == code) {  // (length - 1 <= 63: at most kMaxDepth bounces)
      R.w += 1ull << (at + R.code_bits);
      return true;
    }
  }
  if ((int)cnt < R.max_runs) {
    R.w |= (uint64_t)code << (R.run_bits * (int)cnt);
    R.w += 1ull << 60;
    return true;
  }
  R.w |= 15ull << 60;
  return false;
}

// The records' explicit albedos and pdf weights as two LIFO stacks whose newest entries sit in
// registers (the fold visits records newest first, i.e. in reverse push order): a push into a full
// register part moves its oldest entry to the thread's global slots, a pop refills the register part
// from there.  Scene 7 averages 4.37 records per sample, 3.9 of them weighted and 0.65 explicit
// (DESIGN.md §4.3); with 4 weights and 1 albedo in registers most paths never touch memory, where
// every record store used to leave L2 for HBM at >= 32 B.  Only static register indices (unrolled
// shifts): a dynamically indexed private array would live in scratch.
#ifndef RT_GEN_EXTRA_SL
// pre_common's extra box actions branch-free (config 5, same box, three rounds: 3243-3262 ms per frame
// against 3275-3396 with the branches)
#define RT_GEN_EXTRA_SL 1
#endif
#ifndef RT_GEN_WREG
#define RT_GEN_WREG 4  // pdf weights in registers (config 5, same box: 8 / 4 / 0 -> 274 / 276 / 271 Msamples/s)
#endif
#ifndef RT_GEN_XREG
#define RT_GEN_XREG 1  // explicit albedos in registers
#endif
#ifndef RT_GEN_SLOT_MAJOR
#define RT_GEN_SLOT_MAJOR 0
#endif
constexpr int kWReg = RT_GEN_WREG, kXReg = RT_GEN_XREG;
template <int kN>
struct RegStack {
  float v[kN > 0 ? kN : 1];
  int n;  // entries pushed and not popped (the newest min(n, kN) in v, newest first)
};
template <int kN>
RT_D void rs_push(RegStack<kN> &S, float x, float *spill, uint32_t stride = 1) {
  if constexpr (kN == 0) {
    spill[(uint32_t)S.n * stride] = x;
  } else {
    if (S.n >= kN) spill[(uint32_t)(S.n - kN) * stride] = S.v[kN - 1];
#pragma unroll
    for (int k = kN - 1; k > 0; k--) S.v[k] = S.v[k - 1];
    S.v[0] = x;
  }
  S.n++;
}
template <int kN>
RT_D float rs_pop(RegStack<kN> &S, const float *spill, uint32_t stride = 1) {
  S.n--;
  if constexpr (kN == 0) {
    return spill[(uint32_t)S.n * stride];
  } else {
    const float x = S.v[0];
#pragma unroll
    for (int k = 0; k < kN - 1; k++) S.v[k] = S.v[k + 1];
    if (S.n >= kN) S.v[kN - 1] = spill[(uint32_t)(S.n - kN) * stride];
    return x;
  }
}
template <int kN>
struct XStack {  // explicit albedos
  f3 v[kN > 0 ? kN : 1];
  int n;
};
template <int kN>
RT_D void xs_push(XStack<kN> &S, f3 x, float4 *spill, uint32_t stride = 1) {
  if constexpr (kN == 0) {
    spill[(uint32_t)S.n * stride] = make_float4(x.x, x.y, x.z, 0.0f);
  } else {
    if (S.n >= kN) spill[(uint32_t)(S.n - kN) * stride] = make_float4(S.v[kN - 1].x, S.v[kN - 1].y, S.v[kN - 1].z, 0.0f);
#pragma unroll
    for (int k = kN - 1; k > 0; k--) S.v[k] = S.v[k - 1];
    S.v[0] = x;
  }
  S.n++;
}
template <int kN>
RT_D f3 xs_pop(XStack<kN> &S, const float4 *spill, uint32_t stride = 1) {
  S.n--;
  if constexpr (kN == 0) {
    const float4 e = spill[(uint32_t)S.n * stride];
    return mk(e.x, e.y, e.z);
  } else {
    const f3 x = S.v[0];
#pragma unroll
    for (int k = 0; k < kN - 1; k++) S.v[k] = S.v[k + 1];
    if (S.n >= kN) {
      const float4 e = spill[(uint32_t)(S.n - kN) * stride];
      S.v[kN - 1] = mk(e.x, e.y, e.z);
    }
    return x;
  }
}

// ---- a path's record: what Camera_ray_color's recursion keeps on its stack (src/raytracing.c:39-75)
// per scattered bounce k: the albedo a_k and, on the light-mixture branch, the pdf weight w_k; the fold
// computes c = 0 + (a_k (x) c) * w_k innermost first from the path's tail, as the recursion returns
// (src/raytracing.c:57, :69-71).  Albedos as run-length codes (PathRuns) or on the explicit stack
// (XStack); weights on the weight stack (RegStack), except a weight of exactly 2.0f -- sp / (0.5f sp)
// for a direction that misses every light (lights_pdf 0 at light_prob 0.5), 47 % of scene 7's
// weights -- which is one bit of w2 (bounce index k < kMaxDepth = 64) and takes no stack slot.
// tests/native/stack_check.cpp checks push and fold against a plain array fold at every stack depth.
template <int kW, int kX>
struct PathRecord {
  PathRuns runs;
  RegStack<kW> wst;
  XStack<kX> xst;
  uint64_t w2;      // bit k: bounce k's weight is 2.0f
  uint32_t nonfin;  // channels (bit c: channel c) a non-finite record value poisons; a weight: all three
  int n;            // bounces recorded
};
template <int kW, int kX>
RT_D void rec_init(PathRecord<kW, kX> &P, int albedo_bits) {
  P.runs = runs_init(albedo_bits);
#pragma unroll
  for (int k = 0; k < (kW > 0 ? kW : 1); k++) P.wst.v[k] = 1.0f;
#pragma unroll
  for (int k = 0; k < (kX > 0 ? kX : 1); k++) P.xst.v[k] = mk(0.0f, 0.0f, 0.0f);
  P.wst.n = P.xst.n = 0;
  P.w2 = 0;
  P.nonfin = 0;
  P.n = 0;
}
template <int kW, int kX>
RT_D void rec_clear(PathRecord<kW, kX> &P) {  // a new sample
  P.runs.w = 0;
  P.wst.n = P.xst.n = 0;
  P.w2 = 0;
  P.nonfin = 0;
  P.n = 0;
}
// Bounce P.n: `code` is its albedo code (PathRuns: a solid texture's, the unit albedo's, or explicit),
// plus the weighted bit when it has a pdf weight w (else w is 1.0f and unused).  xrec / xw: the thread's
// kMaxDepth slots for what leaves the register stacks.
template <int kW, int kX>
RT_D void rec_push(PathRecord<kW, kX> &P, uint32_t code, f3 albedo, float w, float4 *xrec, float *xw,
                   uint32_t stride = 1) {
  const uint32_t code_explicit = (1u << P.runs.cb) - 1u, code_weighted = 1u << P.runs.cb;
  if (!runs_push(P.runs, code)) code = code_explicit | code_weighted;  // past the runs: explicit, weighted
  if ((code & code_explicit) == code_explicit) xs_push(P.xst, albedo, xrec, stride);
  if ((code & code_weighted) && w == 2.0f) P.w2 |= 1ull << P.n;
  else if (code & code_weighted) rs_push(P.wst, w, xw, stride);
  P.nonfin |= (uint32_t)!__builtin_isfinite(albedo.x) | ((uint32_t)!__builtin_isfinite(albedo.y) << 1) |
              ((uint32_t)!__builtin_isfinite(albedo.z) << 2) | (__builtin_isfinite(w) ? 0u : 7u);
  P.n++;
}
// The path's colour from its tail (the last bounce's return value: background, emission, or 0 at the
// depth cut).  colors: the solid textures' colours by code - 1.
// Zero tails: when the tail is zero in every channel (a miss into a black background -- scene 7,
// src/main.c:269 --, the depth cut, src/raytracing.c:40-41, the back face of a light) and every record
// value is finite, each step maps +-0 to +0, so c = +0 -- returned without the fold and without
// reloading the records stored beyond the registers (scene 7: 48 % of paths, holding 54 % of those
// entries).  acc + (+0) == acc bit for bit (acc is never -0: it starts at +0).
template <int kW, int kX, typename Colors>
RT_D f3 rec_fold(PathRecord<kW, kX> &P, f3 tail, const Colors &colors, const float4 *xrec, const float *xw,
                 uint32_t stride = 1) {
  if (tail.x == 0.0f && tail.y == 0.0f && tail.z == 0.0f && P.nonfin == 0u) return mk(0.0f, 0.0f, 0.0f);
  const PathRuns &R = P.runs;
  const uint32_t code_explicit = (1u << R.cb) - 1u, code_unit = code_explicit - 1u, code_weighted = 1u << R.cb;
  f3 c = tail;
  const uint32_t cnt = (uint32_t)(R.w >> 60);
  const int nr = cnt == 15u ? R.max_runs : (int)cnt;
  int covered = 0;  // bounces in the runs; those past them are explicit and weighted
  for (int r = 0; r < nr; r++) covered += (int)((R.w >> (R.run_bits * r + R.code_bits)) & 63u) + 1;
  int r = nr - 1, left = 0;  // the run bounce k is in, and its bounces not yet folded
  uint32_t code = code_explicit | code_weighted;
  f3 a = mk(1.0f, 1.0f, 1.0f);
  for (int k = P.n - 1; k >= 0; k--) {
    if (k < covered) {
      if (left == 0) {  // enter the next run down
        code = (uint32_t)(R.w >> (R.run_bits * r)) & R.code_mask;
        left = (int)((R.w >> (R.run_bits * r + R.code_bits)) & 63u) + 1;
        r--;
        const uint32_t ca = code & code_explicit;
        if (ca != code_explicit) a = ca == code_unit ? mk(1.0f, 1.0f, 1.0f) : colors(ca - 1u);
      }
      left--;
    }
    if ((code & code_explicit) == code_explicit) a = xs_pop(P.xst, xrec, stride);
    f3 x = mul(a, c);
    if (code & code_weighted) x = scale(x, (P.w2 >> k) & 1ull ? 2.0f : rs_pop(P.wst, xw, stride));
    c = add(mk(0.0f, 0.0f, 0.0f), x);
  }
  return c;
}

// -DRT_GEN_STATS: per-wave cycle and lane counters of the batched loop (wave-uniform, s_memtime)
enum {
  kGsIterRefill = 0, kGsIterTrace, kGsIterShade,  // cycles of loop iterations by what they ran
  kGsTraceIters, kGsTraceLanes, kGsShadeIters, kGsShadeLanes,
  kGsStepKinds,                                     // sum over trace steps of distinct entry kinds present
  kGsKindBox, kGsKindSphere, kGsKindQuad, kGsKindXform, kGsKindMedium, kGsKindOther,  // lane-steps per kind
  kGsCycRecord, kGsCycEmit, kGsCycScatter, kGsCycLights, kGsCycFold,
  kGsMatLam, kGsMatMetal, kGsMatDiel, kGsMatIso, kGsMatEnd,  // shaded lanes by material
  kGsTexSolid, kGsTexChecker, kGsTexImage, kGsTexPerlin,     // shaded lanes by (first) texture kind
  kGsCycScatterPerlin, kGsPassPerlin, kGsMiss, kGsCycCamera, kGsCycBegin, kGsCycTop, kGsCycClassify, kGsCycCommon, kGsCycRare, kGsRareSteps, kGsCycBounce, kGsCycWrite,
  // per-lane counters from here on (summed over every lane)
  kGsRecords, kGsExplicit, kGsWeighted,
  kGsPaths, kGsPathZero, kGsPathTrunc, kGsPathTruncZero,  // paths with records; zero tail; outgrew the stacks
  kGsSpillSt, kGsSpillStZero,                             // stack entries beyond the registers (all / zero-tail paths)
  kGsW2, kGsFoldSkips,                                    // weights == 2.0f; folds skipped (zero tail)
  kGsN
};
constexpr int kGsPerLane = kGsRecords;

// ---- the phased scan: pre_step (rt_device.h) split into a class test and an execution, so that a
// wave runs the rare, expensive entries -- leaving a transform's subtree, entering one (local_ray +
// three divisions), a constant medium (two boundary roots + logf) -- only when enough of its lanes
// wait at one (rare_min) or nothing else is left, instead of in nearly every step for one lane: at
// scene 7, 1.5 % of lane-steps are media and 1.7 % transforms, yet ~40 % of wave-steps held one of
// each.  A lane's own sequence of entries, t_max updates and rng draws is pre_step's, so deferral
// changes timing only.  Boxes run branch-free and spheres on the exact cores (rt_device.h).

// The hoisted per-frame terms of T.d.
RT_D void pre_frame_terms(PreTrace &T) {
  T.inv = mk(1.0f / T.d.x, 1.0f / T.d.y, 1.0f / T.d.z);
  T.dd = dot(T.d, T.d);
  T.ra = recip_core(T.dd);
  T.fast = T.dd >= kDivLo && T.dd <= kDivHi;
}
// A preorder array: entries as (q0, q1) pairs -- the global S.pre -- or, under RT_GEN_SPLIT, the LDS copy
// as two arrays, every entry's q0 then every entry's q1 `half` entries further (rt_book1.h's item split:
// a ds_read_b128 of random entries then spreads over every bank instead of half of them).
struct PrePairs {
  const float4 *p;
  RT_D float4 q0(uint32_t q) const { return p[2 * q]; }
  RT_D float4 q1(uint32_t q) const { return p[2 * q + 1]; }
};
struct PreSplit {
  const float4 *p;
  uint32_t half;
  RT_D float4 q0(uint32_t q) const { return p[q]; }
  RT_D float4 q1(uint32_t q) const { return p[half + q]; }
};
#ifndef RT_GEN_SPLIT
#define RT_GEN_SPLIT 0
#endif

// Apply the transform of preorder entry `pos` to (o, d): one step of local_ray's chain (translate:
// o - offset; rotate_y: rot_y of o and d), from the entry's inline words.
template <typename PA>
RT_D void pre_apply_xform(PA pre, uint32_t pos, f3 &o, f3 &d) {
  const float4 q0 = pre.q0(pos), q1 = pre.q1(pos);
  if (rt_ref_kind((int32_t)__builtin_bit_cast(uint32_t, q1.w)) == RT_KIND_TRANSLATE) {
    o = sub(o, mk(q0.y, q0.w, q1.x));
  } else {
    o = rot_y(o, q0.y, q0.w);
    d = rot_y(d, q0.y, q0.w);
  }
}
// The ray in the frame whose transform entry is at `pos` (~0: the world), from the world ray:
// local_ray's chain outermost first, walking the entries' enclosing positions (depth <= 8).
template <typename PA>
RT_D void pre_chain_ray(PA pre, uint32_t pos, f3 wo, f3 wd, f3 &o, f3 &d) {
  int depth = 0;
  for (uint32_t q = pos; q != 0xffffffffu && depth < 8; q = __builtin_bit_cast(uint32_t, pre.q0(q).z)) depth++;
  o = wo, d = wd;
  for (int lvl = depth - 1; lvl >= 0; lvl--) {
    uint32_t q = pos;
    for (int k = 0; k < lvl; k++) q = __builtin_bit_cast(uint32_t, pre.q0(q).z);
    pre_apply_xform(pre, q, o, d);
  }
}

// Sphere_hit's two candidate roots (-b -/+ sqrt(disc)) / a for the sphere q = (centre, r^2) on the
// exact cores (a = T.dd, its reciprocal hoisted per frame), the reference expression for lanes
// outside the cores' ranges; false when disc < 0 (no root).
RT_D bool sphere_roots(float4 q, f3 o, f3 d, const PreTrace &T, float &r1, float &r2) {
  const f3 oc = sub(o, mk(q.x, q.y, q.z));
  const float b = dot(oc, d);
  const float c = dot(oc, oc) - q.w;
  const float disc = b * b - T.dd * c;
  float sq = sqrt_core(disc);
  r1 = div_core(-b - sq, T.dd, T.ra), r2 = div_core(-b + sq, T.dd, T.ra);
  const bool ok = (int)T.fast & ((int)(disc == 0.0f) | ((int)(disc >= kSqrtLo) & (int)(disc <= __FLT_MAX__))) &
                  (int)(fabsf(-b - sq) <= kNumHi) & (int)(fabsf(-b + sq) <= kNumHi);
  if (__builtin_expect(!(disc < 0) && !ok, 0)) {
    sq = sqrtf(disc);
    r1 = (-b - sq) / T.dd;
    r2 = (-b + sq) / T.dd;
  }
  return !(disc < 0);
}

// true when the lane's next action is a rare one (q1: its entry, loaded by the caller)
template <int F>
RT_D bool pre_is_rare(const PreTrace &T, float4 q1) {
  if ((F & RT_FEAT_XFORM) && T.p >= T.fend) return true;
  const int kind = rt_ref_kind((int32_t)__builtin_bit_cast(uint32_t, q1.w));
  return ((F & RT_FEAT_XFORM) && (kind == RT_KIND_TRANSLATE || kind == RT_KIND_ROTATE_Y)) ||
         ((F & RT_FEAT_MEDIUM) && kind == RT_KIND_MEDIUM);
}

// One action of the scan (pre_step's, for the entry q0/q1 at T.p); true once past the last entry.
// Leaving transform subtrees is an action of its own: the entry at T.p then runs in a later step.
// pre: the preorder (S.pre, or its LDS copy when the whole of it is there: plain ds_read, no flat).
template <int F, typename PA>
RT_D bool pre_exec(const DScene &S, PA pre, PreTrace &T, f3 wo, f3 wd, float tmin, Pcg32 &g, float4 q0,
                   float4 q1) {
  const uint32_t n = (uint32_t)S.n_pre;
  if (T.p >= n) return true;
  if ((F & RT_FEAT_XFORM) && T.p >= T.fend) {
    uint32_t pp;
    do {  // leaving a transform's subtree: the enclosing frame again (its ref sits in its entry)
      pp = __builtin_bit_cast(uint32_t, pre.q0(T.fpos).z);
      const bool top = pp == 0xffffffffu;
      T.frame = top ? RT_REF_NONE : (int32_t)__builtin_bit_cast(uint32_t, pre.q1(pp).w);
      T.fend = top ? 0xffffffffu : __builtin_bit_cast(uint32_t, pre.q0(pp).x);
      T.fpos = top ? 0u : pp;
    } while (T.p >= T.fend);
    pre_chain_ray(pre, pp, wo, wd, T.o, T.d);
    pre_frame_terms(T);
    return false;
  }
  const int32_t ref = (int32_t)__builtin_bit_cast(uint32_t, q1.w);
  const int kind = rt_ref_kind(ref);
  const int32_t idx = rt_ref_index(ref);
  const f3 o = T.o, d = T.d;
  uint32_t next = T.p + 1;
  float t = 0.0f;
  bool hit = false;
  if ((F & RT_FEAT_BVH) && kind == RT_KIND_BVH) {
    // AABB_hit with the three slabs evaluated together (rt_book1.h: aabb_packed): t_min / t_max
    // only tighten and fmaxf / fminf ignore NaN, so one test at the end equals the early exits
    const float ix = T.inv.x, iy = T.inv.y, iz = T.inv.z;
    const float ax = (q0.x - o.x) * ix, bx = (q0.w - o.x) * ix;
    const float ay = (q0.y - o.y) * iy, by = (q1.x - o.y) * iy;
    const float az = (q0.z - o.z) * iz, bz = (q1.y - o.z) * iz;
    const float lo = fmaxf(fmaxf(fmaxf(tmin, ix < 0 ? bx : ax), iy < 0 ? by : ay), iz < 0 ? bz : az);
    const float hi = fminf(fminf(fminf(T.tmax, ix < 0 ? ax : bx), iy < 0 ? ay : by), iz < 0 ? az : bz);
    if (hi <= lo) next = __builtin_bit_cast(uint32_t, q1.z);
  } else if (kind == RT_KIND_SPHERE) {
    // Sphere_hit (src/hittable.c:120-138) on the exact cores, as rt_book1.h's sphere_test_data;
    // lanes outside the cores' ranges evaluate the reference expression
    const f3 oc = sub(o, mk(q0.x, q0.y, q0.z));
    const float b = dot(oc, d);
    const float c = dot(oc, oc) - q0.w;
    const float disc = b * b - T.dd * c;
    if (!(disc < 0)) {
      float sq = sqrt_core(disc);
      float r1 = div_core(-b - sq, T.dd, T.ra), r2 = div_core(-b + sq, T.dd, T.ra);
      const bool ok = (int)T.fast & ((int)(disc == 0.0f) | ((int)(disc >= kSqrtLo) & (int)(disc <= __FLT_MAX__))) &
                      (int)(fabsf(-b - sq) <= kNumHi) & (int)(fabsf(-b + sq) <= kNumHi);
      if (__builtin_expect(!ok, 0)) {
        sq = sqrtf(disc);
        r1 = (-b - sq) / T.dd;
        r2 = (-b + sq) / T.dd;
      }
      const bool take1 = !(r1 <= tmin || r1 >= T.tmax), take2 = !(r2 <= tmin || r2 >= T.tmax);
      hit = take1 || take2;
      t = take1 ? r1 : r2;
    }
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
    // entering: the current frame is this transform's enclosing one, so applying this transform
    // to the current ray is local_ray's chain one step further (same operations, same order)
    T.frame = ref;
    T.fend = __builtin_bit_cast(uint32_t, q0.x);
    T.fpos = T.p;
    if (kind == RT_KIND_TRANSLATE) {
      T.o = sub(T.o, mk(q0.y, q0.w, q1.x));  // d and its terms unchanged
    } else {
      T.o = rot_y(T.o, q0.y, q0.w);
      T.d = rot_y(T.d, q0.y, q0.w);
      pre_frame_terms(T);
    }
  } else if ((F & RT_FEAT_MEDIUM) && kind == RT_KIND_MEDIUM) {
    // ConstantMedium_hit (src/hittable.c:392-423), as pre_step
    const bool inl = __builtin_bit_cast(uint32_t, q1.y) == 1u;
    float t1, t2, nid;
    bool both;
    if (inl) {
      // the two Sphere_hit calls solve the same quadratic (same o, d, centre): its roots once, on
      // the exact cores (a = |d|^2 = T.dd), then each call's acceptance test on them
      float r1, r2;
      const bool real = sphere_roots(q0, o, d, T, r1, r2);
      const float ninf = -__builtin_inff(), pinf = __builtin_inff();
      const bool a1 = !(r1 <= ninf || r1 >= pinf), a2 = !(r2 <= ninf || r2 >= pinf);
      t1 = a1 ? r1 : r2;
      const float lo2 = t1 + 0.0001f;
      const bool b1 = !(r1 <= lo2 || r1 >= pinf), b2 = !(r2 <= lo2 || r2 >= pinf);
      t2 = b1 ? r1 : r2;
      both = real && (a1 || a2) && (b1 || b2);
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

// The common entries (BVH box, sphere, quad) as one block: every lane evaluates the box slabs, and
// the sphere roots and the quad plane when any lane of the wave sits at a sphere / quad (wave-
// uniform branches), for its entry and keeps the result of its kind -- no per-lane kind branches;
// only the quad's in-plane test (its record: measured no faster when loaded up front) and the
// sphere's out-of-range fallback branch.
// Results equal pre_exec's for the same entry.  Precondition: T.p < n (a tracing lane's entry).
// (Sphere / quad lanes waiting for company while lanes sit at boxes, as rt_book1.h's measured leaf
// wait: 8 / 16 lanes 14 / 58 % slower on config 5, r04.)
template <int F, typename PA>
RT_D bool pre_common(const DScene &S, PA pre, PreTrace &T, float tmin, float4 q0, float4 q1,
                     int extra = 0) {
  const int32_t ref = (int32_t)__builtin_bit_cast(uint32_t, q1.w);
  const int kind = rt_ref_kind(ref);
  const f3 o = T.o, d = T.d;
  // box: q0 = (lo.x, lo.y, lo.z, hi.x), q1 = (hi.y, hi.z, skip, ref)
  const float ix = T.inv.x, iy = T.inv.y, iz = T.inv.z;
  const float ax = (q0.x - o.x) * ix, bx = (q0.w - o.x) * ix;
  const float ay = (q0.y - o.y) * iy, by = (q1.x - o.y) * iy;
  const float az = (q0.z - o.z) * iz, bz = (q1.y - o.z) * iz;
  const float lo = fmaxf(fmaxf(fmaxf(tmin, ix < 0 ? bx : ax), iy < 0 ? by : ay), iz < 0 ? bz : az);
  const float hi = fminf(fminf(fminf(T.tmax, ix < 0 ? ax : bx), iy < 0 ? ay : by), iz < 0 ? az : bz);
  const bool skip = ((F & RT_FEAT_BVH) && kind == RT_KIND_BVH) && hi <= lo;
  // sphere: q0 = (center, r^2); quad: q0 = (normal, D), the record only past the plane test.  Each
  // block runs only when a lane of the wave sits at its kind (a wave-uniform branch: scene 7 +3 %)
  bool hit = false;
  float t = 0.0f;
  if (__ballot(kind == RT_KIND_SPHERE) != 0ull) {
    const f3 oc = sub(o, mk(q0.x, q0.y, q0.z));
    const float b = dot(oc, d);
    const float c = dot(oc, oc) - q0.w;
    const float disc = b * b - T.dd * c;
    float sq = sqrt_core(disc);
    float r1 = div_core(-b - sq, T.dd, T.ra), r2 = div_core(-b + sq, T.dd, T.ra);
    const bool ok = (int)T.fast & ((int)(disc == 0.0f) | ((int)(disc >= kSqrtLo) & (int)(disc <= __FLT_MAX__))) &
                    (int)(fabsf(-b - sq) <= kNumHi) & (int)(fabsf(-b + sq) <= kNumHi);
    if (__builtin_expect(kind == RT_KIND_SPHERE && !(disc < 0) && !ok, 0)) {
      sq = sqrtf(disc);
      r1 = (-b - sq) / T.dd;
      r2 = (-b + sq) / T.dd;
    }
    const bool take1 = !(r1 <= tmin || r1 >= T.tmax), take2 = !(r2 <= tmin || r2 >= T.tmax);
    hit = kind == RT_KIND_SPHERE && !(disc < 0) && (take1 || take2);
    t = take1 ? r1 : r2;
  }
  if ((F & RT_FEAT_QUAD) && __ballot(kind == RT_KIND_QUAD) != 0ull) {
    const f3 nq = mk(q0.x, q0.y, q0.z);
    const float denom = dot(nq, d);
    const float tt = (q0.w - dot(nq, o)) / denom;
    if (kind == RT_KIND_QUAD && !(fabsf(denom) < 1e-8f) && !((tt < tmin) || (tt > T.tmax))) {
      const rt_quad &qd = S.quads[rt_ref_index(ref)];
      const f3 hp = sub(ray_at(o, d, tt), ld3(qd.Q));
      const f3 w = ld3(qd.w);
      const float alpha = dot(w, cross(hp, ld3(qd.v)));
      const float beta = dot(w, cross(ld3(qd.u), hp));
      hit = !((alpha < 0) || (alpha > 1) || (beta < 0) || (beta > 1));
      t = tt;
    }
  }
  if (hit) {
    T.tmax = t;
    T.h.t = t;
    T.h.prim = ref;
    T.h.xform = T.frame;
    T.found = true;
  }
  uint32_t next = skip ? __builtin_bit_cast(uint32_t, q1.z) : T.p + 1;
  // up to `extra` further actions in the same step while the next entry is a box (two thirds of the
  // scan): their LDS reads and slab tests overlap the sphere / quad chains above (T.tmax as those
  // left it); any other entry, or leaving a frame, waits for the next step
  // (the first one straight-line, the rest in a loop: the loop's overhead measured costly at one)
#if RT_GEN_EXTRA_SL
  // (RT_GEN_EXTRA_SL: the two extra box actions branch-free -- every lane reads an entry, its next one
  // or, without one, its current one again -- so the step has no divergent branches there: fewer
  // exec-mask instructions per step, one more LDS read for the lanes that stop)
  bool more = extra > 0 && next < (uint32_t)S.n_pre && next < T.fend;
#pragma unroll
  for (int e = 0; e < 2; e++) {
    const bool go = more && extra > e && next < (uint32_t)S.n_pre && next < T.fend;
    const uint32_t q = go ? next : T.p;
    const float4 r0 = pre.q0(q), r1 = pre.q1(q);
    const float cx = (r0.x - o.x) * ix, dx = (r0.w - o.x) * ix;
    const float cy = (r0.y - o.y) * iy, dy = (r1.x - o.y) * iy;
    const float cz = (r0.z - o.z) * iz, dz = (r1.y - o.z) * iz;
    const float lo2 = fmaxf(fmaxf(fmaxf(tmin, ix < 0 ? dx : cx), iy < 0 ? dy : cy), iz < 0 ? dz : cz);
    const float hi2 = fminf(fminf(fminf(T.tmax, ix < 0 ? cx : dx), iy < 0 ? cy : dy), iz < 0 ? cz : dz);
    more = go && rt_ref_kind((int32_t)__builtin_bit_cast(uint32_t, r1.w)) == RT_KIND_BVH;
    next = more ? (hi2 <= lo2 ? __builtin_bit_cast(uint32_t, r1.z) : next + 1) : next;
  }
#else
  bool more = extra > 0 && next < (uint32_t)S.n_pre && next < T.fend;
  if (more) {
    const float4 r0 = pre.q0(next), r1 = pre.q1(next);
    const float cx = (r0.x - o.x) * ix, dx = (r0.w - o.x) * ix;
    const float cy = (r0.y - o.y) * iy, dy = (r1.x - o.y) * iy;
    const float cz = (r0.z - o.z) * iz, dz = (r1.y - o.z) * iz;
    const float lo2 = fmaxf(fmaxf(fmaxf(tmin, ix < 0 ? dx : cx), iy < 0 ? dy : cy), iz < 0 ? dz : cz);
    const float hi2 = fminf(fminf(fminf(T.tmax, ix < 0 ? cx : dx), iy < 0 ? cy : dy), iz < 0 ? cz : dz);
    more = rt_ref_kind((int32_t)__builtin_bit_cast(uint32_t, r1.w)) == RT_KIND_BVH;
    if (more) next = hi2 <= lo2 ? __builtin_bit_cast(uint32_t, r1.z) : next + 1;
  }
  // the second extra action straight-line as well (extra == 2, the default), further ones looped
  if (more && extra >= 2 && next < (uint32_t)S.n_pre && next < T.fend) {
    const float4 r0 = pre.q0(next), r1 = pre.q1(next);
    const float cx = (r0.x - o.x) * ix, dx = (r0.w - o.x) * ix;
    const float cy = (r0.y - o.y) * iy, dy = (r1.x - o.y) * iy;
    const float cz = (r0.z - o.z) * iz, dz = (r1.y - o.z) * iz;
    const float lo2 = fmaxf(fmaxf(fmaxf(tmin, ix < 0 ? dx : cx), iy < 0 ? dy : cy), iz < 0 ? dz : cz);
    const float hi2 = fminf(fminf(fminf(T.tmax, ix < 0 ? cx : dx), iy < 0 ? cy : dy), iz < 0 ? cz : dz);
    more = rt_ref_kind((int32_t)__builtin_bit_cast(uint32_t, r1.w)) == RT_KIND_BVH;
    if (more) next = hi2 <= lo2 ? __builtin_bit_cast(uint32_t, r1.z) : next + 1;
  }
#endif
#pragma unroll 1
  for (int e = 2; more && e < extra && next < (uint32_t)S.n_pre && next < T.fend; e++) {
    const float4 r0 = pre.q0(next), r1 = pre.q1(next);
    const float cx = (r0.x - o.x) * ix, dx = (r0.w - o.x) * ix;
    const float cy = (r0.y - o.y) * iy, dy = (r1.x - o.y) * iy;
    const float cz = (r0.z - o.z) * iz, dz = (r1.y - o.z) * iz;
    const float lo2 = fmaxf(fmaxf(fmaxf(tmin, ix < 0 ? dx : cx), iy < 0 ? dy : cy), iz < 0 ? dz : cz);
    const float hi2 = fminf(fminf(fminf(T.tmax, ix < 0 ? cx : dx), iy < 0 ? cy : dy), iz < 0 ? cz : dz);
    if (rt_ref_kind((int32_t)__builtin_bit_cast(uint32_t, r1.w)) != RT_KIND_BVH) break;
    next = hi2 <= lo2 ? __builtin_bit_cast(uint32_t, r1.z) : next + 1;
  }
  T.p = next;
  return next >= (uint32_t)S.n_pre;
}

// kBatch (scenes with a preorder, S.pre): the trace runs a few entries per wave iteration
// (pre_step) and a wave shades only once `batch` of its lanes wait -- as rt_book1.h's v3 loop --
// instead of every lane waiting for the wave's longest trace each bounce.
// kAllLds: the whole preorder is in LDS (the 768/1024-thread kernels), so the scan reads only LDS.
template <int F, bool kBatch = false, bool kAllLds = false>
__device__ void render_general(const GeneralView &V, uint8_t *__restrict__ out, float4 *lds = nullptr) {
  const DScene &S = V.S;
  const uint32_t n_lds = kBatch && lds ? (uint32_t)min(V.n_lds, S.n_pre) : 0u;
  PerlinLds pl = PerlinLds{nullptr, nullptr};
  if (kAllLds && V.perlin_lds >= 0) {  // the single Perlin texture's tables, behind the preorder
    uint8_t *pb = (uint8_t *)lds + V.perlin_lds;
    float4 *pg = (float4 *)(pb + 3 * 256);
    const rt_perlin &P = S.perlins[0];
    for (uint32_t q = threadIdx.x; q < 256; q += blockDim.x) {
      pb[q] = (uint8_t)P.perm_x[q], pb[256 + q] = (uint8_t)P.perm_y[q], pb[512 + q] = (uint8_t)P.perm_z[q];
      pg[q] = make_float4(P.grad[q][0], P.grad[q][1], P.grad[q][2], 0.0f);
    }
    pl.perm = pb;
    pl.grad = pg;
  }
  if (n_lds) {  // the top of the preorder (the first BVH levels of every root item) in LDS
#if RT_GEN_SPLIT
    for (uint32_t q = threadIdx.x; q < n_lds; q += blockDim.x) lds[q] = S.pre[2 * q], lds[n_lds + q] = S.pre[2 * q + 1];
#else
    for (uint32_t q = threadIdx.x; q < 2 * n_lds; q += blockDim.x) lds[q] = S.pre[q];
#endif
  }
  if (n_lds || pl.perm) __syncthreads();
  constexpr bool kFull = (F & (RT_FEAT_EMISSIVE | RT_FEAT_LIGHTS)) != 0;
  const int W = S.cam.width;
  const int64_t total = (int64_t)V.n_rows * W;
  const int lane = __lane_id();
  const f3 du = ld3(S.cam.delta_u), dv = ld3(S.cam.delta_v), lf = ld3(S.cam.origin);
  const bool dof = S.cam.dof_angle > 0.0f;
  const float prob = S.cam.light_prob;
  const int spp = S.cam.spp;

  // per-lane path state (path_color's locals, kept across iterations).  A recorded bounce's
  // emission is always +0 (only SurfaceNormal and DiffuseLight emit, and neither scatters:
  // src/material.c:103-142), so the record is (albedo, pdf weight) and the fold adds +0 as the
  // reference's vec3_add(emission_color, scatter_color) does.  Records: albedo codes (kCode*) in
  // registers, explicit ones on register stacks spilling to the thread's slots (a lane's records share
  // cache lines, where private arrays interleave every dword across the wave's lanes).
  // (PathRecord: albedo codes in a register pair, explicit albedos and weights on register stacks whose
  // overflow goes to the thread's kMaxDepth global slots)
  PathRecord<kWReg, kXReg> P;
  rec_init(P, V.code_bits);
  const uint32_t code_explicit = (1u << P.runs.cb) - 1u, code_unit = code_explicit - 1u, code_weighted = 1u << P.runs.cb;
#if RT_GEN_SLOT_MAJOR
  // slot-major: entry k of every thread's slots is one array, so a wave's pushes at equal depth are
  // neighbouring words (thread-contiguous slots put them kMaxDepth entries apart, one line each)
  const uint32_t rec0 = blockIdx.x * blockDim.x + threadIdx.x, rec_stride = gridDim.x * blockDim.x;
#else
  const uint32_t rec0 = (blockIdx.x * blockDim.x + threadIdx.x) * (uint32_t)kMaxDepth, rec_stride = 1u;
#endif
  const auto solid_color = [&](uint32_t t) { return ld3(S.textures[t].color); };
  // extra box actions per step: RT_GEN_FLAT - 1 in the diagnostic build; the product's 2 at compile time,
  // so pre_common's loop for further ones -- and its per-step exec-mask bookkeeping -- compiles away
#ifdef RT_DIAG
  const int extra_boxes = V.flat - 1;
#else
  constexpr int extra_boxes = 2;
#endif
  int depth = 0, s = 0, i = 0, j = 0;
  int64_t pix = 0;
  uint32_t rays = 0;
  Pcg32 g;
  g.state = 0;
  g.inc = 0;
  f3 acc = mk(0.0f, 0.0f, 0.0f), o = acc, d = acc, pixel_pos = acc;
  bool need_pixel = true, need_sample = true, done = false;
  PreTrace T;  // kBatch: the lane's trace in progress (tracing) or finished, not yet shaded (pending)
  T.found = false;
  // the lane's trace state as one integer in a VGPR: as two loop-carried bools the compiler kept lane
  // masks and merged them (s_andn2 / s_and / s_or) at every trace step
  enum : int { kIdle = 0, kTracing = 1, kPending = 2 };
  int tstate = kIdle;
#define tracing (tstate == kTracing)
#define pending (tstate == kPending)
  uint64_t gs_c = 0;
  (void)gs_c;
#ifdef RT_GEN_STATS
  unsigned long long gs[kGsN];
  for (int q = 0; q < kGsN; q++) gs[q] = 0;
  int gs_kind = kGsIterRefill;
  uint64_t gs_t = __builtin_amdgcn_s_memtime();
#define GS_NOW() __builtin_amdgcn_s_memtime()
#define GS_ADD(k, v) (gs[k] += (unsigned long long)(v))
#define GS_CNT(k, pred) GS_ADD(k, __popcll(__ballot(pred)))
#else
#define GS_NOW() 0ull
#define GS_ADD(k, v) ((void)0)
#define GS_CNT(k, pred) ((void)0)
#endif

  for (;;) {
#ifdef RT_GEN_STATS
    {
      const uint64_t now = GS_NOW();
      gs[gs_kind] += now - gs_t;
      gs_t = now;
      gs_kind = kGsIterRefill;
    }
#endif
    // ---- refill (src/raytracing.c:93-94): lanes without a pixel take the next ones
    const uint64_t want = __ballot(need_pixel && !done);
    if (want) {
      const int first = __builtin_ctzll(want);
      int base = 0;
      if (lane == first) base = atomicAdd(V.work_counter, (int)__popcll(want));
      base = __shfl(base, first);
      if (need_pixel && !done) {
        const int64_t k = (int64_t)base + __popcll(want & ((1ull << lane) - 1));
        if (k >= total) {
          done = true;
        } else {
          pix = V.order ? (int64_t)V.order[k] : k;
          const int jj = (int)(pix / W);
          i = (int)(pix - (int64_t)jj * W);
          j = V.row0 + jj * V.row_stride;
          g.seed((uint64_t)(17 + j), (uint64_t)(23 + i));
          pixel_pos = add(add(ld3(S.cam.pixel00), scale(du, (float)i)), scale(dv, (float)j));
          acc = mk(0.0f, 0.0f, 0.0f);
          s = 0;
          if (V.pre_in) {  // the cost pass rendered this pixel's first samples: on from there (same
                           // samples, same summation order; rt_book1.h pre_resume)
            const float4 ps = V.pre_in[pix];
            const uint32_t w = __builtin_bit_cast(uint32_t, ps.w);
            if ((w >> 24) != 0u && (int)(w >> 24) < spp) {
              g.skip(w & 0xffffffu);
              s = (int)(w >> 24);
              acc = mk(ps.x, ps.y, ps.z);
            }
          }
          rays = 0;
          need_pixel = false;
          need_sample = spp > 0;
        }
      }
    }
    if (__ballot(!done) == 0) break;
    if (kBatch) {
      const uint64_t tr = __ballot(!done && tracing);
      const uint64_t ready = __ballot(!done && !tracing);
      const int live = (int)__popcll(tr | ready);
      const int batch = min(V.batch, (3 * live + 3) / 4);
      if (tr != 0 && (int)__popcll(ready) < batch) {  // traversal steps for the lanes still tracing
#ifdef RT_GEN_STATS
        gs_kind = kGsIterTrace;
        GS_ADD(kGsTraceIters, 1);
        GS_ADD(kGsTraceLanes, __popcll(tr));
        for (int k = 0; k < V.steps; k++) {  // entry kinds the tracing lanes meet (peek, no state change)
          const bool on = tracing && T.p < (uint32_t)S.n_pre;
          int kind = -1;
          if (on) {
            const uint32_t q = T.p;
            const float4 q1 = q < n_lds ? lds[RT_GEN_SPLIT ? n_lds + q : 2 * q + 1] : S.pre[2 * q + 1];
            kind = rt_ref_kind((int32_t)__builtin_bit_cast(uint32_t, q1.w));
          }
          const uint64_t b0 = __ballot(on && kind == RT_KIND_BVH), b1 = __ballot(on && kind == RT_KIND_SPHERE),
                         b2 = __ballot(on && kind == RT_KIND_QUAD),
                         b3 = __ballot(on && (kind == RT_KIND_TRANSLATE || kind == RT_KIND_ROTATE_Y)),
                         b4 = __ballot(on && kind == RT_KIND_MEDIUM), ball = __ballot(on);
          GS_ADD(kGsKindBox, __popcll(b0)), GS_ADD(kGsKindSphere, __popcll(b1)), GS_ADD(kGsKindQuad, __popcll(b2));
          GS_ADD(kGsKindXform, __popcll(b3)), GS_ADD(kGsKindMedium, __popcll(b4));
          GS_ADD(kGsKindOther, __popcll(ball & ~(b0 | b1 | b2 | b3 | b4)));
          GS_ADD(kGsStepKinds, (b0 != 0) + (b1 != 0) + (b2 != 0) + (b3 != 0) + (b4 != 0));
          break;  // the first step of the iteration only
        }
#endif
        // iteration after iteration in this inner loop while the shading batch is not full (back
        // through the outer loop's merge after every iteration, the compiler shuffled the lanes'
        // trace state between register sets every step)
        for (;;) {
#pragma unroll 1
          for (int k = 0; k < V.steps; k++) {
            gs_c = GS_NOW();
            // every lane loads (entry 0 when not tracing): both halves as two b128 reads in one round
            // trip (left to itself the compiler split them into four narrower reads)
            const uint32_t q = tracing && T.p < (uint32_t)S.n_pre ? T.p : 0u;
            // (the barrier on whole 128-bit tuples: per-component constraints made the compiler shuffle
            // registers after the loads)
            typedef float f4v __attribute__((ext_vector_type(4)));
            f4v v0, v1;
            if (kAllLds || q < n_lds) {
#if RT_GEN_SPLIT
              v0 = *(const f4v *)&lds[q], v1 = *(const f4v *)&lds[n_lds + q];
#else
              v0 = *(const f4v *)&lds[2 * q], v1 = *(const f4v *)&lds[2 * q + 1];
#endif
            } else {
              v0 = *(const f4v *)&S.pre[2 * q], v1 = *(const f4v *)&S.pre[2 * q + 1];
            }
            asm volatile("" : "+v"(v0), "+v"(v1));
            float4 q0 = make_float4(v0.x, v0.y, v0.z, v0.w), q1 = make_float4(v1.x, v1.y, v1.z, v1.w);
            const bool rare = tracing && pre_is_rare<F>(T, q1);
            const uint64_t rm = __ballot(tracing && rare), cm = __ballot(tracing && !rare);
            if ((rm | cm) == 0) break;
            const bool run_rare = rm != 0 && (cm == 0 || (int)__popcll(rm) >= V.rare_min || k == V.steps - 1);
            bool fin = false;
            GS_ADD(kGsCycClassify, GS_NOW() - gs_c);
            gs_c = GS_NOW();
            if (tracing && !rare) {
              if constexpr (kAllLds && RT_GEN_SPLIT) fin = pre_common<F>(S, PreSplit{lds, n_lds}, T, 1e-3f, q0, q1, extra_boxes);
              else fin = pre_common<F>(S, PrePairs{kAllLds ? lds : S.pre}, T, 1e-3f, q0, q1, extra_boxes);
            }
            GS_ADD(kGsCycCommon, GS_NOW() - gs_c);
            gs_c = GS_NOW();
            if (tracing && rare && run_rare) {
              if constexpr (kAllLds && RT_GEN_SPLIT) fin = pre_exec<F>(S, PreSplit{lds, n_lds}, T, o, d, 1e-3f, g, q0, q1);
              else fin = pre_exec<F>(S, PrePairs{kAllLds ? lds : S.pre}, T, o, d, 1e-3f, g, q0, q1);
            }
            GS_ADD(kGsCycRare, GS_NOW() - gs_c);
            GS_ADD(kGsRareSteps, run_rare);
            if (fin) tstate = kPending;
          }
          const uint64_t tr2 = __ballot(!done && tracing), ready2 = __ballot(!done && !tracing);
          const int batch2 = min(V.batch, (3 * (int)__popcll(tr2 | ready2) + 3) / 4);
          if (tr2 == 0ull || (int)__popcll(ready2) >= batch2) break;
          GS_ADD(kGsTraceIters, 1);
          GS_ADD(kGsTraceLanes, __popcll(tr2));
        }
        continue;
      }
      if (tracing) continue;  // sits out this shading pass
    }
#ifdef RT_GEN_STATS
    if (__ballot(!done)) {
      gs_kind = kGsIterShade;
      GS_ADD(kGsShadeIters, 1);
      GS_CNT(kGsShadeLanes, !done);
      GS_ADD(kGsCycTop, GS_NOW() - gs_t);
    }
#endif
    if (done) continue;
    bool write = spp <= 0 && !need_pixel;  // no samples: the mean is 0/0 (src/raytracing.c:127)
    // ---- camera ray (src/raytracing.c:100-122)
    gs_c = GS_NOW();
    if (need_sample && !write) {
      const float px = g.between(-0.5f, 0.5f);
      const float py = g.between(-0.5f, 0.5f);
      o = lf;
      if (dof) {
        float a, b;
        for (;;) {
          a = g.between(-1.0f, 1.0f);
          b = g.between(-1.0f, 1.0f);
          if (a * a + b * b < 1.0f) break;
        }
        o = add(add(lf, scale(ld3(S.cam.disc_u), a)), scale(ld3(S.cam.disc_v), b));
      }
      d = add(add(add(pixel_pos, scale(du, px)), scale(dv, py)), neg(o));
      depth = S.cam.max_depth;
      rec_clear(P);
      need_sample = false;
    }
    GS_ADD(kGsCycCamera, GS_NOW() - gs_c);
    // ---- one bounce of path_color (rt_device.h; src/raytracing.c:39-75)
#ifdef RT_GEN_STATS
    const uint64_t gs_b = GS_NOW();
#endif
    bool path_done = false;
    f3 tail = mk(0.0f, 0.0f, 0.0f);
    if (write) {
      // straight to the pixel write
    } else if (depth <= 0) {
      path_done = true;
    } else {
      Hit h;
      bool found;
      if (kBatch) {
        if (!pending) {  // start this bounce's trace; it is shaded in a later pass
          gs_c = GS_NOW();
          pre_begin(T, o, d);
          GS_ADD(kGsCycBegin, GS_NOW() - gs_c);
          tstate = kTracing;
          rays++;
          continue;
        }
        tstate = kIdle;
        found = T.found;
        h = T.h;
      } else {
        rays++;
        found = S.pre ? trace_pre<F>(S, o, d, 1e-3f, g, h) : trace<F>(S, o, d, 1e-3f, g, h);
      }
      GS_CNT(kGsMiss, !found);
      if (!found) {
        tail = ld3(S.cam.background);
        path_done = true;
      } else {
        Rec r;
        gs_c = GS_NOW();
        make_record<F>(S, o, d, h, r);
        GS_ADD(kGsCycRecord, GS_NOW() - gs_c);
        gs_c = GS_NOW();
        const f3 e = emit<F>(S, r, pl);
        GS_ADD(kGsCycEmit, GS_NOW() - gs_c);
        f3 dir, albedo;
        bool skip_pdf;
#ifdef RT_GEN_STATS
        const rt_material &gm = S.materials[r.material];
        GS_CNT(kGsMatLam, gm.tag == RT_MAT_LAMBERTIAN), GS_CNT(kGsMatMetal, gm.tag == RT_MAT_METAL);
        GS_CNT(kGsMatDiel, gm.tag == RT_MAT_DIELECTRIC), GS_CNT(kGsMatIso, gm.tag == RT_MAT_ISOTROPIC);
        GS_CNT(kGsMatEnd, gm.tag != RT_MAT_LAMBERTIAN && gm.tag != RT_MAT_METAL && gm.tag != RT_MAT_DIELECTRIC &&
                              gm.tag != RT_MAT_ISOTROPIC);
        const bool textured = gm.tag == RT_MAT_LAMBERTIAN || gm.tag == RT_MAT_METAL || gm.tag == RT_MAT_ISOTROPIC;
        const int tk = textured ? S.textures[gm.texture].kind : -1;
        GS_CNT(kGsTexSolid, tk == RT_TEX_SOLID), GS_CNT(kGsTexChecker, tk == RT_TEX_CHECKER);
        GS_CNT(kGsTexImage, tk == RT_TEX_IMAGE), GS_CNT(kGsTexPerlin, tk == RT_TEX_PERLIN);
        const bool gs_perlin = __ballot(tk == RT_TEX_PERLIN) != 0;
        GS_ADD(kGsPassPerlin, gs_perlin);
#endif
        gs_c = GS_NOW();
        int32_t solid = -1;
        const bool scattered = scatter<F>(S, r, d, g, dir, albedo, skip_pdf, pl, &solid);
#ifdef RT_GEN_STATS
        GS_ADD(gs_perlin ? kGsCycScatterPerlin : kGsCycScatter, GS_NOW() - gs_c);
#endif
        if (!scattered) {
          tail = e;
          path_done = true;
        } else {
          uint32_t code = solid == kUnitAlbedo ? code_unit
                          : (solid >= 0 && (uint32_t)solid + 1u < code_unit ? (uint32_t)solid + 1u : code_explicit);
          float w = 1.0f;
          if (kFull) {
            if ((F & RT_FEAT_LIGHTS) && (S.features & RT_FEAT_LIGHTS) && !skip_pdf) {
              gs_c = GS_NOW();
              if (g.f32() < prob) dir = lights_rand(S, r.p, g);
              const float sp = scatter_pdf(S, r.material, r.normal, dir);
              const float spdf = (1.0f - prob) * sp + prob * lights_pdf(S, r.p, dir);
              w = sp / spdf;
              code |= code_weighted;
              GS_ADD(kGsCycLights, GS_NOW() - gs_c);
            }
          }
          GS_ADD(kGsRecords, 1);  // (per lane: summed over every lane at the end)
          GS_ADD(kGsWeighted, (code & code_weighted) != 0);
          GS_ADD(kGsW2, (code & code_weighted) != 0 && w == 2.0f);
          rec_push(P, code, albedo, w, V.xrec + rec0, V.xw + rec0, rec_stride);
          o = r.p;
          d = dir;
          depth--;
          if (kBatch && depth > 0) {  // the next bounce's trace starts at once
            pre_begin(T, o, d);
            tstate = kTracing;
            rays++;
          }
        }
      }
    }
    GS_ADD(kGsCycBounce, GS_NOW() - gs_b);
    if (!path_done && !write) continue;
    gs_c = GS_NOW();
    if (!write) {
    // ---- fold innermost-first, accumulate, next sample / pixel (src/raytracing.c:124-131)
#ifdef RT_GEN_STATS
    if (P.n > 0) {
      const bool zero_tail = tail.x == 0.0f && tail.y == 0.0f && tail.z == 0.0f;
      const int over = max(0, P.wst.n - kWReg) + max(0, P.xst.n - kXReg);
      GS_ADD(kGsPaths, 1);
      GS_ADD(kGsPathZero, zero_tail);
      GS_ADD(kGsPathTrunc, over > 0);
      GS_ADD(kGsPathTruncZero, over > 0 && zero_tail);
      GS_ADD(kGsSpillSt, over);
      GS_ADD(kGsSpillStZero, zero_tail ? over : 0);
      GS_ADD(kGsFoldSkips, zero_tail && P.nonfin == 0u);
      GS_ADD(kGsExplicit, P.xst.n);
    }
#endif
    const f3 c = rec_fold(P, tail, solid_color, V.xrec + rec0, V.xw + rec0, rec_stride);
    acc = add(acc, c);
    s++;
    GS_ADD(kGsCycFold, GS_NOW() - gs_c);
    if (s < spp) {
      need_sample = true;
      continue;
    }
    }
    gs_c = GS_NOW();
    const float spp_f = (float)spp;
    const float ch[3] = {acc.x, acc.y, acc.z};
    uint8_t *dst = out + pix * 3;
    for (int q = 0; q < 3; q++) {
      float v = sqrtf(ch[q] / spp_f);
      v = v > 0.0f ? v : 0.0f;
      v = v < 0.999f ? v : 0.999f;
      dst[q] = (uint8_t)(int)(256.0f * v);
    }
    if (V.cost_out) V.cost_out[pix] = rays;
    if (V.pre_out) V.pre_out[pix] = make_float4(acc.x, acc.y, acc.z, __builtin_bit_cast(float, pre_word(g.n, (uint32_t)s)));
    need_pixel = true;
    GS_ADD(kGsCycWrite, GS_NOW() - gs_c);
  }
#ifdef RT_GEN_STATS
  if (V.stats)
    for (int q = 0; q < kGsN; q++)
      if (lane == 0 || q >= kGsPerLane) atomicAdd(V.stats + q, gs[q]);
#endif
#undef GS_NOW
#undef GS_ADD
#undef GS_CNT
#undef tracing
#undef pending
}

}  // namespace gen
}  // namespace rt
