// rt_book1.h — the fast path for sphere/BVH scenes (reference scenes 0 and 1: the headline
// Book-1 final scene).  Same arithmetic as rt_device.h (bit-exact with the reference); different
// execution structure, designed for a 64-wide CDNA4 wavefront:
//
//  * persistent lanes + wave-level work stealing: a lane that finishes its pixel takes the next
//    unrendered pixel (one atomic per wave per refill: ballot + mbcnt), so the frame has no tail of
//    half-empty waves and no per-pixel load imbalance (sky vs ground rows);
//  * one flattened loop per lane over (sample, bounce): every iteration a lane traces one ray;
//    lanes whose path ended generate their next camera ray in the same iteration, so a wave never
//    waits for its longest path at a sample boundary (Camera_ray_color's recursion, unrolled);
//  * BVH nodes and sphere (center, r^2) staged once per workgroup in LDS; per-lane DFS stack in LDS
//    ([slot][lane], 16-bit refs: conflict-free); traversal keeps the reference's left-then-right
//    order and shrinking t_max, tests leaf spheres inline, and never pushes the left child;
//  * the path record is a list of material ids (albedo of a Solid texture is a function of the
//    material) in registers (two 4-id chunks) + a per-lane global spill area for deep paths; the
//    colour is folded innermost-first at path end exactly like the recursion.
//
// Eligibility (host-checked, rt_kernel.hip: book1_eligible): spheres only, BVH nodes, lists only at
// the root, Lambertian/Metal/Dielectric with Solid albedo, no lights/emission/textures/transforms.
#pragma once
#include "rt_device.h"

namespace rt {
namespace b1 {

constexpr int kBlock = 256;
constexpr int kWaves = kBlock / 64;
constexpr int kStackSlots = 16;   // per-lane DFS slots in LDS, 32-bit (host checks the need)
constexpr uint16_t kLeafBit = 0x8000;  // 16-bit ref: leaf sphere index | kLeafBit, else node index
constexpr uint16_t kHasLeaf7 = 0x4000; // v7 node refs: the node has a leaf child (its record's spheres are read)

struct FastMat {   // 32 B: material resolved to what the Book-1 path needs
  float albedo[3];  // Solid texture colour; (1,1,1) for Dielectric
  float param;      // fuzz / eta
  int32_t tag;
  int32_t pad[3];
};

// Split render (stream split, render_batched kMode 2; opt-in RT_SPLIT=1).  A pixel's samples share
// one pcg32 stream: sample s starts at stream offset o_s and draws D(o_s), so o_{s+1} = o_s + D(o_s),
// and a sample's colour and draw count are functions of its start offset alone.  A split pixel's
// estimated stream is cut into K segments at offsets B_k.  Segment k > 0 is one chain per offset
// of the window [B_k, B_k + w) (one lane each), sample after sample until the segment's end, each
// storing every sample's colour and draw count at its offset; a chain stops at an offset another
// chain already claimed, so the window's chains coalesce onto the true one.  The head chain is the
// pixel's true chain: it computes segment 0, then takes the finished records in sample order --
// the reference's summation order, so the pixel is bit-identical -- and computes any sample that
// has no finished record itself (a draw count larger than the window, a stream longer than the
// estimate, or a segment still running).  split_walk_kernel / split_replan_kernel finish any pixel
// a round leaves unfinished (with walking heads, none).
struct SplitPx {            // 48 B per work item of a split launch
  float acc[3];             // head chain: colour sum of samples [0, s)
  uint32_t o, s;            // head chain: next sample's start offset and index (s == spp: written)
  uint32_t stop_at;         // head chain stops at this offset (segment 0's end), or kNoStop / kNoCoalesce
  uint32_t base, len;       // records of offsets [segment 0's end, len) at sp_claim / sp_rec [base + o]
  uint32_t len_run;         // offsets below this are covered by segment chains already
  uint32_t w;               // window: chains per segment
  float cps;                // pre-pass traversal steps per sample
  uint32_t rec_lo;          // segment 0's end: records (and claims) exist for offsets >= rec_lo
};
constexpr uint32_t kNoStop = 0xffffffffu;      // stop at a claimed offset only (fix-up rounds)
constexpr uint32_t kNoCoalesce = 0xfffffffeu;  // never stop before spp samples (unsplit pixels, last round)
constexpr uint32_t kSpecBit = 0x80000000u;     // sp_items[].x: segment item (else head item)
constexpr uint32_t kRecFill = 0xffffffffu;     // sp_rec words before their record is written (a NaN no
                                               // arithmetic produces; the draw count is never this)

struct Book1View {
  DScene S;                  // full scene (global memory): sphere aux data, camera
  const float4 *nodes_g;     // 2 float4 per node: (lo.x hi.x lo.y hi.y), (lo.z hi.z left right bits)
  const float4 *spheres_g;   // (center.xyz, r^2)
  const FastMat *mats;
  const uint16_t *root_items;
  int32_t n_nodes, n_spheres, n_root;
  int32_t stack_need;
  int32_t row0, row_stride, n_rows;
  int32_t *work_counter;     // zeroed before each launch
  int32_t shade_batch;       // v3+: shade once this many lanes of a wave are waiting
  int32_t sphere_batch;      // v6: run a sphere phase once this many lanes have a pending sphere
  int32_t reverse;           // hand out work items last-first
  const int32_t *order;      // work item order (longest-first from the cost pre-pass), or null
  uint32_t *cost_out;        // cost pre-pass: traversal steps per work item, or null
  const uint32_t *n_coop;    // v9: the first *n_coop items of `order` are rendered by whole waves
  int32_t *coop_counter;     //     (render_pixel_coop), claimed through this counter
  const uint32_t *coop_waves_dev;  // by the first *coop_waves_dev waves of the grid
  const uint32_t *n_heavy;   // the first *n_heavy items of `order`: waves holding one run at priority 3
  int32_t coop_lanes;        // v5: cooperative traversal once the counter is dry and <= this many lanes live
  int32_t experiment;        // stats builds only: timing experiments that change the image (RT_EXPERIMENT)
  unsigned long long *stats; // diagnostic counters (kStats builds only)
  uint32_t *pixel_cost;      // kStats: per work item {traversal steps, wall_clock64 ticks}
  uint64_t *spill;           // [chunk][global lane]: a deep path's older 4-id chunks (Record)
  const float4 *nodes7_g;    // v7: 4 float4 per record (Node7 below), then one all-zero dummy record
  const uint16_t *root7_items;
  int32_t n_nodes7;          // records incl. the dummy
  const float4 *items9_g;    // v9: the world in traversal preorder, 2 float4 per item (Item9 below)
  int32_t n_items9, n_items9_alloc;  // items, and items incl. the zero pad item at the end
  int32_t spill_lanes;
  int32_t n_bf_leaves;       // whole-wave pixels: leaves for bf_trace; 0: off (coop_trace9 instead)
  uint32_t *px_time;         // diagnostic (RT_PX_TIME=1): per work item {start, end}, wall_clock64 low bits
  const uint4 *wide;         // group trace (rt_group.h): 8-entry treelets over the preorder items
  int32_t n_wide;            // 0: group kernel unavailable for this scene
  const uint16_t *anc;       // group trace: [item][16] ancestor item positions of each leaf (0xffff: none)
  uint32_t *draw_out;        // cost pre-pass (kMode 1): pcg32 draws per work item
  SplitPx *sp_px;            // split render (kMode 2): per work item state
  uint32_t *sp_claim;        //   per stream offset: 0 free, 1 claimed (its record is written)
  float4 *sp_rec;            //   per stream offset: sample colour, draw count (bits in .w)
  const uint4 *sp_items;     //   chains: {pix | kSpecBit, B, E, w} segment, or {pix, -, -, -} head
  const uint32_t *sp_n_items;
  const uint4 *sp_items2;    //   then these (segment chains of re-split pixels, fix-up rounds), or null
  const uint32_t *sp_n_items2;
  uint32_t sp_cap2;          //   (its capacity: the count may run past it)
};

// ---------------------------------------------------------------- wave helpers
RT_D int lane_id() { return __lane_id(); }

// ---------------------------------------------------------------- traversal
struct TraceState {
  f3 o, d, inv;
  float a;       // |d|^2
  float tmax;
  int32_t hit;   // sphere index or -1
};

RT_D void sphere_test_lds(const float4 *sph, int idx, TraceState &T, float tmin) {
  const float4 s = sph[idx];
  const f3 oc = sub(T.o, mk(s.x, s.y, s.z));
  const float b = dot(oc, T.d);
  const float c = dot(oc, oc) - s.w;
  const float disc = b * b - T.a * c;
  if (disc < 0) return;
  const float sq = sqrtf(disc);
  float root = (-b - sq) / T.a;
  if (root <= tmin || root >= T.tmax) {
    root = (-b + sq) / T.a;
    if (root <= tmin || root >= T.tmax) return;
  }
  T.tmax = root;
  T.hit = idx;
}

RT_D bool aabb_lds(float4 lo, float4 hi, const TraceState &T, float tmin) {
  // AABB_hit (src/hittable.c:38-55), slab by slab with the reference's early exit
  float tmax = T.tmax;
  {
    float t0 = (lo.x - T.o.x) * T.inv.x, t1 = (hi.x - T.o.x) * T.inv.x;
    if (T.inv.x < 0) { const float s = t0; t0 = t1; t1 = s; }
    tmin = fmaxf(tmin, t0);
    tmax = fminf(tmax, t1);
    if (tmax <= tmin) return false;
  }
  {
    float t0 = (lo.y - T.o.y) * T.inv.y, t1 = (hi.y - T.o.y) * T.inv.y;
    if (T.inv.y < 0) { const float s = t0; t0 = t1; t1 = s; }
    tmin = fmaxf(tmin, t0);
    tmax = fminf(tmax, t1);
    if (tmax <= tmin) return false;
  }
  {
    float t0 = (lo.z - T.o.z) * T.inv.z, t1 = (hi.z - T.o.z) * T.inv.z;
    if (T.inv.z < 0) { const float s = t0; t0 = t1; t1 = s; }
    tmin = fmaxf(tmin, t0);
    tmax = fminf(tmax, t1);
    if (tmax <= tmin) return false;
  }
  return true;
}

// Closest hit of World.objects (a root list of BVH roots / spheres) in [tmin, inf).
RT_D void trace(const Book1View &V, const float4 *nodes, const float4 *sph, uint32_t *stack, int lane_stride,
                TraceState &T, float tmin) {
  T.tmax = __builtin_inff();
  T.hit = -1;
  for (int k = 0; k < V.n_root; k++) {  // root list, in order (wave-uniform loop)
    uint32_t cur = V.root_items[k];
    int sp = 0;
    for (;;) {
      if (cur & kLeafBit) {
        sphere_test_lds(sph, (int)(cur & 0x7fff), T, tmin);
      } else {
        const float4 na = nodes[2 * cur], nb = nodes[2 * cur + 1];
        const float4 lo = make_float4(na.x, na.z, nb.x, 0.0f), hi = make_float4(na.y, na.w, nb.y, 0.0f);
        if (aabb_lds(lo, hi, T, tmin)) {
          const uint32_t l = __float_as_uint(nb.z), r = __float_as_uint(nb.w);
          if (l & kLeafBit) {
            sphere_test_lds(sph, (int)(l & 0x7fff), T, tmin);
            if (r != 0xffffu) {
              if (r & kLeafBit) {
                sphere_test_lds(sph, (int)(r & 0x7fff), T, tmin);
              } else {
                cur = r;
                continue;
              }
            }
          } else {
            if (r != 0xffffu) {
              stack[sp * lane_stride] = r;
              sp++;
            }
            cur = l;
            continue;
          }
        }
      }
      if (sp == 0) break;
      sp--;
      cur = stack[sp * lane_stride];
    }
  }
}

// ---------------------------------------------------------------- path record
// The path's material ids in push order, in chunks of 4 (16 bits each, newest in the low bits):
// r0 = the current chunk, r1 = the previous one; older chunks go to the per-lane spill area as one
// u64 each (one 8-byte store per 4 bounces beyond the 8th, instead of a 2-byte store per bounce).
struct Record {
  uint64_t r0, r1;
  int n;  // ids pushed
};

RT_D void rec_push(const Book1View &V, Record &R, uint32_t id, int glane) {
  if ((R.n & 3) == 0 && R.n > 0) {  // r0 is a complete chunk: start a new one
    if (R.n >= 8) V.spill[(int64_t)((R.n >> 2) - 2) * V.spill_lanes + glane] = R.r1;  // deep paths only
    R.r1 = R.r0;
    R.r0 = 0;
  }
  R.r0 = (R.r0 << 16) | id;
  R.n++;
}

// c = a_k * c for k = n-1 .. 0 (newest first), the recursion's evaluation order
RT_D f3 rec_fold_chunk(const Book1View &V, uint64_t w, int cnt, f3 c) {
  for (int k = 0; k < cnt; k++) {
    const FastMat &m = V.mats[(uint32_t)(w & 0xffff)];
    c = add(mk(0.0f, 0.0f, 0.0f), mul(ld3(m.albedo), c));
    w >>= 16;
  }
  return c;
}
RT_D f3 rec_fold(const Book1View &V, const Record &R, f3 c, int glane) {
  if (R.n == 0) return c;
  const int cnt0 = R.n - (((R.n - 1) >> 2) << 2);  // ids in the current chunk, 1..4
  c = rec_fold_chunk(V, R.r0, cnt0, c);
  if (R.n > cnt0) c = rec_fold_chunk(V, R.r1, 4, c);
  for (int q = ((R.n - 1) >> 2) - 2; q >= 0; q--)  // spilled chunks, newest first
    c = rec_fold_chunk(V, V.spill[(int64_t)q * V.spill_lanes + glane], 4, c);
  return c;
}

// ---------------------------------------------------------------- scattering (Book-1 materials)
RT_D f3 scatter(const FastMat &m, f3 normal, bool front, f3 r_in, Pcg32 &g) {
  if (m.tag == RT_MAT_LAMBERTIAN) {  // src/material.c:23-37
    const Onb b = onb_from_w(normal);
    const float r1 = g.f32();
    const float r2 = g.f32();
    const float phi = (2.0f * kPi) * r1;
    float sphi, cphi;
    rtm::sincosf(phi, &sphi, &cphi);
    const float sq = sqrtf(r2);
    return onb_local(b, mk(cphi * sq, sphi * sq, sqrtf(1.0f - r2)));
  }
  if (m.tag == RT_MAT_METAL) {  // src/material.c:48-58
    const f3 refl = reflect(normalize(r_in), normal);
    const f3 out = add(refl, scale(rand_unit_vector(g), m.param));
    return dot(out, normal) < 0.0f ? refl : out;
  }
  // DIELECTRIC, src/material.c:62-86
  float eta = m.param;
  if (front) eta = 1.0f / eta;
  const f3 v = normalize(r_in);
  const float cos_t = fminf(-dot(v, normal), 1.0f);
  const float sin_t = sqrtf(1.0f - cos_t * cos_t);
  float sch = (1.0f - eta) / (1.0f + eta);
  sch *= sch;
  sch += (1 - sch) * rtm::powf(1.0f - cos_t, 5.0f);
  if (eta * sin_t > 1.0f || sch > g.f32()) return reflect(v, normal);
  const f3 perp = scale(add(v, scale(normal, cos_t)), eta);
  const f3 para = scale(normal, -sqrtf(fabsf(1.0f - dot(perp, perp))));
  return add(perp, para);
}

// ---------------------------------------------------------------- the persistent kernel body
template <bool kLds>
__device__ void render(const Book1View &V, uint8_t *__restrict__ out, char *lds) {
  const int tid = threadIdx.x;
  const int W = V.S.cam.width;
  const int64_t total = (int64_t)V.n_rows * W;

  // stage the scene (nodes + spheres) in LDS once per workgroup
  // (when !kLds the stack still lives in LDS; only the scene arrays are read from global memory)
  float4 *nodes = (float4 *)lds;
  float4 *sph = nodes + (kLds ? 2 * V.n_nodes : 0);
  uint32_t *stack_base = (uint32_t *)(sph + (kLds ? V.n_spheres : 0));
  if (kLds) {
    for (int k = tid; k < 2 * V.n_nodes; k += kBlock) nodes[k] = V.nodes_g[k];
    for (int k = tid; k < V.n_spheres; k += kBlock) sph[k] = V.spheres_g[k];
    __syncthreads();
  } else {
    nodes = (float4 *)V.nodes_g;
    sph = (float4 *)V.spheres_g;
  }
  uint32_t *stack = stack_base + tid;  // slot k of this lane at stack[k * kBlock]: conflict-free
  const int glane = blockIdx.x * kBlock + tid;
  const int lane = lane_id();

  const rt_camera &cam = V.S.cam;
  const f3 du = ld3(cam.delta_u), dv = ld3(cam.delta_v), lf = ld3(cam.origin);
  const f3 disc_u = ld3(cam.disc_u), disc_v = ld3(cam.disc_v), bg = ld3(cam.background);
  const bool dof = cam.dof_angle > 0.0f;
  const int spp = cam.spp, max_depth = cam.max_depth;
  const float tmin = 1e-3f;

  int64_t pix = -1;  // current work item (index into this launch's rows)
  int i = 0, j = 0, s = 0, depth = 0;
  bool need_pixel = true, need_sample = true;
  Pcg32 g;
  g.state = 0;
  g.inc = 0;
  f3 pixel_pos = mk(0, 0, 0), acc = mk(0, 0, 0), o = mk(0, 0, 0), d = mk(0, 0, 0);
  Record R;
  R.r0 = R.r1 = 0;
  R.n = 0;

  for (;;) {
    // ---- refill: lanes without a pixel take consecutive work items, one atomic per wave
    const uint64_t want = __ballot(need_pixel);
    if (want) {
      const int first = __builtin_ctzll(want);
      int base = 0;
      if (lane == first) base = atomicAdd(V.work_counter, (int)__popcll(want));
      base = __shfl(base, first);
      if (need_pixel) {
        const int rank_in_wave = __popcll(want & ((1ull << lane) - 1));
        pix = base + rank_in_wave;
        if (pix >= total) break;  // no work left for this lane
        const int jj = (int)(pix / W);
        i = (int)(pix - (int64_t)jj * W);
        j = V.row0 + jj * V.row_stride;
        g.seed((uint64_t)(17 + j), (uint64_t)(23 + i));  // src/raytracing.c:94
        pixel_pos = add(add(ld3(cam.pixel00), scale(du, (float)i)), scale(dv, (float)j));
        acc = mk(0.0f, 0.0f, 0.0f);
        s = 0;
        need_pixel = false;
        need_sample = true;
      }
    }
    // ---- camera ray for the next sample (src/raytracing.c:100-122)
    if (need_sample) {
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
        o = add(add(lf, scale(disc_u, a)), scale(disc_v, b));
      }
      d = add(add(add(pixel_pos, scale(du, px)), scale(dv, py)), neg(o));
      depth = max_depth;
      R.n = 0;
      need_sample = false;
    }
    // ---- one bounce (Camera_ray_color body, src/raytracing.c:39-75)
    bool path_done = false;
    f3 tail = mk(0.0f, 0.0f, 0.0f);
    if (depth <= 0) {
      path_done = true;
    } else {
      TraceState T;
      T.o = o;
      T.d = d;
      T.inv = mk(1.0f / d.x, 1.0f / d.y, 1.0f / d.z);
      T.a = dot(d, d);
      trace(V, nodes, sph, stack, kBlock, T, tmin);
      if (T.hit < 0) {
        tail = bg;
        path_done = true;
      } else {
        const rt_sphere &sp = V.S.spheres[T.hit];
        const f3 p = ray_at(o, d, T.tmax);
        const f3 outward = scale(sub(p, ld3(sp.center)), sp.inv_radius);
        const bool front = dot(d, outward) < 0.0f;
        const f3 normal = front ? outward : neg(outward);
        const FastMat &m = V.mats[sp.material];
        const f3 nd = scatter(m, normal, front, d, g);
        rec_push(V, R, (uint32_t)sp.material, glane);
        o = p;
        d = nd;
        depth--;
      }
    }
    if (path_done) {
      acc = add(acc, rec_fold(V, R, tail, glane));
      s++;
      if (s == spp) {  // quantize (src/raytracing.c:127-131)
        const float spp_f = (float)spp;
        const float ch[3] = {acc.x, acc.y, acc.z};
        uint8_t *dst = out + pix * 3;
        for (int c = 0; c < 3; c++) {
          float v = sqrtf(ch[c] / spp_f);
          v = v > 0.0f ? v : 0.0f;
          v = v < 0.999f ? v : 0.999f;
          dst[c] = (uint8_t)(int)(256.0f * v);
        }
        need_pixel = true;
      } else {
        need_sample = true;
      }
    }
  }
}


// quantize one pixel (src/raytracing.c:127-131): mean, gamma 2, clamp-macro semantics, truncate
RT_D uint8_t quantize(float sum, float spp_f) {
  float v = sqrtf(sum / spp_f);
  v = v > 0.0f ? v : 0.0f;
  v = v < 0.999f ? v : 0.999f;
  return (uint8_t)(int)(256.0f * v);
}
RT_D void write_pixel(uint8_t *dst, f3 acc, int spp) {
  const float spp_f = (float)spp;
  dst[0] = quantize(acc.x, spp_f);
  dst[1] = quantize(acc.y, spp_f);
  dst[2] = quantize(acc.z, spp_f);
}

// ================================================================ v3: batched-shading megaloop
// The v2 loop (render) makes every lane of a wave wait for the wave's longest traversal, then run
// every material's shading code: PMC showed ~20% of lanes active per VALU instruction.  v3 keeps
// each lane's traversal state live across iterations and runs, per wave iteration, EITHER
// kSteps traversal steps for the lanes still traversing OR one shading pass for the lanes whose
// ray is resolved -- the latter only once at least `shade_batch` lanes are waiting (wave ballot)
// or nobody is traversing.  Visit order, t_max and arithmetic are exactly v2's (= the reference).
typedef float f2v __attribute__((ext_vector_type(2)));

struct Lane {         // plain scalars: an f3 member here was kept in scratch by the compiler
  float ox, oy, oz;   // current ray origin
  float dx, dy, dz;   // direction
  float ix, iy, iz;   // 1/d (hoisted: same IEEE division as AABB_hit)
  float a, tmax;      // |d|^2, closest hit so far
  float ra;           // refined reciprocal of a (div_core), hoisted per ray
  bool fast;          // a in the range where div_core == '/'
  int32_t hit;        // sphere index or -1
  uint32_t cur;       // ref being visited (16-bit encoding); v6: 0xffff once the DFS is exhausted
  uint32_t pend0, pend1;  // v6: leaf spheres found by the last box step, tested before the next one
  int sp, k;          // LDS stack depth, root-list position
};

// AABB_hit with the slabs evaluated together: t_min / t_max only tighten and fmaxf/fminf ignore a
// NaN operand, so testing tmax <= tmin once after all three slabs returns exactly what the
// reference's per-slab early exit returns.  (lo,hi) pairs are packed: one v_pk_add + v_pk_mul per
// axis.  Swap on a negative 1/d as the reference does (select, not min/max, for NaN parity).
RT_D bool aabb_packed(float4 a, float4 b, const Lane &L, float tmin) {
  const f2v px = (f2v){(a.x - L.ox) * L.ix, (a.y - L.ox) * L.ix};
  const f2v py = (f2v){(a.z - L.oy) * L.iy, (a.w - L.oy) * L.iy};
  const f2v pz = (f2v){(b.x - L.oz) * L.iz, (b.y - L.oz) * L.iz};
  const float t0x = L.ix < 0 ? px.y : px.x, t1x = L.ix < 0 ? px.x : px.y;
  const float t0y = L.iy < 0 ? py.y : py.x, t1y = L.iy < 0 ? py.x : py.y;
  const float t0z = L.iz < 0 ? pz.y : pz.x, t1z = L.iz < 0 ? pz.x : pz.y;
  const float lo = fmaxf(fmaxf(fmaxf(tmin, t0x), t0y), t0z);
  const float hi = fminf(fminf(fminf(L.tmax, t1x), t1y), t1z);
  return !(hi <= lo);
}

RT_D void sphere_test_lane(const float4 *sph, uint32_t ref, Lane &L, float tmin) {
  const int idx = (int)(ref & 0x7fff);
  const float4 s = sph[idx];
  const f3 oc = sub(mk(L.ox, L.oy, L.oz), mk(s.x, s.y, s.z));
  const float b = dot(oc, mk(L.dx, L.dy, L.dz));
  const float c = dot(oc, oc) - s.w;
  const float disc = b * b - L.a * c;
  if (disc < 0) return;
  const float sq = sqrtf(disc);
  float root = (-b - sq) / L.a;
  if (root <= tmin || root >= L.tmax) {
    root = (-b + sq) / L.a;
    if (root <= tmin || root >= L.tmax) return;
  }
  L.tmax = root;
  L.hit = idx;
}

// ---------------------------------------------------------------- exact fast arithmetic (v5)
// What sqrtf() and '/' compile to for f32 on gfx950 (denormals on, correctly rounded): a hardware
// estimate plus a Newton / one-ulp correction core, wrapped in operand scaling for extreme exponents
// and a special-value fix-up (v_div_scale / v_div_fmas / v_div_fixup, and the 2^-96 rescale + class
// test of the sqrt).  On the operand ranges below the wrappers are identities, so the bare cores
// return the same bits; the division's reciprocal refinement depends on the divisor only and is
// hoisted per ray.  Bitwise equality is checked on the device by rt_diag_arith (all floats for the
// sqrt, random pairs for the division: tests/test_render_gpu.py).
constexpr float kDivLo = 0x1p-20f, kDivHi = 0x1p20f;  // divisor range (|d|^2 of a ray)
constexpr float kNumHi = 0x1p40f;                     // numerator magnitude bound
constexpr float kSqrtLo = 0x1p-96f;                   // below it the compiler rescales

RT_D float sqrt_core(float x) {  // == sqrtf(x) for x == 0 or kSqrtLo <= x < inf
  const float r = __builtin_amdgcn_sqrtf(x);
  const float rm = __int_as_float(__float_as_int(r) - 1), rp = __int_as_float(__float_as_int(r) + 1);
  float out = fmaf(-rm, r, x) <= 0.0f ? rm : r;
  out = fmaf(-rp, r, x) > 0.0f ? rp : out;
  return out;
}
RT_D float recip_core(float a) {  // the divisor half of the '/' sequence
  const float y = __builtin_amdgcn_rcpf(a);
  return fmaf(fmaf(-a, y, 1.0f), y, y);
}
RT_D float div_core(float x, float a, float ra) {  // == x / a for a in [kDivLo, kDivHi], |x| <= kNumHi
  const float q0 = x * ra;
  const float q1 = fmaf(fmaf(-a, q0, x), ra, q0);
  return fmaf(fmaf(-a, q1, x), ra, q1);
}
// For |x| < 2^-40 (zero and denormals included) div_core is not bit-exact, but both it and x / a
// are below 2^-18 < t_min in magnitude, so the Sphere_hit root test rejects both: the decision and
// the recorded root (none) are the same.  Only |x| > kNumHi needs the real division.

// Sphere_hit (src/hittable.c:125-150) with the exact cores; lanes outside their ranges (NaN,
// huge numerators, tiny discriminants, degenerate rays) evaluate the reference expression.
template <bool kStats = false>
RT_D void sphere_test_data(float4 s, int idx, Lane &L, float tmin, unsigned long long *st = nullptr);
template <bool kStats = false>
RT_D void sphere_test_v5(const float4 *sph, uint32_t ref, Lane &L, float tmin, unsigned long long *st = nullptr) {
  const int idx = (int)(ref & 0x7fff);
  sphere_test_data<kStats>(sph[idx], idx, L, tmin, st);
}
template <bool kStats>
RT_D void sphere_test_data(float4 s, int idx, Lane &L, float tmin, unsigned long long *st) {
  const f3 oc = sub(mk(L.ox, L.oy, L.oz), mk(s.x, s.y, s.z));
  const float b = dot(oc, mk(L.dx, L.dy, L.dz));
  const float c = dot(oc, oc) - s.w;
  const float disc = b * b - L.a * c;
  if (disc < 0) return;
  float sq = sqrt_core(disc);
  float r1 = div_core(-b - sq, L.a, L.ra), r2 = div_core(-b + sq, L.a, L.ra);
  // (bitwise, not short-circuit: one straight-line guard instead of nested branches)
  const bool ok = (int)L.fast & ((int)(disc == 0.0f) | ((int)(disc >= kSqrtLo) & (int)(disc <= __FLT_MAX__))) &
                  (int)(fabsf(-b - sq) <= kNumHi) & (int)(fabsf(-b + sq) <= kNumHi);
  if (kStats) {
    st[ok ? 12 : 13]++;
    if (!ok && __lane_id() == __builtin_ctzll(__ballot(1))) st[15]++;
  }
  if (__builtin_expect(!ok, 0)) {
    sq = sqrtf(disc);
    r1 = (-b - sq) / L.a;
    r2 = (-b + sq) / L.a;
  }
  // the reference tries root 1, then root 2, each rejected when (root <= t_min || root >= t_max)
  const bool take1 = !(r1 <= tmin || r1 >= L.tmax), take2 = !(r2 <= tmin || r2 >= L.tmax);
  if (take1 || take2) {
    L.tmax = take1 ? r1 : r2;
    L.hit = idx;
  }
}

// One DFS step, v5: the same visit order as trav_step with the control flow reduced to selects --
// the right child is stored unconditionally into the free stack slot (the depth only advances on a
// real push; the stack has one spare slot for it) and the pop reads unconditionally.
template <bool kStats = false>
RT_D bool trav_step_v5(const Book1View &V, const float4 *nodes3, const float4 *sph, uint16_t *stack, Lane &L,
                       float tmin, unsigned long long *st = nullptr) {
  uint32_t t0 = 0xffffu, t1 = 0xffffu;
  bool moved = false;
  const uint32_t cur = L.cur;
  if (__builtin_expect((cur & kLeafBit) != 0, 0)) {  // a sphere directly in the root list
    t0 = cur;
  } else {
    const float4 a = nodes3[2 * cur], b = nodes3[2 * cur + 1];
    const bool hit = aabb_packed(a, b, L, tmin);
    if (kStats && hit) st[22]++;
    const uint32_t l = __float_as_uint(b.z), r = __float_as_uint(b.w);
    const bool lleaf = (l & kLeafBit) != 0, rleaf = (r & kLeafBit) != 0;  // kNone has the leaf bit
    t0 = hit && lleaf ? l : 0xffffu;
    t1 = hit && lleaf && rleaf ? r : 0xffffu;
    moved = hit && !(lleaf && rleaf);
    stack[L.sp * kBlock] = (uint16_t)r;
    L.sp += (hit && !lleaf && r != 0xffffu) ? 1 : 0;
    L.cur = moved ? (lleaf ? r : l) : cur;
  }
  if (kStats && (V.experiment & 1)) t0 = t1 = 0xffffu;  // timing experiment: no sphere tests
  if (t0 != 0xffffu) {
    if (kStats && __lane_id() == __builtin_ctzll(__ballot(1))) st[14]++;
    sphere_test_v5<kStats>(sph, t0, L, tmin, st);
  }
  if (t1 != 0xffffu) {
    if (kStats && __lane_id() == __builtin_ctzll(__ballot(1))) st[14]++;
    sphere_test_v5<kStats>(sph, t1, L, tmin, st);
  }
  if (moved) return false;
  const int top = L.sp - 1;
  const uint32_t popped = stack[(top > 0 ? top : 0) * kBlock];
  if (top >= 0) {
    L.sp = top;
    L.cur = popped;
    return false;
  }
  if (++L.k < V.n_root) {
    L.cur = V.root_items[L.k];
    return false;
  }
  return true;
}

// One DFS step (node box test, or leaf sphere(s)); returns true when the ray's traversal is done.
RT_D bool trav_step(const Book1View &V, const float4 *nodes3, const float4 *sph, uint16_t *stack, Lane &L,
                    float tmin) {
  uint32_t t0 = 0xffffu, t1 = 0xffffu;  // spheres to test in this step, in visit order
  bool moved = false;
  if (L.cur & kLeafBit) {
    t0 = L.cur;
  } else {
    const float4 a = nodes3[2 * L.cur], b = nodes3[2 * L.cur + 1];
    if (aabb_packed(a, b, L, tmin)) {
      const uint32_t l = __float_as_uint(b.z), r = __float_as_uint(b.w);
      if (l & kLeafBit) {
        t0 = l;
        if (r & kLeafBit) {
          if (r != 0xffffu) t1 = r;
        } else {
          L.cur = r;
          moved = true;
        }
      } else {
        if (r != 0xffffu) {
          stack[L.sp * kBlock] = (uint16_t)r;
          L.sp++;
        }
        L.cur = l;
        moved = true;
      }
    }
  }
  if (t0 != 0xffffu) sphere_test_lane(sph, t0, L, tmin);
  if (t1 != 0xffffu) sphere_test_lane(sph, t1, L, tmin);
  if (moved) return false;
  if (L.sp > 0) {
    L.sp--;
    L.cur = stack[L.sp * kBlock];
    return false;
  }
  if (++L.k < V.n_root) {
    L.cur = V.root_items[L.k];
    return false;
  }
  return true;
}

// ---------------------------------------------------------------- v7: one LDS round trip per step
// Per-step latency, not lane occupancy, bounds the v5 loop: a lone wave spends ~1250 clocks per DFS
// step (issue of ~100 VALU + ~40 SALU at 4 clocks each, 4-5 dependent LDS round trips, ~11 exec-mask
// branches).  v7 lays each node out with everything the step can need (Node7, 64 B):
//   q0 = (lo.x, hi.x, lo.y, hi.y)   q1 = (lo.z, hi.z, left ref, right ref)
//   q2 = (cx_l, cx_r, cy_l, cy_r)   q3 = (cz_l, cz_r, r2_l, r2_r)     (leaf children's spheres)
// so a step issues all its LDS reads at once (node + speculative stack pop), tests both leaf spheres
// with packed f32 math, and picks the next node with selects.  Node refs carry kHasLeaf7 so the
// sphere half is only fetched for nodes that have a leaf child (others read the dummy record).
// The two spheres are evaluated independently of t_max (root r = q1 unless q1 <= t_min, then q2)
// and then applied in the reference's order (left, then right against the updated t_max):
// Sphere_hit's accept test `!(root <= t_min || root >= t_max)` on that r is exactly the reference's
// two-root sequence, because q1 <= q2 (monotone rounding) makes a q1 >= t_max rejection final.
typedef float f2v7 __attribute__((ext_vector_type(2)));

// sqrt_core/div_core on a pair; `ok` false for lanes whose operands leave the cores' ranges
RT_D void sphere_pair_roots(f2v7 b, f2v7 disc, const Lane &L, float tmin, bool &ok, f2v7 &root) {
  const float sq0 = sqrt_core(disc.x), sq1 = sqrt_core(disc.y);
  const f2v7 sq = {sq0, sq1};
  const f2v7 n1 = -b - sq, n2 = -b + sq;
  float la = L.a, lra = L.ra;
  asm volatile("" : "+v"(la), "+v"(lra));
  const f2v7 a = {la, la}, ra = {lra, lra};
  f2v7 q0 = n1 * ra;
  f2v7 q1 = __builtin_elementwise_fma(__builtin_elementwise_fma(-a, q0, n1), ra, q0);
  const f2v7 r1 = __builtin_elementwise_fma(__builtin_elementwise_fma(-a, q1, n1), ra, q1);
  q0 = n2 * ra;
  q1 = __builtin_elementwise_fma(__builtin_elementwise_fma(-a, q0, n2), ra, q0);
  const f2v7 r2 = __builtin_elementwise_fma(__builtin_elementwise_fma(-a, q1, n2), ra, q1);
  ok = (int)L.fast & (int)((disc.x == 0.0f) | ((disc.x >= kSqrtLo) & (disc.x <= __FLT_MAX__))) &
       (int)((disc.y == 0.0f) | ((disc.y >= kSqrtLo) & (disc.y <= __FLT_MAX__))) &
       (int)(fmaxf(fmaxf(fabsf(n1.x), fabsf(n1.y)), fmaxf(fabsf(n2.x), fabsf(n2.y))) <= kNumHi);
  root.x = (r1.x <= tmin) ? r2.x : r1.x;
  root.y = (r1.y <= tmin) ? r2.y : r1.y;
}

template <bool kStats = false>
RT_D bool trav_step_v7(const Book1View &V, const float4 *nodes7, uint16_t *stack, Lane &L, float tmin,
                       unsigned long long *st = nullptr) {
  const uint32_t cur = L.cur;
  const int top = L.sp - 1;
  const uint32_t popped = stack[(top > 0 ? top : 0) * kBlock];  // speculative pop
  const float4 *nd = nodes7 + 4 * (cur & 0x3fffu);
  const float4 *ns = (cur & kHasLeaf7) ? nd : nodes7 + 4 * (V.n_nodes7 - 1);  // dummy: no leaves
  const float4 q0 = nd[0], q1 = nd[1], q2 = ns[2], q3 = ns[3];
  const bool hit = aabb_packed(q0, q1, L, tmin);
  const uint32_t l = __float_as_uint(q1.z), r = __float_as_uint(q1.w);
  const bool lleaf = (l & kLeafBit) != 0, rleaf = (r & kLeafBit) != 0;  // kNone has the leaf bit
  const bool t0 = hit && lleaf, t1 = t0 && rleaf && r != 0xffffu;
  if (t0) {
    if (kStats && __lane_id() == __builtin_ctzll(__ballot(1))) st[14]++;
    // Sphere_hit (src/hittable.c:120-151) for the pair (left, right), packed
    const f2v7 cx = {q2.x, q2.y}, cy = {q2.z, q2.w}, cz = {q3.x, q3.y}, r2 = {q3.z, q3.w};
    // register copies of the lane's ray: splatting struct fields straight into vector ops lets the
    // vectorizer widen them into overlapping loads of the Lane struct, which then stays in scratch
    float ox = L.ox, oy = L.oy, oz = L.oz, dx = L.dx, dy = L.dy, dz = L.dz, a = L.a;
    asm volatile("" : "+v"(ox), "+v"(oy), "+v"(oz), "+v"(dx), "+v"(dy), "+v"(dz), "+v"(a));
    const f2v7 ocx = ox - cx, ocy = oy - cy, ocz = oz - cz;
    const f2v7 b = (ocx * dx + ocy * dy) + ocz * dz;
    const f2v7 c = ((ocx * ocx + ocy * ocy) + ocz * ocz) - r2;
    const f2v7 disc = b * b - a * c;
    bool ok;
    f2v7 root;
    sphere_pair_roots(b, disc, L, tmin, ok, root);
    if (kStats) st[ok ? 12 : 13]++;
    if (__builtin_expect(!ok, 0)) {  // the reference expressions, per sphere
      const float s0 = sqrtf(disc.x), s1 = sqrtf(disc.y);
      const float a0 = (-b.x - s0) / L.a, b0 = (-b.x + s0) / L.a;
      const float a1 = (-b.y - s1) / L.a, b1v = (-b.y + s1) / L.a;
      root.x = (a0 <= tmin) ? b0 : a0;
      root.y = (a1 <= tmin) ? b1v : a1;
    }
    if (disc.x < 0.0f) root.x = -__builtin_inff();  // no root: -inf <= t_min rejects it for any t_max
    if (disc.y < 0.0f) root.y = -__builtin_inff();
    if (!(root.x <= tmin || root.x >= L.tmax)) {
      L.tmax = root.x;
      L.hit = (int32_t)(l & 0x7fffu);
    }
    if (t1 && !(root.y <= tmin || root.y >= L.tmax)) {
      L.tmax = root.y;
      L.hit = (int32_t)(r & 0x7fffu);
    }
  }
  const bool moved = hit && !(lleaf && rleaf);
  stack[L.sp * kBlock] = (uint16_t)r;  // free slot: kept only on a real push
  const bool push = hit && !lleaf && r != 0xffffu;
  if (moved) {
    L.sp += push ? 1 : 0;
    L.cur = lleaf ? r : l;
    return false;
  }
  if (top >= 0) {
    L.sp = top;
    L.cur = popped;
    return false;
  }
  if (++L.k < V.n_root) {
    L.cur = V.root7_items[L.k];
    return false;
  }
  return true;
}

// ---------------------------------------------------------------- v9: stackless preorder traversal
// The reference's closest-hit recursion (HittableList_hit over the root items, BVHNode_hit = own box,
// then left, then right: src/hittable.c:74-88, :266-277) visits the hittables in the preorder of the
// world graph, skipping a node's whole subtree when its box misses.  v9 stores that preorder as a
// flat item array, so the traversal is a scan with skips -- no stack, one item per step:
//   node item:  q0 = (lo.x, hi.x, lo.y, hi.y), q1 = (lo.z, hi.z, skip, 0)   next = hit ? p+1 : p+skip
//   leaf item:  q0 = (cx, cy, cz, r^2),        q1 = (-, -, -, idx | 1<<31)   Sphere_hit, next = p+1
// (skip = 1 + the node's subtree size in items).  The box test sees exactly the reference's t_max:
// every item before p in preorder that the reference would test has been tested, in order.
constexpr uint32_t kLeaf9 = 0x80000000u;

template <bool kStats = false>
RT_D bool trav_step_v9(const Book1View &V, const float4 *items, Lane &L, float tmin, unsigned long long *st = nullptr) {
  const uint32_t p = L.cur;
  float4 q0 = items[2 * p], q1 = items[2 * p + 1];
  // both halves in one LDS round trip: without this the compiler sinks the q1.xy / q1.z reads into
  // the branches that use them, i.e. three dependent round trips per step.  (Reading the successor
  // one step ahead measured slower: its moves and the re-read after a skip cost more than the latency.)
  asm volatile("" : "+v"(q0.x), "+v"(q0.y), "+v"(q0.z), "+v"(q0.w), "+v"(q1.x), "+v"(q1.y), "+v"(q1.z), "+v"(q1.w));
  const uint32_t w = __float_as_uint(q1.w);
  uint32_t next = p + 1;
  if (w & kLeaf9) {
    if (kStats) st[6]++;
    if (!(kStats && (V.experiment & 1)))  // timing experiment (stats builds): no sphere tests
      sphere_test_data<kStats>(q0, (int)(w & 0x7fffffffu), L, tmin, st);
  } else {
    if (kStats) st[5]++;
    const bool hit = aabb_packed(q0, q1, L, tmin);
    if (kStats && hit) st[22]++;
    if (!hit) next = p + __float_as_uint(q1.z);
  }
  L.cur = next;
  return next >= (uint32_t)V.n_items9;
}

// ---------------------------------------------------------------- v6: box and sphere phases
// v5 tests the leaf spheres of a node inside the node's step, so every wave step runs the box code
// AND two sphere tests whenever any lane of the wave has a leaf -- with a few lanes active in the
// sphere code.  v6 parks the leaf spheres of a box step in the lane (pend0, pend1) and runs, per wave
// iteration, either a box phase (lanes with nothing pending) or a sphere phase (lanes with a pending
// sphere: one test each), whichever has more lanes.  A lane's own order is untouched: its pending
// spheres are tested before its next box test, in the reference's order, against the same t_max.
RT_D void dfs_advance(const Book1View &V, const uint16_t *stack, Lane &L) {  // pop, next root, or exhausted
  const int top = L.sp - 1;
  const uint32_t popped = stack[(top > 0 ? top : 0) * kBlock];
  if (top >= 0) {
    L.sp = top;
    L.cur = popped;
  } else if (++L.k < V.n_root) {
    L.cur = V.root_items[L.k];
  } else {
    L.cur = 0xffffu;
  }
}

// Box phase of one lane (nothing pending, cur is a node or a root-list sphere).
RT_D void box_step_v6(const Book1View &V, const float4 *nodes3, uint16_t *stack, Lane &L, float tmin) {
  const uint32_t cur = L.cur;
  if (__builtin_expect((cur & kLeafBit) != 0, 0)) {  // a sphere directly in the root list
    L.pend0 = cur;
    dfs_advance(V, stack, L);
    return;
  }
  const float4 a = nodes3[2 * cur], b = nodes3[2 * cur + 1];
  const bool hit = aabb_packed(a, b, L, tmin);
  const uint32_t l = __float_as_uint(b.z), r = __float_as_uint(b.w);
  const bool lleaf = (l & kLeafBit) != 0, rleaf = (r & kLeafBit) != 0;  // kNone has the leaf bit
  L.pend0 = hit && lleaf ? l : 0xffffu;
  L.pend1 = hit && lleaf && rleaf ? r : 0xffffu;
  const bool moved = hit && !(lleaf && rleaf);
  stack[L.sp * kBlock] = (uint16_t)r;  // free slot: kept only on a real push
  L.sp += (hit && !lleaf && r != 0xffffu) ? 1 : 0;
  if (moved)
    L.cur = lleaf ? r : l;
  else
    dfs_advance(V, stack, L);
}

// Sphere phase of one lane (pend0 set): test it, shift the queue.
RT_D void sphere_step_v6(const float4 *sph, Lane &L, float tmin) {
  sphere_test_v5(sph, L.pend0, L, tmin);
  L.pend0 = L.pend1;
  L.pend1 = 0xffffu;
}

// ---------------------------------------------------------------- cooperative traversal (frame tail)
// A lane renders its pixel's samples in sequence (one pcg32 stream per pixel), so the frame ends
// with the slowest pixels' lanes running alone: measured on the headline frame, the pixel counter
// runs dry at ~1/3 of the kernel and the rest is that tail, with per-step latency -- not lane count --
// setting the pace.  Once the counter is dry and a wave has few live lanes, the wave traces each
// remaining ray with all 64 lanes: every node's box interval and every sphere's root are
// independent of t_max, so the lanes compute them all in parallel (kCoopSlots per lane), and one
// wave-uniform walk then replays the reference's DFS (src/hittable.c:74-88, :266-277) on them:
//   box hit at visit   <=>  !(fminf(t_max, X) <= E)   (E = fmaxf chain from t_min, X = fminf chain)
//   sphere accepted    <=>  !(r <= t_min || r >= t_max), r = q1 unless q1 <= t_min, then q2
// (the two-root sequence of Sphere_hit, since q1 <= q2; "no root" is -inf, rejected for any t_max).
typedef float f8v __attribute__((ext_vector_type(8)));
typedef unsigned int u8v __attribute__((ext_vector_type(8)));
constexpr int kCoopSlots = 8;  // 64 x 8 = 512 nodes and 512 spheres at most

RT_D float lane_bcast(float x, int src) { return __int_as_float(__builtin_amdgcn_readlane(__float_as_int(x), src)); }

struct CoopRay {  // wave-uniform copy of the traced ray
  float ox, oy, oz, dx, dy, dz, ix, iy, iz, a, ra;
  bool fast;
};

// Sphere_hit's accepted root for this sphere, independent of t_max (see above)
RT_D float coop_sphere_root(float4 s, const CoopRay &C, float tmin) {
  const f3 oc = sub(mk(C.ox, C.oy, C.oz), mk(s.x, s.y, s.z));
  const float b = dot(oc, mk(C.dx, C.dy, C.dz));
  const float c = dot(oc, oc) - s.w;
  const float disc = b * b - C.a * c;
  if (disc < 0) return -__builtin_inff();
  float sq = sqrt_core(disc);
  float q1 = div_core(-b - sq, C.a, C.ra), q2 = div_core(-b + sq, C.a, C.ra);
  const bool ok = (int)C.fast & ((int)(disc == 0.0f) | ((int)(disc >= kSqrtLo) & (int)(disc <= __FLT_MAX__))) &
                  (int)(fabsf(-b - sq) <= kNumHi) & (int)(fabsf(-b + sq) <= kNumHi);
  if (__builtin_expect(!ok, 0)) {
    sq = sqrtf(disc);
    q1 = (-b - sq) / C.a;
    q2 = (-b + sq) / C.a;
  }
  return (q1 <= tmin) ? q2 : q1;
}

// Trace lane `src`'s ray with the whole wave; returns (t_max, hit) of the reference's traversal.
// `ustack` is a wave-uniform scratch stack (one column of the wave's DFS stacks, free between rays).
RT_D void coop_trace(const Book1View &V, const float4 *nodes3, const float4 *sph, uint16_t *ustack,
                     const Lane &L, int src, float tmin, float &out_tmax, int &out_hit) {
  const int lane = __lane_id();
  CoopRay C;
  C.ox = lane_bcast(L.ox, src), C.oy = lane_bcast(L.oy, src), C.oz = lane_bcast(L.oz, src);
  C.dx = lane_bcast(L.dx, src), C.dy = lane_bcast(L.dy, src), C.dz = lane_bcast(L.dz, src);
  C.ix = lane_bcast(L.ix, src), C.iy = lane_bcast(L.iy, src), C.iz = lane_bcast(L.iz, src);
  C.a = lane_bcast(L.a, src), C.ra = lane_bcast(L.ra, src);
  C.fast = __builtin_amdgcn_readlane((int)L.fast, src) != 0;
  // per-lane tables: node n = k*64 + lane -> (E, X, children), sphere i = k*64 + lane -> root
  f8v E, X, R;
  u8v CH;
#pragma unroll
  for (int k = 0; k < kCoopSlots; k++) {
    const int n = k * 64 + lane;
    float e = 0.0f, x = 0.0f, r = -__builtin_inff();
    unsigned ch = 0xffffffffu;
    if (n < V.n_nodes) {
      const float4 a = nodes3[2 * n], b = nodes3[2 * n + 1];
      const float t0x = (a.x - C.ox) * C.ix, t1x = (a.y - C.ox) * C.ix;
      const float t0y = (a.z - C.oy) * C.iy, t1y = (a.w - C.oy) * C.iy;
      const float t0z = (b.x - C.oz) * C.iz, t1z = (b.y - C.oz) * C.iz;
      const float nx = C.ix < 0 ? t1x : t0x, fx = C.ix < 0 ? t0x : t1x;
      const float ny = C.iy < 0 ? t1y : t0y, fy = C.iy < 0 ? t0y : t1y;
      const float nz = C.iz < 0 ? t1z : t0z, fz = C.iz < 0 ? t0z : t1z;
      e = fmaxf(fmaxf(fmaxf(tmin, nx), ny), nz);
      x = fminf(fminf(fx, fy), fz);
      ch = (__float_as_uint(b.z) & 0xffffu) | (__float_as_uint(b.w) << 16);
    }
    if (n < V.n_spheres) r = coop_sphere_root(sph[n], C, tmin);
    E[k] = e, X[k] = x, R[k] = r, CH[k] = ch;
  }
  // the reference's DFS on the tables (wave-uniform)
  float tmax = __builtin_inff();
  int hit = -1;
  for (int item = 0; item < V.n_root; item++) {
    uint32_t cur = V.root_items[item];
    int sp = 0;
    for (;;) {
      if (cur & kLeafBit) {
        const int si = (int)(cur & 0x7fffu);
        const float r = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(R[si >> 6]), si & 63));
        if (!(r <= tmin || r >= tmax)) tmax = r, hit = si;
      } else {
        const int n = (int)cur;
        const float e = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(E[n >> 6]), n & 63));
        const float x = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(X[n >> 6]), n & 63));
        if (!(fminf(tmax, x) <= e)) {
          const unsigned ch = (unsigned)__builtin_amdgcn_readlane((int)CH[n >> 6], n & 63);
          const uint32_t l = ch & 0xffffu, r = ch >> 16;
          if (l & kLeafBit) {
            const int si = (int)(l & 0x7fffu);
            const float rl = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(R[si >> 6]), si & 63));
            if (!(rl <= tmin || rl >= tmax)) tmax = rl, hit = si;
            if (r != 0xffffu) {
              cur = r;
              continue;  // a right leaf is tested by the next iteration, a right node visited
            }
          } else {
            if (r != 0xffffu) ustack[sp++ * kBlock] = (uint16_t)r;
            cur = l;
            continue;
          }
        }
      }
      if (sp == 0) break;
      cur = (uint32_t)__builtin_amdgcn_readfirstlane((int)ustack[--sp * kBlock]);
    }
  }
  out_tmax = tmax;
  out_hit = hit;
}

// v9 form of the cooperative trace: the preorder scan itself is the walk.  The wave evaluates a
// window of 64 consecutive items (box interval or sphere root, both t_max-independent), then scans
// it with wave-uniform decisions; a skip past the window, or its end, starts the next window.
template <bool kStats = false>
RT_D void coop_trace9(const Book1View &V, const float4 *items, const Lane &L, int src, float tmin,
                      float &out_tmax, int &out_hit, unsigned long long *st = nullptr) {
  const int lane = __lane_id();
  CoopRay C;
  C.ox = lane_bcast(L.ox, src), C.oy = lane_bcast(L.oy, src), C.oz = lane_bcast(L.oz, src);
  C.dx = lane_bcast(L.dx, src), C.dy = lane_bcast(L.dy, src), C.dz = lane_bcast(L.dz, src);
  C.ix = lane_bcast(L.ix, src), C.iy = lane_bcast(L.iy, src), C.iz = lane_bcast(L.iz, src);
  C.a = lane_bcast(L.a, src), C.ra = lane_bcast(L.ra, src);
  C.fast = __builtin_amdgcn_readlane((int)L.fast, src) != 0;
  const int n = V.n_items9;
  float tmax = __builtin_inff();
  int hit = -1;
  int p = 0;
  int guard = 0;  // every scan step advances p, so n steps bound the walk; this only catches bugs
  while (p < n && guard <= n) {
    const int base = p;
    const int q = base + lane;
    if (kStats && lane == 0) st[25]++;
    const long long c_w0 = kStats ? (long long)clock64() : 0;
    float v0 = 0.0f, v1 = 0.0f;  // node: E, X; leaf: root
    uint32_t meta = 0;           // node: skip; leaf: index | kLeaf9
    if (q < n) {
      const float4 q0 = items[2 * q], q1 = items[2 * q + 1];
      meta = __float_as_uint(q1.w);
      if (meta & kLeaf9) {
        v0 = coop_sphere_root(q0, C, tmin);
      } else {
        const float t0x = (q0.x - C.ox) * C.ix, t1x = (q0.y - C.ox) * C.ix;
        const float t0y = (q0.z - C.oy) * C.iy, t1y = (q0.w - C.oy) * C.iy;
        const float t0z = (q1.x - C.oz) * C.iz, t1z = (q1.y - C.oz) * C.iz;
        const float nx = C.ix < 0 ? t1x : t0x, fx = C.ix < 0 ? t0x : t1x;
        const float ny = C.iy < 0 ? t1y : t0y, fy = C.iy < 0 ? t0y : t1y;
        const float nz = C.iz < 0 ? t1z : t0z, fz = C.iz < 0 ? t0z : t1z;
        v0 = fmaxf(fmaxf(fmaxf(tmin, nx), ny), nz);
        v1 = fminf(fminf(fx, fy), fz);
        meta = __float_as_uint(q1.z);
      }
    }
    const int end = min(n, base + 64);
    long long c_w1 = 0;
    if (kStats) {
      __builtin_amdgcn_s_waitcnt(0);
      c_w1 = (long long)clock64();
      if (lane == 0) st[27] += c_w1 - c_w0;
    }
    // decisions for the current t_max in every lane, then a scalar walk along the next-pointers;
    // an accepted sphere changes t_max, so the decisions are redone from there
    const bool leaf = (meta & kLeaf9) != 0;
    const int l = lane;
    while (p < end && guard++ <= n) {
      const bool take = leaf ? !(v0 <= tmin || v0 >= tmax) : !(fminf(tmax, v1) <= v0);
      // next item after this one for the current t_max; an accepted sphere (t_max changes) is
      // encoded as kStop + its position so that the walk below only has to test one bound
      constexpr int kStop = 1 << 20;
      const int next = leaf ? (take ? kStop + l : l + 1) : (take ? l + 1 : l + (int)meta);
      const int wend = end - base;
      int at = p - base;
      while (at < wend) at = __builtin_amdgcn_readlane(next, at);
      if (at < kStop) {  // left the window
        p = base + at;
        break;
      }
      at -= kStop;  // an accepted sphere: t_max shrinks, the walk goes on after it
      tmax = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v0), at));
      hit = (int)((uint32_t)__builtin_amdgcn_readlane((int)meta, at) & 0x7fffffffu);
      p = base + at + 1;
    }
    if (kStats && lane == 0) st[28] += (long long)clock64() - c_w1;
  }
  out_tmax = tmax;
  out_hit = hit;
}

// ---------------------------------------------------------------- whole-wave closest hit by candidates
// The reference's traversal (preorder visit, box culling against the shrinking t_max) returns the
// first-visited sphere of least accepted root.  A sphere's accepted root r (q1, or q2 when q1 <= t_min:
// see above) does not depend on t_max, so take s* = the leaf of least valid r (t_min < r < inf),
// earliest in preorder among equal r.  Every sphere visited before s* is earlier in preorder, so its
// root is > r*, and the t_max at each of s*'s ancestors' visits is > r*.  An ancestor box is then
// entered (!(fminf(t_max, X) <= E), monotone in t_max) whenever fminf(r*, X) > E; if that holds for
// all of s*'s ancestors, s* is visited, accepted (t_max > r* at its visit) and never displaced (no
// root is smaller, equal roots later in preorder fail r >= t_max): the reference returns (r*, s*).
// If the ancestor check fails (a grazing box) or a root is NaN, the exact scan (coop_trace9) runs.
// A miss (no valid root at all) is exact: the reference cannot accept anything.
// Cost per ray, all from LDS: kBfSlots sphere roots per lane (the square root and divisions only
// where some lane's discriminant is >= 0), a 6-step wave argmin, and the ancestor check: the nodes
// q < p* with p* < q + skip(q), found by the lanes among all items before p* -- instead of a ~50-item
// sequential scan whose every decision is a VALU -> scalar round trip.
constexpr int kBfSlots = 8;  // 64 x 8 = 512 leaves at most (host-checked)

RT_D void box_interval(float4 q0, float4 q1, const CoopRay &C, float tmin, float &e, float &x) {
  const float t0x = (q0.x - C.ox) * C.ix, t1x = (q0.y - C.ox) * C.ix;
  const float t0y = (q0.z - C.oy) * C.iy, t1y = (q0.w - C.oy) * C.iy;
  const float t0z = (q1.x - C.oz) * C.iz, t1z = (q1.y - C.oz) * C.iz;
  const float nx = C.ix < 0 ? t1x : t0x, fx = C.ix < 0 ? t0x : t1x;
  const float ny = C.iy < 0 ? t1y : t0y, fy = C.iy < 0 ? t0y : t1y;
  const float nz = C.iz < 0 ? t1z : t0z, fz = C.iz < 0 ? t0z : t1z;
  e = fmaxf(fmaxf(fmaxf(tmin, nx), ny), nz);
  x = fminf(fminf(fx, fy), fz);
}

// Leaf n's item position is kept in a spare word of item n (q1.w of a node item, q1.x of a leaf
// item; host: book1_upload), so the per-ray sphere reads need no table and no registers held across
// the pixel (held spheres would raise the whole kernel's VGPR count and cut the lane waves'
// occupancy).  Returns false when the candidate check cannot decide; the caller then runs the
// exact scan.  Split in two so that the caller can start the hit sphere's material load before the
// ancestor check: bf_candidate returns false (undecided: a NaN root) or the candidate (r*, p*);
// p* = -1 for a miss; bf_verify is the ancestor check of a candidate p* >= 0.
RT_D bool bf_candidate(const Book1View &V, const float4 *items, const CoopRay &C, float tmin, float &out_best,
                       int &out_bp) {
  const int lane = __lane_id();
  float best = __builtin_inff();
  int bp = 0x7fffffff;  // item position of the best leaf (preorder rank)
  bool nan = false;
#pragma unroll 2
  for (int k = 0; k < kBfSlots; k++) {
    if (k * 64 >= V.n_bf_leaves) break;  // wave-uniform
    const int n = k * 64 + lane;
    const bool live = n < V.n_bf_leaves;
    const float4 h = items[2 * (live ? n : 0) + 1];
    const uint32_t hw = __float_as_uint(h.w);
    const int pos = (int)((hw & kLeaf9) ? __float_as_uint(h.x) : hw);
    const float r = coop_sphere_root(items[2 * pos], C, tmin);
    nan |= live && r != r;
    if (live && r > tmin && r < best) best = r, bp = pos;  // strict: the earlier slot wins ties
  }
#pragma unroll
  for (int off = 32; off >= 1; off >>= 1) {  // argmin over (root, preorder position)
    const float ob = __shfl_xor(best, off);
    const int op = __shfl_xor(bp, off);
    if (ob < best || (ob == best && op < bp)) best = ob, bp = op;
  }
  if (__ballot(nan) != 0) return false;
  out_best = __int_as_float(__builtin_amdgcn_readfirstlane(__float_as_int(best)));
  bp = __builtin_amdgcn_readfirstlane(bp);
  out_bp = bp == 0x7fffffff ? -1 : bp;  // no valid root anywhere: a miss
  return true;
}

RT_D bool bf_verify(const float4 *items, const CoopRay &C, float tmin, float best, int bp) {
  const int lane = __lane_id();
  bool bad = false;
  for (int base = 0; base < bp; base += 64) {  // wave-uniform bound
    const int q = base + lane;
    if (q < bp) {
      const float4 q1 = items[2 * q + 1];
      const uint32_t w = __float_as_uint(q1.w);
      if (!(w & kLeaf9) && (uint32_t)bp < (uint32_t)q + __float_as_uint(q1.z)) {  // an ancestor of p*
        float e, x;
        box_interval(items[2 * q], q1, C, tmin, e, x);
        bad |= !(fminf(best, x) > e);
      }
    }
  }
  return __ballot(bad) == 0;
}

// A whole pixel (all its samples, in order) rendered by one wave: the path state is wave-uniform
// (every lane holds the same values and runs the same shading), and each ray is traced with
// coop_trace9.  For the few pixels whose sequential chain is far longer than the frame's fair share
// (the LPT pre-pass finds them), this trades 64 lanes of throughput for a much shorter chain.
RT_D void render_pixel_coop(const Book1View &V, const float4 *items9, int64_t pix, uint8_t *__restrict__ out,
                            int glane) {
  const rt_camera &cam = V.S.cam;
  const int W = cam.width;
  const int jj = (int)(pix / W);
  const int i = (int)(pix - (int64_t)jj * W);
  const int j = V.row0 + jj * V.row_stride;
  const f3 du = ld3(cam.delta_u), dv = ld3(cam.delta_v), lf = ld3(cam.origin);
  const float tmin = 1e-3f;
  Pcg32 g;
  g.seed((uint64_t)(17 + j), (uint64_t)(23 + i));  // src/raytracing.c:94
  f3 acc = mk(0.0f, 0.0f, 0.0f);
  Lane L;
  L.ix = L.iy = L.iz = 0.0f;
  L.hit = -1;
  L.cur = 0;
  L.pend0 = L.pend1 = 0xffffu;
  L.sp = L.k = 0;
  const bool use_bf = V.n_bf_leaves > 0;
  const uint32_t px_start = V.px_time ? (uint32_t)wall_clock64() : 0u;
  for (int s = 0; s < cam.spp; s++) {
    // camera ray (src/raytracing.c:96-122)
    const f3 pixel_pos = add(add(ld3(cam.pixel00), scale(du, (float)i)), scale(dv, (float)j));
    const float px = g.between(-0.5f, 0.5f);
    const float py = g.between(-0.5f, 0.5f);
    f3 o = lf;
    if (cam.dof_angle > 0.0f) {
      float a, b;
      for (;;) {
        a = g.between(-1.0f, 1.0f);
        b = g.between(-1.0f, 1.0f);
        if (a * a + b * b < 1.0f) break;
      }
      o = add(add(lf, scale(ld3(cam.disc_u), a)), scale(ld3(cam.disc_v), b));
    }
    f3 d = add(add(add(pixel_pos, scale(du, px)), scale(dv, py)), neg(o));
    // the path record lives in the lanes: lane k holds the albedo of bounce k (max_depth <= 64)
    float ar = 0.0f, ag = 0.0f, ab = 0.0f;
    int n_b = 0;
    f3 tail = mk(0.0f, 0.0f, 0.0f);
    for (int depth = cam.max_depth; depth > 0;) {  // Camera_ray_color (src/raytracing.c:39-75)
      CoopRay C;
      C.ox = o.x, C.oy = o.y, C.oz = o.z, C.dx = d.x, C.dy = d.y, C.dz = d.z;
      C.ix = 1.0f / d.x, C.iy = 1.0f / d.y, C.iz = 1.0f / d.z;
      C.a = dot(d, d);
      C.fast = C.a >= kDivLo && C.a <= kDivHi;
      C.ra = recip_core(C.a);
      float tmax = __builtin_inff();
      int bp = -1;
      bool decided = use_bf && bf_candidate(V, items9, C, tmin, tmax, bp);
      // the hit sphere (center, 1/r, material) from its LDS item, and its material's load issued
      // before the ancestor check so that its latency overlaps it
      float4 s0 = make_float4(0.0f, 0.0f, 0.0f, 0.0f), s1 = s0;
      FastMat m;
      if (decided && bp >= 0) {
        s0 = items9[2 * bp], s1 = items9[2 * bp + 1];
        m = V.mats[__float_as_int(s1.z)];
        decided = bf_verify(items9, C, tmin, tmax, bp);
      }
      if (!decided) {  // the exact scan
        L.ox = C.ox, L.oy = C.oy, L.oz = C.oz, L.dx = C.dx, L.dy = C.dy, L.dz = C.dz;
        L.ix = C.ix, L.iy = C.iy, L.iz = C.iz, L.a = C.a, L.ra = C.ra, L.fast = C.fast;
        int hit;
        coop_trace9(V, items9, L, 0, tmin, tmax, hit);
        bp = hit;
        if (hit >= 0) {
          const rt_sphere &sp = V.S.spheres[hit];
          s0 = make_float4(sp.center[0], sp.center[1], sp.center[2], 0.0f);
          s1 = make_float4(0.0f, sp.inv_radius, __int_as_float(sp.material), 0.0f);
          m = V.mats[sp.material];
        }
      }
      if (bp < 0) {
        tail = ld3(cam.background);
        break;
      }
      const f3 p = ray_at(o, d, tmax);
      const f3 outward = scale(sub(p, mk(s0.x, s0.y, s0.z)), s1.y);
      const bool front = dot(d, outward) < 0.0f;
      const f3 normal = front ? outward : neg(outward);
      const f3 nd = scatter(m, normal, front, d, g);
      if (__lane_id() == n_b) ar = m.albedo[0], ag = m.albedo[1], ab = m.albedo[2];
      n_b++;
      o = p;
      d = nd;
      depth--;
    }
    // fold innermost first, as the recursion returns: c = 0 + a_k (x) c (rec_fold_chunk)
    f3 c = tail;
    for (int k = n_b - 1; k >= 0; k--) {
      const f3 a = mk(lane_bcast(ar, k), lane_bcast(ag, k), lane_bcast(ab, k));
      c = add(mk(0.0f, 0.0f, 0.0f), mul(a, c));
    }
    acc = add(acc, c);
  }
  if (__lane_id() == 0) {
    write_pixel(out + pix * 3, acc, cam.spp);
    if (V.px_time) V.px_time[2 * pix] = px_start, V.px_time[2 * pix + 1] = (uint32_t)wall_clock64();
  }
}

// The whole-wave kernel (rt_book1_wave_kernel), launched on a second stream next to the lane kernel:
// its first *coop_waves_dev waves claim the first *n_coop items of the order, one pixel per wave,
// heaviest first.  A kernel of its own, so that the whole-wave code's registers do not count
// against the lane kernel's occupancy; the lane kernel leaves it the same number of workgroups.
template <bool kLds>
__device__ void render_wave_items(const Book1View &V, uint8_t *__restrict__ out, char *lds) {
  const int waves = (int)*V.coop_waves_dev;
  if ((int)blockIdx.x * kWaves >= waves) return;  // whole workgroup: before the barrier
  float4 *items9 = (float4 *)lds;
  if (kLds) {
    for (int q = threadIdx.x; q < 2 * V.n_items9_alloc; q += kBlock) items9[q] = V.items9_g[q];
    __syncthreads();
  } else {
    items9 = (float4 *)V.items9_g;
  }
  const int wave = (int)(blockIdx.x * kBlock + threadIdx.x) / 64;
  if (wave >= waves) return;
  const int64_t n_coop = (int64_t)*V.n_coop;
  const int glane = (int)(blockIdx.x * kBlock + threadIdx.x);
  for (;;) {
    int k = 0;
    if (__lane_id() == 0) k = atomicAdd(V.coop_counter, 1);
    k = __shfl(k, 0);
    if (k >= n_coop) break;
    __builtin_amdgcn_s_setprio(3);  // these chains set the frame time: issue before the lane-parallel waves
    render_pixel_coop(V, items9, (int64_t)V.order[k], out, glane);
    __builtin_amdgcn_s_setprio(0);
  }
}

enum : int { kTrav = 0, kWait = 1, kExit = 2 };
constexpr int kNumStats = 29;
constexpr int kSteps = 4;

// kStats: diagnostic build only (RT_BOOK1_STATS=1) — per-lane counters of where wave iterations go,
// accumulated into V.stats with one atomic per lane at exit; never used for timing.
// kMode: 0 frame, 1 cost pre-pass (also counts draws per item), 2 split render (SplitPx above).
template <bool kLds, bool kStats = false, int kStep = 5, int kMode = 0>
__device__ void render_batched(const Book1View &V, uint8_t *__restrict__ out, char *lds) {
  const int tid = threadIdx.x;
  // the last workgroups of the grid leave their CU slots to the whole-wave kernel (render_wave_items)
  if (V.n_coop != nullptr && (int)blockIdx.x >= (int)gridDim.x - (int)((*V.coop_waves_dev + kWaves - 1) / kWaves))
    return;
  const int W = V.S.cam.width;
  const int64_t total = (int64_t)V.n_rows * W;
  // LDS: nodes (lo.x hi.x lo.y hi.y | lo.z hi.z left right) + spheres, then the 16-bit stacks
  float4 *nodes3 = (float4 *)lds;
  float4 *sph = nodes3 + (kLds ? 2 * V.n_nodes : 0);
  uint16_t *stack_base = (uint16_t *)(sph + (kLds ? V.n_spheres : 0));
  float4 *nodes7 = (float4 *)lds;  // v7: Node7 records instead of nodes + spheres
  float4 *items9 = (float4 *)lds;  // v9: preorder items, no stack
  if (kStep == 7) stack_base = (uint16_t *)(nodes7 + (kLds ? 4 * V.n_nodes7 : 0));
  if (kStep == 9) stack_base = (uint16_t *)(items9 + (kLds ? 2 * V.n_items9_alloc : 0));
  if (kLds) {
    if (kStep == 7) {
      for (int q = tid; q < 4 * V.n_nodes7; q += kBlock) nodes7[q] = V.nodes7_g[q];
    } else if (kStep == 9) {
      for (int q = tid; q < 2 * V.n_items9_alloc; q += kBlock) items9[q] = V.items9_g[q];
    } else {
      for (int q = tid; q < 2 * V.n_nodes; q += kBlock) nodes3[q] = V.nodes_g[q];
      for (int q = tid; q < V.n_spheres; q += kBlock) sph[q] = V.spheres_g[q];
    }
    __syncthreads();
  } else {
    nodes3 = (float4 *)V.nodes_g;
    sph = (float4 *)V.spheres_g;
    nodes7 = (float4 *)V.nodes7_g;
    items9 = (float4 *)V.items9_g;
  }
  uint16_t *stack = stack_base + tid;
  const int glane = blockIdx.x * kBlock + tid;
  const int lane = lane_id();
  const rt_camera &cam = V.S.cam;
  const f3 du = ld3(cam.delta_u), dv = ld3(cam.delta_v), lf = ld3(cam.origin);
  const bool dof = cam.dof_angle > 0.0f;
  const int spp = cam.spp, max_depth = cam.max_depth;
  const float tmin = 1e-3f;

  int mode = kWait;
  bool have_result = false;  // false: this lane first needs a pixel
  // stats: 0 trav iterations seen, 1 useful trav steps, 2 shade iterations seen, 3 shading lanes,
  //        4 rays traced, 5 node visits, 6 root-leaf steps, 7 shade passes where this lane was idle,
  //        8/9 shader clocks in traversal / shading iterations (wave-level, counted by lane 0 of
  //        the wave), 10/11 wave-level traversal / shading iterations, 12/13 (v6) wave-level box /
  //        sphere phases, (v5) sphere tests on the fast / exact-fallback path, 14 (v5) wave-level
  //        executions of the sphere code, 15 (v5) wave-level executions of the fallback,
  //        16/17 clock64 / wall_clock64 ticks over the wave's lifetime (lane 0), 18/19 earliest
  //        wave start / latest wave end, 20 latest wave start, 21 first time the pixel counter ran
  //        dry (wall_clock64; the host presets 18 and 21 to ~0), 22 (v5) box tests that hit,
  //        23 cooperative traces, 24 clocks in cooperative traces (lane 0), 25/26 (v9) cooperative
  //        windows / scan steps, 27/28 (v9) clocks in cooperative window evaluation / walks
  unsigned long long st[kNumStats] = {};
  long long t_iter = kStats ? (long long)clock64() : 0;
  const long long t_start = t_iter, w_start = kStats ? (long long)wall_clock64() : 0;
  int last_kind = -1;  // kind of the previous wave iteration (0 traversal, 1 shading)
  uint32_t px_steps = 0;
  long long px_t0 = 0;
  int64_t pix = 0;
  int i = 0, j = 0, s = 0, depth = 0;
  Pcg32 g;
  g.state = 0;
  g.inc = 0;
  g.n = 0;
  // split render: the chain's next sample offset and its end (the pixel's record range is re-read
  // from sp_px at sample boundaries: fewer live registers in the traversal loop)
  uint32_t so = 0, send = 0;
  bool spec = false;
  f3 acc = mk(0, 0, 0);
  Record R;
  R.r0 = R.r1 = 0;
  R.n = 0;
  Lane L;
  L.ox = L.oy = L.oz = L.dx = L.dy = L.dz = L.ix = L.iy = L.iz = 0.0f;
  L.a = L.tmax = L.ra = 0.0f;
  L.fast = false;
  L.hit = -1;
  L.cur = 0;
  L.pend0 = L.pend1 = 0xffffu;
  L.sp = L.k = 0;

  // the heaviest items (the first *n_coop of the order) are rendered by whole waves in the concurrent
  // rt_book1_wave_kernel (render_wave_items); the lanes' own items start after them
  const int64_t work_offset = V.n_coop != nullptr ? (int64_t)*V.n_coop : 0;
  const int64_t n_items1 = kMode == 2 ? (int64_t)*V.sp_n_items : 0;
  const int64_t total_own =
      kMode == 2 ? n_items1 + (V.sp_items2 ? (int64_t)min(*V.sp_n_items2, V.sp_cap2) : 0) : total - work_offset;
  const int64_t n_heavy = (V.order && V.n_heavy) ? (int64_t)*V.n_heavy : 0;
  bool heavy = false;  // this lane's pixel is among the n_heavy longest
  bool prio = false;

  for (;;) {
    const uint64_t trav = __ballot(mode == kTrav);
    const uint64_t wait = __ballot(mode == kWait);
    if (kStats) {  // wave-uniform point: charge the clocks since the last one to the previous iteration
      const long long now = (long long)clock64();
      if (lane == 0 && last_kind >= 0) st[8 + last_kind] += now - t_iter, st[10 + last_kind]++;
      t_iter = now;
    }
    if ((trav | wait) == 0) break;
    if (n_heavy > 0 || (kMode == 2 && V.experiment == 1)) {  // the longest pixels' waves issue first: their chains set the frame time
      const bool want_prio = __ballot(heavy && mode != kExit) != 0;
      if (want_prio != prio) {
        prio = want_prio;
        if (prio)
          __builtin_amdgcn_s_setprio(3);
        else
          __builtin_amdgcn_s_setprio(0);
      }
    }
    // shade once shade_batch lanes wait -- or, when fewer lanes are left (the frame's tail), once
    // 3/4 of them do, so a long path is not held back behind its wave's last traversals
    const int live = (int)__popcll(trav | wait);
    const int batch = min(V.shade_batch, (3 * live + 3) / 4);
    const bool coop = (kStep == 5 || kStep == 9) && kLds && trav != 0 && live <= V.coop_lanes &&
                      __ballot(mode == kExit) != 0;
    if (coop) {  // the frame's tail: trace each remaining ray with the whole wave
      uint16_t *ustack = stack_base + (tid & ~63);
      const long long c0 = kStats ? (long long)clock64() : 0;
      for (uint64_t m = trav; m != 0; m &= m - 1) {
        const int src = __builtin_ctzll(m);
        float t;
        int h;
        if (kStep == 9)
          coop_trace9<kStats>(V, items9, L, src, tmin, t, h, st);
        else
          coop_trace(V, nodes3, sph, ustack, L, src, tmin, t, h);
        if (lane == src) L.tmax = t, L.hit = h, mode = kWait;
        if (kStats && lane == 0) st[23]++;
      }
      if (kStats && lane == 0) st[24] += (long long)clock64() - c0;
    }
    const bool do_trav = !coop && trav != 0 && (int)__popcll(wait) < batch;
    if (kStats) last_kind = do_trav ? 0 : 1;
    if (do_trav) {
      // ---------------- traversal steps for every lane still traversing
      if (kStats && mode != kExit) st[0] += kSteps;
      if (kStep == 6) {
#pragma unroll
        for (int u = 0; u < kSteps; u++) {
          const bool pending = L.pend0 != 0xffffu;
          const uint64_t sph_lanes = __ballot(mode == kTrav && pending);
          const uint64_t box_lanes = __ballot(mode == kTrav && !pending);
          const bool sphere_phase = box_lanes == 0 || (int)__popcll(sph_lanes) >= V.sphere_batch;
          if (kStats && lane == 0) st[sphere_phase ? 13 : 12]++;
          if (sphere_phase) {
            if (mode == kTrav && pending) {
              if (kStats) st[1]++, st[6]++, px_steps++;
              sphere_step_v6(sph, L, tmin);
            }
          } else if (mode == kTrav && !pending) {
            if (kStats) st[1]++, st[5]++, px_steps++;
            box_step_v6(V, nodes3, stack, L, tmin);
          }
          if (mode == kTrav && L.pend0 == 0xffffu && L.cur == 0xffffu) mode = kWait;
        }
      } else if (mode == kTrav) {
#pragma unroll
        for (int u = 0; u < kSteps; u++)
          if (mode == kTrav) {
            px_steps++;  // work-item cost (the LPT pre-pass, stats builds)
            if (kStats) {
              st[1]++;
              if (kStep != 9) {
                if (L.cur & kLeafBit) st[6]++; else st[5]++;
              }
            }
            const bool done = kStep == 9   ? trav_step_v9<kStats>(V, items9, L, tmin, st)
                              : kStep == 7 ? trav_step_v7<kStats>(V, nodes7, stack, L, tmin, st)
                              : kStep == 5 ? trav_step_v5<kStats>(V, nodes3, sph, stack, L, tmin, st)
                                           : trav_step(V, nodes3, sph, stack, L, tmin);
            if (done) mode = kWait;
          }
      }
      continue;
    }
    if (kStats && mode != kExit) {
      st[2]++;
      if (mode == kWait) st[3]++; else st[7]++;
    }
    if (mode != kWait) continue;
    // ---------------- shading pass (Camera_ray_color body after hit(), src/raytracing.c:44-75)
    bool need_pixel = !have_result, need_sample = false;
    if (have_result) {
      bool path_done;
      f3 tail = mk(0.0f, 0.0f, 0.0f);
      if (L.hit < 0) {
        tail = ld3(cam.background);
        path_done = true;
      } else {
        const rt_sphere &sp = V.S.spheres[L.hit];
        const f3 d = mk(L.dx, L.dy, L.dz);
        const f3 p = ray_at(mk(L.ox, L.oy, L.oz), d, L.tmax);
        const f3 outward = scale(sub(p, ld3(sp.center)), sp.inv_radius);
        const bool front = dot(d, outward) < 0.0f;
        const f3 normal = front ? outward : neg(outward);
        const FastMat &m = V.mats[sp.material];
        const f3 nd = scatter(m, normal, front, d, g);
        rec_push(V, R, (uint32_t)sp.material, glane);
        L.ox = p.x, L.oy = p.y, L.oz = p.z;
        L.dx = nd.x, L.dy = nd.y, L.dz = nd.z;
        depth--;
        path_done = depth <= 0;  // the next call would return 0 at depth 0 (src/raytracing.c:40)
      }
      if (kMode == 2 && path_done) {  // split render: the chain check below decides what follows
        const f3 col = rec_fold(V, R, tail, glane);
        if (spec) {  // the record, then claim 2 (relaxed device-coherent stores: no cache maintenance;
                     // a reader that sees claim 2 before all four words checks them for the fill value)
          const uint32_t at = V.sp_px[pix].base + so;
          uint32_t *rw = (uint32_t *)(V.sp_rec + at);
          __hip_atomic_store(rw + 0, __float_as_uint(col.x), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          __hip_atomic_store(rw + 1, __float_as_uint(col.y), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          __hip_atomic_store(rw + 2, __float_as_uint(col.z), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          __hip_atomic_store(rw + 3, g.n - so, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          __hip_atomic_store(&V.sp_claim[at], 2u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        } else {
          acc = add(acc, col);
          s++;
        }
        so = g.n;
        need_sample = true;
      } else if (path_done) {
        acc = add(acc, rec_fold(V, R, tail, glane));
        s++;
        if (s == spp) {  // quantize (src/raytracing.c:127-131)
          write_pixel(out + pix * 3, acc, spp);
          if (V.cost_out) V.cost_out[pix] = px_steps;
          if (kMode == 1) V.draw_out[pix] = g.n;
          if (V.px_time) V.px_time[2 * pix + 1] = (uint32_t)wall_clock64();
          if (kStats) {
            V.pixel_cost[2 * pix] = px_steps;
            V.pixel_cost[2 * pix + 1] = (uint32_t)((long long)wall_clock64() - px_t0);
          }
          need_pixel = true;
        } else {
          need_sample = true;
        }
      }
    }
    while (need_pixel || need_sample) {
      if (need_pixel) {  // work stealing among the lanes that need a pixel right now
        const uint64_t want = __ballot(true);
        const int first = __builtin_ctzll(want);
        int base = 0;
        if (lane == first) base = atomicAdd(V.work_counter, (int)__popcll(want));
        base = __shfl(base, first);
        pix = (int64_t)base + __popcll(want & ((1ull << lane) - 1));
        if (pix >= total_own) {
          if (kStats && mode != kExit) atomicMin(&V.stats[21], (unsigned long long)wall_clock64());
          mode = kExit;
          break;
        }
        uint4 it = make_uint4(0u, 0u, 0u, 0u);
        if (kMode == 2) {  // a chain of the split launch (its items are already in longest-first order)
          it = pix < n_items1 ? V.sp_items[pix] : V.sp_items2[pix - n_items1];
          spec = (it.x & kSpecBit) != 0u;
          pix = (int64_t)(it.x & ~kSpecBit);
          heavy = !spec && V.sp_px[pix].len != 0u;  // a split pixel's head: the critical chain
        } else {
          heavy = pix + work_offset < n_heavy;
          if (V.order) pix = V.order[pix + work_offset];  // longest work items first
          else if (V.reverse) pix = total - 1 - pix;
        }
        const int jj = (int)(pix / W);
        i = (int)(pix - (int64_t)jj * W);
        j = V.row0 + jj * V.row_stride;
        g.seed((uint64_t)(17 + j), (uint64_t)(23 + i));  // src/raytracing.c:94
        acc = mk(0.0f, 0.0f, 0.0f);
        s = 0;
        if (kMode == 2) {
          const SplitPx &P = V.sp_px[pix];
          if (spec) {  // a chain from offset it.y to the segment's end it.z
            so = it.y, send = it.z;
          } else {  // the head chain, from where the last round left it
            acc = mk(P.acc[0], P.acc[1], P.acc[2]);
            so = P.o, s = (int)P.s, send = P.stop_at;
          }
          g.skip(so);
        }
        need_pixel = false;
        px_steps = 0;
        if (V.px_time) V.px_time[2 * pix] = (uint32_t)wall_clock64();
        if (kStats) px_t0 = (long long)wall_clock64();
      }
      if (kMode == 2) {  // the chain check at a sample boundary
        const uint32_t sbase = V.sp_px[pix].base, slen = V.sp_px[pix].len, srec_lo = V.sp_px[pix].rec_lo;
        if (!spec) {
          // the head is the pixel's true chain: it takes the samples segment chains have finished
          // (claim 2: record written) in order, and computes any other itself -- claiming a free
          // offset first, so segment chains that reach it stop there.  (Records exist only past
          // segment 0: sbase + o is a valid index for o >= rec_lo.)
          if (send != kNoCoalesce) {
            for (;;) {
              if (s == spp || !(so >= srec_lo && so < slen)) break;
              uint32_t *cl = &V.sp_claim[sbase + so];
              const uint32_t c = __hip_atomic_load(cl, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
              uint32_t rx = kRecFill, ry = kRecFill, rz = kRecFill, rd = kRecFill;
              if (c == 2u) {
                const uint32_t *rw = (const uint32_t *)(V.sp_rec + (uint32_t)(sbase + so));  // u32 index (wraps)
                rx = __hip_atomic_load(rw + 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                ry = __hip_atomic_load(rw + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                rz = __hip_atomic_load(rw + 2, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                rd = __hip_atomic_load(rw + 3, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
              }
              if (rx == kRecFill || ry == kRecFill || rz == kRecFill || rd == kRecFill) {
                if (c == 0u) (void)atomicCAS(cl, 0u, 1u);  // free: this chain computes it (others stop here)
                break;
              }
              acc = add(acc, mk(__uint_as_float(rx), __uint_as_float(ry), __uint_as_float(rz)));
              so += rd;
              s++;
            }
          }
          if (s == spp) {  // the pixel's last sample: quantize (src/raytracing.c:127-131)
            write_pixel(out + pix * 3, acc, spp);
            V.sp_px[pix].s = (uint32_t)spp;
            need_pixel = true;
            continue;
          }
          g.skip(so - g.n);  // past the samples taken from records
        } else if (!(so < send && so < slen && atomicCAS(&V.sp_claim[sbase + so], 0u, 1u) == 0u)) {
          need_pixel = true;  // a chain ends at its segment's end or at an offset another chain owns
          continue;
        }
      }
      // camera ray (src/raytracing.c:96-122)
      const f3 pixel_pos = add(add(ld3(cam.pixel00), scale(du, (float)i)), scale(dv, (float)j));
      const float px = g.between(-0.5f, 0.5f);
      const float py = g.between(-0.5f, 0.5f);
      f3 o = lf;
      if (dof) {
        float a, b;
        for (;;) {
          a = g.between(-1.0f, 1.0f);
          b = g.between(-1.0f, 1.0f);
          if (a * a + b * b < 1.0f) break;
        }
        o = add(add(lf, scale(ld3(cam.disc_u), a)), scale(ld3(cam.disc_v), b));
      }
      const f3 d = add(add(add(pixel_pos, scale(du, px)), scale(dv, py)), neg(o));
      L.ox = o.x, L.oy = o.y, L.oz = o.z;
      L.dx = d.x, L.dy = d.y, L.dz = d.z;
      depth = max_depth;
      R.n = 0;
      need_sample = false;
      if (kMode != 2 && depth <= 0) {  // Camera_ray_color returns 0 without tracing (host: split needs depth >= 1)
        acc = add(acc, mk(0.0f, 0.0f, 0.0f));
        s++;
        if (s == spp) {
          write_pixel(out + pix * 3, acc, spp);
          need_pixel = true;
        } else {
          need_sample = true;
        }
      }
    }
    if (mode == kExit) continue;
    // set up the traversal of the new ray
    L.ix = 1.0f / L.dx, L.iy = 1.0f / L.dy, L.iz = 1.0f / L.dz;
    L.a = dot(mk(L.dx, L.dy, L.dz), mk(L.dx, L.dy, L.dz));
    L.fast = L.a >= kDivLo && L.a <= kDivHi;
    L.ra = recip_core(L.a);
    L.tmax = __builtin_inff();
    L.hit = -1;
    L.sp = 0;
    L.k = 0;
    L.cur = kStep == 9 ? 0u : kStep == 7 ? V.root7_items[0] : V.root_items[0];
    L.pend0 = L.pend1 = 0xffffu;
    have_result = true;
    if (kStats) st[4]++;
    mode = (kStep == 9 ? V.n_items9 : V.n_root) > 0 ? kTrav : kWait;
  }
  if (kStats) {
    if (lane == 0) {  // 16/17: clock64 and wall_clock64 (100 MHz) ticks over the wave's lifetime
      st[16] = (long long)clock64() - t_start;
      st[17] = (long long)wall_clock64() - w_start;
    }
    for (int q = 0; q < 18; q++) atomicAdd(&V.stats[q], st[q]);
    atomicAdd(&V.stats[22], st[22]);
    atomicAdd(&V.stats[23], st[23]);
    atomicAdd(&V.stats[24], st[24]);
    atomicAdd(&V.stats[25], st[25]);
    atomicAdd(&V.stats[26], st[26]);
    atomicAdd(&V.stats[27], st[27]);
    atomicAdd(&V.stats[28], st[28]);
    if (lane == 0) {  // 18/19: earliest wave start, latest wave end (wall_clock64 ticks)
      atomicMin(&V.stats[18], (unsigned long long)w_start);
      atomicMax(&V.stats[19], (unsigned long long)wall_clock64());
      atomicMax(&V.stats[20], (unsigned long long)w_start);
    }
  }
}

}  // namespace b1
}  // namespace rt
