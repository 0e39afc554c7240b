// rt_group.h — the group kernel for sphere/BVH scenes (reference scenes 0 and 1): eight lanes per
// pixel.  Same results as rt_book1.h (bit-exact with the reference); different trace.
//
// Why: a pixel's samples share one pcg32 stream (src/raytracing.c:93-124), so a pixel is a
// sequential chain of ~2.7k rays (up to ~25k for the heaviest).  The lane kernel runs one chain
// per lane at ~1.5-2.5k clocks per traversal step -- fine when the frame has several pixels per lane
// (one GPU), but when the frame is split over GPUs the slowest chains set the frame time.  Here a
// group of 8 lanes traces one ray in ~7 dependent steps instead of ~50.
//
// The trace.  The reference (HittableList_hit / BVHNode_hit / AABB_hit / Sphere_hit,
// src/hittable.c:38-151) returns the first-visited sphere of least accepted root, visiting in
// preorder and culling boxes against the shrinking t_max.  Let F be the leaves whose ancestors'
// boxes all pass with t_max = inf (!(fminf(inf, X) <= E)); no other leaf is ever visited.  A leaf's
// accepted root r does not depend on t_max (rt_book1.h: bf_trace), so let s* be the leaf of F of
// least valid root, earliest in preorder among equal roots: if every ancestor of s* has E < r*, the
// reference returns s* (each ancestor is then entered at any t_max > r*, which is every t_max it can
// see, since all earlier spheres have larger roots) -- else, or on a NaN root, the exact scan runs.
// F does not depend on the visit order, so the group collects it in any order: the BVH is grouped
// into treelets ("wide nodes", host: book1_upload) of up to 8 entries -- descendants of a tested node
// with up to 3 intermediate nodes each -- and lane k of the group tests entry k (its intermediates'
// boxes, then its own box or sphere), pushing passing internal entries on the group's LDS stack with
// the max E along their path.  tests/native/bf_check.cpp checks the rule against the reference order
// on the CPU (0 mismatches over 2e5 rays; ~7.5 treelets per ray on the headline scene).
#pragma once
#include "rt_book1.h"

namespace rt {
namespace grp {

constexpr int kG = 8;                  // lanes per pixel
constexpr uint32_t kGMask = (1u << kG) - 1u;
constexpr int kBlock = b1::kBlock;     // 256 threads: 32 groups
constexpr int kGroups = kBlock / kG;
constexpr int kStack = 32;             // LDS stack entries per group (overflow: exact scan)
constexpr uint32_t kEmpty = 0xffffffffu;
// treelet slot k (uint4): x = entry k's item position (kEmpty: none), y = its child treelet (internal
// entries), z = its chain (bit c: opened internal node c of the treelet lies between the treelet's
// root and the entry) | leaf << 8, w = the item position of opened internal node k (kEmpty: none).
constexpr int kMaxAnc = 16;  // ancestors per leaf in the verification table (host-checked)

// One ray of this lane's group; returns false when the rule cannot decide (the caller scans).
// out: t_max, and the winning leaf's item position (-1: a miss).  Lane k of the group tests the
// treelet's internal node k and entry k: an entry counts when its chain's internals all pass.  The
// winner's ancestors are then checked against its root (E < r*) from the per-leaf table V.anc.
RT_D bool group_trace(const b1::Book1View &V, const float4 *items, uint32_t *stk, const b1::CoopRay &C, float tmin,
                      float &out_t, int &out_pos) {
  const int lane = __lane_id();
  const int g = lane & (kG - 1), base = lane & ~(kG - 1);
  float best = __builtin_inff();
  int bpos = 0x7fffffff;
  bool nan = false, overflow = false;
  uint32_t cur = 0;  // treelet 0: the root list's items
  int sp = 0;
  bool active = true;
  while (__ballot(active) != 0) {
    bool push = false, ipass = true;
    uint32_t child = 0;
    uint4 e = make_uint4(kEmpty, 0u, 0u, kEmpty);
    if (active) {
      e = V.wide[cur * kG + g];
      if (e.w != kEmpty) {
        float be, bx;
        b1::box_interval(items[2 * e.w], items[2 * e.w + 1], C, tmin, be, bx);
        ipass = fminf(__builtin_inff(), bx) > be;
      }
    }
    const uint32_t fail = (uint32_t)(__ballot(!ipass) >> base) & kGMask;  // the group's failing internals
    if (active && e.x != kEmpty && (e.z & fail & 0xffu) == 0u) {
      const float4 q0 = items[2 * e.x];
      if (e.z & 0x100u) {
        const float r = b1::coop_sphere_root(q0, C, tmin);
        nan |= r != r;
        if (r > tmin && (r < best || (r == best && (int)e.x < bpos))) best = r, bpos = (int)e.x;
      } else {
        float be, bx;
        b1::box_interval(q0, items[2 * e.x + 1], C, tmin, be, bx);
        if (fminf(__builtin_inff(), bx) > be) push = true, child = e.y;
      }
    }
    // push the group's passing internal entries (a ballot slice per group), then pop one
    const uint32_t m = (uint32_t)(__ballot(push) >> base) & kGMask;
    if (push) {
      const int at = sp + __popc(m & ((1u << g) - 1u));
      if (at < kStack)
        stk[at] = child;
      else
        overflow = true;
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    if (active) {
      sp += __popc(m);
      if (sp > kStack) sp = kStack;  // (overflow already flagged: the result is discarded)
      if (sp == 0) {
        active = false;
      } else {
        sp--;
        cur = stk[sp];
      }
    }
    __builtin_amdgcn_wave_barrier();  // the next iteration's pushes may overwrite the popped slot
  }
  // group reduction over (root, preorder position)
#pragma unroll
  for (int off = kG / 2; off >= 1; off >>= 1) {
    const float ob = __shfl_xor(best, off);
    const int op = __shfl_xor(bpos, off);
    if (ob < best || (ob == best && op < bpos)) best = ob, bpos = op;
  }
  bool bad = nan || overflow;
  if (bpos != 0x7fffffff) {  // the winner's ancestors (all passed t_max-free): E < r* at each
#pragma unroll
    for (int q = 0; q < kMaxAnc; q += kG) {
      const uint32_t a = V.anc[(uint32_t)bpos * kMaxAnc + q + g];
      if (a != 0xffffu) {
        float be, bx;
        b1::box_interval(items[2 * a], items[2 * a + 1], C, tmin, be, bx);
        bad |= !(fminf(best, bx) > be);
      }
    }
  }
  if ((__ballot(bad) >> base) & kGMask) return false;
  if (bpos == 0x7fffffff) {
    out_t = __builtin_inff();
    out_pos = -1;
    return true;
  }
  out_t = best;
  out_pos = bpos;
  return true;
}

// The persistent group kernel: each group of 8 lanes claims pixels (longest first, V.order) and
// renders each one's samples in sequence, exactly as Camera_render (src/raytracing.c:86-135).
template <bool kLds>
__device__ void render_groups(const b1::Book1View &V, uint8_t *__restrict__ out, char *lds) {
  const int tid = threadIdx.x;
  // as the lane kernel: the last workgroups leave their slots to the whole-wave kernel, and the
  // groups' items start after the whole-wave ones (rt_book1.h: render_wave_items)
  if (V.n_coop != nullptr &&
      (int)blockIdx.x >= (int)gridDim.x - (int)((*V.coop_waves_dev + b1::kWaves - 1) / b1::kWaves))
    return;
  const int64_t work_offset = V.n_coop != nullptr ? (int64_t)*V.n_coop : 0;
  float4 *items = (float4 *)lds;
  uint32_t *stacks = (uint32_t *)(items + (kLds ? 2 * V.n_items9_alloc : 0));
  if (kLds) {
    for (int q = tid; q < 2 * V.n_items9_alloc; q += kBlock) items[q] = V.items9_g[q];
    __syncthreads();
  } else {
    items = (float4 *)V.items9_g;
  }
  uint32_t *stk = stacks + (tid / kG) * kStack;
  const int lane = __lane_id();
  const int g = lane & (kG - 1), base = lane & ~(kG - 1);
  const int spill_lane = (int)(blockIdx.x * kBlock + tid) / kG;  // one record spill column per group
  const rt_camera &cam = V.S.cam;
  const int W = cam.width;
  const int64_t total = (int64_t)V.n_rows * W - work_offset;
  const f3 du = ld3(cam.delta_u), dv = ld3(cam.delta_v), lf = ld3(cam.origin);
  const float tmin = 1e-3f;
  bool alive = true, need_pixel = true;
  int64_t pix = 0;
  int i = 0, j = 0, s = 0, depth = 0;
  Pcg32 gen;
  gen.state = gen.inc = 0;
  f3 acc = mk(0.0f, 0.0f, 0.0f), o = mk(0.0f, 0.0f, 0.0f), d = o;
  b1::Record R;
  R.r0 = R.r1 = 0;
  R.n = 0;
  bool need_ray = true;
  while (__ballot(alive) != 0) {
    // ---- pixel claims: one atomic per wave for the groups that need one
    const uint64_t want = __ballot(alive && need_pixel && g == 0);
    if (want != 0) {
      const int first = __builtin_ctzll(want);
      int b0 = 0;
      if (lane == first) b0 = atomicAdd(V.work_counter, (int)__popcll(want));
      b0 = __shfl(b0, first);
      int64_t k = (int64_t)b0 + __popcll(want & ((1ull << base) - 1));  // this group's rank among them
      k = __shfl(k, base);
      if (alive && need_pixel) {
        if (k >= total) {
          alive = false;
        } else {
          pix = V.order ? (int64_t)V.order[k + work_offset] : k;
          const int jj = (int)(pix / W);
          i = (int)(pix - (int64_t)jj * W);
          j = V.row0 + jj * V.row_stride;
          gen.seed((uint64_t)(17 + j), (uint64_t)(23 + i));  // src/raytracing.c:94
          acc = mk(0.0f, 0.0f, 0.0f);
          s = 0;
          need_pixel = false;
          need_ray = true;
          if (V.px_time && g == 0) V.px_time[2 * pix] = (uint32_t)wall_clock64();
        }
      }
    }
    if (!alive) continue;
    if (need_ray) {  // camera ray (src/raytracing.c:96-122)
      const f3 pixel_pos = add(add(ld3(cam.pixel00), scale(du, (float)i)), scale(dv, (float)j));
      const float px = gen.between(-0.5f, 0.5f);
      const float py = gen.between(-0.5f, 0.5f);
      o = lf;
      if (cam.dof_angle > 0.0f) {
        float a, b;
        for (;;) {
          a = gen.between(-1.0f, 1.0f);
          b = gen.between(-1.0f, 1.0f);
          if (a * a + b * b < 1.0f) break;
        }
        o = add(add(lf, scale(ld3(cam.disc_u), a)), scale(ld3(cam.disc_v), b));
      }
      d = add(add(add(pixel_pos, scale(du, px)), scale(dv, py)), neg(o));
      depth = cam.max_depth;
      R.n = 0;
      need_ray = false;
    }
    f3 tail = mk(0.0f, 0.0f, 0.0f);
    bool path_done = depth <= 0;  // Camera_ray_color returns 0 without tracing at depth 0
    if (!path_done) {
      b1::CoopRay C;
      C.ox = o.x, C.oy = o.y, C.oz = o.z, C.dx = d.x, C.dy = d.y, C.dz = d.z;
      C.ix = 1.0f / d.x, C.iy = 1.0f / d.y, C.iz = 1.0f / d.z;
      C.a = dot(d, d);
      C.fast = C.a >= b1::kDivLo && C.a <= b1::kDivHi;
      C.ra = b1::recip_core(C.a);
      float tmax;
      int pos;
      if (!group_trace(V, items, stk, C, tmin, tmax, pos)) {  // the exact scan (rare)
        b1::Lane L;
        L.ox = C.ox, L.oy = C.oy, L.oz = C.oz, L.dx = C.dx, L.dy = C.dy, L.dz = C.dz;
        L.ix = C.ix, L.iy = C.iy, L.iz = C.iz, L.a = C.a, L.ra = C.ra, L.fast = C.fast;
        L.tmax = __builtin_inff();
        L.hit = -1;
        L.cur = 0;
        if (V.n_items9 > 0)
          while (!b1::trav_step_v9(V, items, L, tmin)) {
          }
        tmax = L.tmax;
        pos = -1;
        if (L.hit >= 0) {  // find its item for the shading data below (the leaf's LDS record)
          pos = -2 - L.hit;
        }
      }
      if (pos == -1) {
        tail = ld3(cam.background);
        path_done = true;
      } else {
        f3 center;
        float inv_r;
        int mat;
        if (pos >= 0) {
          const float4 q0 = items[2 * pos], q1 = items[2 * pos + 1];
          center = mk(q0.x, q0.y, q0.z);
          inv_r = q1.y;
          mat = __float_as_int(q1.z);
        } else {
          const rt_sphere &sp = V.S.spheres[-2 - pos];
          center = ld3(sp.center);
          inv_r = sp.inv_radius;
          mat = sp.material;
        }
        const f3 p = ray_at(o, d, tmax);
        const f3 outward = scale(sub(p, center), inv_r);
        const bool front = dot(d, outward) < 0.0f;
        const f3 normal = front ? outward : neg(outward);
        const b1::FastMat &m = V.mats[mat];
        const f3 nd = b1::scatter(m, normal, front, d, gen);
        b1::rec_push(V, R, (uint32_t)mat, spill_lane);
        o = p;
        d = nd;
        depth--;
        path_done = depth <= 0;
      }
    }
    if (path_done) {
      acc = add(acc, b1::rec_fold(V, R, tail, spill_lane));
      s++;
      need_ray = true;
      if (s == cam.spp) {  // quantize (src/raytracing.c:127-131)
        if (g == 0) {
          b1::write_pixel(out + pix * 3, acc, cam.spp);
          if (V.px_time) V.px_time[2 * pix + 1] = (uint32_t)wall_clock64();
        }
        need_pixel = true;
      }
    }
  }
}

}  // namespace grp
}  // namespace rt
