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
  int32_t batch;             // kBatch: shade once this many lanes of a wave wait (RT_GEN_BATCH)
  int32_t steps;             // kBatch: preorder entries per lane per traversal iteration (RT_GEN_STEPS)
  int32_t n_lds;             // kBatch: the first n_lds preorder entries are staged in LDS (RT_GEN_LDS)
};

// kBatch (scenes with a preorder, S.pre): the trace runs a few entries per wave iteration
// (pre_step) and a wave shades only once `batch` of its lanes wait -- as rt_book1.h's v3 loop --
// instead of every lane waiting for the wave's longest trace each bounce.
template <int F, bool kBatch = false>
__device__ void render_general(const GeneralView &V, uint8_t *__restrict__ out, float4 *lds = nullptr) {
  const DScene &S = V.S;
  const uint32_t n_lds = kBatch && lds ? (uint32_t)min(V.n_lds, S.n_pre) : 0u;
  if (n_lds) {  // the top of the preorder (the first BVH levels of every root item) in LDS
    for (uint32_t q = threadIdx.x; q < 2 * n_lds; q += blockDim.x) lds[q] = S.pre[q];
    __syncthreads();
  }
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
  // reference's vec3_add(emission_color, scatter_color) does.
  f3 rec_a[kMaxDepth];
  float rec_w[kFull ? kMaxDepth : 1];
  uint64_t weighted = 0;
  int n = 0, depth = 0, s = 0, i = 0, j = 0;
  int64_t pix = 0;
  uint32_t rays = 0;
  Pcg32 g;
  g.state = 0;
  g.inc = 0;
  f3 acc = mk(0.0f, 0.0f, 0.0f), o = acc, d = acc, pixel_pos = acc;
  bool need_pixel = true, need_sample = true, done = false;
  PreTrace T;  // kBatch: the lane's trace in progress (tracing) or finished, not yet shaded (pending)
  T.found = false;
  bool tracing = false, pending = false;

  for (;;) {
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
        if (tracing) {
#pragma unroll 1
          for (int k = 0; k < V.steps; k++)
            if (pre_step<F>(S, T, o, d, 1e-3f, g, lds, n_lds)) {
              tracing = false;
              pending = true;
              break;
            }
        }
        continue;
      }
      if (tracing) continue;  // sits out this shading pass
    }
    if (done) continue;
    bool write = spp <= 0 && !need_pixel;  // no samples: the mean is 0/0 (src/raytracing.c:127)
    // ---- camera ray (src/raytracing.c:100-122)
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
      n = 0;
      weighted = 0;
      need_sample = false;
    }
    // ---- one bounce of path_color (rt_device.h; src/raytracing.c:39-75)
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
          pre_begin(T, o, d);
          tracing = true;
          rays++;
          continue;
        }
        pending = false;
        found = T.found;
        h = T.h;
      } else {
        rays++;
        found = S.pre ? trace_pre<F>(S, o, d, 1e-3f, g, h) : trace<F>(S, o, d, 1e-3f, g, h);
      }
      if (!found) {
        tail = ld3(S.cam.background);
        path_done = true;
      } else {
        Rec r;
        make_record<F>(S, o, d, h, r);
        const f3 e = emit<F>(S, r);
        f3 dir, albedo;
        bool skip_pdf;
        if (!scatter<F>(S, r, d, g, dir, albedo, skip_pdf)) {
          tail = e;
          path_done = true;
        } else {
          rec_a[n] = albedo;
          if (kFull) {
            if ((F & RT_FEAT_LIGHTS) && (S.features & RT_FEAT_LIGHTS) && !skip_pdf) {
              if (g.f32() < prob) dir = lights_rand(S, r.p, g);
              const float sp = scatter_pdf(S, r.material, r.normal, dir);
              const float spdf = (1.0f - prob) * sp + prob * lights_pdf(S, r.p, dir);
              rec_w[n] = sp / spdf;
              weighted |= 1ull << n;
            }
          }
          n++;
          o = r.p;
          d = dir;
          depth--;
          if (kBatch && depth > 0) {  // the next bounce's trace starts at once
            pre_begin(T, o, d);
            tracing = true;
            rays++;
          }
        }
      }
    }
    if (!path_done && !write) continue;
    if (!write) {
    // ---- fold innermost-first, accumulate, next sample / pixel (src/raytracing.c:124-131)
    f3 c = tail;
    for (int k = n - 1; k >= 0; k--) {
      f3 x = mul(rec_a[k], c);
      if (kFull && ((weighted >> k) & 1)) x = scale(x, rec_w[k]);
      c = add(mk(0.0f, 0.0f, 0.0f), x);
    }
    acc = add(acc, c);
    s++;
    if (s < spp) {
      need_sample = true;
      continue;
    }
    }
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
    need_pixel = true;
  }
}

}  // namespace gen
}  // namespace rt
