// rt_kernel.hip — gfx950 render kernels + the C ABI declared in include/rt_hip.h.
//
// Work decomposition: one lane = one pixel (the reference's per-pixel pcg32 stream is sequential
// across that pixel's samples, so pixels are the only parallel axis: SURVEY §0.6).  A launch
// covers a set of image rows row0 + k*row_stride; multi-GPU runs give GPU g the rows j % G == g
// (interleaved) and need no collective: each GPU writes its own compact rows.
//
// Kernel variants are compiled per feature set (rt_flat.h rt_feature_bits) so the Book-1 scenes
// do not carry quad / transform / medium / light-sampling code.
#include <hip/hip_runtime.h>

#include <math.h>
#include <stdarg.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>

#include <mutex>
#include <functional>
#include <vector>

#include "../../include/rt_hip.h"
#include "rt_book1.h"
#include "rt_group.h"
#include "rt_general.h"
#include "rt_device.h"

using namespace rt;

// ------------------------------------------------------------------------------ errors
static thread_local char g_err[1024];

extern "C" void rt_set_error(const char *fmt, ...) {
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(g_err, sizeof g_err, fmt, ap);
  va_end(ap);
}
extern "C" const char *rt_last_error(void) { return g_err; }
extern "C" int rt_abi_version(void) { return RT_ABI_VERSION; }

#define HIP_OK(expr)                                                                               \
  do {                                                                                             \
    hipError_t e_ = (expr);                                                                        \
    if (e_ != hipSuccess) {                                                                        \
      rt_set_error("%s failed: %s (%s:%d)", #expr, hipGetErrorString(e_), __FILE__, __LINE__);     \
      return -1;                                                                                   \
    }                                                                                              \
  } while (0)

// ------------------------------------------------------------------------------ kernels
constexpr int kBlock = 256;

template <int F>
__global__ __launch_bounds__(kBlock) void rt_render_rows_kernel(DScene S, int row0, int row_stride, int n_rows,
                                                                uint8_t *__restrict__ out) {
  const int W = S.cam.width;
  const int64_t pix = (int64_t)blockIdx.x * kBlock + threadIdx.x;
  if (pix >= (int64_t)n_rows * W) return;
  const int jj = (int)(pix / W);
  const int i = (int)(pix - (int64_t)jj * W);
  render_pixel<F>(S, i, row0 + jj * row_stride, out + pix * 3);
}

// Persistent Book-1 kernel (rt_book1.h): grid = resident workgroups, lanes steal pixels.
// kOcc > 0: ask the register allocator for that many waves per SIMD (launch-bounds minimum).
template <bool kLds, int kVer, bool kStats = false, int kOcc = 0>
__global__ __launch_bounds__(b1::kBlock, kOcc > 0 ? kOcc : 1) void rt_book1_kernel(b1::Book1View V, uint8_t *__restrict__ out) {
  extern __shared__ __attribute__((aligned(16))) char lds[];
  if (kVer >= 3)  // batched megaloop; kStep 3 / 5 / 6 = traversal step generation
    b1::render_batched<kLds, kStats, kVer>(V, out, lds);
  else
    b1::render<kLds>(V, out, lds);
}

// The group kernel (rt_group.h): eight lanes per pixel, for frames with few pixels per lane.
template <bool kLds>
__global__ __launch_bounds__(grp::kBlock) void rt_book1_group_kernel(b1::Book1View V, uint8_t *__restrict__ out) {
  extern __shared__ __attribute__((aligned(16))) char lds[];
  grp::render_groups<kLds>(V, out, lds);
}

// The whole-wave items of a Book-1 launch (rt_book1.h: render_wave_items), concurrent with the lane
// kernel on a second stream.
template <bool kLds>
__global__ __launch_bounds__(b1::kBlock) void rt_book1_wave_kernel(b1::Book1View V, uint8_t *__restrict__ out) {
  extern __shared__ __attribute__((aligned(16))) char lds[];
  b1::render_wave_items<kLds>(V, out, lds);
}

// The LPT cost pre-pass: the same persistent kernel at low spp, under its own name so profiles
// separate it from the frame's launch.
template <bool kLds, int kVer>
__global__ __launch_bounds__(b1::kBlock) void rt_book1_cost_kernel(b1::Book1View V, uint8_t *__restrict__ out) {
  extern __shared__ __attribute__((aligned(16))) char lds[];
  b1::render_batched<kLds, false, kVer, 1>(V, out, lds);
}

// Split render (rt_book1.h: SplitPx): the chains of one round -- head chains and segment windows.
template <bool kLds>
__global__ __launch_bounds__(b1::kBlock, 5) void rt_book1_split_kernel(b1::Book1View V, uint8_t *__restrict__ out) {
  extern __shared__ __attribute__((aligned(16))) char lds[];
  b1::render_batched<kLds, false, 9, 2>(V, out, lds);
}

// Split render: expand the host's entries (a head chain, or a segment's window {pix, B, E, w}) into
// one chain per window start offset, in the entries' (longest-first) order.
__global__ void split_expand_kernel(const uint4 *ent, const uint32_t *pre, uint32_t n, uint4 *items) {
  for (uint32_t e = blockIdx.x * blockDim.x + threadIdx.x; e < n; e += gridDim.x * blockDim.x) {
    const uint4 x = ent[e];
    const uint32_t w = x.w ? x.w : 1u, at = pre[e];
    for (uint32_t q = 0; q < w; q++) items[at + q] = make_uint4(x.x, x.y + q, x.z, 1u);
  }
}

// Split render, before a fix-up round: the chains for the pixels the walk left unfinished.  A pixel
// whose stream ran past the offsets its segment chains covered (the pre-pass under-estimated it) is
// split again from its exact position, with the stream length now estimated from its own samples;
// any other continues as a head chain (it coalesces with the records at the next claimed offset).
// The heads stay in the walk's list (sp_items); the new segment chains go to sp_items2 (one wave per
// pixel writes them).  A reservation past `cap` is filled with empty chains (start past end).
__global__ void split_replan_kernel(b1::Book1View V, const uint4 *heads, const uint32_t *n_heads, uint4 *items,
                                    uint32_t *n_items, uint32_t cap, float cstar, float margin, int kmax, int last_round) {
  const uint32_t n = *n_heads;
  const uint32_t spp = (uint32_t)V.S.cam.spp;
  const int lane = __lane_id();
  const uint32_t waves = gridDim.x * (blockDim.x / 64);
  for (uint32_t k = (blockIdx.x * blockDim.x + threadIdx.x) / 64; k < n; k += waves) {
    const uint32_t pix = heads[k].x;
    b1::SplitPx &P = V.sp_px[pix];
    if (last_round || !(P.o < P.len && P.s > 0 && P.s < spp)) continue;
    const uint32_t r = spp - P.s, w = P.w, o = P.o;
    const double mu = (double)o / (double)P.s;
    const uint32_t run = (uint32_t)fmin((double)(P.len - o), ceil((double)r * mu * margin) + w);
    int K = (int)fmin((double)kmax, ceil((double)r * P.cps / cstar));
    K = (int)fmin((double)K, floor((double)run / (4.0 * w)));
    if (K < 2) continue;  // a head chain through the rest
    const uint32_t L = (run + K - 1) / K;
    const uint32_t need = (uint32_t)(K - 1) * w;
    uint32_t at = 0;
    if (lane == 0) at = atomicAdd(n_items, need);
    at = __shfl(at, 0);
    const bool ok = at + need <= cap;
    for (uint32_t q = lane; q < need; q += 64) {
      if (at + q >= cap) break;
      const uint32_t seg = 1u + q / w, t = q % w;
      const uint32_t B = o + seg * L, E = seg + 1 == (uint32_t)K ? o + run : o + (seg + 1) * L;
      items[at + q] = ok ? make_uint4(pix | b1::kSpecBit, B + t, E, 1u) : make_uint4(pix | b1::kSpecBit, 1u, 0u, 1u);
    }
    if (ok && lane == 0) {
      P.stop_at = o + L;
      P.len_run = o + run;
    }
  }
}

// Split render, after a round: follow each listed pixel's true chain through the sample records,
// adding the colours in sample order (the reference's sum, src/raytracing.c:124).  A pixel whose
// chain reaches spp samples is written; one that reaches an offset without a record (never
// evaluated) is listed for the next round as a head chain from there.
__global__ void split_walk_kernel(b1::Book1View V, uint8_t *__restrict__ out, const uint4 *in, const uint32_t *n_in,
                                  uint4 *next, uint32_t *n_next, int last_round) {
  const uint32_t n = *n_in;
  const uint32_t spp = (uint32_t)V.S.cam.spp;
  for (uint32_t k = blockIdx.x * blockDim.x + threadIdx.x; k < n; k += gridDim.x * blockDim.x) {
    const uint32_t pix = in[k].x & ~b1::kSpecBit;
    b1::SplitPx &P = V.sp_px[pix];
    uint32_t s = P.s, o = P.o;
    if (s >= spp) continue;  // written by its head chain
    const uint32_t base = P.base, len = P.len;
    f3 acc = mk(P.acc[0], P.acc[1], P.acc[2]);
    while (s < spp && o < len && V.sp_claim[base + o] == 2u) {
      const float4 r = V.sp_rec[base + o];  // (after the round's kernel: every claimed record is complete)
      acc = add(acc, mk(r.x, r.y, r.z));
      o += __float_as_uint(r.w);
      s++;
    }
    if (s == spp) {
      b1::write_pixel(out + (size_t)pix * 3, acc, (int)spp);
      P.s = spp;
    } else {
      P.acc[0] = acc.x, P.acc[1] = acc.y, P.acc[2] = acc.z;
      P.o = o, P.s = s;
      P.stop_at = last_round ? b1::kNoCoalesce : b1::kNoStop;  // a head chain that stops at a claimed offset
      next[atomicAdd(n_next, 1u)] = make_uint4(pix, 0u, 0u, 0u);
    }
  }
}

// Persistent general kernel (rt_general.h): grid = resident workgroups, lanes steal pixels.
template <int F, bool kBatch = false>
__global__ __launch_bounds__(gen::kBlock, kBatch ? 3 : 1) void rt_general_kernel(gen::GeneralView V, uint8_t *__restrict__ out) {
  extern __shared__ __attribute__((aligned(16))) char lds[];
  gen::render_general<F, kBatch>(V, out, (float4 *)lds);
}

__global__ void rt_diag_libm_kernel(int fn, const float *x, float *out, int64_t n) {
  const int64_t k = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (k >= n) return;
  const float v = x[k];
  if (fn == 0) {
    float s, c;
    rtm::sincosf(v, &s, &c);
    out[2 * k] = s;
    out[2 * k + 1] = c;
  } else if (fn == 1) {
    out[k] = rtm::powf(v, 5.0f);
  } else if (fn == 2) {
    out[k] = rtm::logf(v);
  } else if (fn == 3) {
    out[k] = rtm::sinf(v);
  } else if (fn == 4) {  // atan2f(y = x[2k], x = x[2k+1]) for k < n/2
    if (2 * k + 1 < n) out[k] = rtm::atan2f(x[2 * k], x[2 * k + 1]);
  } else {
    out[k] = rtm::acosf(v);
  }
}

// Exactness checks of the Book-1 v5 arithmetic (rt_book1.h: sqrt_core / div_core / sphere_test_v5)
// against what the compiler emits for sqrtf() and '/' -- run on the device, count mismatches.
//  fn 0: sqrt_core(x) vs sqrtf(x), x = the float with bits start + k, where x is in the core's domain
//  fn 1: div_core vs '/' on hashed pairs (a in [kDivLo, kDivHi], |x| in [2^-40, kNumHi] or 0)
//  fn 2: sphere_test_v5 vs the v3 sphere test (outcome: hit index and t_max bits) on hashed rays,
//        half of them starting on the sphere's surface (the scattered-ray case: c ~ 0)
RT_D uint64_t diag_hash(uint64_t x) {  // splitmix64 finaliser
  x += 0x9e3779b97f4a7c15ull;
  x = (x ^ (x >> 30)) * 0xbf58476d1ce4e5b9ull;
  x = (x ^ (x >> 27)) * 0x94d049bb133111ebull;
  return x ^ (x >> 31);
}
RT_D float diag_float(uint64_t h, int emin, int emax) {  // random sign/mantissa, exponent in [emin, emax]
  const int e = emin + (int)((h >> 40) % (uint64_t)(emax - emin + 1));
  return __uint_as_float((uint32_t)((h >> 63) << 31) | (uint32_t)((e + 127) << 23) | (uint32_t)(h & 0x7fffff));
}
__global__ void rt_diag_arith_kernel(int fn, uint64_t start, uint64_t count, uint64_t seed,
                                     unsigned long long *mism) {
  if (fn == 3) {  // timing: a dependent v_readlane chain, clocks per hop
    const int lane = __lane_id();
    const int next = (lane + 1 + (int)(seed & 7)) & 63;
    int at = 0;
    const long long t0 = (long long)clock64();
    for (uint64_t k = 0; k < count; k++) at = __builtin_amdgcn_readlane(next, at);
    const long long t1 = (long long)clock64();
    if (lane == 0) mism[0] = (unsigned long long)((t1 - t0) * 1000 / (long long)(count ? count : 1)) + (at == 1000 ? 1 : 0);
    return;
  }
  unsigned long long bad = 0;
  for (uint64_t k = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; k < count; k += (uint64_t)gridDim.x * blockDim.x) {
    if (fn == 0) {
      const float x = __uint_as_float((uint32_t)(start + k));
      if (!(x == 0.0f || (x >= b1::kSqrtLo && x <= __FLT_MAX__))) continue;
      bad += __float_as_uint(b1::sqrt_core(x)) != __float_as_uint(sqrtf(x));
    } else if (fn == 1) {
      const uint64_t h1 = diag_hash(seed ^ (start + k)), h2 = diag_hash(h1);
      const float a = fabsf(diag_float(h1, -20, 19));
      float x = diag_float(h2, -40, 39);
      if ((h2 & 0xff00000) == 0) x = 0.0f;
      bad += __float_as_uint(b1::div_core(x, a, b1::recip_core(a))) != __float_as_uint(x / a);
    } else {
      const uint64_t h1 = diag_hash(seed ^ (start + k)), h2 = diag_hash(h1), h3 = diag_hash(h2), h4 = diag_hash(h3);
      const float4 sph = make_float4(diag_float(h1, -2, 3), diag_float(h1 >> 7, -2, 3), diag_float(h1 >> 13, -2, 3), 0.0f);
      const float r = fabsf(diag_float(h2, -4, 9));
      float4 sp = sph;
      sp.w = r * r;
      f3 d = mk(diag_float(h3, -3, 2), diag_float(h3 >> 9, -3, 2), diag_float(h3 >> 17, -3, 2));
      f3 o;
      if (h4 & 1) {  // on the surface (up to rounding), like a scattered ray
        const float inv = 1.0f / sqrtf(dot(d, d));
        const f3 n = mk(d.z * inv, d.x * inv, d.y * inv);
        o = add(mk(sph.x, sph.y, sph.z), scale(n, r));
      } else {
        o = mk(diag_float(h4, -3, 6), diag_float(h4 >> 11, -3, 6), diag_float(h4 >> 21, -3, 6));
      }
      b1::Lane A;
      A.ox = o.x, A.oy = o.y, A.oz = o.z, A.dx = d.x, A.dy = d.y, A.dz = d.z;
      A.ix = A.iy = A.iz = 0.0f;
      A.a = dot(d, d);
      A.ra = b1::recip_core(A.a);
      A.fast = A.a >= b1::kDivLo && A.a <= b1::kDivHi;
      A.tmax = (h4 & 2) ? __builtin_inff() : fabsf(diag_float(h4 >> 5, -4, 10));
      A.hit = -1;
      A.cur = 0;
      A.sp = A.k = 0;
      b1::Lane B = A;
      b1::sphere_test_v5(&sp, 0, A, 1e-3f);
      b1::sphere_test_lane(&sp, 0, B, 1e-3f);
      bad += (A.hit != B.hit) || (__float_as_uint(A.tmax) != __float_as_uint(B.tmax));
    }
  }
  if (bad) atomicAdd(mism, bad);
}

// Longest-first work order (rt_render_rows_async): bucket work items by log2(cost) with 3 mantissa
// bits (256 buckets), highest bucket first.  Order inside a bucket is arbitrary (atomics): any order
// renders the same image, the order only decides which pixels start first.
__device__ __forceinline__ uint32_t lpt_bucket(uint32_t c) {
  c |= 1u;
  const int e = 31 - __clz(c);
  const uint32_t frac = e >= 3 ? (c >> (e - 3)) & 7u : (c << (3 - e)) & 7u;
  const uint32_t k = (uint32_t)e * 8u + frac;
  return k > 255u ? 255u : k;
}
static uint32_t host_lpt_bucket(uint32_t c) {  // lpt_bucket on the host
  c |= 1u;
  const int e = 31 - __builtin_clz(c);
  const uint32_t frac = e >= 3 ? (c >> (e - 3)) & 7u : (c << (3 - e)) & 7u;
  const uint32_t k = (uint32_t)e * 8u + frac;
  return k > 255u ? 255u : k;
}
__global__ void lpt_hist_kernel(const uint32_t *cost, int n, uint32_t *hist, unsigned long long *sums) {
  __shared__ uint32_t h[256];
  __shared__ unsigned long long w[256];
  for (int k = threadIdx.x; k < 256; k += blockDim.x) h[k] = 0, w[k] = 0;
  __syncthreads();
  for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) {
    const uint32_t b = lpt_bucket(cost[i]);
    atomicAdd(&h[b], 1u);
    atomicAdd(&w[b], (unsigned long long)cost[i]);
  }
  __syncthreads();
  for (int k = threadIdx.x; k < 256; k += blockDim.x) {
    if (h[k]) atomicAdd(&hist[k], h[k]);
    if (w[k]) atomicAdd(&sums[k], w[k]);
  }
}

// Cost model of one launch for the split between whole-wave pixels (render_pixel_coop) and lane (or
// group) pixels, in clocks per pre-pass step (measured on the headline frame): the
// frame ends when the slowest lane pixel's chain (lat_step), the lanes' aggregate work (thr_step per
// lane), the whole-wave queue and the heaviest whole-wave pixel's chain (coop_step) are all done.
// LPT scratch: 256 bucket counts, 256 running offsets, 4 split counters (u32 [512..515]), then from
// u32 544 the 256 per-bucket step sums (u64): 2176 + 2048 bytes
constexpr size_t kLptHistBytes = 8192;

struct LptModel {
  float spp_ratio;  // frame spp / pre-pass spp (costs are pre-pass steps)
  int grid_waves;
  float lat_step;   // clocks per step of the slowest lane (group) pixels under load: their chain
  float thr_step;   // clocks per step per lane (group) of all lanes' (groups') aggregate rate
  float coop_step;  // clocks per step of a whole-wave pixel (its chain, and its wave's rate)
  int lanes_per_wave;  // pixels in flight per non-cooperative wave: 64 lanes, or 8 groups
  int debug;           // RT_DEBUG: print the model's inputs and choice
};
// clocks per pre-pass step, fitted to frame times on one MI355X (scripts/tail_probe.py measures the
// per-pixel rates: lane pixels ~1.6-4k by load, group ~0.6-1.1k, whole-wave ~120-180)
constexpr float kLaneLat = 1900.0f, kLaneThr = 2714.0f, kGroupLat = 850.0f, kGroupThr = 850.0f;
constexpr float kCoopStep = 180.0f, kCoopStepLane = 250.0f;

// one thread: offsets, highest bucket first; hist[512] = items in buckets above the chosen split
// (rendered by whole waves), hist[513] = their claim counter, hist[514] = items above `prio_bucket`
// (raised priority), hist[515] = whole waves.  coop_bucket / coop_waves < 0: chosen by the model.
__global__ void lpt_scan_kernel(uint32_t *hist, const unsigned long long *sums, int coop_bucket, int coop_waves,
                                int prio_bucket, LptModel m) {
  if (threadIdx.x != 0) return;
  uint32_t run = 0, heavy = 0;
  for (int k = 255; k >= 0; k--) {
    hist[256 + k] = run;
    run += hist[k];
    if (k > prio_bucket) heavy += hist[k];
  }
  double total = 0.0;
  for (int k = 0; k < 256; k++) total += (double)sums[k];
  int best_b = coop_bucket >= 0 ? coop_bucket : 255, best_w = coop_waves >= 0 ? coop_waves : 0;
  if (coop_bucket < 0 || coop_waves < 0) {
    // highest non-empty bucket at or below each bucket (the largest lane pixel of a split)
    int16_t top_of[256];
    for (int k = 0, t = -1; k < 256; k++) top_of[k] = (int16_t)(t = hist[k] ? k : t);
    const double top_all = top_of[255] < 0 ? 0.0
                                           : ldexp((double)(9 + (top_of[255] & 7)) / 8.0, top_of[255] >> 3) * m.spp_ratio;
    double best_t = 1e300;
    for (int wc = 0; wc <= m.grid_waves / 2; wc = wc ? 2 * wc : 128) {
      if (coop_waves >= 0 && wc != coop_waves) continue;
      double coop_work = 0.0;  // steps above the split
      for (int b = 255; b >= -1; b--) {
        if (b < 255) coop_work += (double)sums[b + 1];
        if (coop_bucket >= 0 && b != coop_bucket) continue;
        if (wc == 0 && coop_work > 0.0) break;
        // the largest lane pixel: the top of bucket b (or of the highest non-empty one)
        const int top = b < 0 ? -1 : top_of[b];
        const double maxc = top < 0 ? 0.0 : ldexp((double)(9 + (top & 7)) / 8.0, top >> 3) * m.spp_ratio;
        const double lanes = (double)(m.grid_waves - wc) * m.lanes_per_wave;
        const double t_dfs = fmax(maxc * m.lat_step, (total - coop_work) * m.spp_ratio * m.thr_step / lanes);
        // whole waves: their queue, and the heaviest pixel's own chain
        const double t_coop = wc ? fmax(coop_work * m.spp_ratio * m.coop_step / wc, top_all * m.coop_step) : 0.0;
        const double t = fmax(t_dfs, t_coop);
        if (t < best_t) best_t = t, best_b = b, best_w = wc;
      }
    }
  }
  uint32_t coop = 0;
  for (int k = 255; k > best_b; k--) coop += hist[k];
  if (m.debug)
    printf("[lpt_scan] ratio %f grid_waves %d lat %f thr %f coop %f lpw %d total %f best_b %d best_w %d\n", m.spp_ratio,
           m.grid_waves, m.lat_step, m.thr_step, m.coop_step, m.lanes_per_wave, total, best_b, best_w);
  hist[512] = best_w > 0 ? coop : 0;
  hist[513] = 0;
  hist[514] = heavy;
  hist[515] = (uint32_t)best_w;
}

__global__ void lpt_scatter_kernel(const uint32_t *cost, int n, uint32_t *hist, int32_t *order) {
  for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x)
    order[atomicAdd(&hist[256 + lpt_bucket(cost[i])], 1u)] = i;
}

// The whole-wave items (the first hist[512] of the order) exactly longest first: the buckets keep
// an arbitrary order among items of up to 12.5 % different cost, and with a few whole waves per
// hundred items the heaviest pixel could start only after a wave's first item (measured at N = 8:
// started at 72 ms, the frame's last item).  One workgroup, bitonic sort of up to kCoopSort items.
constexpr int kCoopSort = 8192;
__global__ __launch_bounds__(1024) void lpt_coop_sort_kernel(const uint32_t *cost, const uint32_t *hist, int32_t *order) {
  __shared__ uint32_t key[kCoopSort];
  __shared__ int32_t val[kCoopSort];
  const int n = (int)min(hist[512], (uint32_t)kCoopSort);
  if (n < 2) return;
  int m = 2;
  while (m < n) m <<= 1;
  for (int i = threadIdx.x; i < m; i += blockDim.x) {
    key[i] = i < n ? cost[order[i]] : 0u;  // padding sorts last (descending)
    val[i] = i < n ? order[i] : -1;
  }
  __syncthreads();
  for (int k = 2; k <= m; k <<= 1)
    for (int j = k >> 1; j > 0; j >>= 1) {
      for (int i = threadIdx.x; i < m; i += blockDim.x) {
        const int l = i ^ j;
        if (l > i) {
          const bool desc = (i & k) == 0;  // descending overall
          const uint32_t a = key[i], b = key[l];
          if (desc ? a < b : a > b) {
            key[i] = b, key[l] = a;
            const int32_t t = val[i];
            val[i] = val[l], val[l] = t;
          }
        }
      }
      __syncthreads();
    }
  for (int i = threadIdx.x; i < n; i += blockDim.x) order[i] = val[i];
}

// ------------------------------------------------------------------------------ device scene
struct rt_device_scene {
  int device;
  DScene view;
  void *arena;
  size_t arena_bytes;
  int features;
  int width, height;
  // Book-1 fast path (rt_book1.h), when the scene qualifies
  bool book1 = false;
  bool book1_lds = false;
  int book1_ver = 9;
  int book1_occ = 0;         // register-allocation occupancy target of the launched variant (0: default)
  bool book1_stats = false;  // diagnostic counters build (RT_BOOK1_STATS=1)
  b1::Book1View b1view;
  void *b1_arena = nullptr;
  // longest-first work order from a low-spp cost pre-pass (RT_LPT, RT_LPT_SPP)
  bool lpt = false;
  int lpt_spp = 8;
  uint32_t *lpt_cost = nullptr;  // steps per work item (W*H)
  int32_t *lpt_order = nullptr;  // work item order (W*H)
  uint32_t *lpt_hist = nullptr;  // 256 bucket counts, 256 running offsets, cooperative count + counter
  int coop_steps = -1;           // pre-pass steps per sample above which a pixel goes to a whole wave (-1: model)
  int coop_waves = -1;           // waves that render those pixels first (0: off, -1: model)
  int prio_steps = 0;            // pre-pass steps per sample above which a pixel's wave runs at priority 3
  hipEvent_t ev_main[2] = {nullptr, nullptr};  // bracket the last frame launch (rt_scene_last_launch_ms)
  // persistent general path (rt_general.h) for scenes outside the Book-1 path
  bool general = false;
  void *gen_arena = nullptr;
  int32_t *gen_counter = nullptr;
  int gen_grid = 0;
  int b1_grid = 0;
  size_t b1_lds_bytes = 0;
  uint32_t *px_time = nullptr;  // RT_PX_TIME diagnostic: {start, end} per work item
  int group_mode = 2;                 // RT_MODE: 0 lane kernel, 1 group kernel, 2 auto (by pixels per lane)
  int g_grid = 0;                     // group kernel: resident workgroups, LDS bytes per workgroup
  size_t g_lds_bytes = 0;
  hipStream_t wave_stream = nullptr;  // the whole-wave kernel's stream (forked from / joined to the caller's)
  hipEvent_t ev_fork = nullptr, ev_join = nullptr;
  // split render (rt_book1.h: SplitPx), RT_SPLIT: 0 off (default), 1 every LPT launch, 2 launches with fewer
  // pixels than lanes
  int split_mode = 0;
  float split_beta = 0.7f;    // a chain's target cost, as a fraction of the frame's throughput time
  float split_margin = 1.1f;  // first-round chains cover this times the pre-pass estimate of the stream length
  float split_alloc = 1.0f;   // records per pixel: this times the estimate (a re-split continues into them)
  float split_fixc = 0.25f;   // a re-split's chain target, as a fraction of the first round's
  float split_wfact = 2.0f;   // window: this times the pre-pass draws per sample
  int split_kmax = 64, split_rounds = 0;  // rounds queued before the host checks (heads walk: usually none)
  uint32_t *draw_out = nullptr;  // pre-pass draws per work item (W*H)
  void *sp_arena = nullptr;
  size_t sp_bytes = 0;
  std::vector<uint32_t> h_cost, h_draws;
  std::vector<b1::SplitPx> h_px;
  std::vector<uint4> h_items, h_walk;
  std::vector<uint32_t> h_pre;
  uint32_t h_cnt[256];  // device counters: [0] chains, [1] split pixels, [2 + r] / [128 + r] round r's
  int split_rounds_used = 0;
  int sp_grid = 0;  // resident workgroups of rt_book1_split_kernel
  void *pre_arena = nullptr;  // the general path's preorder entries (rt_device.h: trace_pre)
  int gen_batch = 0;          // general kernel: batched shading threshold (0: one bounce per iteration)
  int gen_steps = 8;          // general kernel: preorder entries per traversal iteration
  int gen_lds = 0;            // general kernel: preorder entries staged in LDS
};

static size_t align_up(size_t x, size_t a) { return (x + a - 1) / a * a; }

static bool ref_ok(const rt_flat_scene *s, int32_t ref, bool allow_none) {
  if (ref == RT_REF_NONE) return allow_none;
  const int32_t i = rt_ref_index(ref);
  switch (rt_ref_kind(ref)) {
  case RT_KIND_BVH: return i < s->n_bvh;
  case RT_KIND_SPHERE: return i < s->n_spheres;
  case RT_KIND_QUAD: return i < s->n_quads;
  case RT_KIND_LIST: return i < s->n_lists;
  case RT_KIND_TRANSLATE: return i < s->n_translates;
  case RT_KIND_ROTATE_Y: return i < s->n_rotates;
  case RT_KIND_MEDIUM: return i < s->n_media;
  default: return false;
  }
}

// Every index the kernel will follow is checked here, so a malformed scene fails on the host
// instead of faulting the GPU.
static int validate(const rt_flat_scene *s) {
  const rt_camera &c = s->camera;
  if (c.width <= 0 || c.height <= 0 || c.spp <= 0) return rt_set_error("bad image size / spp"), -1;
  if (c.max_depth > kMaxDepth)
    return rt_set_error("max_depth %d exceeds the kernel's path record (%d)", c.max_depth, kMaxDepth), -1;
  if (s->stack_needed > kStackMax)
    return rt_set_error("scene needs %d traversal stack slots, kernel has %d", s->stack_needed, kStackMax), -1;
  if (!ref_ok(s, s->root, false) || rt_ref_kind(s->root) != RT_KIND_LIST) return rt_set_error("bad root"), -1;
  if (s->lights < 0 || s->lights >= s->n_lists) return rt_set_error("bad lights list"), -1;
  for (int k = 0; k < s->n_bvh; k++)
    if (!ref_ok(s, s->bvh[k].left, false) || !ref_ok(s, s->bvh[k].right, true)) return rt_set_error("bad bvh ref"), -1;
  for (int k = 0; k < s->n_lists; k++)
    if (s->lists[k].first < 0 || s->lists[k].count < 0 || s->lists[k].first + s->lists[k].count > s->n_list_items)
      return rt_set_error("bad list range"), -1;
  for (int k = 0; k < s->n_list_items; k++)
    if (!ref_ok(s, s->list_items[k], true)) return rt_set_error("bad list item"), -1;
  for (int k = 0; k < s->n_translates; k++)
    if (!ref_ok(s, s->translates[k].child, false) || !ref_ok(s, s->translates[k].parent_xform, true))
      return rt_set_error("bad translate"), -1;
  for (int k = 0; k < s->n_rotates; k++)
    if (!ref_ok(s, s->rotates[k].child, false) || !ref_ok(s, s->rotates[k].parent_xform, true))
      return rt_set_error("bad rotate"), -1;
  for (int k = 0; k < s->n_media; k++) {
    const rt_medium &m = s->media[k];
    const int bk = rt_ref_kind(m.boundary);
    if (!ref_ok(s, m.boundary, false) || (bk != RT_KIND_SPHERE && bk != RT_KIND_QUAD) || m.phase_material < 0 ||
        m.phase_material >= s->n_materials)
      return rt_set_error("bad medium"), -1;
  }
  for (int k = 0; k < s->n_spheres; k++)
    if (s->spheres[k].material < 0 || s->spheres[k].material >= s->n_materials) return rt_set_error("bad material"), -1;
  for (int k = 0; k < s->n_quads; k++)
    if (s->quads[k].material < 0 || s->quads[k].material >= s->n_materials) return rt_set_error("bad material"), -1;
  for (int k = 0; k < s->n_materials; k++) {
    const rt_material &m = s->materials[k];
    const bool needs_tex = m.tag == RT_MAT_LAMBERTIAN || m.tag == RT_MAT_METAL || m.tag == RT_MAT_DIFFUSE_LIGHT ||
                           m.tag == RT_MAT_ISOTROPIC;
    if (m.tag < 0 || m.tag > RT_MAT_ISOTROPIC) return rt_set_error("bad material tag"), -1;
    if (needs_tex && (m.texture < 0 || m.texture >= s->n_textures)) return rt_set_error("bad texture index"), -1;
  }
  for (int k = 0; k < s->n_textures; k++) {
    const rt_texture &t = s->textures[k];
    if (t.kind == RT_TEX_CHECKER && (t.a < 0 || t.a >= s->n_textures || t.b < 0 || t.b >= s->n_textures))
      return rt_set_error("bad checker"), -1;
    if (t.kind == RT_TEX_IMAGE) {
      if (t.a < 0 || t.a >= s->n_images) return rt_set_error("bad image index"), -1;
      const rt_image &im = s->images[t.a];
      if (im.width <= 0 || im.height <= 0 || im.offset < 0 ||
          im.offset + (int64_t)im.width * im.height * 3 > s->n_image_bytes)
        return rt_set_error("bad image extent"), -1;
    }
    if (t.kind == RT_TEX_PERLIN) {
      if (t.a < 0 || t.a >= s->n_perlins) return rt_set_error("bad perlin index"), -1;
      const rt_perlin &p = s->perlins[t.a];
      for (int q = 0; q < 256; q++)
        if ((unsigned)p.perm_x[q] > 255 || (unsigned)p.perm_y[q] > 255 || (unsigned)p.perm_z[q] > 255)
          return rt_set_error("bad perlin permutation"), -1;
    }
    if (t.kind < RT_TEX_SOLID || t.kind > RT_TEX_PERLIN) return rt_set_error("bad texture kind"), -1;
  }
  return 0;
}

// ------------------------------------------------------------------------------ Book-1 packing
static bool env_flag(const char *name, bool dflt) {
  const char *e = getenv(name);
  if (!e || !*e) return dflt;
  return !(e[0] == '0' || e[0] == 'n' || e[0] == 'N' || e[0] == 'f' || e[0] == 'F');
}

// 16-bit ref used by the fast traversal: node index, or sphere index | 0x8000, or 0xffff (none)
static bool pack_ref(int32_t ref, uint32_t *out) {
  if (ref == RT_REF_NONE) return *out = 0xffffu, true;
  const int32_t i = rt_ref_index(ref);
  if (rt_ref_kind(ref) == RT_KIND_BVH && i < 0x7fff) return *out = (uint32_t)i, true;
  if (rt_ref_kind(ref) == RT_KIND_SPHERE && i < 0x7fff) return *out = (uint32_t)i | b1::kLeafBit, true;
  return false;
}

// stack slots the fast traversal needs below `ref` (rt_book1.h: trace never pushes a left child)
static int b1_stack_need(const rt_flat_scene *s, int32_t ref, int depth_guard) {
  if (ref == RT_REF_NONE || rt_ref_kind(ref) != RT_KIND_BVH || depth_guard > 4096) return 0;
  const rt_bvh_node &n = s->bvh[rt_ref_index(ref)];
  const bool left_leaf = rt_ref_kind(n.left) == RT_KIND_SPHERE;
  if (left_leaf) return b1_stack_need(s, n.right, depth_guard + 1);
  if (n.right == RT_REF_NONE) return b1_stack_need(s, n.left, depth_guard + 1);
  const int l = 1 + b1_stack_need(s, n.left, depth_guard + 1), r = b1_stack_need(s, n.right, depth_guard + 1);
  return l > r ? l : r;
}

static float bits_as_float(uint32_t u) {
  float f;
  memcpy(&f, &u, 4);
  return f;
}

static bool book1_eligible(const rt_flat_scene *s) {
  if (s->features & ~kFeatBook1) return false;
  if (s->n_lists != 2 || s->n_quads || s->n_translates || s->n_rotates || s->n_media) return false;  // root + lights
  if (s->lists[s->lights].count != 0) return false;
  if (s->n_spheres >= 0x7fff || s->n_bvh >= 0x7fff || s->camera.max_depth > kMaxDepth) return false;
  if (s->n_bvh + s->lists[rt_ref_index(s->root)].count + 1 >= (int)b1::kHasLeaf7) return false;  // v7 refs
  for (int k = 0; k < s->n_materials; k++) {
    const rt_material &m = s->materials[k];
    if (m.tag != RT_MAT_LAMBERTIAN && m.tag != RT_MAT_METAL && m.tag != RT_MAT_DIELECTRIC) return false;
    if (m.tag != RT_MAT_DIELECTRIC && s->textures[m.texture].kind != RT_TEX_SOLID) return false;
  }
  for (int k = 0; k < s->n_bvh; k++) {
    uint32_t a, b;
    if (!pack_ref(s->bvh[k].left, &a) || !pack_ref(s->bvh[k].right, &b) || a == 0xffffu) return false;
  }
  const rt_list &root = s->lists[rt_ref_index(s->root)];
  for (int k = 0; k < root.count; k++) {
    uint32_t a;
    if (!pack_ref(s->list_items[root.first + k], &a) || a == 0xffffu) return false;
    if (b1_stack_need(s, s->list_items[root.first + k], 0) > b1::kStackSlots) return false;
  }
  return env_flag("RT_BOOK1", true);
}

// Build and upload the Book-1 arrays; sets d->book1 on success (failure just keeps the general path).
static int book1_upload(rt_device_scene *d, const rt_flat_scene *s) {
  const rt_list &root = s->lists[rt_ref_index(s->root)];
  std::vector<float4> nodes(2 * (size_t)s->n_bvh);
  for (int k = 0; k < s->n_bvh; k++) {
    const rt_bvh_node &n = s->bvh[k];
    uint32_t l, r;
    pack_ref(n.left, &l);
    pack_ref(n.right, &r);
    nodes[2 * k] = make_float4(n.lo[0], n.hi[0], n.lo[1], n.hi[1]);  // the reference's AABB values[axis][lo/hi]
    nodes[2 * k + 1] = make_float4(n.lo[2], n.hi[2], bits_as_float(l), bits_as_float(r));
  }
  // v7 records (rt_book1.h: Node7): own box + child refs, then the leaf children's spheres as
  // (left, right) pairs; a sphere directly in the root list gets a record with an infinite box
  std::vector<float4> nodes7;
  std::vector<uint16_t> roots7;
  {
    auto has_leaf = [&](int node) {
      return rt_ref_kind(s->bvh[node].left) == RT_KIND_SPHERE || rt_ref_kind(s->bvh[node].right) == RT_KIND_SPHERE;
    };
    auto ref7 = [&](int32_t ref) -> uint32_t {
      if (ref == RT_REF_NONE) return 0xffffu;
      const int32_t i = rt_ref_index(ref);
      if (rt_ref_kind(ref) == RT_KIND_SPHERE) return (uint32_t)i | b1::kLeafBit;
      return (uint32_t)i | (has_leaf(i) ? b1::kHasLeaf7 : 0u);
    };
    auto sphere_of = [&](int32_t ref, float *c, float *r2) {
      if (ref != RT_REF_NONE && rt_ref_kind(ref) == RT_KIND_SPHERE) {
        const rt_sphere &sp = s->spheres[rt_ref_index(ref)];
        c[0] = sp.center[0], c[1] = sp.center[1], c[2] = sp.center[2], *r2 = sp.radius_sq;
      } else {
        c[0] = c[1] = c[2] = 0.0f, *r2 = 0.0f;
      }
    };
    auto push_record = [&](const float lo[3], const float hi[3], int32_t left, int32_t right, uint32_t l, uint32_t r) {
      float cl[3], cr[3], rl, rr;
      sphere_of(left, cl, &rl);
      sphere_of(right, cr, &rr);
      nodes7.push_back(make_float4(lo[0], hi[0], lo[1], hi[1]));
      nodes7.push_back(make_float4(lo[2], hi[2], bits_as_float(l), bits_as_float(r)));
      nodes7.push_back(make_float4(cl[0], cr[0], cl[1], cr[1]));
      nodes7.push_back(make_float4(cl[2], cr[2], rl, rr));
    };
    for (int k = 0; k < s->n_bvh; k++) {
      const rt_bvh_node &n = s->bvh[k];
      push_record(n.lo, n.hi, n.left, n.right, ref7(n.left), ref7(n.right));
    }
    const float inf = __builtin_inff(), lo_inf[3] = {-inf, -inf, -inf}, hi_inf[3] = {inf, inf, inf};
    for (int k = 0; k < root.count; k++) {
      const int32_t item = s->list_items[root.first + k];
      if (rt_ref_kind(item) == RT_KIND_BVH) {
        roots7.push_back((uint16_t)ref7(item));
      } else {  // Sphere_hit straight from the list == an always-hit box around it (rt_book1.h)
        roots7.push_back((uint16_t)((nodes7.size() / 4) | b1::kHasLeaf7));
        push_record(lo_inf, hi_inf, item, RT_REF_NONE, ref7(item), 0xffffu);
      }
    }
    if (roots7.empty()) roots7.push_back(0);
    const float zero[3] = {0.0f, 0.0f, 0.0f};
    push_record(zero, zero, RT_REF_NONE, RT_REF_NONE, 0xffffu, 0xffffu);  // the dummy record (no leaf children)
  }
  // v9 items (rt_book1.h: trav_step_v9): the root list's hittables in traversal preorder
  std::vector<float4> items9;
  std::vector<uint32_t> bf_item;  // whole-wave candidate trace (rt_book1.h: bf_trace): leaf item positions
  {
    std::function<void(int32_t)> emit = [&](int32_t ref) {
      if (ref == RT_REF_NONE) return;
      const int32_t i = rt_ref_index(ref);
      if (rt_ref_kind(ref) == RT_KIND_SPHERE) {
        const rt_sphere &sp = s->spheres[i];
        const float4 c = make_float4(sp.center[0], sp.center[1], sp.center[2], sp.radius_sq);
        items9.push_back(c);
        // (x: bf_trace position slot, y: 1/r and z: material for the whole-wave shading, w: index)
        items9.push_back(make_float4(0.0f, sp.inv_radius, bits_as_float((uint32_t)sp.material),
                                     bits_as_float((uint32_t)i | b1::kLeaf9)));
        bf_item.push_back((uint32_t)(items9.size() / 2 - 1));
        return;
      }
      const rt_bvh_node &n = s->bvh[i];
      const size_t at = items9.size();
      items9.push_back(make_float4(n.lo[0], n.hi[0], n.lo[1], n.hi[1]));
      items9.push_back(make_float4(n.lo[2], n.hi[2], 0.0f, 0.0f));
      emit(n.left);
      emit(n.right);  // RT_REF_NONE for the collapsed n == 1 duplicate (rt_flatten.c)
      items9[at + 1].z = bits_as_float((uint32_t)((items9.size() - at) / 2));
    };
    for (int k = 0; k < root.count; k++) emit(s->list_items[root.first + k]);
    // one zero item past the end: the step reads its successor before knowing it exists
    items9.push_back(make_float4(0.0f, 0.0f, 0.0f, 0.0f));
    items9.push_back(make_float4(0.0f, 0.0f, 0.0f, 0.0f));
  }
  // bf_trace: leaf n's item position in a spare word of item n (q1.w of a node, q1.x of a leaf)
  for (size_t n = 0; n < bf_item.size() && 2 * n + 1 < items9.size(); n++) {
    float4 &h = items9[2 * n + 1];
    uint32_t hw;
    memcpy(&hw, &h.w, 4);
    if (hw & b1::kLeaf9)
      h.x = bits_as_float(bf_item[n]);
    else
      h.w = bits_as_float(bf_item[n]);
  }
  // group trace treelets (rt_group.h): greedy treelets of <= 8 entries over the preorder items, each
  // entry with <= 3 opened internal nodes between it and the treelet's (already tested) root; and the
  // per-leaf ancestor table for the winner's check
  std::vector<uint4> wide;
  std::vector<uint16_t> anc;
  {
    const int n_items = (int)(items9.size() / 2) - 1;  // without the pad item
    auto is_leaf = [&](int p) {
      uint32_t w;
      memcpy(&w, &items9[2 * p + 1].w, 4);
      return (w & b1::kLeaf9) != 0;
    };
    auto size_of = [&](int p) {
      if (is_leaf(p)) return 1;
      uint32_t k;
      memcpy(&k, &items9[2 * p + 1].z, 4);
      return (int)k;
    };
    auto kids = [&](int p, int out[2]) {
      const int l = p + 1;
      int n = 0;
      out[n++] = l;
      if (l + size_of(l) < p + size_of(p)) out[n++] = l + size_of(l);
      return n;
    };
    struct E {
      int item, n_chain;
      uint32_t need;
    };
    bool ok = n_items > 0 && n_items < 0xffff;
    std::function<int(const std::vector<int> &)> make = [&](const std::vector<int> &level1) -> int {
      if (!ok || level1.size() > (size_t)grp::kG) return ok = false, -1;
      std::vector<E> es;
      std::vector<int> internals;
      for (int c : level1) es.push_back({c, 0, 0u});
      for (;;) {  // open the internal entry with the largest subtree while the treelet has room
        int pick = -1;
        for (int k = 0; k < (int)es.size(); k++) {
          int kc[2];
          if (is_leaf(es[k].item) || es[k].n_chain >= 3 || (int)es.size() + kids(es[k].item, kc) - 1 > grp::kG)
            continue;
          if (pick < 0 || size_of(es[k].item) > size_of(es[pick].item)) pick = k;
        }
        if (pick < 0 || (int)internals.size() >= grp::kG) break;
        const E old = es[pick];
        int kc[2];
        const int nc = kids(old.item, kc);
        const uint32_t bit = 1u << internals.size();
        internals.push_back(old.item);
        std::vector<E> repl;
        for (int c = 0; c < nc; c++) repl.push_back({kc[c], old.n_chain + 1, old.need | bit});
        es.erase(es.begin() + pick);
        es.insert(es.begin() + pick, repl.begin(), repl.end());
      }
      const int id = (int)(wide.size() / grp::kG);
      for (int k = 0; k < grp::kG; k++)
        wide.push_back(make_uint4(grp::kEmpty, 0u, 0u, k < (int)internals.size() ? (uint32_t)internals[k] : grp::kEmpty));
      for (int k = 0; k < (int)es.size(); k++) {
        const E &e = es[k];
        uint32_t child = 0;
        if (!is_leaf(e.item)) {
          int kc[2];
          const int nc = kids(e.item, kc);
          const int c = make(std::vector<int>(kc, kc + nc));
          if (c < 0) return -1;
          child = (uint32_t)c;
        }
        uint4 &w = wide[(size_t)id * grp::kG + k];
        w.x = (uint32_t)e.item, w.y = child, w.z = e.need | (is_leaf(e.item) ? 0x100u : 0u);
      }
      return id;
    };
    std::vector<int> tops;
    for (int p = 0; p < n_items; p += size_of(p)) tops.push_back(p);
    if (make(tops) != 0 || !ok) wide.clear();
    // ancestors of every leaf, root first
    if (!wide.empty()) {
      anc.assign((size_t)(n_items + 1) * grp::kMaxAnc, 0xffffu);
      std::vector<int> path;
      std::function<void(int)> walk = [&](int p) {
        if (!ok) return;
        if (is_leaf(p)) {
          if ((int)path.size() > grp::kMaxAnc) return void(ok = false);
          for (size_t q = 0; q < path.size(); q++) anc[(size_t)p * grp::kMaxAnc + q] = (uint16_t)path[q];
          return;
        }
        path.push_back(p);
        int kc[2];
        const int nc = kids(p, kc);
        for (int c = 0; c < nc; c++) walk(kc[c]);
        path.pop_back();
      };
      for (int t : tops) walk(t);
      if (!ok) wide.clear(), anc.clear();
    }
  }
  std::vector<float4> sph(s->n_spheres);
  for (int k = 0; k < s->n_spheres; k++)
    sph[k] = make_float4(s->spheres[k].center[0], s->spheres[k].center[1], s->spheres[k].center[2],
                         s->spheres[k].radius_sq);
  std::vector<b1::FastMat> mats(s->n_materials);
  for (int k = 0; k < s->n_materials; k++) {
    const rt_material &m = s->materials[k];
    b1::FastMat f;
    memset(&f, 0, sizeof f);
    f.tag = m.tag;
    f.param = m.param;
    if (m.tag == RT_MAT_DIELECTRIC) {
      f.albedo[0] = f.albedo[1] = f.albedo[2] = 1.0f;  // Dielectric_scatter: *color = vec3(1, 1, 1)
    } else {
      const rt_texture &t = s->textures[m.texture];
      f.albedo[0] = t.color[0];
      f.albedo[1] = t.color[1];
      f.albedo[2] = t.color[2];
    }
    mats[k] = f;
  }
  std::vector<uint16_t> roots(root.count > 0 ? root.count : 1);
  int need = 0;
  for (int k = 0; k < root.count; k++) {
    uint32_t a;
    pack_ref(s->list_items[root.first + k], &a);
    roots[k] = (uint16_t)a;
    const int nk = b1_stack_need(s, s->list_items[root.first + k], 0);
    need = nk > need ? nk : need;
  }

  // geometry: LDS-resident when it fits next to the stack (gfx950: 160 KiB per CU)
  const size_t scene_bytes_v5 = nodes.size() * sizeof(float4) + sph.size() * sizeof(float4);
  const size_t scene_bytes_v7 = nodes7.size() * sizeof(float4);
  const size_t scene_bytes_v9 = items9.size() * sizeof(float4);
  {
    const char *ev = getenv("RT_BOOK1_V");
    d->book1_ver = (ev && *ev) ? atoi(ev) : 9;
    if (d->book1_ver != 2 && d->book1_ver != 3 && d->book1_ver != 5 && d->book1_ver != 6 && d->book1_ver != 7)
      d->book1_ver = 9;
  }
  const size_t scene_bytes = d->book1_ver == 9 ? scene_bytes_v9 : d->book1_ver == 7 ? scene_bytes_v7 : scene_bytes_v5;
  // v2 keeps 32-bit stack slots, v3+ 16-bit ones (+1 slot: v5+ store the right child unconditionally)
  // only the slots this scene's DFS can reach (host-computed `need` <= kStackSlots) take LDS
  const size_t stack_bytes = d->book1_ver == 9 ? 0 : (size_t)(need + 1) * b1::kBlock * (d->book1_ver >= 3 ? 2 : 4);
  d->book1_lds = env_flag("RT_BOOK1_LDS", true) && scene_bytes + stack_bytes <= 64 * 1024;
  d->book1_stats = env_flag("RT_BOOK1_STATS", false) && d->book1_ver >= 5 && d->book1_lds;
  d->b1_lds_bytes = align_up((d->book1_lds ? scene_bytes : 0) + stack_bytes, 16);

  hipDeviceProp_t prop;
  HIP_OK(hipGetDeviceProperties(&prop, d->device));
  int per_cu = 0;
  {
    const char *eo = getenv("RT_BOOK1_OCC");
    d->book1_occ = (eo && *eo) ? atoi(eo) : 0;
    if (d->book1_ver != 5 || d->book1_stats || (d->book1_occ != 5 && d->book1_occ != 6)) d->book1_occ = 0;
  }
  const void *fn = d->book1_stats ? (d->book1_ver == 9   ? (const void *)rt_book1_kernel<true, 9, true>
                                     : d->book1_ver == 6 ? (const void *)rt_book1_kernel<true, 6, true>
                                     : d->book1_ver == 7 ? (const void *)rt_book1_kernel<true, 7, true>
                                                         : (const void *)rt_book1_kernel<true, 5, true>)
                   : d->book1_occ == 5 ? (d->book1_lds ? (const void *)rt_book1_kernel<true, 5, false, 5> : (const void *)rt_book1_kernel<false, 5, false, 5>)
                   : d->book1_occ == 6 ? (d->book1_lds ? (const void *)rt_book1_kernel<true, 5, false, 6> : (const void *)rt_book1_kernel<false, 5, false, 6>)
                   : d->book1_ver == 9 ? (d->book1_lds ? (const void *)rt_book1_kernel<true, 9> : (const void *)rt_book1_kernel<false, 9>)
                   : d->book1_ver == 7 ? (d->book1_lds ? (const void *)rt_book1_kernel<true, 7> : (const void *)rt_book1_kernel<false, 7>)
                   : d->book1_ver == 6 ? (d->book1_lds ? (const void *)rt_book1_kernel<true, 6> : (const void *)rt_book1_kernel<false, 6>)
                   : d->book1_ver == 5 ? (d->book1_lds ? (const void *)rt_book1_kernel<true, 5> : (const void *)rt_book1_kernel<false, 5>)
                   : d->book1_ver == 3 ? (d->book1_lds ? (const void *)rt_book1_kernel<true, 3> : (const void *)rt_book1_kernel<false, 3>)
                                       : (d->book1_lds ? (const void *)rt_book1_kernel<true, 2> : (const void *)rt_book1_kernel<false, 2>);
  HIP_OK(hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, fn, b1::kBlock, d->b1_lds_bytes));
  if (per_cu < 1) per_cu = 1;
  d->b1_grid = prop.multiProcessorCount * per_cu;
  const int spill_lanes = d->b1_grid * b1::kBlock;
  const size_t spill_bytes = (size_t)(kMaxDepth / 4) * spill_lanes * sizeof(uint64_t);  // Record chunks

  size_t off[16], total = 0;
  const size_t cost_bytes = d->book1_stats ? (size_t)s->camera.width * s->camera.height * 2 * sizeof(uint32_t) : 0;
  const size_t sizes[16] = {nodes.size() * sizeof(float4), sph.size() * sizeof(float4), mats.size() * sizeof(b1::FastMat),
                           roots.size() * sizeof(uint16_t), 256, spill_bytes, cost_bytes,  // [4]: counter + stats
                           nodes7.size() * sizeof(float4), roots7.size() * sizeof(uint16_t),
                           items9.size() * sizeof(float4),
                           (size_t)s->camera.width * s->camera.height * sizeof(uint32_t),   // [10] LPT cost
                           (size_t)s->camera.width * s->camera.height * sizeof(int32_t),    // [11] LPT order
                           kLptHistBytes,                                                    // [12] LPT buckets
                           wide.size() * sizeof(uint4), anc.size() * sizeof(uint16_t),      // [13] [14] group
                           (size_t)s->camera.width * s->camera.height * sizeof(uint32_t)};  // [15] pre-pass draws
  for (int k = 0; k < 16; k++) {
    off[k] = total;
    total = align_up(total + (sizes[k] ? sizes[k] : 16), 256);
  }
  void *arena = nullptr;
  HIP_OK(hipMalloc(&arena, total));
  char *b = (char *)arena;
  if (sizes[0]) HIP_OK(hipMemcpy(b + off[0], nodes.data(), sizes[0], hipMemcpyHostToDevice));
  if (sizes[1]) HIP_OK(hipMemcpy(b + off[1], sph.data(), sizes[1], hipMemcpyHostToDevice));
  if (sizes[2]) HIP_OK(hipMemcpy(b + off[2], mats.data(), sizes[2], hipMemcpyHostToDevice));
  HIP_OK(hipMemcpy(b + off[3], roots.data(), sizes[3], hipMemcpyHostToDevice));
  HIP_OK(hipMemcpy(b + off[7], nodes7.data(), sizes[7], hipMemcpyHostToDevice));
  HIP_OK(hipMemcpy(b + off[8], roots7.data(), sizes[8], hipMemcpyHostToDevice));
  if (sizes[9]) HIP_OK(hipMemcpy(b + off[9], items9.data(), sizes[9], hipMemcpyHostToDevice));
  if (sizes[13]) HIP_OK(hipMemcpy(b + off[13], wide.data(), sizes[13], hipMemcpyHostToDevice));
  if (sizes[14]) HIP_OK(hipMemcpy(b + off[14], anc.data(), sizes[14], hipMemcpyHostToDevice));
  d->b1_arena = arena;
  b1::Book1View &V = d->b1view;
  V.S = d->view;
  V.nodes_g = (const float4 *)(b + off[0]);
  V.spheres_g = (const float4 *)(b + off[1]);
  V.mats = (const b1::FastMat *)(b + off[2]);
  V.root_items = (const uint16_t *)(b + off[3]);
  V.work_counter = (int32_t *)(b + off[4]);
  V.stats = (unsigned long long *)(b + off[4] + 64);
  V.spill = (uint64_t *)(b + off[5]);
  V.pixel_cost = d->book1_stats ? (uint32_t *)(b + off[6]) : nullptr;
  V.nodes7_g = (const float4 *)(b + off[7]);
  V.root7_items = (const uint16_t *)(b + off[8]);
  V.n_nodes7 = (int32_t)(nodes7.size() / 4);
  V.items9_g = (const float4 *)(b + off[9]);
  V.wide = (const uint4 *)(b + off[13]);
  V.n_wide = (int32_t)(wide.size() / grp::kG);
  V.anc = (const uint16_t *)(b + off[14]);
  {  // the group kernel (rt_group.h), for frames with few pixels per lane
    const char *em = getenv("RT_MODE");
    d->group_mode = (em && !strcmp(em, "lane")) ? 0 : (em && !strcmp(em, "group")) ? 1 : 2;
    if (V.n_wide == 0 || d->book1_ver != 9 || d->book1_stats) d->group_mode = 0;
    if (d->group_mode != 0) {
      const bool lds = d->book1_lds;
      d->g_lds_bytes = align_up((lds ? items9.size() * sizeof(float4) : 0) +
                                    (size_t)grp::kGroups * grp::kStack * sizeof(uint32_t), 16);
      int per = 0;
      HIP_OK(hipOccupancyMaxActiveBlocksPerMultiprocessor(
          &per, lds ? (const void *)rt_book1_group_kernel<true> : (const void *)rt_book1_group_kernel<false>,
          grp::kBlock, d->g_lds_bytes));
      d->g_grid = prop.multiProcessorCount * (per < 1 ? 1 : per);
      if (d->g_grid * grp::kGroups > spill_lanes) d->g_grid = spill_lanes / grp::kGroups;  // record spill columns
    }
  }
  if (d->book1_ver == 9 && !d->book1_stats) {  // whole-wave items run concurrently on a second stream
    // high priority: the whole-wave workgroups take CU slots ahead of the lane / group kernel's
    // (their chains set the frame time; measured at N = 8 their first items started at ~70 ms)
    int prio_lo = 0, prio_hi = 0;
    HIP_OK(hipDeviceGetStreamPriorityRange(&prio_lo, &prio_hi));
    HIP_OK(hipStreamCreateWithPriority(&d->wave_stream, hipStreamNonBlocking,
                                       env_flag("RT_WAVE_PRIO", true) ? prio_hi : prio_lo));
    HIP_OK(hipEventCreateWithFlags(&d->ev_fork, hipEventDisableTiming));
    HIP_OK(hipEventCreateWithFlags(&d->ev_join, hipEventDisableTiming));
  }
  V.px_time = nullptr;
  if (env_flag("RT_PX_TIME", false)) {
    HIP_OK(hipMalloc(&d->px_time, (size_t)s->camera.width * s->camera.height * 2 * sizeof(uint32_t)));
    V.px_time = d->px_time;
  }
  // whole-wave pixels trace by candidates (bf_trace) when every leaf fits the wave's slots
  V.n_bf_leaves = !bf_item.empty() && bf_item.size() <= (size_t)64 * b1::kBfSlots && env_flag("RT_BF", true)
                      ? (int32_t)bf_item.size() : 0;
  d->lpt_cost = (uint32_t *)(b + off[10]);
  d->lpt_order = (int32_t *)(b + off[11]);
  d->lpt_hist = (uint32_t *)(b + off[12]);
  d->draw_out = (uint32_t *)(b + off[15]);
  {
    int per = 0;
    HIP_OK(hipOccupancyMaxActiveBlocksPerMultiprocessor(&per, (const void *)rt_book1_split_kernel<true>, b1::kBlock,
                                                        d->b1_lds_bytes));
    d->sp_grid = prop.multiProcessorCount * (per < 1 ? 1 : per);
    if (d->sp_grid > d->b1_grid) d->sp_grid = d->b1_grid;  // the record spill area has b1_grid columns
  }
  V.draw_out = d->draw_out;
  V.sp_px = nullptr;
  V.sp_claim = nullptr;
  V.sp_rec = nullptr;
  V.sp_items = nullptr;
  V.sp_n_items = nullptr;
  {
    const char *e = getenv("RT_SPLIT");
    d->split_mode = (e && *e) ? atoi(e) : 0;  // opt-in: measured no faster than the group kernel
    if (d->book1_ver != 9 || !d->book1_lds || d->book1_stats) d->split_mode = 0;
    if ((e = getenv("RT_SPLIT_BETA")) && *e) d->split_beta = (float)atof(e);
    if ((e = getenv("RT_SPLIT_MARGIN")) && *e) d->split_margin = (float)atof(e);
    if ((e = getenv("RT_SPLIT_ALLOC")) && *e) d->split_alloc = (float)atof(e);
    if ((e = getenv("RT_SPLIT_FIXC")) && *e) d->split_fixc = (float)atof(e);
    if ((e = getenv("RT_SPLIT_W")) && *e) d->split_wfact = (float)atof(e);
    if ((e = getenv("RT_SPLIT_KMAX")) && *e) d->split_kmax = atoi(e);
    if ((e = getenv("RT_SPLIT_ROUNDS")) && *e) d->split_rounds = atoi(e);
    if (d->split_kmax < 1) d->split_kmax = 1;
    if (d->split_rounds < 1) d->split_rounds = 1;
    if (d->split_rounds > 16) d->split_rounds = 16;
    if (d->split_margin < 0.5f) d->split_margin = 0.5f;
    if (d->split_alloc < d->split_margin) d->split_alloc = d->split_margin;
  }
  d->lpt = env_flag("RT_LPT", true) && (d->book1_ver == 9 || d->book1_ver == 5) && d->book1_occ == 0;
  {
    const char *el = getenv("RT_LPT_SPP");
    d->lpt_spp = (el && *el) ? atoi(el) : 8;
    if (d->lpt_spp < 1) d->lpt_spp = 1;
  }
  V.order = nullptr;
  V.cost_out = nullptr;
  V.n_coop = nullptr;
  V.coop_counter = nullptr;
  V.coop_waves_dev = nullptr;
  {
    const char *e1 = getenv("RT_COOP_STEPS"), *e2 = getenv("RT_COOP_WAVES");
    d->coop_steps = (e1 && *e1) ? atoi(e1) : -1;  // -1: split chosen by the cost model (lpt_scan_kernel)
    d->coop_waves = (e2 && *e2) ? atoi(e2) : -1;
    if (d->book1_ver != 9 || !d->book1_lds) d->coop_waves = 0;
    const char *e3 = getenv("RT_PRIO_STEPS");
    d->prio_steps = (e3 && *e3) ? atoi(e3) : 0;  // off by default: measured no gain
  }
  V.n_heavy = nullptr;
  V.n_items9 = (int32_t)(items9.size() / 2) - 1;  // without the trailing pad item
  V.n_items9_alloc = (int32_t)(items9.size() / 2);
  V.spill_lanes = spill_lanes;
  V.n_nodes = s->n_bvh;
  V.n_spheres = s->n_spheres;
  V.n_root = root.count;
  V.stack_need = need;
  {
    const char *eb = getenv("RT_SHADE_BATCH");
    V.shade_batch = (eb && *eb) ? atoi(eb) : 48;
    V.shade_batch = V.shade_batch < 1 ? 1 : (V.shade_batch > 64 ? 64 : V.shade_batch);  // >= 1: progress
    const char *ex = getenv("RT_EXPERIMENT");
    V.experiment = (ex && *ex) ? atoi(ex) : 0;  // bit 0 (stats builds): no sphere tests; bit 1: coop printf
    const char *ec = getenv("RT_COOP_LANES");
    V.coop_lanes = (ec && *ec) ? atoi(ec) : 0;  // off: measured slower than the DFS lanes
    if ((d->book1_ver == 5 && (s->n_bvh > 64 * b1::kCoopSlots || s->n_spheres > 64 * b1::kCoopSlots)) ||
        (d->book1_ver != 5 && d->book1_ver != 9) || !d->book1_lds)
      V.coop_lanes = 0;
    const char *eo = getenv("RT_PIXEL_ORDER");
    V.reverse = (eo && !strcmp(eo, "rev")) ? 1 : 0;
    const char *es = getenv("RT_SPHERE_BATCH");
    V.sphere_batch = (es && *es) ? atoi(es) : 16;
    V.sphere_batch = V.sphere_batch < 1 ? 1 : (V.sphere_batch > 64 ? 64 : V.sphere_batch);
  }
  d->book1 = true;
  if (env_flag("RT_DEBUG", false))
    fprintf(stderr, "[rtc] book1 v%d%s lds=%d bytes=%zu grid=%d (%d/CU) stack_need=%d occ=%d shade_batch=%d coop=%d\n",
            d->book1_ver, d->book1_stats ? "+stats" : "", (int)d->book1_lds, d->b1_lds_bytes, d->b1_grid, per_cu, need,
            d->book1_occ, V.shade_batch, V.coop_lanes);
  return 0;
}

extern "C" int rt_device_count(void) {
  int n = 0;
  if (hipGetDeviceCount(&n) != hipSuccess) return 0;
  return n;
}

extern "C" void rt_scene_release(rt_device_scene *d);

// Buffers of the persistent general path: work counter, longest-first cost / order / buckets.
static int general_upload(rt_device_scene *d, const rt_flat_scene *s) {
  const size_t npix = (size_t)s->camera.width * s->camera.height;
  const size_t sizes[4] = {256, npix * sizeof(uint32_t), npix * sizeof(int32_t), kLptHistBytes};
  size_t off[4], total = 0;
  for (int k = 0; k < 4; k++) {
    off[k] = total;
    total = align_up(total + sizes[k], 256);
  }
  void *arena = nullptr;
  HIP_OK(hipMalloc(&arena, total));
  char *b = (char *)arena;
  d->gen_arena = arena;
  d->gen_counter = (int32_t *)(b + off[0]);
  d->lpt_cost = (uint32_t *)(b + off[1]);
  d->lpt_order = (int32_t *)(b + off[2]);
  d->lpt_hist = (uint32_t *)(b + off[3]);
  d->lpt = env_flag("RT_LPT", true);
  {
    const char *el = getenv("RT_LPT_SPP");
    d->lpt_spp = (el && *el) ? atoi(el) : 8;
    if (d->lpt_spp < 1) d->lpt_spp = 1;
  }
  hipDeviceProp_t prop;
  HIP_OK(hipGetDeviceProperties(&prop, d->device));
  int per_cu = 0;
  {
    const char *eb = getenv("RT_GEN_BATCH");
    d->gen_batch = (eb && *eb) ? atoi(eb) : 56;
    if (d->gen_batch < 0) d->gen_batch = 0;
    if (d->gen_batch > 64) d->gen_batch = 64;
    if (!d->view.pre) d->gen_batch = 0;  // the batched loop runs the preorder scan
    const char *el = getenv("RT_GEN_LDS");
    d->gen_lds = d->gen_batch ? ((el && *el) ? atoi(el) : 1024) : 0;
    if (d->gen_lds < 0) d->gen_lds = 0;
    if (d->gen_lds > d->view.n_pre) d->gen_lds = d->view.n_pre;
    if (d->gen_lds > 2048) d->gen_lds = 2048;  // 64 KB: the default dynamic LDS limit
    const char *es = getenv("RT_GEN_STEPS");
    d->gen_steps = (es && *es) ? atoi(es) : 8;
    if (d->gen_steps < 1) d->gen_steps = 1;
  }
  const bool fb = (d->features & ~kFeatBook1) == 0;
  const void *fn = d->gen_batch ? (fb ? (const void *)rt_general_kernel<kFeatBook1, true> : (const void *)rt_general_kernel<kFeatAll, true>)
                                : (fb ? (const void *)rt_general_kernel<kFeatBook1> : (const void *)rt_general_kernel<kFeatAll>);
  HIP_OK(hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, fn, gen::kBlock, (size_t)d->gen_lds * 2 * sizeof(float4)));
  if (per_cu < 1) per_cu = 1;
  d->gen_grid = prop.multiProcessorCount * per_cu;
  d->general = true;
  if (env_flag("RT_DEBUG", false))
    fprintf(stderr, "[rtc] general persistent kernel: grid=%d (%d/CU), features=0x%x\n", d->gen_grid, per_cu,
            d->features);
  return 0;
}

extern "C" rt_device_scene *rt_scene_upload(const rt_flat_scene *s, int device) {
  if (s == NULL) {
    rt_set_error("rt_scene_upload: NULL scene");
    return NULL;
  }
  if (validate(s) != 0) return NULL;
  if (hipSetDevice(device) != hipSuccess) {
    rt_set_error("hipSetDevice(%d) failed", device);
    return NULL;
  }
  struct Part {
    const void *src;
    size_t bytes;
    size_t off;
  };
  Part parts[13] = {
      {s->bvh, sizeof(rt_bvh_node) * s->n_bvh, 0},       {s->spheres, sizeof(rt_sphere) * s->n_spheres, 0},
      {s->quads, sizeof(rt_quad) * s->n_quads, 0},       {s->lists, sizeof(rt_list) * s->n_lists, 0},
      {s->list_items, sizeof(int32_t) * s->n_list_items, 0},
      {s->translates, sizeof(rt_translate) * s->n_translates, 0},
      {s->rotates, sizeof(rt_rotate_y) * s->n_rotates, 0}, {s->media, sizeof(rt_medium) * s->n_media, 0},
      {s->materials, sizeof(rt_material) * s->n_materials, 0},
      {s->textures, sizeof(rt_texture) * s->n_textures, 0}, {s->images, sizeof(rt_image) * s->n_images, 0},
      {s->perlins, sizeof(rt_perlin) * s->n_perlins, 0},   {s->image_bytes, (size_t)s->n_image_bytes, 0}};
  size_t total = 0;
  for (auto &p : parts) {
    p.off = total;
    total = align_up(total + p.bytes, 256);
  }
  total = total ? total : 256;
  void *arena = NULL;
  if (hipMalloc(&arena, total) != hipSuccess) {
    rt_set_error("hipMalloc(%zu) failed on device %d", total, device);
    return NULL;
  }
  for (auto &p : parts)
    if (p.bytes && hipMemcpy((char *)arena + p.off, p.src, p.bytes, hipMemcpyHostToDevice) != hipSuccess) {
      (void)hipFree(arena);
      rt_set_error("scene upload failed on device %d", device);
      return NULL;
    }
  rt_device_scene *d = new rt_device_scene();
  d->device = device;
  d->arena = arena;
  d->arena_bytes = total;
  d->features = s->features;
  d->width = s->camera.width;
  d->height = s->camera.height;
  const void *dev_arrays[13];
  for (int k = 0; k < 13; k++) dev_arrays[k] = (char *)arena + parts[k].off;
  d->view = make_view(*s, dev_arrays);
  if (!book1_eligible(s) && env_flag("RT_GEN_PRE", true)) {  // the general path's preorder (trace_pre)
    std::vector<float4> pre;
    build_preorder(*s, pre);
    if (!pre.empty()) {
      if (hipMalloc(&d->pre_arena, pre.size() * sizeof(float4)) != hipSuccess ||
          hipMemcpy(d->pre_arena, pre.data(), pre.size() * sizeof(float4), hipMemcpyHostToDevice) != hipSuccess) {
        rt_set_error("preorder upload failed on device %d", device);
        rt_scene_release(d);
        return NULL;
      }
      d->view.pre = (const float4 *)d->pre_arena;
      d->view.n_pre = (int32_t)(pre.size() / 2);
    }
  }
  if (hipEventCreate(&d->ev_main[0]) != hipSuccess || hipEventCreate(&d->ev_main[1]) != hipSuccess)
    d->ev_main[0] = d->ev_main[1] = nullptr;
  if (book1_eligible(s) && book1_upload(d, s) != 0) {
    rt_scene_release(d);
    return NULL;
  }
  if (!d->book1 && env_flag("RT_GENERAL", true) && general_upload(d, s) != 0) {
    rt_scene_release(d);
    return NULL;
  }
  return d;
}

extern "C" void rt_scene_release(rt_device_scene *d) {
  if (!d) return;
  (void)hipSetDevice(d->device);
  (void)hipFree(d->arena);
  if (d->b1_arena) (void)hipFree(d->b1_arena);
  if (d->gen_arena) (void)hipFree(d->gen_arena);
  if (d->px_time) (void)hipFree(d->px_time);
  if (d->sp_arena) (void)hipFree(d->sp_arena);
  if (d->pre_arena) (void)hipFree(d->pre_arena);
  if (d->wave_stream) (void)hipStreamDestroy(d->wave_stream);
  if (d->ev_fork) (void)hipEventDestroy(d->ev_fork);
  if (d->ev_join) (void)hipEventDestroy(d->ev_join);
  for (hipEvent_t e : d->ev_main)
    if (e) (void)hipEventDestroy(e);
  delete d;
}

// One Book-1 launch of the scene's variant (work counter and stats reset first).
static int launch_book1(rt_device_scene *d, const b1::Book1View &V, uint8_t *d_out, hipStream_t st,
                        bool cost_pass = false) {
  HIP_OK(hipMemsetAsync(V.work_counter, 0, d->book1_stats ? 256 : sizeof(int32_t), st));
  if (d->book1_stats) {
    HIP_OK(hipMemsetAsync(V.stats + 18, 0xff, sizeof(unsigned long long), st));
    HIP_OK(hipMemsetAsync(V.stats + 21, 0xff, sizeof(unsigned long long), st));
  }
    const dim3 g1((unsigned)d->b1_grid), blk(b1::kBlock);
  if (cost_pass) {  // the variants that have an ordered refill (render_batched)
    if (d->book1_ver == 9 && d->book1_lds)
      hipLaunchKernelGGL((rt_book1_cost_kernel<true, 9>), g1, blk, d->b1_lds_bytes, st, V, d_out);
    else if (d->book1_ver == 9)
      hipLaunchKernelGGL((rt_book1_cost_kernel<false, 9>), g1, blk, d->b1_lds_bytes, st, V, d_out);
    else if (d->book1_lds)
      hipLaunchKernelGGL((rt_book1_cost_kernel<true, 5>), g1, blk, d->b1_lds_bytes, st, V, d_out);
    else
      hipLaunchKernelGGL((rt_book1_cost_kernel<false, 5>), g1, blk, d->b1_lds_bytes, st, V, d_out);
    HIP_OK(hipGetLastError());
    return 0;
  }
#define RT_B1_LAUNCH(LDS, VER, ST, ...) \
  hipLaunchKernelGGL((rt_book1_kernel<LDS, VER, ST, ##__VA_ARGS__>), g1, blk, d->b1_lds_bytes, st, V, d_out)
    switch (d->book1_occ * 100 + d->book1_ver * 4 + (d->book1_lds ? 1 : 0) + (d->book1_stats ? 2 : 0)) {
      case 500 + 5 * 4 + 1: RT_B1_LAUNCH(true, 5, false, 5); break;
      case 500 + 5 * 4 + 0: RT_B1_LAUNCH(false, 5, false, 5); break;
      case 600 + 5 * 4 + 1: RT_B1_LAUNCH(true, 5, false, 6); break;
      case 600 + 5 * 4 + 0: RT_B1_LAUNCH(false, 5, false, 6); break;
      case 6 * 4 + 3: RT_B1_LAUNCH(true, 6, true); break;
      case 5 * 4 + 3: RT_B1_LAUNCH(true, 5, true); break;
      case 9 * 4 + 1: RT_B1_LAUNCH(true, 9, false); break;
      case 9 * 4 + 0: RT_B1_LAUNCH(false, 9, false); break;
      case 9 * 4 + 3: RT_B1_LAUNCH(true, 9, true); break;
      case 7 * 4 + 1: RT_B1_LAUNCH(true, 7, false); break;
      case 7 * 4 + 0: RT_B1_LAUNCH(false, 7, false); break;
      case 7 * 4 + 3: RT_B1_LAUNCH(true, 7, true); break;
      case 6 * 4 + 1: RT_B1_LAUNCH(true, 6, false); break;
      case 6 * 4 + 0: RT_B1_LAUNCH(false, 6, false); break;
      case 5 * 4 + 1: RT_B1_LAUNCH(true, 5, false); break;
      case 5 * 4 + 0: RT_B1_LAUNCH(false, 5, false); break;
      case 3 * 4 + 1: RT_B1_LAUNCH(true, 3, false); break;
      case 3 * 4 + 0: RT_B1_LAUNCH(false, 3, false); break;
      case 2 * 4 + 1: RT_B1_LAUNCH(true, 2, false); break;
      case 2 * 4 + 0: RT_B1_LAUNCH(false, 2, false); break;
      default: return rt_set_error("book1 variant %d not built", d->book1_ver), -1;
    }
#undef RT_B1_LAUNCH
  HIP_OK(hipGetLastError());
  return 0;
}

// Split render of one launch (rt_book1.h: SplitPx).  A pre-pass at lpt_spp measures each pixel's
// traversal steps and pcg32 draws; the host cuts every pixel whose chain would outlast the frame's
// throughput time into segments (and orders all chains longest first); then one round of chains,
// the walk, and split_rounds fix-up rounds, all queued on the stream.  Returns 1 (nothing launched
// after the pre-pass) when the plan does not fit its limits; the caller renders unsplit.
static int launch_split(rt_device_scene *d, b1::Book1View V, uint8_t *d_out, hipStream_t st, int64_t npix) {
  {
    b1::Book1View P = V;
    P.S.cam.spp = d->lpt_spp;
    P.cost_out = d->lpt_cost;
    P.draw_out = d->draw_out;
    if (launch_book1(d, P, d_out, st, true) != 0) return -1;
  }
  const size_t n = (size_t)npix;
  d->h_cost.resize(n);
  d->h_draws.resize(n);
  HIP_OK(hipMemcpyAsync(d->h_cost.data(), d->lpt_cost, n * sizeof(uint32_t), hipMemcpyDeviceToHost, st));
  HIP_OK(hipMemcpyAsync(d->h_draws.data(), d->draw_out, n * sizeof(uint32_t), hipMemcpyDeviceToHost, st));
  HIP_OK(hipStreamSynchronize(st));
  const double ratio = (double)V.S.cam.spp / (double)d->lpt_spp;
  double sum = 0.0;
  for (size_t p = 0; p < n; p++) sum += (double)d->h_cost[p];
  // a chain's target cost (pre-pass steps): its latency at kLaneLat per step against the lanes'
  // throughput time for the whole launch at kLaneThr per step
  const double lanes = (double)d->sp_grid * b1::kBlock;
  const double cstar = fmax(1.0, d->split_beta * sum * kLaneThr / (lanes * kLaneLat));
  std::vector<b1::SplitPx> &px = d->h_px;
  px.resize(n);
  std::vector<uint16_t> kseg(n);
  uint32_t hist[256] = {0};
  uint64_t n_items = 0, rec_total = 0;
  d->h_walk.clear();
  for (size_t p = 0; p < n; p++) {
    const double c = (double)d->h_cost[p];
    int K = (int)fmin((double)d->split_kmax, ceil(c / cstar));
    b1::SplitPx &P = px[p];
    P.acc[0] = P.acc[1] = P.acc[2] = 0.0f;
    P.o = P.s = 0u;
    P.stop_at = b1::kNoCoalesce;
    P.base = P.len = P.len_run = 0u;
    const double mu = fmax(1.0, (double)d->h_draws[p] / d->lpt_spp);  // draws per sample
    const uint32_t w = (uint32_t)fmin(512.0, fmax(8.0, ceil(d->split_wfact * mu)));
    P.w = w;
    P.cps = (float)(c / V.S.cam.spp);  // pre-pass steps per frame sample
    P.rec_lo = 0xffffffffu;
    const double est = (double)d->h_draws[p] * ratio;
    const double len = ceil(est * d->split_margin) + w;
    if (K > 1) K = (int)fmin((double)K, floor(len / (4.0 * w)));  // segments of at least 4 windows
    if (K < 2) K = 1;
    kseg[p] = (uint16_t)K;
    if (K > 1) {
      const uint32_t L = (uint32_t)ceil(len / K);
      P.len_run = (uint32_t)len;
      P.len = (uint32_t)fmax(len, ceil(est * d->split_alloc) + 2.0 * w);
      P.stop_at = L;
      P.rec_lo = L;
      P.base = (uint32_t)(rec_total - L);  // records of offsets [L, len) only (u32 wrap-around)
      rec_total += P.len - L;
      d->h_walk.push_back(make_uint4((uint32_t)p, 0u, 0u, 0u));
    }
    const uint32_t b = host_lpt_bucket((uint32_t)fmin(4294967295.0, c / K));
    hist[b] += (uint32_t)K;
    n_items += (uint64_t)K;
  }
  if (rec_total >= ((uint64_t)15 << 28) || n_items >= ((uint64_t)1 << 31)) {  // u32 record indices
    if (env_flag("RT_DEBUG", false)) fprintf(stderr, "[rtc] split: plan too large (%llu records), unsplit\n", (unsigned long long)rec_total);
    return 1;
  }
  const uint64_t n_ent = n_items;
  // longest chains first: bucket offsets from the top bucket down
  uint32_t start[256];
  for (int k = 255, run = 0; k >= 0; k--) start[k] = (uint32_t)run, run += (int)hist[k];
  d->h_items.resize((size_t)n_items);  // entries: heads, and one per segment window
  for (size_t p = 0; p < n; p++) {
    const int K = kseg[p];
    const uint32_t b = host_lpt_bucket((uint32_t)fmin(4294967295.0, (double)d->h_cost[p] / K));
    if (K > 1) {  // the segment windows first, then the head: the head walks the segments' records
      const b1::SplitPx &P = px[p];
      const uint32_t L = P.stop_at;
      const uint32_t w = (uint32_t)fmin(512.0, fmax(8.0, ceil(d->split_wfact * fmax(1.0, (double)d->h_draws[p] / d->lpt_spp))));
      for (int k = 1; k < K; k++) {
        const uint32_t B = (uint32_t)k * L, E = k + 1 == K ? P.len_run : (uint32_t)(k + 1) * L;
        d->h_items[start[b]++] = make_uint4((uint32_t)p | b1::kSpecBit, B, E, w);
      }
    }
    d->h_items[start[b]++] = make_uint4((uint32_t)p, 0u, 0u, 0u);
  }
  const size_t n_split = d->h_walk.size();
  d->h_pre.resize((size_t)n_ent);
  uint64_t n_chains = 0;
  for (size_t e = 0; e < (size_t)n_ent; e++) d->h_pre[e] = (uint32_t)n_chains, n_chains += d->h_items[e].w ? d->h_items[e].w : 1u;
  if (n_chains >= ((uint64_t)1 << 31)) return 1;
  // device buffers: px, items, walk list, two fix-up lists, counters, claims, records
  size_t off[10], total = 0;
  const size_t sizes[10] = {n * sizeof(b1::SplitPx), (size_t)n_chains * sizeof(uint4), (n_split + 1) * sizeof(uint4),
                           2 * (n_split + 1) * sizeof(uint4), 256 * sizeof(uint32_t),
                           (size_t)rec_total * sizeof(uint32_t), (size_t)rec_total * sizeof(float4),
                           (size_t)n_ent * sizeof(uint4), (size_t)n_ent * sizeof(uint32_t),
                           (size_t)n_chains * sizeof(uint4)};  // [9] re-split chains of a fix-up round
  for (int k = 0; k < 10; k++) off[k] = total, total = align_up(total + (sizes[k] ? sizes[k] : 16), 256);
  if (total > d->sp_bytes) {
    if (d->sp_arena) HIP_OK(hipFree(d->sp_arena));
    d->sp_arena = nullptr;
    d->sp_bytes = 0;
    HIP_OK(hipMalloc(&d->sp_arena, total));
    d->sp_bytes = total;
  }
  char *b = (char *)d->sp_arena;
  uint32_t *cnt = (uint32_t *)(b + off[4]);
  d->h_cnt[0] = (uint32_t)n_chains;
  d->h_cnt[1] = (uint32_t)n_split;
  for (int k = 2; k < 256; k++) d->h_cnt[k] = 0u;
  HIP_OK(hipMemcpyAsync(b + off[0], px.data(), sizes[0], hipMemcpyHostToDevice, st));
  HIP_OK(hipMemcpyAsync(b + off[7], d->h_items.data(), sizes[7], hipMemcpyHostToDevice, st));
  HIP_OK(hipMemcpyAsync(b + off[8], d->h_pre.data(), sizes[8], hipMemcpyHostToDevice, st));
  {
    const unsigned eb = (unsigned)(n_ent / 256 + 1 < 4096 ? n_ent / 256 + 1 : 4096);
    hipLaunchKernelGGL(split_expand_kernel, dim3(eb), dim3(256), 0, st, (const uint4 *)(b + off[7]),
                       (const uint32_t *)(b + off[8]), (uint32_t)n_ent, (uint4 *)(b + off[1]));
    HIP_OK(hipGetLastError());
  }
  if (n_split) HIP_OK(hipMemcpyAsync(b + off[2], d->h_walk.data(), n_split * sizeof(uint4), hipMemcpyHostToDevice, st));
  HIP_OK(hipMemcpyAsync(cnt, d->h_cnt, 256 * sizeof(uint32_t), hipMemcpyHostToDevice, st));
  if (env_flag("RT_DEBUG", false))
    fprintf(stderr, "[rtc] split: %zu px, %zu split, %llu entries, %llu chains, %llu records (%.1f MB), chain target %.0f steps\n", n,
            n_split, (unsigned long long)n_ent, (unsigned long long)n_chains, (unsigned long long)rec_total, total / 1e6, cstar * ratio);
  if (d->ev_main[0]) HIP_OK(hipEventRecord(d->ev_main[0], st));
  if (rec_total) {
    HIP_OK(hipMemsetAsync(b + off[5], 0, sizes[5], st));
    HIP_OK(hipMemsetAsync(b + off[6], 0xff, sizes[6], st));  // kRecFill
  }
  V.sp_px = (b1::SplitPx *)(b + off[0]);
  V.sp_claim = (uint32_t *)(b + off[5]);
  V.sp_rec = (float4 *)(b + off[6]);
  V.order = nullptr;
  V.n_coop = nullptr;
  V.n_heavy = nullptr;
  V.cost_out = nullptr;
  V.sp_items2 = nullptr;
  V.sp_n_items2 = nullptr;
  V.sp_cap2 = 0u;
  uint4 *items2 = (uint4 *)(b + off[9]);
  uint4 *walk0 = (uint4 *)(b + off[2]);
  uint4 *fix[2] = {(uint4 *)(b + off[3]), (uint4 *)(b + off[3]) + (n_split + 1)};
  const dim3 gs((unsigned)d->sp_grid), blk(b1::kBlock);
  const unsigned wb = (unsigned)(n_split / 256 + 1 < 2048 ? n_split / 256 + 1 : 2048);
  const int rounds = d->split_rounds;
  const bool dbg = env_flag("RT_DEBUG", false);
  auto dbg_mark = [&](const char *what, int r) {  // diagnostic: synchronous timing of each step
    static double t_last = 0.0;
    (void)hipStreamSynchronize(st);
    timespec ts;
    clock_gettime(CLOCK_MONOTONIC, &ts);
    const double t = ts.tv_sec * 1e3 + ts.tv_nsec * 1e-6;
    uint32_t c[136];
    (void)hipMemcpy(c, cnt, sizeof c, hipMemcpyDeviceToHost);
    if (what) fprintf(stderr, "[rtc] split %s %d: %.2f ms (counts %u %u | fix %u %u %u %u | resplit %u %u %u)\n", what, r,
                      t - t_last, c[0], c[1], c[2], c[3], c[4], c[5], c[129], c[130], c[131]);
    t_last = t;
  };
  if (dbg) dbg_mark(nullptr, 0);
  // round r: (r > 0: re-split the unfinished pixels) chains, then the walk; its unfinished pixels are
  // round r+1's heads.  The first `rounds` rounds are queued without a host sync; then the host
  // checks the count and queues more while pixels remain; round kMaxRounds-1 walks with
  // last_round set, so round kMaxRounds's heads run to the end without stopping.
  constexpr int kMaxRounds = 100;
  auto queue_round = [&](int r) -> int {
    V.sp_items = r == 0 ? (const uint4 *)(b + off[1]) : fix[(r - 1) % 2];
    V.sp_n_items = r == 0 ? cnt : cnt + 1 + r;
    if (r > 0) {  // re-split pixels' segment chains (split_replan_kernel, counter cnt[128 + r])
      hipLaunchKernelGGL(split_replan_kernel, dim3(wb), dim3(256), 0, st, V, fix[(r - 1) % 2], cnt + 1 + r, items2,
                         cnt + 128 + r, (uint32_t)n_chains, (float)(cstar * d->split_fixc), d->split_margin,
                         d->split_kmax, (int)(r == kMaxRounds));
      HIP_OK(hipGetLastError());
      V.sp_items2 = items2;
      V.sp_n_items2 = cnt + 128 + r;
      V.sp_cap2 = (uint32_t)n_chains;
      if (dbg) dbg_mark("replan", r);
    }
    HIP_OK(hipMemsetAsync(V.work_counter, 0, sizeof(int32_t), st));
    hipLaunchKernelGGL(rt_book1_split_kernel<true>, gs, blk, d->b1_lds_bytes, st, V, d_out);
    HIP_OK(hipGetLastError());
    if (dbg) dbg_mark("chains", r);
    if (r < kMaxRounds) {  // the walk over this round's split pixels; misses become next round's heads
      hipLaunchKernelGGL(split_walk_kernel, dim3(wb), dim3(256), 0, st, V, d_out, r == 0 ? walk0 : fix[(r - 1) % 2],
                         r == 0 ? cnt + 1 : cnt + 1 + r, fix[r % 2], cnt + 2 + r, (int)(r + 1 == kMaxRounds));
      HIP_OK(hipGetLastError());
      if (dbg) dbg_mark("walk", r);
    }
    return 0;
  };
  int r = 0;
  for (; r <= rounds && r <= kMaxRounds; r++)
    if (queue_round(r) != 0) return -1;
  while (n_split && r <= kMaxRounds) {  // more rounds while the last walk left pixels unfinished
    uint32_t left = 0;
    HIP_OK(hipMemcpyAsync(&left, cnt + 1 + r, sizeof left, hipMemcpyDeviceToHost, st));
    HIP_OK(hipStreamSynchronize(st));
    if (left == 0) break;
    if (queue_round(r) != 0) return -1;
    r++;
  }
  d->split_rounds_used = r;
  if (d->ev_main[1]) HIP_OK(hipEventRecord(d->ev_main[1], st));
  return 0;
}

static void launch_general(const rt_device_scene *d, bool all, dim3 g, dim3 b, hipStream_t st, gen::GeneralView V,
                           uint8_t *d_out) {
  V.batch = d->gen_batch;
  V.steps = d->gen_steps;
  V.n_lds = d->gen_lds;
  const size_t lds_bytes = (size_t)d->gen_lds * 2 * sizeof(float4);
  if (all && d->gen_batch)
    hipLaunchKernelGGL((rt_general_kernel<kFeatAll, true>), g, b, lds_bytes, st, V, d_out);
  else if (all)
    hipLaunchKernelGGL((rt_general_kernel<kFeatAll, false>), g, b, 0, st, V, d_out);
  else if (d->gen_batch)
    hipLaunchKernelGGL((rt_general_kernel<kFeatBook1, true>), g, b, lds_bytes, st, V, d_out);
  else
    hipLaunchKernelGGL((rt_general_kernel<kFeatBook1, false>), g, b, 0, st, V, d_out);
}

extern "C" int rt_render_rows_async(rt_device_scene *d, int row0, int row_stride, int n_rows, uint8_t *d_out,
                                    void *stream) {
  if (!d || !d_out) return rt_set_error("rt_render_rows_async: NULL argument"), -1;
  if (n_rows <= 0) return 0;
  if (row0 < 0 || row_stride <= 0 || (int64_t)row0 + (int64_t)(n_rows - 1) * row_stride >= d->height)
    return rt_set_error("rows %d + k*%d (k < %d) outside image height %d", row0, row_stride, n_rows, d->height), -1;
  HIP_OK(hipSetDevice(d->device));
  const int64_t npix = (int64_t)n_rows * d->width;
  const dim3 grid((unsigned)((npix + kBlock - 1) / kBlock)), block(kBlock);
  hipStream_t st = (hipStream_t)stream;
  if (d->book1) {
    if (npix >= (int64_t)1 << 31) return rt_set_error("too many pixels for one launch"), -1;
    b1::Book1View V = d->b1view;
    V.row0 = row0;
    V.row_stride = row_stride;
    V.n_rows = n_rows;
    // the group kernel when the launch has fewer pixels than the lane kernel has lanes (a frame split
    // over several GPUs): there the sequential per-pixel chains, not the lanes' throughput, set the time
    const bool use_group =
        d->group_mode == 1 || (d->group_mode == 2 && npix < (int64_t)d->b1_grid * b1::kBlock);
    // the split render where the chains, not the lanes, bound the launch (RT_SPLIT)
    if (d->split_mode != 0 && d->lpt && V.S.cam.spp >= 4 * d->lpt_spp && npix >= 4096 && V.S.cam.max_depth >= 1 &&
        (d->split_mode == 1 || npix < (int64_t)d->b1_grid * b1::kBlock)) {
      const int rc = launch_split(d, V, d_out, st, npix);
      if (rc <= 0) return rc;
    }
    // longest-first order: a low-spp pass measures each work item's traversal steps
    if (d->lpt && V.S.cam.spp >= 4 * d->lpt_spp && npix >= 4096) {
      b1::Book1View P = V;
      P.S.cam.spp = d->lpt_spp;
      P.cost_out = d->lpt_cost;
      if (launch_book1(d, P, d_out, st, true) != 0) return -1;
      HIP_OK(hipMemsetAsync(d->lpt_hist, 0, kLptHistBytes, st));
      unsigned long long *sums = (unsigned long long *)(d->lpt_hist + 512 + 32);  // after the 516 counters
      const int n = (int)npix, nb = (int)((npix + 255) / 256 < 1024 ? (npix + 255) / 256 : 1024);
      hipLaunchKernelGGL(lpt_hist_kernel, dim3(nb), dim3(256), 0, st, d->lpt_cost, n, d->lpt_hist, sums);
      const int64_t thr = (int64_t)d->coop_steps * d->lpt_spp;
      const int coop_bucket = d->coop_steps < 0 ? -1 : (thr < (int64_t)UINT32_MAX ? (int)host_lpt_bucket((uint32_t)thr) : 255);
      LptModel model;
      model.spp_ratio = (float)V.S.cam.spp / (float)d->lpt_spp;
      model.grid_waves = (use_group ? d->g_grid : d->b1_grid) * (b1::kBlock / 64);
      model.lat_step = use_group ? kGroupLat : kLaneLat;
      model.thr_step = use_group ? kGroupThr : kLaneThr;
      model.coop_step = use_group ? kCoopStep : kCoopStepLane;
      model.lanes_per_wave = use_group ? 64 / grp::kG : 64;
      model.debug = env_flag("RT_DEBUG", false) ? 1 : 0;
      if (const char *em = getenv(use_group ? "RT_MODEL_GROUP" : "RT_MODEL_LANE"))  // "lat,thr,coop" (tuning)
        sscanf(em, "%f,%f,%f", &model.lat_step, &model.thr_step, &model.coop_step);
      const int64_t pthr = (int64_t)d->prio_steps * d->lpt_spp;
      const int prio_bucket = d->prio_steps > 0 && pthr < (int64_t)UINT32_MAX ? (int)host_lpt_bucket((uint32_t)pthr) : 256;
      hipLaunchKernelGGL(lpt_scan_kernel, dim3(1), dim3(64), 0, st, d->lpt_hist, sums, coop_bucket,
                         d->coop_waves, prio_bucket, model);
      hipLaunchKernelGGL(lpt_scatter_kernel, dim3(nb), dim3(256), 0, st, d->lpt_cost, n, d->lpt_hist, d->lpt_order);
      if (d->coop_waves != 0 && d->wave_stream && env_flag("RT_COOP_SORT", true))
        hipLaunchKernelGGL(lpt_coop_sort_kernel, dim3(1), dim3(1024), 0, st, d->lpt_cost, d->lpt_hist, d->lpt_order);
      HIP_OK(hipGetLastError());
      V.order = d->lpt_order;
      V.n_heavy = d->prio_steps > 0 ? d->lpt_hist + 514 : nullptr;
      if (env_flag("RT_DEBUG", false)) {  // diagnostic: synchronous peek at the cooperative count
        uint32_t nc = 0;
        HIP_OK(hipStreamSynchronize(st));
        HIP_OK(hipMemcpy(&nc, d->lpt_hist + 512, sizeof nc, hipMemcpyDeviceToHost));
        uint32_t nh = 0, nw = 0;
        HIP_OK(hipMemcpy(&nh, d->lpt_hist + 514, sizeof nh, hipMemcpyDeviceToHost));
        HIP_OK(hipMemcpy(&nw, d->lpt_hist + 515, sizeof nw, hipMemcpyDeviceToHost));
        fprintf(stderr, "[rtc] lpt: %lld items, %u cooperative on %u waves (RT_COOP_STEPS %d, RT_COOP_WAVES %d; <0: "
                "model), %u at raised priority\n", (long long)npix, nc, nw, d->coop_steps, d->coop_waves, nh);
      }
      if (d->coop_waves != 0 && d->wave_stream) {
        V.n_coop = d->lpt_hist + 512;
        V.coop_counter = (int32_t *)(d->lpt_hist + 513);
        V.coop_waves_dev = d->lpt_hist + 515;
      }
    }
    if (d->ev_main[0]) HIP_OK(hipEventRecord(d->ev_main[0], st));
    const bool split = V.n_coop != nullptr;
    if (split) {  // whole-wave items: a concurrent kernel on the second stream (rt_book1.h: render_wave_items)
      HIP_OK(hipEventRecord(d->ev_fork, st));
      HIP_OK(hipStreamWaitEvent(d->wave_stream, d->ev_fork, 0));
      // as many workgroups as the model may give it; the lane kernel leaves it that many CU slots
      const dim3 gw((unsigned)(d->b1_grid / 2 > 0 ? d->b1_grid / 2 : 1)), blk(b1::kBlock);
      if (d->book1_lds)
        hipLaunchKernelGGL((rt_book1_wave_kernel<true>), gw, blk, d->b1_lds_bytes, d->wave_stream, V, d_out);
      else
        hipLaunchKernelGGL((rt_book1_wave_kernel<false>), gw, blk, d->b1_lds_bytes, d->wave_stream, V, d_out);
      HIP_OK(hipGetLastError());
    }
    if (use_group) {  // eight lanes per pixel (rt_group.h)
      HIP_OK(hipMemsetAsync(V.work_counter, 0, sizeof(int32_t), st));
      const dim3 gg((unsigned)d->g_grid), gb(grp::kBlock);
      if (d->book1_lds)
        hipLaunchKernelGGL((rt_book1_group_kernel<true>), gg, gb, d->g_lds_bytes, st, V, d_out);
      else
        hipLaunchKernelGGL((rt_book1_group_kernel<false>), gg, gb, d->g_lds_bytes, st, V, d_out);
      HIP_OK(hipGetLastError());
    } else if (launch_book1(d, V, d_out, st) != 0) {
      return -1;
    }
    if (split) {
      HIP_OK(hipEventRecord(d->ev_join, d->wave_stream));
      HIP_OK(hipStreamWaitEvent(st, d->ev_join, 0));
    }
    if (d->ev_main[1]) HIP_OK(hipEventRecord(d->ev_main[1], st));
    return 0;
  }
  if (d->general) {
    gen::GeneralView G;
    G.S = d->view;
    G.row0 = row0;
    G.row_stride = row_stride;
    G.n_rows = n_rows;
    G.work_counter = d->gen_counter;
    G.order = nullptr;
    G.cost_out = nullptr;
    const bool all = (d->features & ~kFeatBook1) != 0;
    const dim3 gg((unsigned)d->gen_grid), gb(gen::kBlock);
    if (d->lpt && G.S.cam.spp >= 4 * d->lpt_spp && npix >= 4096) {  // longest-first order (rays per pixel)
      gen::GeneralView P = G;
      P.S.cam.spp = d->lpt_spp;
      P.cost_out = d->lpt_cost;
      HIP_OK(hipMemsetAsync(d->gen_counter, 0, sizeof(int32_t), st));
      if (all)
        launch_general(d, true, gg, gb, st, P, d_out);
      else
        launch_general(d, false, gg, gb, st, P, d_out);
      HIP_OK(hipMemsetAsync(d->lpt_hist, 0, kLptHistBytes, st));
      unsigned long long *sums = (unsigned long long *)(d->lpt_hist + 512 + 32);
      const int n = (int)npix, nb = (int)((npix + 255) / 256 < 1024 ? (npix + 255) / 256 : 1024);
      hipLaunchKernelGGL(lpt_hist_kernel, dim3(nb), dim3(256), 0, st, d->lpt_cost, n, d->lpt_hist, sums);
      LptModel model;
      model.spp_ratio = 1.0f;
      model.grid_waves = d->gen_grid * (gen::kBlock / 64);
      model.lat_step = kLaneLat;
      model.thr_step = kLaneThr;
      model.coop_step = kCoopStep;
      model.lanes_per_wave = 64;
      model.debug = 0;
      hipLaunchKernelGGL(lpt_scan_kernel, dim3(1), dim3(64), 0, st, d->lpt_hist, sums, 255, 0, 256, model);
      hipLaunchKernelGGL(lpt_scatter_kernel, dim3(nb), dim3(256), 0, st, d->lpt_cost, n, d->lpt_hist, d->lpt_order);
      HIP_OK(hipGetLastError());
      G.order = d->lpt_order;
    }
    HIP_OK(hipMemsetAsync(d->gen_counter, 0, sizeof(int32_t), st));
    if (d->ev_main[0]) HIP_OK(hipEventRecord(d->ev_main[0], st));
    if (all)
      launch_general(d, true, gg, gb, st, G, d_out);
    else
      launch_general(d, false, gg, gb, st, G, d_out);
    HIP_OK(hipGetLastError());
    if (d->ev_main[1]) HIP_OK(hipEventRecord(d->ev_main[1], st));
    return 0;
  }
  if ((d->features & ~kFeatBook1) == 0)
    hipLaunchKernelGGL(rt_render_rows_kernel<kFeatBook1>, grid, block, 0, st, d->view, row0, row_stride, n_rows, d_out);
  else
    hipLaunchKernelGGL(rt_render_rows_kernel<kFeatAll>, grid, block, 0, st, d->view, row0, row_stride, n_rows, d_out);
  HIP_OK(hipGetLastError());
  return 0;
}

// ------------------------------------------------------------------------------ whole frame
static std::mutex g_timing_mu;
static std::vector<double> g_kernel_ms(64, 0.0);

extern "C" double rt_last_kernel_ms(int device) {
  std::lock_guard<std::mutex> lk(g_timing_mu);
  return (device >= 0 && device < (int)g_kernel_ms.size()) ? g_kernel_ms[device] : 0.0;
}

extern "C" int rt_render(const rt_flat_scene *s, int n_gpus, uint8_t *out_host) {
  if (!s || !out_host) return rt_set_error("rt_render: NULL argument"), -1;
  const int avail = rt_device_count();
  if (avail <= 0) return rt_set_error("rt_render: no HIP device visible (this library has no CPU path)"), -1;
  const int H = s->camera.height, W = s->camera.width;
  int G = (n_gpus <= 0 || n_gpus > avail) ? avail : n_gpus;
  if (G > H) G = H;
  struct PerGpu {
    rt_device_scene *scene = nullptr;
    uint8_t *d_out = nullptr;
    hipStream_t stream = nullptr;
    hipEvent_t t0 = nullptr, t1 = nullptr;
    int n_rows = 0;
  };
  std::vector<PerGpu> per(G);
  int rc = 0;
  for (int g = 0; g < G && rc == 0; g++) {  // upload + launch on every GPU first
    PerGpu &p = per[g];
    p.n_rows = (H - g + G - 1) / G;
    p.scene = rt_scene_upload(s, g);
    if (!p.scene) {
      rc = -1;
      break;
    }
    if (hipStreamCreateWithFlags(&p.stream, hipStreamNonBlocking) != hipSuccess ||
        hipMalloc(&p.d_out, (size_t)p.n_rows * W * 3) != hipSuccess || hipEventCreate(&p.t0) != hipSuccess ||
        hipEventCreate(&p.t1) != hipSuccess) {
      rt_set_error("rt_render: stream/buffer setup failed on device %d", g);
      rc = -1;
      break;
    }
    (void)hipEventRecord(p.t0, p.stream);
    if (rt_render_rows_async(p.scene, g, G, p.n_rows, p.d_out, p.stream) != 0) {
      rc = -1;
      break;
    }
    (void)hipEventRecord(p.t1, p.stream);
  }
  std::vector<uint8_t> rows;
  for (int g = 0; g < G; g++) {  // then drain: D2H compact rows, scatter to j % G == g
    PerGpu &p = per[g];
    if (rc == 0 && p.scene) {
      (void)hipSetDevice(g);
      rows.resize((size_t)p.n_rows * W * 3);
      hipError_t e = hipStreamSynchronize(p.stream);
      if (e == hipSuccess) e = hipMemcpy(rows.data(), p.d_out, rows.size(), hipMemcpyDeviceToHost);
      if (e != hipSuccess) {
        rt_set_error("rt_render: device %d: %s", g, hipGetErrorString(e));
        rc = -1;
      } else {
        float ms = 0.0f;
        (void)hipEventElapsedTime(&ms, p.t0, p.t1);
        {
          std::lock_guard<std::mutex> lk(g_timing_mu);
          if (g < (int)g_kernel_ms.size()) g_kernel_ms[g] = ms;
        }
        for (int k = 0; k < p.n_rows; k++)
          memcpy(out_host + (size_t)(g + k * G) * W * 3, rows.data() + (size_t)k * W * 3, (size_t)W * 3);
      }
    }
    if (p.scene) (void)hipSetDevice(g);
    if (p.t0) (void)hipEventDestroy(p.t0);
    if (p.t1) (void)hipEventDestroy(p.t1);
    if (p.d_out) (void)hipFree(p.d_out);
    if (p.stream) (void)hipStreamDestroy(p.stream);
    rt_scene_release(p.scene);
  }
  return rc;
}

// Diagnostic counters of the last RT_BOOK1_STATS=1 launch on this scene (b1::kNumStats x u64; see rt_book1.h).
extern "C" int rt_book1_stats(rt_device_scene *d, unsigned long long *out, int n) {
  if (!d || !d->book1 || !d->book1_stats) return rt_set_error("no stats build active (RT_BOOK1_STATS=1)"), -1;
  HIP_OK(hipSetDevice(d->device));
  if (n < 0 || n > b1::kNumStats) return rt_set_error("rt_book1_stats: n must be in [0, %d]", b1::kNumStats), -1;
  HIP_OK(hipMemcpy(out, d->b1view.stats, n * sizeof(unsigned long long), hipMemcpyDeviceToHost));
  return 0;
}

extern "C" int rt_diag_libm(int fn, const float *x_host, float *out_host, int64_t n, int device) {
  if (n <= 0) return 0;
  HIP_OK(hipSetDevice(device));
  const int64_t nout = (fn == 0) ? 2 * n : n;
  float *dx = NULL, *dy = NULL;
  HIP_OK(hipMalloc(&dx, n * sizeof(float)));
  HIP_OK(hipMalloc(&dy, nout * sizeof(float)));
  HIP_OK(hipMemcpy(dx, x_host, n * sizeof(float), hipMemcpyHostToDevice));
  hipLaunchKernelGGL(rt_diag_libm_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, 0, fn, dx, dy, n);
  HIP_OK(hipGetLastError());
  HIP_OK(hipMemcpy(out_host, dy, nout * sizeof(float), hipMemcpyDeviceToHost));
  HIP_OK(hipFree(dx));
  HIP_OK(hipFree(dy));
  return 0;
}

extern "C" int rt_diag_arith(int fn, uint64_t start, uint64_t count, uint64_t seed, unsigned long long *mismatches,
                             int device) {
  if (fn < 0 || fn > 3 || mismatches == NULL) return rt_set_error("rt_diag_arith: bad arguments"), -1;
  HIP_OK(hipSetDevice(device));
  unsigned long long *dm = NULL;
  HIP_OK(hipMalloc(&dm, sizeof *dm));
  HIP_OK(hipMemset(dm, 0, sizeof *dm));
  hipLaunchKernelGGL(rt_diag_arith_kernel, dim3(fn == 3 ? 1 : 4096), dim3(fn == 3 ? 64 : 256), 0, 0, fn, start, count,
                     seed, dm);
  HIP_OK(hipGetLastError());
  HIP_OK(hipMemcpy(mismatches, dm, sizeof *dm, hipMemcpyDeviceToHost));
  HIP_OK(hipFree(dm));
  return 0;
}

extern "C" int rt_book1_pixel_cost(rt_device_scene *d, uint32_t *out, int64_t n_items) {
  if (!d || !d->book1 || !d->book1_stats) return rt_set_error("no stats build active (RT_BOOK1_STATS=1)"), -1;
  if (n_items < 0 || n_items > (int64_t)d->width * d->height) return rt_set_error("rt_book1_pixel_cost: bad count"), -1;
  HIP_OK(hipSetDevice(d->device));
  HIP_OK(hipDeviceSynchronize());
  HIP_OK(hipMemcpy(out, d->b1view.pixel_cost, (size_t)n_items * 2 * sizeof(uint32_t), hipMemcpyDeviceToHost));
  return 0;
}

extern "C" int rt_scene_px_time(rt_device_scene *d, uint32_t *times, uint32_t *cost, int32_t *order,
                                uint32_t *n_coop, int64_t n) {
  if (!d || !d->book1) return rt_set_error("rt_scene_px_time: not a Book-1 scene"), -1;
  if (n < 0 || n > (int64_t)d->width * d->height) return rt_set_error("rt_scene_px_time: bad count"), -1;
  HIP_OK(hipSetDevice(d->device));
  HIP_OK(hipDeviceSynchronize());
  if (times) {
    if (!d->px_time) return rt_set_error("rt_scene_px_time: upload with RT_PX_TIME=1"), -1;
    HIP_OK(hipMemcpy(times, d->px_time, (size_t)n * 2 * sizeof(uint32_t), hipMemcpyDeviceToHost));
  }
  if (cost) HIP_OK(hipMemcpy(cost, d->lpt_cost, (size_t)n * sizeof(uint32_t), hipMemcpyDeviceToHost));
  if (order) HIP_OK(hipMemcpy(order, d->lpt_order, (size_t)n * sizeof(int32_t), hipMemcpyDeviceToHost));
  if (n_coop) HIP_OK(hipMemcpy(n_coop, d->lpt_hist + 512, sizeof(uint32_t), hipMemcpyDeviceToHost));
  return 0;
}

// Name of the kernel rt_render_rows_async launches for this scene (as rocprofv3 reports it).
extern "C" const char *rt_scene_kernel(const rt_device_scene *d) {
  static thread_local char buf[160];
  if (!d) return "";
  if (!d->book1)
    snprintf(buf, sizeof buf, "%s<%d>", d->general ? "rt_general_kernel" : "rt_render_rows_kernel",
             (d->features & ~kFeatBook1) == 0 ? (int)kFeatBook1 : (int)kFeatAll);
  else
    snprintf(buf, sizeof buf, "rt_book1_kernel<%s, %d, %s, %d>", d->book1_lds ? "true" : "false", d->book1_ver,
             d->book1_stats ? "true" : "false", d->book1_occ);
  return buf;
}

// Milliseconds of the last frame launch of rt_render_rows_async on this scene (after it completed);
// excludes the LPT cost pre-pass.  -1 when unavailable.
extern "C" double rt_scene_last_launch_ms(rt_device_scene *d) {
  if (!d || !d->ev_main[0] || !d->ev_main[1]) return -1.0;
  float ms = 0.0f;
  if (hipEventElapsedTime(&ms, d->ev_main[0], d->ev_main[1]) != hipSuccess) return -1.0;
  return (double)ms;
}
