// rt_kernel.hip — gfx950 render kernels + the C ABI declared in include/rt_hip.h.
//
// Work decomposition: a pixel's samples share one pcg32 stream (src/raytracing.c:93-124), so the
// unit of parallel work is a pixel -- or, in the chain render, a segment of a pixel's sample stream
// (rt_book1.h: ChainPx).  A launch covers a set of image rows row0 + k*row_stride; multi-GPU runs
// give GPU g the rows j % G == g (interleaved) and need no collective: each GPU
// writes its own compact rows.
//
// Kernels (rt_scene_kernel names the frame kernel of a scene):
//   rt_book1_chain_kernel  Book-1 scenes, lane = chain segment (default); chain_* planner / fold
//   rt_book1_kernel        Book-1 scenes at low spp / small images, lane = pixel (or RT_MODE=lane)
//   rt_book1_cost_kernel   the low-spp pre-pass that measures every pixel's cost
//   rt_general_kernel      every other scene (Book-2 features)
// Every tuning knob (RT_* environment variables) is read once, at scene upload.
#include <hip/hip_runtime.h>

#include <math.h>
#include <stdarg.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <algorithm>
#include <array>
#include <chrono>
#include <cstddef>
#include <functional>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include "../../include/rt_hip.h"
#include "rt_book1.h"
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

// max_depth > kMaxDepth: one pixel per thread, grid-stride over the launch, the path record in a
// global-memory slot of max_depth entries per thread (rt_device.h: DeepRec).
template <int F>
__global__ __launch_bounds__(kBlock) void rt_render_deep_kernel(DScene S, int row0, int row_stride, int n_rows,
                                                                uint8_t *__restrict__ out, DeepRec *rec) {
  const int W = S.cam.width;
  const int64_t tid = (int64_t)blockIdx.x * kBlock + threadIdx.x, nthreads = (int64_t)gridDim.x * kBlock;
  DeepRec *mine = rec + tid * S.cam.max_depth;
  for (int64_t pix = tid; pix < (int64_t)n_rows * W; pix += nthreads) {
    const int jj = (int)(pix / W);
    const int i = (int)(pix - (int64_t)jj * W);
    render_pixel<F, true>(S, i, row0 + jj * row_stride, out + pix * 3, mine);
  }
}

// Persistent Book-1 kernels (rt_book1.h): grid = resident workgroups, lanes steal work items.  The
// chain kernel, its cost pre-pass and the lane kernel run at 5 waves per SIMD (96 VGPRs; the chain
// kernel spills 15, none in the traversal loop: 270 ms vs 282 ms at 4 waves; with the
// SLP vectorizer's packed f32 ops it needed 128 and spilled 65 at 5); launches with few pixels per lane
// (N >= 2 shares) use the 3-wave instantiation (launch_chain).
template <bool kLds>
__global__ __launch_bounds__(b1::kBlock, 5) void rt_book1_kernel(b1::Book1View V, uint8_t *__restrict__ out) {
  extern __shared__ __attribute__((aligned(16))) char lds[];
  b1::render_batched<kLds, 0>(V, out, lds);
}
template <bool kLds, int kOcc = 5>
__global__ __launch_bounds__(b1::kBlock, kOcc) void rt_book1_chain_kernel(b1::Book1View V, uint8_t *__restrict__ out) {
  extern __shared__ __attribute__((aligned(16))) char lds[];
  b1::render_batched<kLds, 2>(V, out, lds);
}
// The cost pre-pass: the same loop at low spp, under its own name so profiles separate it.
template <bool kLds, int kOcc = 5>
__global__ __launch_bounds__(b1::kBlock, kOcc) void rt_book1_cost_kernel(b1::Book1View V, uint8_t *__restrict__ out) {
  extern __shared__ __attribute__((aligned(16))) char lds[];
  b1::render_batched<kLds, 1>(V, out, lds);
}
// After a chain launch: one lane per split pixel (rt_book1.h: chain_fold_px).  (One wave per pixel, its
// lanes loading 64 records for a serial fold in lane order, took 1.44 ms for the N = 8 share's 101 k
// pixels: 17 dependent load round trips per pixel, 12 pixels per wave in turn.)
__global__ __launch_bounds__(64) void chain_fold_kernel(b1::Book1View V, uint8_t *__restrict__ out,
                                                        const uint32_t *split, const uint32_t *cnt,
                                                        b1::ChainCont *cont, uint32_t *n_cont) {
  const uint32_t n = cnt[1];
  for (uint32_t k = blockIdx.x * blockDim.x + threadIdx.x; k < n; k += gridDim.x * blockDim.x) {
    b1::ChainCont q;
    if (!b1::chain_fold_px(V, split[k], out, q)) cont[atomicAdd(n_cont, 1u)] = q;
  }
}

// Persistent general kernel (rt_general.h): grid = resident workgroups, lanes steal pixels.
// kThreads = kBigBlock: one 768-thread workgroup per CU (3 waves per SIMD, as the 256-thread variant
// at occupancy 3) holding the scene's WHOLE preorder in LDS (up to 160 KiB per workgroup on gfx950;
// scene 7's 4946 entries are 158 KiB), so no traversal step waits on L2.  (1024 threads, 4 waves per
// SIMD at 128 VGPRs without spills: 3.91 s vs 3.61-3.66 s for config 5)
constexpr int kBigBlock = 768;
template <int F, bool kBatch = false, int kThreads = gen::kBlock>
__global__ __launch_bounds__(kThreads, kThreads == gen::kBlock ? (kBatch ? 3 : 1) : 1) void rt_general_kernel(
    gen::GeneralView V, uint8_t *__restrict__ out) {
  extern __shared__ __attribute__((aligned(16))) char lds[];
  gen::render_general<F, kBatch, kBatch && kThreads != gen::kBlock>(V, out, (float4 *)lds);
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

// Exactness checks of the Book-1 arithmetic (rt_book1.h: sqrt_core / div_core / sphere_test_data)
// against what the compiler emits for sqrtf() and '/' -- run on the device, count mismatches.
//  fn 0: sqrt_core(x) vs sqrtf(x), x = the float with bits start + k, where x is in the core's domain
//  fn 1: div_core vs '/' on hashed pairs (a in [kDivLo, kDivHi], |x| in [2^-40, kNumHi] or 0)
//  fn 2: sphere_test_data vs the reference-form sphere test (outcome: hit index and t_max bits) on
//        hashed rays, half of them starting on the sphere's surface (the scattered-ray case: c ~ 0)
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
      b1::Lane B = A;
      b1::sphere_test_data(sp, 0, A, 1e-3f);
      b1::sphere_test_lane(&sp, 0, B, 1e-3f);
      bad += (A.hit != B.hit) || (__float_as_uint(A.tmax) != __float_as_uint(B.tmax));
    }
  }
  if (bad) atomicAdd(mism, bad);
}

// ------------------------------------------------------------------------------ longest-first order
// Bucket work items by log2(cost) with 3 mantissa bits (256 buckets), highest bucket first.  Order
// inside a bucket is arbitrary (atomics): any order renders the same image, the order only decides
// which items start first.
RT_D uint32_t lpt_bucket(uint32_t c) {
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

// The pre-pass cost as the planner uses it (RT_COST_SMOOTH = h > 0, diagnostic build): the larger of a
// pixel's own 16-spp cost and the mean over its row neighbours +-h -- a pixel whose few samples were
// cheap, among expensive neighbours, is planned (split, started) like its neighbours.
__global__ void cost_smooth_kernel(uint32_t *cost, const uint32_t *own, int n, int width, int h) {
  for (int p = blockIdx.x * blockDim.x + threadIdx.x; p < n; p += gridDim.x * blockDim.x) {
    const int row = p / width, x = p - row * width;
    const int x0 = max(0, x - h), x1 = min(width - 1, x + h);
    uint64_t sum = 0;
    for (int q = x0; q <= x1; q++) sum += own[row * width + q];
    const uint32_t avg = (uint32_t)(sum / (uint64_t)(x1 - x0 + 1));
    cost[p] = max(own[p], avg);
  }
}

// LPT scratch (u32): 256 bucket counts, 256 running offsets, then from u32 544 the 256 per-bucket
// step sums (u64).
constexpr size_t kLptHistBytes = 8192;

// Per-step clock rates of the chain kernel under load, fitted to frame times on one MI355X (DESIGN.md
// §5): the slowest lane chain's latency and the lanes' aggregate throughput per pre-pass traversal
// step, and a whole-wave chain's rate.
constexpr float kLaneLat = 1900.0f, kLaneThr = 2714.0f, kCoopStep = 250.0f;
// Launch classes by pixels per lane of the 5-wave grid (pl; headline frame: N = 1 2.47, N = 2 1.24, N = 4 0.62,
// N = 8 0.31): the one-GPU frame (pl >= chain_occ_px, 2), the N = 2 / 4 shares (kTailPx <= pl < 2) and the
// N = 8 share (pl < kTailPx).  Since r05 every class runs the 5-wave kernel (the shares ran the 3-wave
// instantiation since r03; same box, max rank ms, two rounds, each class at its best plan: 3 waves N = 2
// 145.7 / 144.2, N = 4 87.9 / 89.5, N = 8 56.5 / 56.4; 5 waves 142.6 / 142.8, 85.3 / 85.7, 55.0 / 55.0).
// Tail shaping (ChainModel.alpha) for the N = 2 / 4 shares.  Same box, max rank ms, three rounds, r05 at 3
// waves: N = 2 alpha 0: 164.4-167.1, 1.5: 150.7-153.4, 2: 162.3-165.1, 3: 167.1-169.6; N = 4
// 0: 94.0-95.3, 1.5: 93.5-94.5; N = 8 (two rounds) 0: 61.0-61.3, 1.5: 62.4-63.1 (5 waves: 60.1 / 60.0 vs
// 55.0 / 55.0); N = 1 1.5: 257.6-258.4 vs 252.0-252.8 ms per frame.  With r06's live-lane priority (the fullest
// waves issue first) the optimum moved to 2 (same box, two rounds, N = 4 / 2 max rank ms: 1.5 79.1 / 79.9 and 133.7 /
// 133.7; 2 77.7 / 77.8 and 130.4 / 129.5; 2.5 77.5 / 77.4 and 131.6 / 132.2; profiles/r06/sweep_alpha_r06.txt).
#ifndef RT_TAIL_ALPHA
#define RT_TAIL_ALPHA 2.0f
#endif
constexpr float kTailAlpha = RT_TAIL_ALPHA, kTailPx = 0.5f;
// Heavy pixels (ChainModel.heavy) in the shares: a pixel planned at >= 8 lane segments gets twice as many.
// Its waves hold only heavy lanes (image-tile order) and run up to 3x slower per traversal step than the
// planner's model (N = 8 rank 7: 0.45-0.70 ms per sample for 340-670 steps).  Same box, N = 8
// max rank ms, two rounds (3 waves): off 60.9 / 60.5, 1.5: 60.7 / 59.7, 2: 59.7 / 59.4, 2 from 4 segments:
// 64.6 / 64.1; N = 2 unchanged (147-148).
constexpr float kHeavy = 2.0f;
// Tail migration (rt_book1.h: MigRec): a drained wave hands its chains to helper waves once at most this many
// of its lanes are live (and 70 % of the grid's waves have finished).  The one-GPU frame: 32 since the lane
// waves' live-lane priority (rt_book1.h RT_LIVE_PRIO; same box, two rounds, Msamples/s: 24 3480 / 3494, 32
// 3498 / 3491, 40 3495 / 3494, 48 3471 / 3471; without the priority 48 was best: 16 3358 / 3364, 32 3389 / 3391,
// 48 3419 / 3406, 63 3414 / 3380); the rank shares: 16 (with the priority, N = 8 / 4 / 2 max rank ms: 8 51.4 /
// 80.7 / 135.6, 16 49.9 / 82.3 / 134.9, 24 51.3 / 83.9 / 135.8, 32 52.7 / 85.8 / 137.2).
constexpr int kMigLive = 32, kMigLiveShare = 16;

// one thread: running offsets, highest bucket first (longest first)
__global__ void lpt_scan_kernel(uint32_t *hist) {
  if (threadIdx.x != 0) return;
  uint32_t run = 0;
  for (int k = 255; k >= 0; k--) {
    hist[256 + k] = run;
    run += hist[k];
  }
}

// Image tiles for the scatters' visiting order: index q of a tile-ordered sweep -> the pixel (n = none).
// Tiles of tw x (256 / tw) pixels (tw a power of two <= 256), row-major; tile_w = 0: q itself.  The
// items of one cost bucket that one block (or wave) adds are adjacent in the order, so they come from
// one patch of the image and their rays share BVH nodes (same-box A/B).
struct TileSweep {
  int n, tile_w, tw, th, tpr, rows, span;
  RT_D TileSweep(int n_, int tile_w_, int tw_) : n(n_), tile_w(tile_w_), tw(tw_) {
    th = 256 / tw;
    tpr = tile_w > 0 ? (tile_w + tw - 1) / tw : 0;
    rows = tile_w > 0 ? (n + tile_w - 1) / tile_w : 0;  // (a partial last row: pixel() bounds-checks)
    span = tile_w > 0 ? tpr * ((rows + th - 1) / th) * 256 : n;
  }
  RT_D int pixel(int q) const {
    if (tile_w <= 0) return q < n ? q : n;
    const int tile = q >> 8, r = q & 255, tx = (tile % tpr) * tw + r % tw, ty = (tile / tpr) * th + r / tw;
    const int i = ty * tile_w + tx;
    return tx < tile_w && ty < rows && i < n ? i : n;
  }
};

// The general path's longest-first order: two-level like chain_scatter_kernel -- a block's pixels per cost
// bucket counted in LDS, one global atomic per bucket and block (one global atomic per pixel on the 256
// running offsets took 3.1 ms of a config-5 frame).
__global__ __launch_bounds__(256) void lpt_scatter_kernel(const uint32_t *cost, int n, uint32_t *hist, int32_t *order,
                                                          int tile_w, int tw) {
  __shared__ uint32_t cnt_l[256], base_l[256];
  const TileSweep T(n, tile_w, tw);
  for (int q0 = blockIdx.x * blockDim.x; q0 < T.span; q0 += gridDim.x * blockDim.x) {
    for (int k = threadIdx.x; k < 256; k += blockDim.x) cnt_l[k] = 0u;
    __syncthreads();
    const int i = T.pixel(q0 + (int)threadIdx.x);
    uint32_t b = 0u, loc = 0u;
    if (i < n) {
      b = (uint32_t)lpt_bucket(cost[i]);
      loc = atomicAdd(&cnt_l[b], 1u);
    }
    __syncthreads();
    for (int k = threadIdx.x; k < 256; k += blockDim.x)
      if (cnt_l[k]) base_l[k] = atomicAdd(&hist[256 + k], cnt_l[k]);
    __syncthreads();
    if (i < n) order[base_l[b] + loc] = i;
    __syncthreads();
  }
}

// Bitonic sort (descending) in LDS, one workgroup: the chain planner's whole-wave items exactly
// longest first (the buckets keep an arbitrary order among items of up to 12.5 % different cost, and
// with a few whole waves per hundred items the heaviest pixel could start only after a wave's first
// item: measured at N = 8, started at 72 ms, the frame's last item).
template <typename K, typename T>
__device__ void bitonic_desc(K *key, T *val, int m) {
  for (int k = 2; k <= m; k <<= 1)
    for (int j = k >> 1; j > 0; j >>= 1) {
      for (int i = threadIdx.x; i < m; i += blockDim.x) {
        const int l = i ^ j;
        if (l > i) {
          const bool desc = (i & k) == 0;
          const K a = key[i], b = key[l];
          if (desc ? a < b : a > b) {
            key[i] = b, key[l] = a;
            const T t = val[i];
            val[i] = val[l], val[l] = t;
          }
        }
      }
      __syncthreads();
    }
}
// ------------------------------------------------------------------------------ chain planner
// Device-side plan of a chain launch (rt_book1.h: ChainPx), after the cost pre-pass and lpt_hist:
//   chain_params_kernel   the lane chain target c* (pre-pass steps) from the launch's total work;
//   chain_plan_kernel     per pixel: K = ceil(cost / c*) lane segments, or -- past kmax_lane --
//                         whole-wave segments against c*_w = c* * lat / coop; allocates records and
//                         end words, lists the split pixels, histograms the chains by cost;
//   chain_scan_kernel     offsets (whole-wave items first, then lane items longest first) and the
//                         whole-wave kernel's wave count;
//   chain_scatter_kernel  the items, a pixel's K chains adjacent (they start together);
//   chain_wave_sort_kernel, chain_dirty_kernel.
// Counters (u32, ch_cnt): see kCn* below; [256, 512) lane bucket counts, [512, 768) their offsets.
enum : int {
  kCnItems = 0, kCnSplit = 1, kCnFilled = 2, kCnRec = 14 /* u64 */, kCnSeg = 3, kCnCont = 4, kCnWave = 5, kCnWaveNext = 6,
  kCnCoopWaves = 7, kCnCoopCounter = 8, kCnNCoop = 9, kCnWaveWork = 10 /* u64 */, kCnCstar = 12, kCnCstarW = 13,
  kCnHist = 256, kCnOff = 512, kCnCstarB = 768 /* per cost bucket: the lane chain target c*_b (f32) */, kCnWords = 1024
};

struct ChainModel {
  float ratio;          // frame spp / pre-pass spp
  int grid_waves;       // waves of the lane kernel's grid
  float lat, thr, coop; // clocks per pre-pass step: lane chain latency, per-lane throughput, whole wave
  float beta;           // a lane chain's latency target, as a fraction of the launch's throughput time
  float margin;         // records per segment: margin * spp / K + slack
  int slack;
  int kmax_lane, kmax_wave;
  int kmin;             // every lane pixel gets at least this many segments (launches with few pixels)
  int spp;
  int min_seg;          // samples per segment at least
  int width, smooth;    // launch row width; draw estimates averaged over +-smooth pixels of the row
  float est_scale;      // stream length estimate x this
  float alpha, floor;   // tail shaping (alpha > 0): bucket b's chain target min(beta, max(floor, alpha (1 - F_b))) T,
                        // F_b = the share of the launch's work in costlier buckets (they start before it)
  float pad;            // pixels of >= pad_k segments: segments of the planned length over pad x the estimate
  int pad_k;
  float cover;          // pixels of >= cover_k segments: segments up to max(own, estimate) x cover (0: off)
  int cover_k;
  float heavy;          // lane pixels of >= heavy_k segments: heavy x as many (shorter) segments (1: off)
  int heavy_k;
  int bucket_shift;     // cost buckets merged 2^this at a time (coarser buckets: longer runs of one image tile)
  uint32_t rec_cap;     // records available
  uint32_t seg_cap;     // end words available
};

__global__ void chain_params_kernel(const unsigned long long *sums, uint32_t *cnt, ChainModel m) {
  if (threadIdx.x != 0) return;
  double total = 0.0;
  for (int k = 0; k < 256; k++) total += (double)sums[k];
  const double lanes = (double)m.grid_waves * 64.0;
  const float cstar = (float)fmax(1.0, m.beta * total * m.thr / (lanes * m.lat));
  cnt[kCnCstar] = __float_as_uint(cstar);
  cnt[kCnCstarW] = __float_as_uint(cstar * m.lat / m.coop);
  // tail shaping: items start longest first, so a pixel of bucket b starts after about F_b of the
  // launch's work and has (1 - F_b) T left -- its lane chains get that much (alpha x), down to floor T
  double above = 0.0;
  for (int b = 255; b >= 0; b--) {
    float c = cstar;
    if (m.alpha > 0.0f && total > 0.0) {
      const float f = (float)(above / total);
      const float t = fminf(m.beta, fmaxf(m.floor, m.alpha * (1.0f - f)));
      c = (float)fmax(1.0, (double)cstar * t / m.beta);
    }
    cnt[kCnCstarB + b] = __float_as_uint(c);
    above += (double)sums[b];
  }
}

__global__ __launch_bounds__(256) void chain_plan_kernel(const uint32_t *cost, const uint32_t *draws, int n,
                                                         uint32_t *cnt, ChainModel m, b1::ChainPx *px,
                                                         uint64_t *seg, uint32_t *kk, uint32_t *split) {
  __shared__ uint32_t h[256];
  __shared__ unsigned long long wwork;
  for (int k = threadIdx.x; k < 256; k += blockDim.x) h[k] = 0;
  if (threadIdx.x == 0) wwork = 0;
  __syncthreads();
  for (int p = blockIdx.x * blockDim.x + threadIdx.x; p < n; p += gridDim.x * blockDim.x) {
    const uint32_t c = cost[p];
    const float cstar = __uint_as_float(cnt[kCnCstarB + lpt_bucket(c)]), cstar_w = __uint_as_float(cnt[kCnCstarW]);
    int K = (int)fminf(ceilf((float)c / cstar), 1e6f);
    bool wave = false;
    if (K > m.kmax_lane && m.kmax_wave > 0) {  // too long for lane chains: whole-wave chains
      wave = true;
      K = min((int)fminf(ceilf((float)c / cstar_w), 1e6f), m.kmax_wave);
    }
    if (!wave && K < m.kmin) K = m.kmin;  // fill: at least kmin segments when pixels are fewer than lanes
    // heavy pixels run slower per traversal step than the model says (their waves hold only heavy
    // lanes: DESIGN.md §5.2), so their lane segments are made shorter still
    if (!wave && m.heavy > 1.0f && K >= m.heavy_k) K = min(m.kmax_lane, (int)ceilf((float)K * m.heavy));
    K = min(K, max(m.kmax_lane, m.kmax_wave));  // (the item and end-word arrays are sized for this)
    K = max(1, min(K, m.spp / m.min_seg));
    // the stream's length at full spp: the pre-pass draws per sample, averaged over the pixel's row
    // neighbours (+-smooth): draw counts are heavy-tailed (glass, metal), and 8 samples of one pixel
    // misjudge a long stream by 2x and more; the neighbours see the same surfaces
    double dsum = 0.0;
    int dn = 0;
    {
      const int row = p / m.width, x = p - row * m.width;
      const int x0 = max(0, x - m.smooth), x1 = min(m.width - 1, x + m.smooth);
      for (int q = x0; q <= x1; q++) dsum += (double)draws[row * m.width + q], dn++;
    }
    const double est = dsum / dn * m.ratio * m.est_scale;
    if (K > 1 && est * 2.0 >= 4294967295.0) K = 1;   // u32 offsets
    uint32_t seg_len = K > 1 ? (uint32_t)ceil(est / K) : 0u;
    // padded plan: the estimate's error lands on the last segment, K times its share of the stream
    // (DESIGN.md §5), so a pixel of many segments gets more segments of the same length, reaching past
    // the estimate: the true end falls inside one of them, and those past it stop when the pixel is done
    // (a whole-wave pixel's segments stay within kmax_wave; the padded stream keeps the u32 guard)
    if (m.pad > 1.0f && K >= m.pad_k && est * m.pad * 2.0 < 4294967295.0) {
      const int kcap = wave ? m.kmax_wave : max(m.kmax_lane, m.kmax_wave);
      const int kp = max(K, min(min((int)ceilf((float)K * m.pad), kcap), max(K, m.spp / m.min_seg)));
      seg_len = (uint32_t)ceil(est * m.pad / kp);
      K = kp;
    }
    seg_len = (seg_len + 1u) & ~1u;  // even: most draw counts are even
    if (seg_len < 2u) K = 1;
    // covered plan: a pixel whose own pre-pass stream is longer than its neighbours' average (the
    // estimate) gets more segments of the same length, up to max(own, estimate) x cover, so that its
    // true end falls inside one of them instead of the last segment running the difference alone
    if (m.cover > 0.0f && K >= m.cover_k && K > 1) {
      const double own = (double)draws[p] * m.ratio * m.est_scale;
      const double reach = fmax(own, est) * m.cover;
      const int kcap = max(K, min(wave ? m.kmax_wave : max(m.kmax_lane, m.kmax_wave), m.spp / m.min_seg));
      const int kc = (int)fmin(ceil(reach / seg_len), (double)kcap);
      if (kc > K && (double)kc * seg_len * 2.0 < 4294967295.0) K = kc;
    }
    if (K > 1) {
      // a segment holds at most the pixel's spp true samples (+ its garbage samples before it couples):
      // with spp + slack records no list fills up whatever the estimate's error (margin < 1 in tests
      // only: short lists force continuations); the last segment takes what remains of the stream
      const uint32_t cap = (uint32_t)ceilf(fminf(m.margin, (float)K) * (float)m.spp / (float)K) + (uint32_t)m.slack;
      const uint32_t cap_last = max(cap, (uint32_t)m.spp + (uint32_t)m.slack);
      const uint32_t need = (uint32_t)(K - 2) * cap + cap_last;
      const unsigned long long r0 = atomicAdd((unsigned long long *)&cnt[kCnRec], (unsigned long long)need);
      const bool fits = r0 + need <= (unsigned long long)m.rec_cap;
      const uint32_t n_end = (uint32_t)K;  // end words
      const uint32_t e0 = fits ? atomicAdd(&cnt[kCnSeg], n_end) : 0xffffffffu;
      if (!fits || (uint64_t)e0 + n_end > (uint64_t)m.seg_cap) {
        K = 1;  // out of record / end-word space: this pixel stays whole (the reservation is left unused)
      } else {
        b1::ChainPx P;
        P.K = (uint32_t)K;
        P.seg_len = seg_len;
        P.rec0 = (uint32_t)r0;
        P.cap = cap;
        P.end0 = e0;
        P.check = (uint32_t)(3 * (m.spp / K) / 4);
        P.cap_last = cap_last;
        P.pad = 0u;
        px[p] = P;
        for (uint32_t k = 0; k < n_end; k++) seg[e0 + k] = 0ull;
        split[atomicAdd(&cnt[kCnSplit], 1u)] = (uint32_t)p;
      }
    }
    if (K == 1) wave = wave && c > 0u;
    kk[p] = (uint32_t)K | (wave ? 0x80000000u : 0u);
    const uint32_t cc = c / (uint32_t)K;
    if (wave) {
      atomicAdd(&cnt[kCnWave], (uint32_t)K);
      atomicAdd(&wwork, (unsigned long long)c);
    } else {
      atomicAdd(&h[lpt_bucket(cc) >> m.bucket_shift << m.bucket_shift], (uint32_t)K);
    }
  }
  __syncthreads();
  for (int k = threadIdx.x; k < 256; k += blockDim.x)
    if (h[k]) atomicAdd(&cnt[kCnHist + k], h[k]);
  if (threadIdx.x == 0 && wwork) atomicAdd((unsigned long long *)&cnt[kCnWaveWork], wwork);
}

__global__ void chain_scan_kernel(uint32_t *cnt, const unsigned long long *sums, ChainModel m) {
  if (threadIdx.x != 0) return;
  const uint32_t n_wave = cnt[kCnWave];
  uint32_t run = n_wave;
  for (int b = 255; b >= 0; b--) {
    cnt[kCnOff + b] = run;
    run += cnt[kCnHist + b];
  }
  cnt[kCnItems] = run;
  cnt[kCnNCoop] = n_wave;
  cnt[kCnWaveNext] = 0;
  cnt[kCnCoopCounter] = 0;
  // every whole-wave item gets a wave of the chain kernel from the start (up to half the grid): they
  // are the launch's longest chains, and a wave that runs out of them goes on to lane items
  const uint32_t half = (uint32_t)m.grid_waves / 2u;
  cnt[kCnCoopWaves] = n_wave < half ? n_wave : half;
}

__global__ __launch_bounds__(256) void chain_scatter_kernel(const uint32_t *cost, int n, uint32_t *cnt, const uint32_t *kk,
                                                            uint2 *items, uint64_t *wave_key, int tile_w, int tw, int bshift) {
  // two-level: the block's items per bucket are counted in LDS, one global atomic per bucket and
  // block reserves their range (one global atomic per pixel on 256 bucket words serialised: 3 ms
  // for a full frame).  tile_w > 0 (the launch's row width): a block takes an image tile
  // (TileSweep) instead of 256 pixels of a row
  __shared__ uint32_t cnt_l[257], base_l[257];
  const int stride = gridDim.x * blockDim.x;
  const TileSweep T(n, tile_w, tw);
  for (int p0 = blockIdx.x * blockDim.x; p0 < T.span; p0 += stride) {
    for (int k = threadIdx.x; k < 257; k += blockDim.x) cnt_l[k] = 0u;
    __syncthreads();
    const int p = T.pixel(p0 + (int)threadIdx.x);
    uint32_t K = 0u, b = 256u, loc = 0u, cc = 0u;
    if (p < n) {
      K = kk[p] & 0xffffu;
      const bool wave = (kk[p] >> 31) != 0u;
      cc = cost[p] / K;
      b = wave ? 256u : lpt_bucket(cc) >> bshift << bshift;  // 256: the whole-wave list
      loc = atomicAdd(&cnt_l[b], K);
    }
    __syncthreads();
    for (int k = threadIdx.x; k < 257; k += blockDim.x)
      if (cnt_l[k]) base_l[k] = atomicAdd(k == 256 ? &cnt[kCnWaveNext] : &cnt[kCnOff + k], cnt_l[k]);
    __syncthreads();
    if (p < n) {
      const uint32_t at = base_l[b] + loc;
      for (uint32_t k = 0; k < K; k++) {
        items[at + k] = make_uint2((uint32_t)p, K == 1u ? b1::kItemUnsplit : k);
        if (b == 256u) wave_key[at + k] = ((uint64_t)cc << 32) | (uint32_t)(0xffffffffu - (at + k));
      }
    }
    __syncthreads();
  }
}

// the whole-wave items exactly longest first (a pixel's chains stay adjacent, in segment order)
constexpr int kWaveSort = 4096;  // 64 KB of LDS
__global__ __launch_bounds__(1024) void chain_wave_sort_kernel(const uint32_t *cnt, uint2 *items, const uint64_t *wave_key) {
  __shared__ uint64_t key[kWaveSort], val[kWaveSort];
  const int n = (int)min(cnt[kCnWave], (uint32_t)kWaveSort);
  if (n < 2) return;
  int m = 2;
  while (m < n) m <<= 1;
  for (int i = threadIdx.x; i < m; i += blockDim.x) {
    key[i] = i < n ? wave_key[i] : 0u;
    val[i] = i < n ? ((uint64_t)items[i].x << 32) | items[i].y : 0u;
  }
  __syncthreads();
  bitonic_desc(key, val, m);
  for (int i = threadIdx.x; i < n; i += blockDim.x) items[i] = make_uint2((uint32_t)(val[i] >> 32), (uint32_t)val[i]);
}

// The records this launch reserved (and may write), for the next launch's cost pre-pass to set back to
// kRecFill (rt_book1.h: clean_records).  The arena's records [0, hw) are clean when a launch starts; a
// fresh arena has hw = 0 and is not filled when it is allocated (a 24-GiB memset per new arena cost the
// drop-in path milliseconds per call: DESIGN.md §5.3): the records this launch reserves past hw are filled
// by chain_fill_kernel right after the plan, [lo, hi) = [hw, max(hw, n)), and hw moves up to hi.
// dirty[0]: the reservation (what the next pre-pass cleans), dirty[1]: hw, dirty[2..3]: this launch's fill.
enum : int { kDirtyN = 0, kDirtyHw = 1, kDirtyLo = 2, kDirtyHi = 3, kDirtyWords = 4 };
__global__ void chain_dirty_kernel(uint32_t *cnt, uint32_t *dirty, uint32_t cap) {
  if (blockIdx.x != 0 || threadIdx.x != 0) return;
  const unsigned long long c = *(const unsigned long long *)&cnt[kCnRec];
  const uint32_t n = c < cap ? (uint32_t)c : cap;  // (the count includes reservations past the capacity)
  cnt[kCnFilled] = n;
  const uint32_t hw = dirty[kDirtyHw], hi = n > hw ? n : hw;
  dirty[kDirtyN] = n;
  dirty[kDirtyLo] = hw;
  dirty[kDirtyHi] = hi;
  dirty[kDirtyHw] = hi;
}
// (records [lo, hi) to kRecFill; nothing to do -- every launch on a warm arena -- exits at once)
__global__ __launch_bounds__(256) void chain_fill_kernel(float4 *col, const uint32_t *dirty) {
  const uint64_t lo = dirty[kDirtyLo], hi = dirty[kDirtyHi];
  const float4 fill = make_float4(0.0f, 0.0f, 0.0f, __uint_as_float(b1::kRecFill));
  for (uint64_t i = lo + (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < hi; i += (uint64_t)gridDim.x * blockDim.x)
    col[i] = fill;
}

constexpr size_t kCounterBytes = 128 + b1::kMigWords * sizeof(uint32_t);  // work counter line + migration words
constexpr size_t kCounterSlot = (kCounterBytes + 255) / 256 * 256;

// After a migrating chain launch: did every work item finish?  A lane or helper counts each item it
// completes (rt_book1.h: mig_item_done); fewer than the launch's items means work was lost, which the
// scene's status word records (rt_scene_check surfaces it; rt_render / Camera_render fail loudly).
// status[0]: error bits (1: items unfinished), status[1]: items missing (summed over launches).
enum : uint32_t { kStatusIncomplete = 1u };
__global__ void chain_check_kernel(const uint32_t *mig, const uint32_t *n_items, const uint32_t *n_coop,
                                   uint32_t *status) {
  if (threadIdx.x != 0) return;
  const uint32_t total = *n_items - (n_coop ? *n_coop : 0u);
  const uint32_t done = mig[b1::kMigDone];
  if (done != total) {
    atomicOr(&status[0], kStatusIncomplete);
    atomicAdd(&status[1], total > done ? total - done : 1u);
  }
}

// ------------------------------------------------------------------------------ configuration
[[maybe_unused]] static bool env_flag(const char *name, bool dflt) {  // (the diagnostic build's switches)
  const char *e = getenv(name);
  if (!e || !*e) return dflt;
  return !(e[0] == '0' || e[0] == 'n' || e[0] == 'N' || e[0] == 'f' || e[0] == 'F');
}
static int env_int(const char *name, int dflt) {
  const char *e = getenv(name);
  return (e && *e) ? atoi(e) : dflt;
}
[[maybe_unused]] static float env_float(const char *name, float dflt) {
  const char *e = getenv(name);
  return (e && *e) ? (float)atof(e) : dflt;
}

enum : int { kModeLane = 0, kModeChain = 2, kModeAuto = 3 };

// Every knob, read once per scene upload (INTEGRATION.md lists them): the diagnostic build (-DRT_DIAG)
// only; the product library runs the defaults below (since r06: DESIGN.md §5.4).
struct Config {
  bool book1 = true, book1_lds = true, general = true, gen_pre = true;
  bool lpt = true, bf = true, bf_cuts = true, px_time = false, debug = false;
  bool pre_resume = true;     // chain items go on from the cost pre-pass's samples (RT_PRE_RESUME=0: off)
  int lpt_spp = 16, shade_batch = 48;
  // the chain launch's cost pre-pass spp (capped at a quarter of the frame's; lpt_spp is the least a chain
  // launch needs): its samples are the frame's first ones (pre_resume), so a longer pre-pass only costs its
  // lower efficiency and buys a better plan -- headline, same box, two-three rounds: 16 spp 3252-3267
  // Msamples/s, 32 3293-3304, 48 3297-3313, 64 3322-3330, 128 3326-3330 (the 6000-step budget stops most
  // pixels near 44 samples); the general path's longest-first pre-pass stays at lpt_spp (config 5: 16 spp
  // 302-311, 32 304-307, 64 293-300).  RT_LPT_SPP sets both.
  int chain_pre_spp = 64;
  int mode = kModeAuto;
  // chain_beta: a lane chain's latency target as a fraction of the launch's throughput time; 0 = by the
  // launch's class (launch_chain, kTailPx): 0.7 for 0.5-2 pixels per lane of the 5-wave grid -- the N = 2 / 4
  // shares (N = 4 95.2-96.1 ms at 0.7 vs 98.4-102.5 at 0.9) --, else 0.9 (N = 1: fewer splits, same box
  // 244.6-245.2 vs 246.6-247.8 ms at 0.7, 1.0 mixed; N = 8 the same within noise)
  float chain_beta = 0.0f, chain_margin = 1e9f;
  // chain_alpha: tail shaping of the plan (ChainModel.alpha; < 0: by the launch's class, kTailAlpha for
  // 0.5-2 pixels per lane, off otherwise); chain_floor: its smallest lane chain target, a fraction of the
  // throughput time
  float chain_alpha = -1.0f, chain_floor = 0.1f;  // margin: records per segment / (spp / K); >= K: spp
  int chain_kmax = 32, chain_kmax_wave = 8, chain_min_seg = 16, chain_slack = 64, chain_smooth = 4;
  float chain_est = 1.0f;
  // chain_cover: pixels of >= chain_cover_k segments get segments up to max(own, estimate) x this (0: off);
  // chain_heavy: lane pixels of >= chain_heavy_k segments get this x as many (< 1: by the launch's class,
  // kHeavy for the rank shares -- < 2 pixels per lane --, off for the one-GPU frame; 1: off)
  float chain_cover = 1.1f;
  int chain_cover_k = 8;
  float chain_heavy = -1.0f;
  int chain_heavy_k = 8;
  float chain_pad = 1.2f;  // padded plan (chain_plan_kernel; 1: off) for pixels of >= chain_pad_k segments
  int chain_pad_k = 8;
  float chain_fill = 1.0f;   // kmin = ceil(lanes x fill / pixels) segments per pixel (0: off)
  size_t chain_mb = 24576;  // record arena budget (MiB; the planner keeps pixels whole beyond it)
  int gen_batch = 56, gen_steps = 16, gen_lds = 1024, gen_rare = 8, gen_flat = 3;
  bool gen_big = true;  // general path: whole preorder in one 768-thread workgroup's LDS when it fits
  bool gen_perlin = true;  // ... and the Perlin tables behind it when they fit too
  int mig_live = -1;  // tail migration (rt_book1.h: MigRec): lanes left in a wave when it hands them over
                      //   (< 0: by the launch's class, kMigLive / kMigLiveShare; 0: off)
  int mig_idle = 30;  //   ... once this percentage of the grid's waves has finished: 30 since the live-lane priority
                      //   (same box, two rounds, N = 1 step / N = 8 / 4 / 2 max rank ms: 70 231.3 / 50.1 / 81.8 /
                      //   135.0, 40 231.5 / 48.8 / 80.4 / 133.9, 30 231.3 / 48.7 / 80.3 / 134.0, 20 231.0 / 49.4 /
                      //   79.8 / 133.7, 0 231.1 / 48.8 / 79.5 / 133.5); 70 in r05-r06 before it (50 until r05: N = 1
                      //   p50 230.3-231.9 at 70 vs 231.8-232.8, N = 2 142.0 / 142.1 vs 143.4 / 143.7, 85-90 slower)
  int mig_poll_us = 500;  //   a sparse wave's reads of the helper count until the gate opens (20 until r05:
                         //   N = 8 58.7-59.2 vs 56.0-57.2 ms, same box; 100 / 1000 / 2000 between / equal)
  int chain_blocks3 = 0;  // (diagnostic) blocks per CU of the shares' chain kernel (0: as many as fit)
  int chain_walk = 4;  // a segment past its check walks its pixel's links every this many samples (power of
                       // 2; 8 / 16 measured equal)
  int mig_help = 80;  //   this percentage of the grid's waves stays resident as helpers: 80 since the live-lane
                      //   priority and the 30-% gate (same box, two rounds each, two calls, N = 1 step / N = 8 / 4 / 2
                      //   max rank ms: 40 230.5 / 48.6 / 80.0 / 134.0, 80 231.0 / 48.1 / 79.2 / 133.7, 100 230.4 /
                      //   48.2 / 79.3 / 133.6); 40 before
  int mig_sleep = 64; //   helpers' poll interval (x ~3.4 us)
  int mig_wait_us = 4000000;  // a helper idle this long leaves (taking back its unclaimed credit)
  int mig_drop = 0;   // fault injection (tests only): helpers drop this many migrated items
  int cost_budget = 6000;  // cost pre-pass: traversal steps per pixel before extrapolating (0: none)
  int cost_smooth = 4;     // planner cost = max(own, row mean +-cost_smooth) (cost_smooth_kernel; 0: own)
  int bucket_shift = 0;     // chain planner cost buckets merged 2^this at a time
  int tile_order = 32;      // > 0: chain items of one cost bucket grouped by image tiles this wide, 256 / it high (chain_scatter_kernel)
  int chain_occ = 0;          // chain kernel waves per SIMD: 3 or 5 (0: 5; r03-r05a ran the shares at 3:
                              //   same box, N = 1 / 2 / 4 / 8 with r03's plans: 3 waves 268 / 168 / 100 / 68.5 ms,
                              //   4 waves 274-277 / 172-180 / 102-104 / 69-70, 5 waves 265-267 / 172-177 / 105 /
                              //   70-73; with r05's plans 5 waves are ahead, kTailPx)
  float chain_occ_px = 2.0f;  // launches of fewer pixels per lane of the 5-wave grid are rank shares (kTailPx)
  static Config from_env() {
    Config c;
#ifdef RT_DIAG
    // The product library reads none of these: its plan follows the launch's class alone (launch_chain,
    // kTailPx).  The diagnostic build (librtc_amd_diag.so, -DRT_DIAG) reads the planner /
    // scheduling parameters measured in DESIGN.md ...
    c.lpt_spp = env_int("RT_LPT_SPP", c.lpt_spp);
    if (c.lpt_spp < 1) c.lpt_spp = 1;
    if (getenv("RT_LPT_SPP")) c.chain_pre_spp = c.lpt_spp;
    c.chain_beta = env_float("RT_CHAIN_BETA", c.chain_beta);
    c.chain_alpha = env_float("RT_CHAIN_ALPHA", c.chain_alpha);
    c.chain_floor = env_float("RT_CHAIN_FLOOR", c.chain_floor);
    c.chain_occ = env_int("RT_CHAIN_OCC", c.chain_occ);
    c.chain_heavy = env_float("RT_CHAIN_HEAVY", c.chain_heavy);
    c.chain_cover = env_float("RT_CHAIN_COVER", c.chain_cover);
    c.chain_cover_k = env_int("RT_CHAIN_COVER_K", c.chain_cover_k);
    c.chain_heavy_k = env_int("RT_CHAIN_HEAVY_K", c.chain_heavy_k);
    c.mig_live = env_int("RT_MIG_LIVE", c.mig_live);
    c.mig_live = c.mig_live < -1 ? 0 : (c.mig_live > 63 ? 63 : c.mig_live);
    c.mig_idle = env_int("RT_MIG_IDLE", c.mig_idle);
    c.mig_poll_us = env_int("RT_MIG_POLL_US", c.mig_poll_us);
    c.chain_walk = env_int("RT_CHAIN_WALK", c.chain_walk);
    if (c.chain_walk < 1 || (c.chain_walk & (c.chain_walk - 1))) c.chain_walk = 4;
    c.mig_help = env_int("RT_MIG_HELP", c.mig_help);
    c.mig_sleep = env_int("RT_MIG_SLEEP", c.mig_sleep);
    if (c.mig_sleep < 1) c.mig_sleep = 1;
    c.mig_wait_us = env_int("RT_MIG_WAIT_US", c.mig_wait_us);
    if (c.mig_wait_us < 0) c.mig_wait_us = 0;
    // ... and path selection for tests, the A/B switches of the measured alternatives, timelines, fault
    // injection
    c.mig_drop = env_int("RT_FAULT_MIG_DROP", 0);
    if (c.mig_drop < 0) c.mig_drop = 0;
    c.cost_budget = env_int("RT_COST_BUDGET", c.cost_budget);
    c.cost_smooth = env_int("RT_COST_SMOOTH", c.cost_smooth);
    c.tile_order = env_int("RT_TILE_ORDER", c.tile_order);
    c.bucket_shift = min(max(env_int("RT_BUCKET_SHIFT", c.bucket_shift), 0), 4);
    if (c.tile_order == 1) c.tile_order = 16;
    if (c.tile_order < 0 || c.tile_order > 256 || (c.tile_order & (c.tile_order - 1))) c.tile_order = 0;
    c.cost_smooth = c.cost_smooth < 0 ? 0 : (c.cost_smooth > 64 ? 64 : c.cost_smooth);
    c.book1 = env_flag("RT_BOOK1", true);
    c.book1_lds = env_flag("RT_BOOK1_LDS", true);
    c.general = env_flag("RT_GENERAL", true);
    c.gen_pre = env_flag("RT_GEN_PRE", true);
    c.lpt = env_flag("RT_LPT", true);
    c.pre_resume = env_flag("RT_PRE_RESUME", true);
    c.bf = env_flag("RT_BF", true);
    c.bf_cuts = env_flag("RT_BF_CUTS", true);
    c.px_time = env_flag("RT_PX_TIME", false);
    c.debug = env_flag("RT_DEBUG", false);
    c.shade_batch = env_int("RT_SHADE_BATCH", c.shade_batch);
    c.shade_batch = c.shade_batch < 1 ? 1 : (c.shade_batch > 64 ? 64 : c.shade_batch);  // >= 1: progress
    if (const char *m = getenv("RT_MODE")) {
      if (!strcmp(m, "lane")) c.mode = kModeLane;
      else if (!strcmp(m, "chain")) c.mode = kModeChain;
    }
    c.chain_margin = env_float("RT_CHAIN_MARGIN", c.chain_margin);
    if (c.chain_margin < 1.0f) c.chain_margin = 1.0f;
    c.chain_kmax = env_int("RT_CHAIN_KMAX", c.chain_kmax);
    c.chain_kmax_wave = env_int("RT_CHAIN_KMAX_WAVE", c.chain_kmax_wave);
    c.chain_kmax = c.chain_kmax < 1 ? 1 : (c.chain_kmax > 64 ? 64 : c.chain_kmax);
    c.chain_kmax_wave = c.chain_kmax_wave < 1 ? 1 : (c.chain_kmax_wave > 64 ? 64 : c.chain_kmax_wave);
    c.chain_min_seg = env_int("RT_CHAIN_MIN_SEG", c.chain_min_seg);
    if (c.chain_min_seg < 4) c.chain_min_seg = 4;
    c.chain_mb = (size_t)env_int("RT_CHAIN_MB", (int)c.chain_mb);
    c.chain_smooth = env_int("RT_CHAIN_SMOOTH", c.chain_smooth);
    if (c.chain_smooth < 0) c.chain_smooth = 0;
    c.chain_est = env_float("RT_CHAIN_EST", c.chain_est);
    c.chain_pad = env_float("RT_CHAIN_PAD", c.chain_pad);
    c.chain_pad = c.chain_pad < 1.0f ? 1.0f : (c.chain_pad > 2.0f ? 2.0f : c.chain_pad);  // (1, 2]: 1 = off
    c.chain_pad_k = env_int("RT_CHAIN_PAD_K", c.chain_pad_k);
    c.chain_fill = env_float("RT_CHAIN_FILL", c.chain_fill);
    c.chain_occ_px = env_float("RT_CHAIN_OCC_PX", c.chain_occ_px);
    c.chain_blocks3 = env_int("RT_CHAIN_BLOCKS3", c.chain_blocks3);
    c.chain_slack = env_int("RT_CHAIN_SLACK", c.chain_slack);  // (tests: tiny lists force continuations)
    if (c.chain_slack < 1) c.chain_slack = 1;
    c.gen_batch = env_int("RT_GEN_BATCH", c.gen_batch);
    c.gen_batch = c.gen_batch < 0 ? 0 : (c.gen_batch > 64 ? 64 : c.gen_batch);
    c.gen_lds = env_int("RT_GEN_LDS", c.gen_lds);
    c.gen_big = env_flag("RT_GEN_BIG", true);
    c.gen_perlin = env_flag("RT_GEN_PERLIN_LDS", true);
    c.gen_steps = env_int("RT_GEN_STEPS", c.gen_steps);
    if (c.gen_steps < 1) c.gen_steps = 1;
    c.gen_rare = env_int("RT_GEN_RARE", c.gen_rare);
    c.gen_flat = env_int("RT_GEN_FLAT", c.gen_flat);
    if (c.gen_flat < 1) c.gen_flat = 1;
#endif
    return c;
  }
};

// ------------------------------------------------------------------------------ device scene
struct rt_device_scene {
  int device;
  Config cfg;
  DScene view;
  void *arena;
  size_t arena_bytes;
  int features;
  int width, height;
  hipEvent_t ev_main[2] = {nullptr, nullptr};  // bracket the last frame launch (rt_scene_last_launch_ms)
  // the last kLaunchRing launches' brackets as device timestamps (stamp_kernel: wall_clock64, 100 MHz) --
  // rt_scene_launch_history; one u64 pair per launch in the scene's status allocation, no extra events
  static constexpr int kLaunchRing = 64;
  uint64_t *ts_ring = nullptr;
  uint64_t n_launches = 0;
  hipEvent_t ev_done = nullptr;                // end of the last launch: the next one waits for it
  bool launched = false;
  uint32_t *status = nullptr;  // device: completion status of the launches (chain_check_kernel)
  // Book-1 path (rt_book1.h), when the scene qualifies
  bool book1 = false;
  b1::Book1View b1view;
  void *b1_arena = nullptr;
  b1::BfCut *bf_cuts = nullptr;  // the candidate trace's subtree cuts
  size_t b1_lds_bytes = 0;
  int b1_grid = 0, chain_grid = 0;  // chain_grid: the current chain launch's (one of the two below)
  int chain_grid5 = 0, chain_grid3 = 0, chain_occ = 5;  // chain kernel grids at 5 / 3 waves per SIMD
  uint32_t *lpt_cost = nullptr;  // pre-pass steps per work item (W*H)
  int32_t *lpt_order = nullptr;  // work item order (W*H)
  uint32_t *lpt_hist = nullptr;  // buckets, offsets, whole-wave counters, sums
  uint32_t *draw_out = nullptr;  // pre-pass draws per work item (W*H)
  float4 *pre_state = nullptr;   // pre-pass colour sum and position per work item (W*H; rt_book1.h pre_resume)
  uint32_t *cost_own = nullptr;  // RT_COST_SMOOTH: the pre-pass's own costs (W*H), lpt_cost the smoothed ones
  DeepRec *deep_rec = nullptr;   // max_depth > kMaxDepth: path records (rt_render_deep_kernel)
  int64_t deep_threads = 0;
  b1::MigRec *mig_q = nullptr;   // tail migration queue (rt_book1.h: MigRec)
  uint32_t mig_epoch = 0;        //   its entries are tagged with a per-launch epoch
  uint32_t *px_time = nullptr;   // RT_PX_TIME diagnostic: {start, end, migrated} per work item
  uint32_t *seg_time = nullptr;  //   and per chain segment
  // chain render scratch (rt_book1.h: ChainPx), sized for the whole frame at upload; records on demand
  void *ch_arena = nullptr;
  uint32_t *ch_cnt = nullptr, *ch_k = nullptr, *ch_split = nullptr;
  uint32_t *ch_dirty = nullptr;  // records the last chain launch reserved (the next pre-pass cleans them)
  b1::ChainPx *ch_px = nullptr;
  uint2 *ch_items = nullptr;
  uint64_t *ch_seg = nullptr, *ch_wave_key = nullptr;
  float4 *ch_acc0 = nullptr;
  b1::ChainCont *ch_cont = nullptr;
  uint32_t ch_seg_cap = 0;
  void *ch_rec_arena = nullptr;
  size_t ch_rec_cap = 0;     // records
  size_t ch_rec_demand = 0;  // records the last chain launch wanted (read back after rt_render_share's launches)
  // (every chain launch also copies its plan's reservation to pinned host memory, for the next launch on this scene
  // to see without a host sync: rt_render_rows_async callers get the arena grown too)
  unsigned long long *rec_demand_host = nullptr;
  hipEvent_t ev_demand = nullptr;
  bool demand_pending = false;
  // general path (rt_general.h) for scenes outside the Book-1 path
  bool general = false;
  void *gen_arena = nullptr;
  int32_t *gen_counter = nullptr;
  int gen_grid = 0, gen_block = 256;
  float4 *gen_xrec = nullptr;  // explicit path records of the general kernel (rt_general.h: GeneralView.xrec / xw)
  float *gen_xw = nullptr;
  float4 *gen_pre = nullptr;   // the general cost pass's colour sums and positions per pixel (GeneralView.pre_out)
  void *pre_arena = nullptr;  // the general path's preorder entries (rt_device.h: trace_pre)
  int gen_lds = 0;
  size_t gen_lds_bytes = 0;   // dynamic LDS of the general kernel
  int32_t gen_perlin_lds = -1;  // byte offset of the Perlin tables in it, or -1
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
  if (c.max_depth > kMaxDepthDeep)
    return rt_set_error("max_depth %d exceeds the deep kernel's path record (%d)", c.max_depth, kMaxDepthDeep), -1;
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

// ------------------------------------------------------------------------------ host packing
static float bits_as_float(uint32_t u) {
  float f;
  memcpy(&f, &u, 4);
  return f;
}

// Everything a device upload needs that is computed on the host, built once per scene (rt_render
// shares one pack between its per-device threads).
struct HostPack {
  Config cfg;
  bool book1 = false;
  std::vector<float4> items9;     // Book-1: the world in traversal preorder (rt_book1.h: trav_step_v9)
  int n_bf = 0;                   // leaves for the whole-wave candidate trace (0: off)
  std::vector<b1::BfCut> bf_cuts; // and its subtree cuts (empty: every leaf each ray)
  std::vector<b1::FastMat> mats;
  std::vector<float4> pre;        // general path preorder (rt_device.h: build_preorder)
};

static bool book1_eligible(const rt_flat_scene *s, const Config &cfg) {
  if (!cfg.book1) return false;
  if (s->features & ~kFeatBook1) return false;
  if (s->n_lists != 2 || s->n_quads || s->n_translates || s->n_rotates || s->n_media) return false;  // root + lights
  if (s->lists[s->lights].count != 0) return false;
  if (s->n_spheres >= 0x7fffffff / 2 || s->camera.max_depth > kMaxDepth) return false;
  for (int k = 0; k < s->n_materials; k++) {
    const rt_material &m = s->materials[k];
    if (m.tag != RT_MAT_LAMBERTIAN && m.tag != RT_MAT_METAL && m.tag != RT_MAT_DIELECTRIC) return false;
    if (m.tag != RT_MAT_DIELECTRIC && s->textures[m.texture].kind != RT_TEX_SOLID) return false;
    if (k > 0xffff) return false;  // 16-bit material ids in the path record
  }
  for (int k = 0; k < s->n_bvh; k++) {
    const int32_t l = s->bvh[k].left, r = s->bvh[k].right;
    if (l == RT_REF_NONE || (rt_ref_kind(l) != RT_KIND_BVH && rt_ref_kind(l) != RT_KIND_SPHERE)) return false;
    if (r != RT_REF_NONE && rt_ref_kind(r) != RT_KIND_BVH && rt_ref_kind(r) != RT_KIND_SPHERE) return false;
  }
  const rt_list &root = s->lists[rt_ref_index(s->root)];
  for (int k = 0; k < root.count; k++) {
    const int32_t it = s->list_items[root.first + k];
    if (it == RT_REF_NONE || (rt_ref_kind(it) != RT_KIND_BVH && rt_ref_kind(it) != RT_KIND_SPHERE)) return false;
  }
  return true;
}

// Book-1 arrays: the preorder items and the materials.
static void book1_pack(const rt_flat_scene *s, HostPack &H) {
  const rt_list &root = s->lists[rt_ref_index(s->root)];
  std::vector<float4> &items9 = H.items9;
  std::vector<uint32_t> bf_item;  // whole-wave candidate trace: leaf item positions
  {
    std::function<void(int32_t)> emit = [&](int32_t ref) {
      if (ref == RT_REF_NONE) return;
      const int32_t i = rt_ref_index(ref);
      if (rt_ref_kind(ref) == RT_KIND_SPHERE) {
        const rt_sphere &sp = s->spheres[i];
        items9.push_back(make_float4(sp.center[0], sp.center[1], sp.center[2], sp.radius_sq));
        // (x: bf position slot, y: 1/r and z: material for the whole-wave shading, w: index)
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
    // sibling leaves (rt_book1.h: kLeafPair): a leaf followed by a leaf in preorder
    for (size_t k = 0; k + 1 < items9.size() / 2; k++) {
      uint32_t a, b;
      memcpy(&a, &items9[2 * k + 1].w, 4);
      memcpy(&b, &items9[2 * k + 3].w, 4);
      if ((a & b1::kLeaf9) && (b & b1::kLeaf9)) items9[2 * k + 1].w = bits_as_float(a | b1::kLeafPair);
    }
    // one zero item past the end: the step reads its successor before knowing it exists
    items9.push_back(make_float4(0.0f, 0.0f, 0.0f, 0.0f));
    items9.push_back(make_float4(0.0f, 0.0f, 0.0f, 0.0f));
  }
  // whole-wave trace: leaf n's item position in a spare word of item n (q1.w of a node, q1.x of a leaf)
  for (size_t n = 0; n < bf_item.size() && 2 * n + 1 < items9.size(); n++) {
    float4 &h = items9[2 * n + 1];
    uint32_t hw;
    memcpy(&hw, &h.w, 4);
    if (hw & b1::kLeaf9)
      h.x = bits_as_float(bf_item[n]);
    else
      h.w = bits_as_float(bf_item[n]);
  }
  H.n_bf = !bf_item.empty() && bf_item.size() <= (size_t)64 * b1::kBfSlots && H.cfg.bf ? (int)bf_item.size() : 0;
  // subtree cuts for the candidate trace (rt_book1.h: BfCut): from the top-level items, split the cut of most
  // leaves into its children while at most 64 cuts result and a cut holds more than 4 leaves
  if (H.n_bf > 0 && H.cfg.bf_cuts) {
    const int n = (int)(items9.size() / 2) - 1;  // (without the pad item)
    auto word = [&](int q, int c) { uint32_t w; memcpy(&w, (const char *)&items9[2 * q + 1] + 4 * c, 4); return w; };
    auto leaf = [&](int q) { return (word(q, 3) & b1::kLeaf9) != 0; };
    auto size_of = [&](int q) { return leaf(q) ? 1 : (int)word(q, 2); };
    std::vector<int> lb((size_t)n + 1, 0);  // leaves before item q (the candidate trace's numbering)
    for (int q = 0; q < n; q++) lb[q + 1] = lb[q] + (leaf(q) ? 1 : 0);
    std::vector<int> cuts;
    for (int q = 0; q < n; q += size_of(q)) cuts.push_back(q);
    auto leaves = [&](int q) { return lb[q + size_of(q)] - lb[q]; };
    bool ok = !cuts.empty() && cuts.size() <= 64 && lb[n] == H.n_bf;
    while (ok) {
      int at = -1;
      for (size_t k = 0; k < cuts.size(); k++)
        if (!leaf(cuts[k]) && (at < 0 || leaves(cuts[k]) > leaves(cuts[at]))) at = (int)k;
      if (at < 0 || leaves(cuts[at]) <= 4) break;
      const int q = cuts[at];
      std::vector<int> kids;
      for (int c = q + 1; c < q + size_of(q); c += size_of(c)) kids.push_back(c);
      if (cuts.size() - 1 + kids.size() > 64) break;
      cuts.erase(cuts.begin() + at);
      cuts.insert(cuts.end(), kids.begin(), kids.end());
    }
    std::sort(cuts.begin(), cuts.end());
    for (size_t k = 0; ok && k < cuts.size(); k++) {
      b1::BfCut c;
      memset(&c, 0, sizeof c);
      const int q = cuts[k];
      c.q = (uint16_t)q, c.l0 = (uint16_t)lb[q], c.l1 = (uint16_t)lb[q + size_of(q)];
      for (int a = 0; a < q && ok; a++)
        if (!leaf(a) && a + size_of(a) > q) {
          if (c.n_anc >= b1::kBfAnc) ok = false;
          else c.anc[c.n_anc++] = (uint16_t)a;
        }
      ok = ok && n < 65535;
      H.bf_cuts.push_back(c);
    }
    if (!ok) H.bf_cuts.clear();
  }
  H.mats.resize(s->n_materials);
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
    H.mats[k] = f;
  }
}

static int host_pack(const rt_flat_scene *s, HostPack &H) {
  if (s == NULL) return rt_set_error("NULL scene"), -1;
  if (validate(s) != 0) return -1;
  H.cfg = Config::from_env();
  H.book1 = book1_eligible(s, H.cfg);
  if (H.book1) book1_pack(s, H);
  else if (H.cfg.gen_pre) build_preorder(*s, H.pre);
  return 0;
}

// ------------------------------------------------------------------------------ upload
extern "C" int rt_device_count(void) {
  int n = 0;
  if (hipGetDeviceCount(&n) != hipSuccess) return 0;
  return n;
}

extern "C" void rt_scene_release(rt_device_scene *d);

// Book-1 device state: the pack's arrays, the persistent grids, the LPT and chain scratch.

static int book1_upload(rt_device_scene *d, const rt_flat_scene *s, const HostPack &H) {
  const Config &cfg = d->cfg;
  const size_t items_bytes = H.items9.size() * sizeof(float4);
  const bool lds = cfg.book1_lds && items_bytes <= 64 * 1024;  // gfx950: 160 KiB per CU, 64 KiB per workgroup
  d->b1_lds_bytes = align_up(lds ? items_bytes : 0, 16);
  hipDeviceProp_t prop;
  HIP_OK(hipGetDeviceProperties(&prop, d->device));
  int per_cu = 0, per_cu_chain = 0, per_cu_chain3 = 0;
  HIP_OK(hipOccupancyMaxActiveBlocksPerMultiprocessor(
      &per_cu, lds ? (const void *)rt_book1_kernel<true> : (const void *)rt_book1_kernel<false>, b1::kBlock,
      d->b1_lds_bytes));
  HIP_OK(hipOccupancyMaxActiveBlocksPerMultiprocessor(
      &per_cu_chain, lds ? (const void *)rt_book1_chain_kernel<true> : (const void *)rt_book1_chain_kernel<false>,
      b1::kBlock, d->b1_lds_bytes));
  HIP_OK(hipOccupancyMaxActiveBlocksPerMultiprocessor(
      &per_cu_chain3, lds ? (const void *)rt_book1_chain_kernel<true, 3> : (const void *)rt_book1_chain_kernel<false, 3>,
      b1::kBlock, d->b1_lds_bytes));
  d->b1_grid = prop.multiProcessorCount * (per_cu < 1 ? 1 : per_cu);
  d->chain_grid5 = prop.multiProcessorCount * (per_cu_chain < 1 ? 1 : per_cu_chain);
  d->chain_grid3 = prop.multiProcessorCount * (per_cu_chain3 < 1 ? 1 : per_cu_chain3);
#ifdef RT_DIAG
  if (cfg.chain_blocks3 > 0 && cfg.chain_blocks3 < per_cu_chain3)  // (A/B: fewer waves per SIMD for the shares)
    d->chain_grid3 = prop.multiProcessorCount * cfg.chain_blocks3;
#endif
  d->chain_grid = d->chain_grid5;
  const int chain_max = d->chain_grid5 > d->chain_grid3 ? d->chain_grid5 : d->chain_grid3;
  const int spill_grid = d->b1_grid > chain_max ? d->b1_grid : chain_max;
  const int spill_lanes = spill_grid * b1::kBlock;
  // path record chunks beyond the two in registers (Record): ceil(max_depth / 4) - 2 per lane
  const int chunks = (s->camera.max_depth + 3) / 4 - 2;
  const size_t spill_bytes = (size_t)(chunks > 0 ? chunks : 0) * spill_lanes * sizeof(uint64_t);
  const size_t npix = (size_t)s->camera.width * s->camera.height;
  const size_t sizes[8] = {items_bytes, H.mats.size() * sizeof(b1::FastMat), kCounterSlot, spill_bytes,
                           npix * sizeof(uint32_t),   // [4] pre-pass cost
                           npix * sizeof(int32_t),    // [5] LPT order
                           kLptHistBytes,             // [6] LPT buckets
                           npix * sizeof(uint32_t)};  // [7] pre-pass draws
  size_t off[8], total = 0;
  for (int k = 0; k < 8; k++) {
    off[k] = total;
    total = align_up(total + (sizes[k] ? sizes[k] : 16), 256);
  }
  void *arena = nullptr;
  HIP_OK(hipMalloc(&arena, total));
  d->b1_arena = arena;
  char *b = (char *)arena;
  {  // on the device as two arrays: every item's q0, then every item's q1 (rt_book1.h: it_q0 / it_q1)
    const size_t na = H.items9.size() / 2;
    std::vector<float4> soa(2 * na);
    for (size_t k = 0; k < na; k++) soa[k] = H.items9[2 * k], soa[na + k] = H.items9[2 * k + 1];
    HIP_OK(hipMemcpy(b + off[0], soa.data(), sizes[0], hipMemcpyHostToDevice));
  }
  if (sizes[1]) HIP_OK(hipMemcpy(b + off[1], H.mats.data(), sizes[1], hipMemcpyHostToDevice));
  b1::Book1View &V = d->b1view;
  memset(&V, 0, sizeof V);
  V.S = d->view;
  V.items9_g = (const float4 *)(b + off[0]);
  V.n_items9 = (int32_t)(H.items9.size() / 2) - 1;  // without the trailing pad item
  V.n_items9_alloc = (int32_t)(H.items9.size() / 2);
  V.mats = (const b1::FastMat *)(b + off[1]);
  V.work_counter = (int32_t *)(b + off[2]);  // (the counter; the migration words from the next line on)
  V.mig = (uint32_t *)(b + off[2] + 128);
  V.mig_live = cfg.mig_live < 0 ? kMigLiveShare : cfg.mig_live;  // (launch_chain sets it by the launch's class)
  if (cfg.mig_live != 0) {  // one queue entry per lane of the grid: an item migrates at most once per launch...
    V.mig_cap = (uint32_t)spill_lanes;  // ...and only against an idle helper wave (push beyond: the lane keeps it)
    HIP_OK(hipMalloc(&d->mig_q, (size_t)V.mig_cap * sizeof(b1::MigRec)));
    HIP_OK(hipMemset(d->mig_q, 0, (size_t)V.mig_cap * sizeof(b1::MigRec)));  // epoch 0: no entry
    V.mig_q = d->mig_q;
  }
  V.spill = (uint64_t *)(b + off[3]);
  V.spill_lanes = spill_lanes;
  V.shade_batch = cfg.shade_batch;
  V.n_bf_leaves = H.n_bf;
  if (!H.bf_cuts.empty()) {
    HIP_OK(hipMalloc(&d->bf_cuts, H.bf_cuts.size() * sizeof(b1::BfCut)));
    HIP_OK(hipMemcpy(d->bf_cuts, H.bf_cuts.data(), H.bf_cuts.size() * sizeof(b1::BfCut), hipMemcpyHostToDevice));
    V.bf_cuts = d->bf_cuts;
    V.n_bf_cuts = (int32_t)H.bf_cuts.size();
  }
  d->lpt_cost = (uint32_t *)(b + off[4]);
  d->lpt_order = (int32_t *)(b + off[5]);
  d->lpt_hist = (uint32_t *)(b + off[6]);
  d->draw_out = (uint32_t *)(b + off[7]);
  if (cfg.cost_smooth > 0) HIP_OK(hipMalloc(&d->cost_own, npix * sizeof(uint32_t)));
  if (cfg.pre_resume) HIP_OK(hipMalloc(&d->pre_state, npix * sizeof(float4)));
  V.pre_state = nullptr;  // (set per launch: the cost pass writes it, the chain launch after it reads it)
  if (cfg.px_time) {
    HIP_OK(hipMalloc(&d->px_time, npix * b1::kTimeWords * sizeof(uint32_t)));
    V.px_time = d->px_time;
  }
#ifdef RT_LOOP_STATS
  HIP_OK(hipMalloc(&V.loop_stats, 32 * sizeof(unsigned long long)));
  HIP_OK(hipMemset(V.loop_stats, 0, 32 * sizeof(unsigned long long)));
#endif
  // chain scratch for the whole frame (a launch covers at most every pixel)
  {
    const int kmax = cfg.chain_kmax > cfg.chain_kmax_wave ? cfg.chain_kmax : cfg.chain_kmax_wave;
    const size_t nitem = npix * (size_t)kmax, nseg = npix * (size_t)kmax;
    d->ch_seg_cap = nseg < 0xffffffffu ? (uint32_t)nseg : 0xffffffffu;
    const size_t cs[9] = {(kCnWords + 64) * sizeof(uint32_t), npix * sizeof(uint32_t), npix * sizeof(uint32_t),
                          npix * sizeof(b1::ChainPx), nitem * sizeof(uint2), nseg * sizeof(uint64_t),
                          nitem * sizeof(uint64_t), npix * sizeof(float4), npix * sizeof(b1::ChainCont)};
    size_t co[9], ct = 0;
    for (int k = 0; k < 9; k++) co[k] = ct, ct = align_up(ct + cs[k], 256);
    HIP_OK(hipMalloc(&d->ch_arena, ct));
    char *c = (char *)d->ch_arena;
    d->ch_cnt = (uint32_t *)(c + co[0]);
    d->ch_dirty = d->ch_cnt + kCnWords;  // (past the words each plan zeroes)
    HIP_OK(hipMemset(d->ch_dirty, 0, kDirtyWords * sizeof(uint32_t)));
    HIP_OK(hipHostMalloc((void **)&d->rec_demand_host, sizeof(unsigned long long), hipHostMallocDefault));
    *d->rec_demand_host = 0ull;
    HIP_OK(hipEventCreateWithFlags(&d->ev_demand, hipEventDisableTiming));
    d->ch_k = (uint32_t *)(c + co[1]);
    d->ch_split = (uint32_t *)(c + co[2]);
    d->ch_px = (b1::ChainPx *)(c + co[3]);
    d->ch_items = (uint2 *)(c + co[4]);
    d->ch_seg = (uint64_t *)(c + co[5]);
    d->ch_wave_key = (uint64_t *)(c + co[6]);
    d->ch_acc0 = (float4 *)(c + co[7]);
    d->ch_cont = (b1::ChainCont *)(c + co[8]);
    if (cfg.px_time) {
      HIP_OK(hipMalloc(&d->seg_time, nseg * b1::kTimeWords * sizeof(uint32_t)));
      V.seg_time = d->seg_time;
    }
  }
  d->book1 = true;
  if (cfg.debug)
    fprintf(stderr, "[rtc] book1 lds=%d bytes=%zu grid=%d chain_grid=%d bf=%d spill_chunks=%d\n", (int)lds,
            d->b1_lds_bytes, d->b1_grid, d->chain_grid, H.n_bf, chunks);
  return 0;
}

// Buffers of the persistent general path: work counter, longest-first cost / order / buckets.
static int general_upload(rt_device_scene *d, const rt_flat_scene *s) {
  const Config &cfg = d->cfg;
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
  hipDeviceProp_t prop;
  HIP_OK(hipGetDeviceProperties(&prop, d->device));
  const int batch = d->view.pre ? cfg.gen_batch : 0;  // the batched loop runs the preorder scan
  int lds = batch ? cfg.gen_lds : 0;
  if (lds < 0) lds = 0;
  if (lds > d->view.n_pre) lds = d->view.n_pre;
  if (lds > 2048) lds = 2048;  // 64 KB per 256-thread workgroup (three per CU)
  const bool fb = (d->features & ~kFeatBook1) == 0;
  const size_t pre_bytes = (size_t)d->view.n_pre * 2 * sizeof(float4);
  d->gen_block = gen::kBlock;
  if (batch && cfg.gen_big && d->view.n_pre > lds && pre_bytes <= (size_t)prop.sharedMemPerBlock) {
    d->gen_block = kBigBlock;  // the whole preorder in one workgroup's LDS
    lds = d->view.n_pre;
  }
  d->gen_lds = lds;
  const bool big = d->gen_block == kBigBlock;
  size_t lds_bytes = (size_t)lds * 2 * sizeof(float4);
  // the single Perlin texture's tables in LDS behind the whole preorder, when they fit (scene 7: 158 KiB
  // of preorder + 4.75 KiB of tables in 160 KiB)
  d->gen_perlin_lds = -1;
  if (big && cfg.gen_perlin && s->n_perlins == 1 && lds_bytes + kPerlinLdsBytes <= (size_t)prop.sharedMemPerBlock) {
    d->gen_perlin_lds = (int32_t)lds_bytes;
    lds_bytes += kPerlinLdsBytes;
  }
  d->gen_lds_bytes = lds_bytes;
  const void *fn = big ? (fb ? (const void *)rt_general_kernel<kFeatBook1, true, kBigBlock>
                             : (const void *)rt_general_kernel<kFeatAll, true, kBigBlock>)
                 : batch ? (fb ? (const void *)rt_general_kernel<kFeatBook1, true> : (const void *)rt_general_kernel<kFeatAll, true>)
                         : (fb ? (const void *)rt_general_kernel<kFeatBook1> : (const void *)rt_general_kernel<kFeatAll>);
  if (lds_bytes > 65536) HIP_OK(hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds_bytes));
  int per_cu = 0;
  HIP_OK(hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, fn, d->gen_block, lds_bytes));
  if (per_cu < 1) per_cu = 1;
  d->gen_grid = prop.multiProcessorCount * per_cu;
  // explicit path records (rt_general.h: PathRuns), kMaxDepth albedos and weights per thread of the grid
  const size_t threads = (size_t)d->gen_grid * d->gen_block;
  HIP_OK(hipMalloc(&d->gen_xrec, threads * kMaxDepth * (sizeof(float4) + sizeof(float))));
  d->gen_xw = (float *)(d->gen_xrec + threads * kMaxDepth);
  if (cfg.pre_resume && cfg.lpt)
    HIP_OK(hipMalloc(&d->gen_pre, (size_t)s->camera.width * s->camera.height * sizeof(float4)));
  d->general = true;
  if (cfg.debug)
    fprintf(stderr, "[rtc] general persistent kernel: grid=%d (%d/CU) block=%d lds entries=%d of %d, perlin in lds %d, "
            "features=0x%x\n", d->gen_grid, per_cu, d->gen_block, d->gen_lds, d->view.n_pre, d->gen_perlin_lds >= 0,
            d->features);
  return 0;
}

static rt_device_scene *upload_packed(const rt_flat_scene *s, const HostPack &H, int device) {
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
  d->cfg = H.cfg;
  d->arena = arena;
  d->arena_bytes = total;
  d->features = s->features;
  d->width = s->camera.width;
  d->height = s->camera.height;
  const void *dev_arrays[13];
  for (int k = 0; k < 13; k++) dev_arrays[k] = (char *)arena + parts[k].off;
  d->view = make_view(*s, dev_arrays);
  if (!H.pre.empty()) {  // the general path's preorder (trace_pre)
    if (hipMalloc(&d->pre_arena, H.pre.size() * sizeof(float4)) != hipSuccess ||
        hipMemcpy(d->pre_arena, H.pre.data(), H.pre.size() * sizeof(float4), hipMemcpyHostToDevice) != hipSuccess) {
      rt_set_error("preorder upload failed on device %d", device);
      rt_scene_release(d);
      return NULL;
    }
    d->view.pre = (const float4 *)d->pre_arena;
    d->view.n_pre = (int32_t)(H.pre.size() / 2);
  }
  // status words (256 B), then the launch timestamp ring
  const size_t status_bytes = 256 + rt_device_scene::kLaunchRing * 2 * sizeof(uint64_t);
  if (hipEventCreate(&d->ev_main[0]) != hipSuccess || hipEventCreate(&d->ev_main[1]) != hipSuccess ||
      hipEventCreateWithFlags(&d->ev_done, hipEventDisableTiming) != hipSuccess ||
      hipMalloc(&d->status, status_bytes) != hipSuccess || hipMemset(d->status, 0, status_bytes) != hipSuccess) {
    rt_set_error("event / status word creation failed on device %d", device);
    rt_scene_release(d);
    return NULL;
  }
  if (H.book1 && book1_upload(d, s, H) != 0) {
    rt_scene_release(d);
    return NULL;
  }
  if (s->camera.max_depth > kMaxDepth) {  // deep paths: rt_render_deep_kernel and its record slots
    const size_t per = (size_t)s->camera.max_depth * sizeof(DeepRec);
    const size_t npix = (size_t)s->camera.width * s->camera.height;
    size_t threads = ((size_t)1 << 30) / per;  // 1 GiB of records
    threads = threads < npix ? threads : npix;
    threads = (threads + kBlock - 1) / kBlock * kBlock;
    if (hipMalloc(&d->deep_rec, threads * per) != hipSuccess) {
      rt_set_error("hipMalloc of the deep path records failed on device %d", device);
      rt_scene_release(d);
      return NULL;
    }
    d->deep_threads = (int64_t)threads;
    return d;
  }
  if (!d->book1 && H.cfg.general && general_upload(d, s) != 0) {
    rt_scene_release(d);
    return NULL;
  }
  return d;
}

extern "C" rt_device_scene *rt_scene_upload(const rt_flat_scene *s, int device) {
  HostPack H;
  if (host_pack(s, H) != 0) return NULL;
  return upload_packed(s, H, device);
}

extern "C" void rt_scene_release(rt_device_scene *d) {
  if (!d) return;
  (void)hipSetDevice(d->device);
  if (d->launched && d->ev_done) (void)hipEventSynchronize(d->ev_done);  // no launch of this scene in flight
  (void)hipFree(d->arena);
  if (d->b1_arena) (void)hipFree(d->b1_arena);
  if (d->bf_cuts) (void)hipFree(d->bf_cuts);
  if (d->gen_arena) (void)hipFree(d->gen_arena);
  if (d->gen_xrec) (void)hipFree(d->gen_xrec);
  if (d->gen_pre) (void)hipFree(d->gen_pre);
  if (d->px_time) (void)hipFree(d->px_time);
  if (d->cost_own) (void)hipFree(d->cost_own);
  if (d->pre_state) (void)hipFree(d->pre_state);
  if (d->seg_time) (void)hipFree(d->seg_time);
  if (d->mig_q) (void)hipFree(d->mig_q);
  if (d->deep_rec) (void)hipFree(d->deep_rec);
  if (d->pre_arena) (void)hipFree(d->pre_arena);
  if (d->ch_arena) (void)hipFree(d->ch_arena);
  if (d->ch_rec_arena) (void)hipFree(d->ch_rec_arena);
  if (d->rec_demand_host) (void)hipHostFree(d->rec_demand_host);
  if (d->ev_demand) (void)hipEventDestroy(d->ev_demand);
  if (d->status) (void)hipFree(d->status);
  if (d->ev_done) (void)hipEventDestroy(d->ev_done);
  for (hipEvent_t e : d->ev_main)
    if (e) (void)hipEventDestroy(e);
  delete d;
}

// ------------------------------------------------------------------------------ launches
// The chain launch's cost pre-pass spp (Config.chain_pre_spp, at most a quarter of the frame's spp, at
// least lpt_spp; the exact-plan diagnostic: the frame's spp).
static int chain_pre_spp(const rt_device_scene *d, int spp) {
  const Config &c = d->cfg;
  if (c.lpt_spp >= spp) return spp;
  const int p = c.chain_pre_spp < spp / 4 ? c.chain_pre_spp : spp / 4;
  return p > c.lpt_spp ? p : c.lpt_spp;
}

static void launch_cost_pass(const rt_device_scene *d, b1::Book1View P, uint8_t *d_out, hipStream_t st) {
  (void)hipMemsetAsync(P.work_counter, 0, kCounterBytes, st);  // (the previous launch left it past its items)
  P.S.cam.spp = chain_pre_spp(d, P.S.cam.spp);
  P.cost_out = d->cost_own ? d->cost_own : d->lpt_cost;
  P.draw_out = d->draw_out;
  P.pre_state = d->pre_state;
  P.cost_budget = d->cfg.cost_budget > 0 ? (uint32_t)d->cfg.cost_budget : 0xffffffffu;
  P.n_coop = nullptr;
  P.clean_col = (float4 *)d->ch_rec_arena;  // the previous chain launch's records back to kRecFill
  P.clean_n = d->ch_dirty;
  // at the chain kernel's occupancy, on its grid
  // (at the chain kernel's occupancy: the 3-wave instantiation for the shares; neither spills)
  const dim3 g((unsigned)d->chain_grid), blk(b1::kBlock);
  if (d->chain_occ == 3) {
    if (d->b1_lds_bytes) hipLaunchKernelGGL((rt_book1_cost_kernel<true, 3>), g, blk, d->b1_lds_bytes, st, P, d_out);
    else hipLaunchKernelGGL((rt_book1_cost_kernel<false, 3>), g, blk, 0, st, P, d_out);
    return;
  }
  if (d->b1_lds_bytes) hipLaunchKernelGGL((rt_book1_cost_kernel<true>), g, blk, d->b1_lds_bytes, st, P, d_out);
  else hipLaunchKernelGGL((rt_book1_cost_kernel<false>), g, blk, 0, st, P, d_out);
}

static void launch_chain_kernel(const rt_device_scene *d, const b1::Book1View &V, uint8_t *d_out, hipStream_t st) {
  const dim3 gc((unsigned)d->chain_grid), blk(b1::kBlock);
  const size_t lds = d->b1_lds_bytes;
  if (d->chain_occ == 3) {
    if (lds) hipLaunchKernelGGL((rt_book1_chain_kernel<true, 3>), gc, blk, lds, st, V, d_out);
    else hipLaunchKernelGGL((rt_book1_chain_kernel<false, 3>), gc, blk, 0, st, V, d_out);
    return;
  }
  if (lds) hipLaunchKernelGGL((rt_book1_chain_kernel<true>), gc, blk, lds, st, V, d_out);
  else hipLaunchKernelGGL((rt_book1_chain_kernel<false>), gc, blk, 0, st, V, d_out);
}

// Records of a chain launch, up to the RT_CHAIN_MB budget (the planner keeps pixels whole when they run out).
// The plan reserves spp + slack records for every segment past a pixel's first, and a launch's segments number
// at most (kmin - 1) x npix + about 1.5 x lanes (the fill to one item per lane, then c* = beta T: a lane's worth
// of cost per segment).  Measured reservations of the headline frame: 0.16 / 7.4 / 9.0 / 6.1 GB at N = 1 / 2 / 4
// / 8, against 8.4 / 8.4 / 11.8 / 13.5 GB of that bound; until r06 the arena took the whole
// 24-GiB budget, which every cached scene then held and every cold call allocated and freed.  A launch that
// wanted more than the arena held (ch_rec_demand, read back by rt_render_share after its launch) grows the
// next one's.  Small launches (worst case <= 4 GiB) get the worst case: every pixel split as far as allowed.
static int chain_records(rt_device_scene *d, size_t npix, int spp, hipStream_t st) {
  const Config &cfg = d->cfg;
  // the reservation a previous launch's plan wanted, if its copy has landed (queried, never waited on: the
  // launch stays asynchronous; a launch enqueued before it lands is planned on the old arena)
  if (d->demand_pending && hipEventQuery(d->ev_demand) == hipSuccess) {
    d->demand_pending = false;
    const size_t want = (size_t)*d->rec_demand_host;
    if (want > d->ch_rec_cap && want > d->ch_rec_demand) d->ch_rec_demand = want;
  }
  const size_t kmax = (size_t)(cfg.chain_kmax > cfg.chain_kmax_wave ? cfg.chain_kmax : cfg.chain_kmax_wave);
  const double seg_recs = fmin((double)cfg.chain_margin * spp / 2.0, (double)spp) + cfg.chain_slack;
  const size_t per_px = (size_t)ceil((double)(kmax - 1) * seg_recs) + (size_t)spp + (size_t)cfg.chain_slack;
  size_t want = npix * per_px;  // the worst case
  const size_t small = ((size_t)4 << 30) / sizeof(float4);
  if (want > small) {
    const double lanes = (double)d->chain_grid5 * b1::kBlock;
    const double kmin = cfg.chain_fill > 0.0f ? ceil(lanes * cfg.chain_fill / (double)npix) : 1.0;
    const double segs = (kmin > 1.0 ? kmin - 1.0 : 0.0) * (double)npix + 1.5 * lanes;
    size_t bound = (size_t)(segs * ((double)spp + cfg.chain_slack)) + (size_t)spp + (size_t)cfg.chain_slack;
    const size_t grow = d->ch_rec_demand + d->ch_rec_demand / 4;
    if (bound < grow) bound = grow;
    if (bound < small) bound = small;
    if (want > bound) want = bound;
  }
  const size_t budget = cfg.chain_mb * ((size_t)1 << 20) / sizeof(float4);
  if (want > budget) want = budget;
  if (want > 0xfff00000u) want = 0xfff00000u;  // u32 record indices
  if (want <= d->ch_rec_cap) return 0;
  if (d->ch_rec_arena) HIP_OK(hipFree(d->ch_rec_arena));
  d->ch_rec_arena = nullptr;
  d->ch_rec_cap = 0;
  HIP_OK(hipMalloc(&d->ch_rec_arena, want * sizeof(float4) + 256));
  d->ch_rec_cap = want;
  // a fresh arena: nothing clean yet (hw 0: chain_fill_kernel fills what each launch reserves past hw),
  // nothing for the next pre-pass to set back
  HIP_OK(hipMemsetAsync(d->ch_dirty, 0, kDirtyWords * sizeof(uint32_t), st));
  return 0;
}

// Chain launch (rt_book1.h: ChainPx): cost pre-pass, device-side plan, the chains (lanes + whole
// waves), the fold, and a continuation launch for whatever the fold could not finish.  No host sync.
// The chain kernel's waves per SIMD for a launch of npix pixels (RT_CHAIN_OCC, else by pixels per lane).
static int chain_occupancy(const rt_device_scene *d, int64_t npix) {
  (void)npix;  // (every launch class at 5 since r05: the kTailPx note)
  return d->cfg.chain_occ == 3 ? 3 : 5;
}

// A launch's bracket: the ev_main event (rt_scene_last_launch_ms) and a device timestamp in the
// scene's ring (rt_scene_launch_history): one thread writes wall_clock64 with a vector store.
__global__ void stamp_kernel(uint64_t *p) {
  if (threadIdx.x == 0) *p = (uint64_t)wall_clock64();
}
static hipError_t mark_launch(rt_device_scene *d, int which, hipStream_t st) {
  if (d->ev_main[which]) {
    const hipError_t e = hipEventRecord(d->ev_main[which], st);
    if (e != hipSuccess) return e;
  }
  if (!d->ts_ring) return hipSuccess;
  hipLaunchKernelGGL(stamp_kernel, dim3(1), dim3(64), 0, st, d->ts_ring + which);
  return hipGetLastError();
}

static int launch_chain(rt_device_scene *d, b1::Book1View V, uint8_t *d_out, hipStream_t st, int64_t npix) {
  const Config &cfg = d->cfg;
  if (chain_records(d, (size_t)npix, V.S.cam.spp, st) != 0) return -1;
  // waves per SIMD: 5 hide more latency (headline frame 266 vs 275 ms at 4), 3 run each lane chain
  // faster with no spills at all (168 VGPRs) -- what a launch with few pixels per lane needs (its time
  // is its longest chains)
  d->chain_occ = chain_occupancy(d, npix);
  d->chain_grid = d->chain_occ == 5 ? d->chain_grid5 : d->chain_grid3;
  if (d->px_time) {  // (diagnostic timelines: a fresh record per launch)
    HIP_OK(hipMemsetAsync(d->px_time, 0, (size_t)d->width * d->height * b1::kTimeWords * sizeof(uint32_t), st));
    HIP_OK(hipMemsetAsync(d->seg_time, 0, (size_t)d->ch_seg_cap * b1::kTimeWords * sizeof(uint32_t), st));
  }
  // (every chain launch runs its cost pre-pass: it sets the previous launch's reservation back to kRecFill,
  // and chain_fill_kernel below fills only what lies past the clean high-water mark -- a chain launch
  // without this pre-pass would read the previous launch's records)
  launch_cost_pass(d, V, d_out, st);
  HIP_OK(hipGetLastError());
  HIP_OK(hipMemsetAsync(d->lpt_hist, 0, kLptHistBytes, st));
  HIP_OK(hipMemsetAsync(d->ch_cnt, 0, kCnWords * sizeof(uint32_t), st));
  unsigned long long *sums = (unsigned long long *)(d->lpt_hist + 512 + 32);
  const int n = (int)npix, nb = (int)((npix + 255) / 256 < 1024 ? (npix + 255) / 256 : 1024);
  if (d->cost_own)
    hipLaunchKernelGGL(cost_smooth_kernel, dim3(nb), dim3(256), 0, st, d->lpt_cost, (const uint32_t *)d->cost_own, n,
                       V.S.cam.width, cfg.cost_smooth);
  hipLaunchKernelGGL(lpt_hist_kernel, dim3(nb), dim3(256), 0, st, d->lpt_cost, n, d->lpt_hist, sums);
  ChainModel m;
  m.ratio = (float)V.S.cam.spp / (float)chain_pre_spp(d, V.S.cam.spp);
  m.grid_waves = d->chain_grid * (b1::kBlock / 64);
  m.lat = kLaneLat;
  m.thr = kLaneThr;
  m.coop = kCoopStep;
  // the launch's class (kTailPx above): pixels per lane of the 5-wave grid
  const double px_lane = (double)npix / ((double)d->chain_grid5 * b1::kBlock);
  const bool share = px_lane < (double)cfg.chain_occ_px, mid_share = share && px_lane >= (double)kTailPx;
  m.beta = cfg.chain_beta > 0.0f ? cfg.chain_beta : (mid_share ? 0.7f : 0.9f);
  m.alpha = cfg.chain_alpha >= 0.0f ? cfg.chain_alpha : (mid_share ? kTailAlpha : 0.0f);
  m.floor = cfg.chain_floor;
  m.margin = cfg.chain_margin;
  m.slack = cfg.chain_slack;
  m.width = V.S.cam.width;
  m.smooth = cfg.chain_smooth;
  m.est_scale = cfg.chain_est;
  m.pad = cfg.chain_pad;
  m.cover = cfg.chain_cover;
  m.cover_k = cfg.chain_cover_k < 2 ? 2 : cfg.chain_cover_k;
  m.heavy = cfg.chain_heavy >= 1.0f ? cfg.chain_heavy : (share ? kHeavy : 1.0f);
  if (cfg.mig_live < 0) V.mig_live = share ? kMigLiveShare : kMigLive;
  m.heavy_k = cfg.chain_heavy_k < 2 ? 2 : cfg.chain_heavy_k;
  m.pad_k = cfg.chain_pad_k < 2 ? 2 : cfg.chain_pad_k;
  m.kmax_lane = cfg.chain_kmax;
  {  // enough items to give every lane of the grid one: light pixels' 1000-sample chains were the
     // launch's longest items at N = 8 (per-sample overhead, not traversal steps, sets their latency)
    const double lanes = (double)d->chain_grid * b1::kBlock;
    m.kmin = cfg.chain_fill > 0.0f ? (int)ceil(lanes * cfg.chain_fill / (double)npix) : 1;
    if (m.kmin < 1) m.kmin = 1;
  }
  m.kmax_wave = d->b1_lds_bytes ? cfg.chain_kmax_wave : 0;  // no whole waves without the LDS scene
  m.spp = V.S.cam.spp;
  m.min_seg = cfg.chain_min_seg;
  m.bucket_shift = cfg.bucket_shift;
  m.rec_cap = (uint32_t)d->ch_rec_cap;
  m.seg_cap = d->ch_seg_cap;
  float4 *col = (float4 *)d->ch_rec_arena;
  hipLaunchKernelGGL(chain_params_kernel, dim3(1), dim3(64), 0, st, sums, d->ch_cnt, m);
  hipLaunchKernelGGL(chain_plan_kernel, dim3(nb), dim3(256), 0, st, d->lpt_cost, d->draw_out, n, d->ch_cnt, m, d->ch_px,
                     d->ch_seg, d->ch_k, d->ch_split);
  hipLaunchKernelGGL(chain_scan_kernel, dim3(1), dim3(64), 0, st, d->ch_cnt, sums, m);
  hipLaunchKernelGGL(chain_scatter_kernel, dim3(nb), dim3(256), 0, st, d->lpt_cost, n, d->ch_cnt, d->ch_k, d->ch_items,
                     d->ch_wave_key, cfg.tile_order ? V.S.cam.width : 0, cfg.tile_order ? cfg.tile_order : 16,
                     m.bucket_shift);
  hipLaunchKernelGGL(chain_wave_sort_kernel, dim3(1), dim3(1024), 0, st, d->ch_cnt, d->ch_items, d->ch_wave_key);
  hipLaunchKernelGGL(chain_dirty_kernel, dim3(1), dim3(64), 0, st, d->ch_cnt, d->ch_dirty, (uint32_t)d->ch_rec_cap);
  hipLaunchKernelGGL(chain_fill_kernel, dim3(2048), dim3(256), 0, st, col, (const uint32_t *)d->ch_dirty);
  HIP_OK(hipGetLastError());
  if (d->rec_demand_host && !d->demand_pending) {  // (the plan's reservation, for the next launch's arena: above)
    HIP_OK(hipMemcpyAsync(d->rec_demand_host, d->ch_cnt + kCnRec, sizeof(unsigned long long), hipMemcpyDeviceToHost, st));
    HIP_OK(hipEventRecord(d->ev_demand, st));
    d->demand_pending = true;
  }
  if (cfg.debug) {  // diagnostic: synchronous peek at the plan
    uint32_t c[16];
    HIP_OK(hipStreamSynchronize(st));
    HIP_OK(hipMemcpy(c, d->ch_cnt, sizeof c, hipMemcpyDeviceToHost));
    fprintf(stderr, "[rtc] chain plan: %lld px, %u items, %u split px, %llu records (cap %zu), %u wave items on %u waves, "
            "c* %.1f c*_w %.1f\n", (long long)npix, c[kCnItems], c[kCnSplit], *(unsigned long long *)&c[kCnRec], d->ch_rec_cap, c[kCnWave],
            c[kCnCoopWaves], bits_as_float(c[kCnCstar]), bits_as_float(c[kCnCstarW]));
  }
  V.ch_px = d->ch_px;
  V.ch_items = d->ch_items;
  V.ch_n_items = d->ch_cnt + kCnItems;
  V.pre_state = d->pre_state;  // the chain items go on from the pre-pass's samples
  V.ch_seg = d->ch_seg;
  V.ch_col = col;
  V.ch_acc0 = d->ch_acc0;
  V.ch_cont = nullptr;
  V.ch_n_cont = nullptr;
  V.n_coop = d->ch_cnt + kCnNCoop;
  V.coop_counter = (int32_t *)(d->ch_cnt + kCnCoopCounter);
  V.coop_waves_dev = d->ch_cnt + kCnCoopWaves;
  V.mig_epoch = ++d->mig_epoch;
  V.mig_idle = (int32_t)((int64_t)d->chain_grid * (b1::kBlock / 64) * cfg.mig_idle / 100);
  V.mig_poll = (uint32_t)(cfg.mig_poll_us > 1 ? cfg.mig_poll_us : 1) * 100u;
  V.walk_mask = (uint32_t)(cfg.chain_walk > 1 ? cfg.chain_walk : 1) - 1u;
  V.mig_sleep = cfg.mig_sleep;
  V.mig_max_help = (int32_t)((int64_t)d->chain_grid * (b1::kBlock / 64) * cfg.mig_help / 100);
  V.mig_wait = (uint64_t)cfg.mig_wait_us * 100u;  // wall_clock64: 100 MHz
  V.mig_drop = (uint32_t)cfg.mig_drop;
  HIP_OK(mark_launch(d, 0, st));
  const bool lds = d->b1_lds_bytes != 0;
  if (!lds) V.n_coop = nullptr;  // (the planner gives no whole-wave items without the LDS scene)
  HIP_OK(hipMemsetAsync(V.work_counter, 0, kCounterBytes, st));  // counter + migration words
  launch_chain_kernel(d, V, d_out, st);  // (whole-wave items in its first waves: rt_book1.h coop_items)
  HIP_OK(hipGetLastError());
  if (V.mig_live > 0)  // (before the continuation launch resets the migration words)
    hipLaunchKernelGGL(chain_check_kernel, dim3(1), dim3(64), 0, st, (const uint32_t *)V.mig, V.ch_n_items, V.n_coop,
                       d->status);
  hipEvent_t dbg_ev[3] = {nullptr, nullptr, nullptr};  // (RT_DEBUG: chains / fold / continuations)
  if (cfg.debug) {
    for (auto &e : dbg_ev) HIP_OK(hipEventCreate(&e));
    HIP_OK(hipEventRecord(dbg_ev[0], st));
    if (V.mig) {
      std::vector<uint32_t> mw(b1::kMigWords);
      HIP_OK(hipStreamSynchronize(st));
      HIP_OK(hipMemcpy(mw.data(), V.mig, mw.size() * 4, hipMemcpyDeviceToHost));
      uint64_t pushed = 0, popped = 0;
      for (int m = 0; m < b1::kMigBoxes; m++) {
        const uint32_t *bx = &mw[b1::kMigBox0 + m * b1::kMigBoxWords];
        pushed += bx[b1::kMigPush] < V.mig_cap / b1::kMigBoxes ? bx[b1::kMigPush] : V.mig_cap / b1::kMigBoxes;
        popped += bx[b1::kMigPop];
      }
      fprintf(stderr, "[rtc] chain launch migration: helpers %u pushed %llu popped %llu done %u\n", mw[b1::kMigHelpers],
              (unsigned long long)pushed, (unsigned long long)popped, mw[b1::kMigDone]);
      uint64_t ms[6];  // (diagnostic build with RT_PX_TIME: the migrated items' rays and shader clocks)
      memcpy(ms, &mw[b1::kMigStat], sizeof(ms));
      if (ms[0])
        fprintf(stderr, "[rtc] migrated items: rays %llu exact scans %llu; clocks per ray: candidate %.0f ancestors %.0f "
                "exact %.0f item %.0f\n", (unsigned long long)ms[0], (unsigned long long)ms[1], (double)ms[2] / ms[0],
                (double)ms[3] / ms[0], (double)ms[4] / ms[0], (double)ms[5] / ms[0]);
    }
  }
  hipLaunchKernelGGL(chain_fold_kernel, dim3((unsigned)(npix / 64 + 1 < 8192 ? npix / 64 + 1 : 8192)), dim3(64), 0, st,
                     V, d_out, (const uint32_t *)d->ch_split, (const uint32_t *)d->ch_cnt, d->ch_cont,
                     d->ch_cnt + kCnCont);
  if (cfg.debug) HIP_OK(hipEventRecord(dbg_ev[1], st));
  // continuation items (normally none: the launch exits at once)
  b1::Book1View C = V;
  C.n_coop = nullptr;
  C.pre_state = nullptr;  // (continuations start from the fold's exact positions)
  C.ch_cont = d->ch_cont;
  C.ch_n_cont = d->ch_cnt + kCnCont;
  C.mig_epoch = ++d->mig_epoch;
  HIP_OK(hipMemsetAsync(V.work_counter, 0, kCounterBytes, st));  // counter + migration words
  launch_chain_kernel(d, C, d_out, st);
  HIP_OK(hipGetLastError());
  if (C.mig_live > 0)
    hipLaunchKernelGGL(chain_check_kernel, dim3(1), dim3(64), 0, st, (const uint32_t *)C.mig, C.ch_n_cont,
                       (const uint32_t *)nullptr, d->status);
  HIP_OK(mark_launch(d, 1, st));
  if (cfg.debug) {
    HIP_OK(hipEventRecord(dbg_ev[2], st));
    HIP_OK(hipStreamSynchronize(st));
    float t_chains = 0.0f, t_fold = 0.0f, t_cont = 0.0f;
    HIP_OK(hipEventElapsedTime(&t_chains, d->ev_main[0], dbg_ev[0]));
    HIP_OK(hipEventElapsedTime(&t_fold, dbg_ev[0], dbg_ev[1]));
    HIP_OK(hipEventElapsedTime(&t_cont, dbg_ev[1], dbg_ev[2]));
    for (auto &e : dbg_ev) HIP_OK(hipEventDestroy(e));
    fprintf(stderr, "[rtc] chain launch ms: chains %.2f fold %.2f continuations %.2f\n", t_chains, t_fold, t_cont);
#ifdef RT_LOOP_STATS
    {  // cumulative over the scene's launches; kMode 2 row
      unsigned long long q[32];
      HIP_OK(hipMemcpy(q, V.loop_stats, sizeof q, hipMemcpyDeviceToHost));
      const unsigned long long *r = q + 16;
      const double cyc = (double)(r[2] + r[5]);
      fprintf(stderr, "[rtc] loop stats (cumulative): trav iters %llu lanes/iter %.1f cycles %.1f%% | shade passes %llu "
              "lanes/pass %.1f cycles %.1f%% | live lanes/iter %.1f\n", r[0], r[0] ? (double)r[1] / r[0] : 0.0,
              100.0 * r[2] / cyc, r[3], r[3] ? (double)r[4] / r[3] : 0.0, 100.0 * r[5] / cyc,
              (r[0] + r[3]) ? (double)r[6] / (r[0] + r[3]) : 0.0);
      const unsigned long long *w = q + 24;
      fprintf(stderr, "[rtc] loop stats (cumulative): wave-steps %llu, stepping lanes/step %.1f; steps running the sphere "
              "block %.1f%%, leaf lanes in those %.2f\n", w[0], w[0] ? (double)w[1] / w[0] : 0.0,
              w[0] ? 100.0 * w[2] / w[0] : 0.0, w[2] ? (double)w[3] / w[2] : 0.0);
      fprintf(stderr, "[rtc] loop stats (cumulative): leaf lane-steps at the first of two sibling leaves %.1f%%; "
              "sphere-block steps whose leaf lanes all are %.1f%%\n", w[3] ? 100.0 * w[4] / w[3] : 0.0,
              w[2] ? 100.0 * w[5] / w[2] : 0.0);
    }
#endif

    uint32_t c[16];
    HIP_OK(hipStreamSynchronize(st));
    HIP_OK(hipMemcpy(c, d->ch_cnt, sizeof c, hipMemcpyDeviceToHost));
    // where the chains ended: per split pixel, records written vs the spp the pixel needs
    std::vector<uint32_t> split(c[kCnSplit]);
    std::vector<b1::ChainPx> px(npix);
    std::vector<uint64_t> seg(c[kCnSeg] < d->ch_seg_cap ? c[kCnSeg] : d->ch_seg_cap);
    HIP_OK(hipMemcpy(split.data(), d->ch_split, split.size() * 4, hipMemcpyDeviceToHost));
    HIP_OK(hipMemcpy(px.data(), d->ch_px, px.size() * sizeof(b1::ChainPx), hipMemcpyDeviceToHost));
    HIP_OK(hipMemcpy(seg.data(), d->ch_seg, seg.size() * 8, hipMemcpyDeviceToHost));
    double recs = 0.0, head = 0.0;
    uint64_t linked = 0, nolink = 0, segs = 0, khist[9] = {0};
    for (uint32_t p : split) {
      const b1::ChainPx &P = px[p];
      khist[P.K < 8 ? P.K : 8]++;
      for (uint32_t k = 0; k < P.K; k++) {
        const uint64_t w = seg[P.end0 + k];
        (k ? recs : head) += b1::end_n(w);
        segs++;
        if (w & b1::kEndNoLink) nolink++; else linked++;
      }
    }
    fprintf(stderr, "[rtc] chain launch: %u continuation items; split px %zu: samples %.3f x spp (head %.3f), segments "
            "%llu (%llu coupled, %llu unlinked); K hist 2:%llu 3:%llu 4:%llu 5:%llu 6:%llu 7:%llu 8+:%llu\n", c[kCnCont],
            split.size(), (recs + head) / (double)split.size() / V.S.cam.spp, head / (double)split.size() / V.S.cam.spp,
            (unsigned long long)segs, (unsigned long long)linked, (unsigned long long)nolink,
            (unsigned long long)khist[2], (unsigned long long)khist[3], (unsigned long long)khist[4],
            (unsigned long long)khist[5], (unsigned long long)khist[6], (unsigned long long)khist[7],
            (unsigned long long)khist[8]);
  }
  return 0;
}

// Lane launch (low spp, small launches, RT_MODE=lane): pixels in row order, one per lane.
static int launch_lane(rt_device_scene *d, b1::Book1View V, uint8_t *d_out, hipStream_t st) {
  const bool lds = d->b1_lds_bytes != 0;
  V.n_coop = nullptr;
  HIP_OK(mark_launch(d, 0, st));
  HIP_OK(hipMemsetAsync(V.work_counter, 0, kCounterBytes, st));  // counter + migration words
  const dim3 g1((unsigned)d->b1_grid), blk(b1::kBlock);
  if (lds) hipLaunchKernelGGL((rt_book1_kernel<true>), g1, blk, d->b1_lds_bytes, st, V, d_out);
  else hipLaunchKernelGGL((rt_book1_kernel<false>), g1, blk, 0, st, V, d_out);
  HIP_OK(hipGetLastError());
  HIP_OK(mark_launch(d, 1, st));
  return 0;
}

static void launch_general(const rt_device_scene *d, bool all, dim3 g, dim3 b, hipStream_t st, gen::GeneralView V,
                           uint8_t *d_out) {
  V.batch = d->view.pre ? d->cfg.gen_batch : 0;
  V.steps = d->cfg.gen_steps;
  V.rare_min = d->cfg.gen_rare;
  V.flat = d->cfg.gen_flat;
  V.n_lds = d->gen_lds;
  V.perlin_lds = d->gen_perlin_lds;
  const size_t lds_bytes = d->gen_lds_bytes;
  if (V.batch && d->gen_block == kBigBlock) {
    const dim3 bb(kBigBlock);
    if (all) hipLaunchKernelGGL((rt_general_kernel<kFeatAll, true, kBigBlock>), g, bb, lds_bytes, st, V, d_out);
    else hipLaunchKernelGGL((rt_general_kernel<kFeatBook1, true, kBigBlock>), g, bb, lds_bytes, st, V, d_out);
    return;
  }
  if (all && V.batch)
    hipLaunchKernelGGL((rt_general_kernel<kFeatAll, true>), g, b, lds_bytes, st, V, d_out);
  else if (all)
    hipLaunchKernelGGL((rt_general_kernel<kFeatAll, false>), g, b, 0, st, V, d_out);
  else if (V.batch)
    hipLaunchKernelGGL((rt_general_kernel<kFeatBook1, true>), g, b, lds_bytes, st, V, d_out);
  else
    hipLaunchKernelGGL((rt_general_kernel<kFeatBook1, false>), g, b, 0, st, V, d_out);
}

// The frame kernel rt_render_rows_async uses for a launch of npix pixels on this scene.
static int pick_mode(const rt_device_scene *d, int64_t npix) {
  const Config &cfg = d->cfg;
  const int spp = d->view.cam.spp;
  // (a pre-pass of at most a quarter of the frame's spp -- or, in the diagnostic build only, exactly its
  // spp: the "exact stream lengths" plan of scripts/gpu_r04.sh, RT_LPT_SPP = spp)
#ifdef RT_DIAG
  const bool exact_plan = cfg.lpt_spp == spp && spp >= 64;
#else
  const bool exact_plan = false;
#endif
  const bool chain_ok = cfg.lpt && (spp >= 4 * cfg.lpt_spp || exact_plan) &&
                        spp >= 2 * cfg.chain_min_seg && npix >= 4096 && d->view.cam.max_depth >= 1;
  if (cfg.mode == kModeChain) return chain_ok ? kModeChain : kModeLane;
  if (cfg.mode == kModeLane) return kModeLane;
  // auto: the chain render whenever it applies (measured ahead of the lane kernel at every N, from
  // 1.16x at N = 1 to 2.2x at N = 8: DESIGN.md §5); the lane kernel for low spp / small launches
  return chain_ok ? kModeChain : kModeLane;
}

static int render_rows(rt_device_scene *d, int row0, int row_stride, int n_rows, uint8_t *d_out, hipStream_t st) {
  const int64_t npix = (int64_t)n_rows * d->width;
  if (d->book1) {
    if (npix >= (int64_t)1 << 31) return rt_set_error("too many pixels for one launch"), -1;
    b1::Book1View V = d->b1view;
    V.row0 = row0;
    V.row_stride = row_stride;
    V.n_rows = n_rows;
    const int mode = pick_mode(d, npix);
    if (mode == kModeChain) return launch_chain(d, V, d_out, st, npix);
    return launch_lane(d, V, d_out, st);
  }
  if (d->general) {
    const Config &cfg = d->cfg;
    gen::GeneralView G;
    G.S = d->view;
    G.row0 = row0;
    G.row_stride = row_stride;
    G.n_rows = n_rows;
    G.work_counter = d->gen_counter;
    G.order = nullptr;
    G.cost_out = nullptr;
    G.pre_out = nullptr;
    G.pre_in = nullptr;
    G.stats = nullptr;
    G.xrec = d->gen_xrec;
    G.xw = d->gen_xw;
    G.code_bits = d->view.n_textures <= 13 ? 4 : 8;
    const bool all = (d->features & ~kFeatBook1) != 0;
    const dim3 gg((unsigned)d->gen_grid), gb(gen::kBlock);
    if (cfg.lpt && G.S.cam.spp >= 4 * cfg.lpt_spp && npix >= 4096) {  // longest-first order (rays per pixel)
      gen::GeneralView P = G;
      P.S.cam.spp = cfg.lpt_spp;
      P.cost_out = d->lpt_cost;
      P.pre_out = d->gen_pre;  // (its samples are the pixels' first ones: the launch below goes on from them)
      HIP_OK(hipMemsetAsync(d->gen_counter, 0, sizeof(int32_t), st));
      launch_general(d, all, gg, gb, st, P, d_out);
      HIP_OK(hipMemsetAsync(d->lpt_hist, 0, kLptHistBytes, st));
      unsigned long long *sums = (unsigned long long *)(d->lpt_hist + 512 + 32);
      const int n = (int)npix, nb = (int)((npix + 255) / 256 < 1024 ? (npix + 255) / 256 : 1024);
      hipLaunchKernelGGL(lpt_hist_kernel, dim3(nb), dim3(256), 0, st, d->lpt_cost, n, d->lpt_hist, sums);
      hipLaunchKernelGGL(lpt_scan_kernel, dim3(1), dim3(64), 0, st, d->lpt_hist);
      hipLaunchKernelGGL(lpt_scatter_kernel, dim3(nb), dim3(256), 0, st, d->lpt_cost, n, d->lpt_hist, d->lpt_order,
                         cfg.tile_order ? G.S.cam.width : 0, cfg.tile_order ? cfg.tile_order : 16);
      HIP_OK(hipGetLastError());
      G.order = d->lpt_order;
      G.pre_in = d->gen_pre;
    }
    HIP_OK(hipMemsetAsync(d->gen_counter, 0, sizeof(int32_t), st));
#ifdef RT_GEN_STATS
    static unsigned long long *gen_stats = nullptr;  // diagnostic build only (one device)
    if (!gen_stats) HIP_OK(hipMalloc(&gen_stats, gen::kGsN * sizeof(unsigned long long)));
    HIP_OK(hipMemsetAsync(gen_stats, 0, gen::kGsN * sizeof(unsigned long long), st));
    G.stats = gen_stats;
#endif
    HIP_OK(mark_launch(d, 0, st));
    launch_general(d, all, gg, gb, st, G, d_out);
    HIP_OK(hipGetLastError());
#ifdef RT_GEN_STATS
    if (cfg.debug) {
      unsigned long long q[gen::kGsN];
      HIP_OK(hipStreamSynchronize(st));
      HIP_OK(hipMemcpy(q, gen_stats, sizeof q, hipMemcpyDeviceToHost));
      static const char *names[gen::kGsN] = {
          "cyc_iter_refill", "cyc_iter_trace", "cyc_iter_shade", "trace_iters", "trace_lanes", "shade_iters",
          "shade_lanes", "step_kinds", "kind_box", "kind_sphere", "kind_quad", "kind_xform", "kind_medium",
          "kind_other", "cyc_record", "cyc_emit", "cyc_scatter", "cyc_lights", "cyc_fold", "mat_lam", "mat_metal",
          "mat_diel", "mat_iso", "mat_end", "tex_solid", "tex_checker", "tex_image", "tex_perlin",
          "cyc_scatter_perlin", "pass_perlin", "miss", "cyc_camera", "cyc_begin", "cyc_top", "cyc_classify",
          "cyc_common", "cyc_rare", "rare_steps", "cyc_bounce", "cyc_write", "records", "explicit", "weighted",
          "paths", "path_zero", "path_trunc", "path_trunc_zero", "spill_st", "spill_st_zero", "w2", "fold_skips"};
      fprintf(stderr, "[rtc] gen stats:");
      for (int k = 0; k < gen::kGsN; k++) fprintf(stderr, " %s=%llu", names[k], q[k]);
      fprintf(stderr, "\n");
    }
#endif
    HIP_OK(mark_launch(d, 1, st));
    return 0;
  }
  if (d->deep_rec) {
    const int64_t th = d->deep_threads < npix ? (d->deep_threads + kBlock - 1) / kBlock * kBlock : npix;
    const dim3 gd((unsigned)((th + kBlock - 1) / kBlock)), bd(kBlock);
    if ((d->features & ~kFeatBook1) == 0)
      hipLaunchKernelGGL(rt_render_deep_kernel<kFeatBook1>, gd, bd, 0, st, d->view, row0, row_stride, n_rows, d_out,
                         d->deep_rec);
    else
      hipLaunchKernelGGL(rt_render_deep_kernel<kFeatAll>, gd, bd, 0, st, d->view, row0, row_stride, n_rows, d_out,
                         d->deep_rec);
    HIP_OK(hipGetLastError());
    return 0;
  }
  const dim3 grid((unsigned)((npix + kBlock - 1) / kBlock)), block(kBlock);
  if ((d->features & ~kFeatBook1) == 0)
    hipLaunchKernelGGL(rt_render_rows_kernel<kFeatBook1>, grid, block, 0, st, d->view, row0, row_stride, n_rows, d_out);
  else
    hipLaunchKernelGGL(rt_render_rows_kernel<kFeatAll>, grid, block, 0, st, d->view, row0, row_stride, n_rows, d_out);
  HIP_OK(hipGetLastError());
  return 0;
}

// A scene's launches share its scratch (work counters, plans, records), so a launch first waits for
// the scene's previous launch (ev_done) -- whatever stream that one was queued on.
extern "C" int rt_render_rows_async(rt_device_scene *d, int row0, int row_stride, int n_rows, uint8_t *d_out,
                                    void *stream) {
  if (!d || !d_out) return rt_set_error("rt_render_rows_async: NULL argument"), -1;
  if (n_rows <= 0) return 0;
  if (row0 < 0 || row_stride <= 0 || (int64_t)row0 + (int64_t)(n_rows - 1) * row_stride >= d->height)
    return rt_set_error("rows %d + k*%d (k < %d) outside image height %d", row0, row_stride, n_rows, d->height), -1;
  HIP_OK(hipSetDevice(d->device));
  hipStream_t st = (hipStream_t)stream;
  if (d->launched) HIP_OK(hipStreamWaitEvent(st, d->ev_done, 0));
  // this launch's timestamps go to the next slot of the ring (mark_launch)
  d->ts_ring = (uint64_t *)((char *)d->status + 256) + 2 * (d->n_launches++ % rt_device_scene::kLaunchRing);
  HIP_OK(hipMemsetAsync(d->ts_ring, 0, 2 * sizeof(uint64_t), st));  // (a launch without a bracket reads -1)
  const int rc = render_rows(d, row0, row_stride, n_rows, d_out, st);
  HIP_OK(hipEventRecord(d->ev_done, st));
  d->launched = true;
  return rc;
}

// Completion status of the scene's launches so far (chain_check_kernel): waits for the last launch,
// then returns 0, or -1 with the number of unfinished work items in the error message, and clears it.
extern "C" int rt_scene_check(rt_device_scene *d) {
  if (!d) return rt_set_error("rt_scene_check: NULL scene"), -1;
  HIP_OK(hipSetDevice(d->device));
  if (d->launched) HIP_OK(hipEventSynchronize(d->ev_done));
  uint32_t st[2] = {0u, 0u};
  HIP_OK(hipMemcpy(st, d->status, sizeof st, hipMemcpyDeviceToHost));
  if (st[0] == 0u) return 0;
  HIP_OK(hipMemset(d->status, 0, sizeof st));
  return rt_set_error("render incomplete on device %d: %u work item(s) of a chain launch never finished "
                      "(status 0x%x); the frame is not valid", d->device, st[1], st[0]), -1;
}

// ------------------------------------------------------------------------------ device-scene cache
// A share -- rows j % n_shares == share of a frame, on one device -- keeps its device scene (arrays, plan
// scratch and the chain-record arena, which stays clean between launches), its output rows and its stream
// after the call, keyed by every byte of the flat scene, the share, and the RT_* environment the scene's
// Config is read from.  The next rt_render / rt_render_share with an identical key renders at once: a
// driver that calls Camera_render frame after frame pays the upload, the allocations and the first
// launch's record fill once.  One layout (key, n_shares) per device: a call with another
// layout frees the device's idle slots first.  RT_SCENE_CACHE=0: nothing is kept (every call uploads and
// frees); rt_render_cache_release() frees what is kept.
struct ShareSlot {
  int device = -1, share = -1, n_shares = 0;
  std::string key;
  rt_device_scene *scene = nullptr;
  hipStream_t stream = nullptr;
  uint8_t *d_out = nullptr;
  bool busy = false, cached = false;
};
static std::mutex g_cache_mu;
static std::vector<ShareSlot *> &cache_slots() {  // (never destroyed: no HIP call from a static destructor)
  static std::vector<ShareSlot *> *v = new std::vector<ShareSlot *>();
  return *v;
}

static void slot_free(ShareSlot *e) {
  (void)hipSetDevice(e->device);
  if (e->scene) rt_scene_release(e->scene);  // (waits for the scene's last launch)
  if (e->d_out) (void)hipFree(e->d_out);
  if (e->stream) (void)hipStreamDestroy(e->stream);
  delete e;
}

extern char **environ;
static std::string scene_key(const rt_flat_scene *s, int per_dev) {
  std::string k;
  auto add = [&k](const void *p, size_t n) {
    if (p && n) k.append((const char *)p, n);
  };
  add(s, offsetof(rt_flat_scene, bvh));  // camera, root, lights, features, counts
  add(s->bvh, sizeof(rt_bvh_node) * s->n_bvh);
  add(s->spheres, sizeof(rt_sphere) * s->n_spheres);
  add(s->quads, sizeof(rt_quad) * s->n_quads);
  add(s->lists, sizeof(rt_list) * s->n_lists);
  add(s->list_items, sizeof(int32_t) * s->n_list_items);
  add(s->translates, sizeof(rt_translate) * s->n_translates);
  add(s->rotates, sizeof(rt_rotate_y) * s->n_rotates);
  add(s->media, sizeof(rt_medium) * s->n_media);
  add(s->materials, sizeof(rt_material) * s->n_materials);
  add(s->textures, sizeof(rt_texture) * s->n_textures);
  add(s->images, sizeof(rt_image) * s->n_images);
  add(s->perlins, sizeof(rt_perlin) * s->n_perlins);
  add(s->image_bytes, (size_t)s->n_image_bytes);
  std::vector<std::string> env;
  for (char **e = environ; e && *e; e++)
    if (!strncmp(*e, "RT_", 3)) env.emplace_back(*e);
  std::sort(env.begin(), env.end());
  for (const std::string &e : env) k.append(e).push_back('\0');
  add(&per_dev, sizeof per_dev);
  return k;
}

// A slot for (device, share, n_shares): the cached one when its key matches and no other call holds it,
// else a new one (cached when the cache is on and no identical slot is in use).
static ShareSlot *slot_acquire(const std::string *key, int device, int share, int n_shares) {
  std::vector<ShareSlot *> stale;
  ShareSlot *e = nullptr;
  {
    std::lock_guard<std::mutex> lk(g_cache_mu);
    std::vector<ShareSlot *> &v = cache_slots();
    bool in_use = false;
    for (size_t i = 0; i < v.size();) {
      ShareSlot *c = v[i];
      const bool same = key && c->n_shares == n_shares && c->key == *key;
      if (c->device == device && same && c->share == share) {
        if (!c->busy) e = c, e->busy = true;
        else in_use = true;
      }
      if (c->device == device && !same && !c->busy) {  // another layout on this device: freed
        stale.push_back(c);
        v.erase(v.begin() + (ptrdiff_t)i);
        continue;
      }
      i++;
    }
    if (!e) {
      e = new ShareSlot();
      e->device = device, e->share = share, e->n_shares = n_shares, e->busy = true;
      if (key && !in_use) e->key = *key, e->cached = true, v.push_back(e);
    }
  }
  for (ShareSlot *c : stale) slot_free(c);
  return e;
}

static void slot_release(ShareSlot *e, bool ok) {
  if (e->cached) {
    std::lock_guard<std::mutex> lk(g_cache_mu);
    if (ok) {
      e->busy = false;
      return;
    }
    std::vector<ShareSlot *> &v = cache_slots();  // (a failed share's scene is not reused)
    v.erase(std::remove(v.begin(), v.end(), e), v.end());
  }
  slot_free(e);
}

extern "C" void rt_render_cache_release(void) {
  std::vector<ShareSlot *> idle;
  {
    std::lock_guard<std::mutex> lk(g_cache_mu);
    std::vector<ShareSlot *> &v = cache_slots();
    for (ShareSlot *c : v) (c->busy ? (void)(c->cached = false) : idle.push_back(c));  // (a busy one: freed on release)
    v.clear();
  }
  for (ShareSlot *c : idle) slot_free(c);
}

// ------------------------------------------------------------------------------ whole frame
static std::mutex g_timing_mu;
static std::vector<double> g_kernel_ms(64, 0.0);
static std::vector<std::array<double, 4>> g_share_ms(64, std::array<double, 4>{0.0, 0.0, 0.0, 0.0});

extern "C" double rt_last_kernel_ms(int device) {
  std::lock_guard<std::mutex> lk(g_timing_mu);
  return (device >= 0 && device < (int)g_kernel_ms.size()) ? g_kernel_ms[device] : 0.0;
}

extern "C" int rt_last_share_ms(int share, double *ms) {
  if (!ms) return rt_set_error("rt_last_share_ms: NULL argument"), -1;
  std::lock_guard<std::mutex> lk(g_timing_mu);
  if (share < 0 || share >= (int)g_share_ms.size()) return rt_set_error("rt_last_share_ms: share %d", share), -1;
  for (int k = 0; k < 4; k++) ms[k] = g_share_ms[share][k];
  return 0;
}

static double now_ms() {
  return std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

// One share on one device: upload (or reuse), launch, copy its compact rows straight into rows
// share + k * n_shares of the caller's buffer (disjoint rows: no lock), check completion.
// pack() gives the host preprocessing (computed at most once per rt_render call, only on a miss).
static int render_share(const rt_flat_scene *s, const std::function<const HostPack *()> &pack, const std::string *key,
                        int g, int G, int device, uint8_t *out_host, std::string &err) {
  const double t_start = now_ms();
  const int H_img = s->camera.height, W = s->camera.width;
  const int n_rows = (H_img - g + G - 1) / G;
  ShareSlot *e = slot_acquire(key, device, g, G);
  int rc = 0;
  if (!e->scene) {
    const HostPack *H = pack();
    e->scene = H ? upload_packed(s, *H, device) : nullptr;
    if (!e->scene ||
        hipStreamCreateWithFlags(&e->stream, hipStreamNonBlocking) != hipSuccess ||
        hipMalloc(&e->d_out, (size_t)n_rows * W * 3) != hipSuccess) {
      if (e->scene) rt_set_error("rt_render: stream/buffer setup failed on device %d", device);
      rc = -1;
    }
  }
  const double t_setup = now_ms();
  double t_done = t_setup;
  hipEvent_t t0 = nullptr, t1 = nullptr;
  if (rc == 0 && (hipSetDevice(device) != hipSuccess || hipEventCreate(&t0) != hipSuccess ||
                  hipEventCreate(&t1) != hipSuccess)) {
    rt_set_error("rt_render: event setup failed on device %d", device);
    rc = -1;
  }
  if (rc == 0) {
    (void)hipEventRecord(t0, e->stream);
    rc = rt_render_rows_async(e->scene, g, G, n_rows, e->d_out, e->stream);
    (void)hipEventRecord(t1, e->stream);
  }
  if (rc == 0) {
    hipError_t x = hipEventSynchronize(t1);
    t_done = now_ms();
    const size_t row = (size_t)W * 3;
    if (x == hipSuccess)
      x = hipMemcpy2DAsync(out_host + (size_t)g * row, row * (size_t)G, e->d_out, row, row, (size_t)n_rows,
                           hipMemcpyDeviceToHost, e->stream);
    if (x == hipSuccess) x = hipStreamSynchronize(e->stream);
    if (x != hipSuccess) {
      rt_set_error("rt_render: share %d (device %d): %s", g, device, hipGetErrorString(x));
      rc = -1;
    } else if (rt_scene_check(e->scene) != 0) {  // never a partial image with rc 0
      rc = -1;
    } else if (e->scene->ch_cnt) {  // the records the launch's plan wanted: a kept scene's next arena
      unsigned long long want = 0;
      if (hipMemcpy(&want, e->scene->ch_cnt + kCnRec, sizeof want, hipMemcpyDeviceToHost) == hipSuccess &&
          want > e->scene->ch_rec_cap)
        e->scene->ch_rec_demand = (size_t)want;
    }
  }
  if (rc == 0) {
    float ms = 0.0f;
    (void)hipEventElapsedTime(&ms, t0, t1);
    const double t_end = now_ms();
    std::lock_guard<std::mutex> lk(g_timing_mu);
    if (g < (int)g_kernel_ms.size()) {
      g_kernel_ms[g] = ms;
      g_share_ms[g] = {t_setup - t_start, t_done - t_setup, t_end - t_done, t_end - t_start};
    }
  }
  if (rc != 0) err = rt_last_error();
  (void)hipSetDevice(device);
  if (t0) (void)hipEventDestroy(t0);
  if (t1) (void)hipEventDestroy(t1);
  slot_release(e, rc == 0);
  return rc;
}

// RT_REHEARSE_DEVICES=N (N > 0): behave as if N devices were visible -- share g runs on device
// g % (visible devices), still one host thread and one device scene per share -- so the multi-device
// path (threads, per-share upload, streams, error aggregation) runs on a box with fewer GPUs.
// Shares on one device split its chain-record budget.  Timings are then contended.
extern "C" int rt_render(const rt_flat_scene *s, int n_gpus, uint8_t *out_host) {
  if (!s || !out_host) return rt_set_error("rt_render: NULL argument"), -1;
  const int avail = rt_device_count();
  if (avail <= 0) return rt_set_error("rt_render: no HIP device visible (this library has no CPU path)"), -1;
  const int rehearse = env_int("RT_REHEARSE_DEVICES", 0);
  const int visible = rehearse > 0 ? rehearse : avail;
  int G = (n_gpus <= 0 || n_gpus > visible) ? visible : n_gpus;
  if (G > s->camera.height) G = s->camera.height;
  const int per_dev = (G + avail - 1) / avail;  // shares per device (> 1 only when rehearsing)
  std::string key;
  const bool cache = env_int("RT_SCENE_CACHE", 1) != 0;
  if (cache) key = scene_key(s, per_dev);
  // host preprocessing at most once, shared by every device, and only when a share has no cached scene
  HostPack H;
  int pack_rc = 0;
  std::once_flag once;
  auto pack = [&]() -> const HostPack * {
    std::call_once(once, [&] {
      pack_rc = host_pack(s, H);
      if (per_dev > 1) H.cfg.chain_mb /= (size_t)per_dev;
    });
    return pack_rc == 0 ? &H : nullptr;
  };
  std::vector<int> rc(G, 0);
  std::vector<std::string> err(G);
  if (G == 1) {
    rc[0] = render_share(s, pack, cache ? &key : nullptr, 0, 1, 0, out_host, err[0]);
  } else {  // one host thread per share: uploads and launches proceed in parallel
    std::vector<std::thread> th;
    for (int g = 0; g < G; g++)
      th.emplace_back([&, g] { rc[g] = render_share(s, pack, cache ? &key : nullptr, g, G, g % avail, out_host, err[g]); });
    for (auto &t : th) t.join();
  }
  for (int g = 0; g < G; g++)
    if (rc[g] != 0) return rt_set_error("%s", err[g].c_str()), -1;
  return 0;
}

// One share of rt_render's partition, for a driver that runs one process (or thread) per GPU: rows
// j % n_shares == share of the frame on `device`, written into those rows of out_host (a whole frame's
// buffer; the other rows are left as they are).  Same cache and completion check as rt_render.
extern "C" int rt_render_share(const rt_flat_scene *s, int share, int n_shares, int device, uint8_t *out_host) {
  if (!s || !out_host) return rt_set_error("rt_render_share: NULL argument"), -1;
  if (n_shares < 1 || share < 0 || share >= n_shares || share >= s->camera.height)
    return rt_set_error("rt_render_share: share %d of %d (image height %d)", share, n_shares, s->camera.height), -1;
  const int avail = rt_device_count();
  if (avail <= 0) return rt_set_error("rt_render_share: no HIP device visible (this library has no CPU path)"), -1;
  if (device < 0 || device >= avail) return rt_set_error("rt_render_share: device %d of %d", device, avail), -1;
  std::string key;
  const bool cache = env_int("RT_SCENE_CACHE", 1) != 0;
  if (cache) key = scene_key(s, 1);
  HostPack H;
  int pack_rc = 1;
  auto pack = [&]() -> const HostPack * {
    if (pack_rc == 1) pack_rc = host_pack(s, H);
    return pack_rc == 0 ? &H : nullptr;
  };
  std::string err;
  const int rc = render_share(s, pack, cache ? &key : nullptr, share, n_shares, device, out_host, err);
  if (rc != 0) rt_set_error("%s", err.c_str());
  return rc;
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
  if (fn < 0 || fn > 2 || mismatches == NULL) return rt_set_error("rt_diag_arith: bad arguments"), -1;
  HIP_OK(hipSetDevice(device));
  unsigned long long *dm = NULL;
  HIP_OK(hipMalloc(&dm, sizeof *dm));
  HIP_OK(hipMemset(dm, 0, sizeof *dm));
  hipLaunchKernelGGL(rt_diag_arith_kernel, dim3(4096), dim3(256), 0, 0, fn, start, count, seed, dm);
  HIP_OK(hipGetLastError());
  HIP_OK(hipMemcpy(mismatches, dm, sizeof *dm, hipMemcpyDeviceToHost));
  HIP_OK(hipFree(dm));
  return 0;
}

// Diagnostics of the last chain launch (RT_PX_TIME=1 at upload): one row of 16 u32 per work item, in
// item order -- pixel, segment, K, whole-wave (1) or lane (0), start, end (wall_clock64 ticks, low 32
// bits), records (samples for segment 0 / unsplit), end flags (bit 0 linked, bit 1 ended), link
// segment, link record, segment length, the pixel's pre-pass draws and own cost, the migration tick,
// the planner's cost, 1 reserved (rt_hip.h).
// Returns the number of items (rows written: min(items, max_rows)), or -1.
extern "C" int64_t rt_scene_chain_diag(rt_device_scene *d, uint32_t *rows, int64_t max_rows) {
  if (!d || !d->book1 || !d->px_time || !d->seg_time) return rt_set_error("rt_scene_chain_diag: upload with RT_PX_TIME=1"), -1;
  HIP_OK(hipSetDevice(d->device));
  HIP_OK(hipDeviceSynchronize());
  uint32_t c[kCnWords];
  HIP_OK(hipMemcpy(c, d->ch_cnt, sizeof c, hipMemcpyDeviceToHost));
  const size_t npix = (size_t)d->width * d->height, n_items = c[kCnItems], n_seg = c[kCnSeg] < d->ch_seg_cap ? c[kCnSeg] : d->ch_seg_cap;
  std::vector<uint2> items(n_items);
  std::vector<b1::ChainPx> px(npix);
  std::vector<uint64_t> seg(n_seg);
  std::vector<uint32_t> pt(b1::kTimeWords * npix), sgt(b1::kTimeWords * n_seg), draws(npix), costs(npix), own(npix);
  HIP_OK(hipMemcpy(draws.data(), d->draw_out, npix * sizeof(uint32_t), hipMemcpyDeviceToHost));
  HIP_OK(hipMemcpy(costs.data(), d->lpt_cost, npix * sizeof(uint32_t), hipMemcpyDeviceToHost));
  // (cost smoothing on: lpt_cost holds the planner's max(own, row mean); the pixel's own is cost_own)
  HIP_OK(hipMemcpy(own.data(), d->cost_own ? d->cost_own : d->lpt_cost, npix * sizeof(uint32_t), hipMemcpyDeviceToHost));
  HIP_OK(hipMemcpy(items.data(), d->ch_items, n_items * sizeof(uint2), hipMemcpyDeviceToHost));
  HIP_OK(hipMemcpy(px.data(), d->ch_px, npix * sizeof(b1::ChainPx), hipMemcpyDeviceToHost));
  HIP_OK(hipMemcpy(seg.data(), d->ch_seg, n_seg * sizeof(uint64_t), hipMemcpyDeviceToHost));
  HIP_OK(hipMemcpy(pt.data(), d->px_time, b1::kTimeWords * npix * sizeof(uint32_t), hipMemcpyDeviceToHost));
  HIP_OK(hipMemcpy(sgt.data(), d->seg_time, b1::kTimeWords * n_seg * sizeof(uint32_t), hipMemcpyDeviceToHost));
  const uint32_t spp = (uint32_t)d->view.cam.spp;
  for (size_t k = 0; k < n_items && (int64_t)k < max_rows; k++) {
    const uint32_t p = items[k].x, sg = items[k].y;
    uint32_t *r = rows + 16 * k;
    r[0] = p;
    r[3] = k < c[kCnNCoop] ? 1u : 0u;
    r[8] = r[9] = r[10] = 0u;
    r[11] = draws[p];
    r[12] = own[p];
    r[13] = r[15] = 0u;  // (15: where the item started, b1::hw_where)
    r[14] = costs[p];
    if (sg & b1::kItemUnsplit) {
      r[1] = 0, r[2] = 1, r[4] = pt[4 * p], r[5] = pt[4 * p + 1], r[6] = spp, r[7] = 2u, r[13] = pt[4 * p + 2], r[15] = pt[4 * p + 3];
    } else {
      const b1::ChainPx &P = px[p];
      const uint64_t w = P.end0 + sg < n_seg ? seg[P.end0 + sg] : 0ull;
      r[1] = sg, r[2] = P.K;
      r[4] = P.end0 + sg < n_seg ? sgt[4 * (P.end0 + sg)] : 0u;
      r[5] = P.end0 + sg < n_seg ? sgt[4 * (P.end0 + sg) + 1] : 0u;
      r[13] = P.end0 + sg < n_seg ? sgt[4 * (P.end0 + sg) + 2] : 0u;
      r[15] = P.end0 + sg < n_seg ? sgt[4 * (P.end0 + sg) + 3] : 0u;
      r[6] = b1::end_n(w);
      r[7] = ((w & b1::kEndEnded) && !(w & b1::kEndNoLink) ? 1u : 0u) | ((w & b1::kEndEnded) ? 2u : 0u);
      r[8] = b1::end_t(w), r[9] = b1::end_c(w), r[10] = P.seg_len;
    }
  }
  const size_t k = n_items;
  return (int64_t)k;
}

// Name of the frame kernel rt_render_rows_async launched last on this scene -- or, before any launch,
// the one it would launch over the whole image -- as rocprofv3 reports it (the chain kernel's
// occupancy depends on the launch's pixel count: a rank's share can get the 3-wave instantiation).
extern "C" const char *rt_scene_kernel(const rt_device_scene *d) {
  static thread_local char buf[160];
  if (!d) return "";
  if (d->deep_rec) {
    snprintf(buf, sizeof buf, "rt_render_deep_kernel<%d>", (d->features & ~kFeatBook1) == 0 ? (int)kFeatBook1 : (int)kFeatAll);
    return buf;
  }
  if (!d->book1) {
    snprintf(buf, sizeof buf, "%s<%d%s>", d->general ? "rt_general_kernel" : "rt_render_rows_kernel",
             (d->features & ~kFeatBook1) == 0 ? (int)kFeatBook1 : (int)kFeatAll,
             d->general && d->gen_block == kBigBlock ? ", true, 768"
             : d->general && d->view.pre && d->cfg.gen_batch ? ", true" : d->general ? ", false" : "");
    return buf;
  }
  const int64_t npix = (int64_t)d->width * d->height;
  const int mode = pick_mode(d, npix);
  const char *lds = d->b1_lds_bytes ? "true" : "false";
  if (mode == kModeChain)  // (every template argument, as rocprofv3 demangles the name: kLds, kOcc)
    snprintf(buf, sizeof buf, "rt_book1_chain_kernel<%s, %d>", lds, d->launched ? d->chain_occ : chain_occupancy(d, npix));
  else
    snprintf(buf, sizeof buf, "rt_book1_kernel<%s>", lds);
  return buf;
}

// Milliseconds of the last frame launch of rt_render_rows_async on this scene (after it completed);
// excludes the cost pre-pass and the plan.  -1 when unavailable.
extern "C" double rt_scene_last_launch_ms(rt_device_scene *d) {
  if (!d || !d->ev_main[0] || !d->ev_main[1]) return -1.0;
  float ms = 0.0f;
  if (hipEventElapsedTime(&ms, d->ev_main[0], d->ev_main[1]) != hipSuccess) return -1.0;
  return (double)ms;
}

// The frame-kernel milliseconds of this scene's last min(max, launches, 64) launches, oldest first
// (after they completed; from the device timestamps of mark_launch); returns how many were written, or -1.
extern "C" int rt_scene_launch_history(rt_device_scene *d, double *ms, int max) {
  if (!d || !ms || max < 0) return rt_set_error("rt_scene_launch_history: bad argument"), -1;
  const int R = rt_device_scene::kLaunchRing;
  const int n = (int)(d->n_launches < (uint64_t)R ? d->n_launches : (uint64_t)R);
  const int m = n < max ? n : max;
  HIP_OK(hipSetDevice(d->device));
  if (d->launched) HIP_OK(hipEventSynchronize(d->ev_done));
  std::vector<uint64_t> ts(2 * R);
  HIP_OK(hipMemcpy(ts.data(), (char *)d->status + 256, ts.size() * sizeof(uint64_t), hipMemcpyDeviceToHost));
  for (int k = 0; k < m; k++) {
    const int slot = (int)((d->n_launches - (uint64_t)m + (uint64_t)k) % (uint64_t)R);
    const uint64_t a = ts[2 * slot], b = ts[2 * slot + 1];
    ms[k] = a && b >= a ? (double)(b - a) * 1e-5 : -1.0;  // wall_clock64: 100 MHz
  }
  return m;
}
