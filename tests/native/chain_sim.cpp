// chain_sim — TEST INFRASTRUCTURE.  Runs the chain-render protocol of the gfx950 kernel
// (ray-tracing-c_amd/csrc/rt_book1.h: chain_boundary / chain_couple / chain_walk_done /
// chain_record, the same code the kernel compiles) on the CPU with AddressSanitizer, over a small
// frame of a Book-1 scene, with adversarial plans: random segment counts, stream-length estimates
// off by up to 2x, tiny record lists (forcing continuations) and a random interleaving of the chains
// (random start delays, one sample per scheduling step).  Then the fold and the continuations, as chain_fold_kernel and the continuation launch do.  tests/test_kernel_logic.py compares the image
// with the oracle: the protocol must be exact whatever the plan and the timing.
// It is not part of the product and is never linked into librtc_amd.so.
//   chain_sim <scene> <width> <spp> <depth> <out.rgb> <seed> <kmin> <kmax> <margin> <slack> [pad] [pre]
// pad > 1: stream-length estimates off by up to 2x are then spread over pad x the estimate (the
// planner's padded plan for many-segment pixels: segments past the true stream end).
// pre > 0: a cost pre-pass of `pre` samples per pixel (a random 0..pre of them for some pixels, as the
// pre-pass's step budget cuts heavy pixels short) leaves its colour sum and position, and segment 0 /
// unsplit chains go on from there (rt_book1.h: pre_word / pre_resume) -- the pre-pass position can lie
// past segment 1's start.
#include "../../ray-tracing-c_amd/csrc/rt_book1.h"
#include "../../include/rt_hip.h"

#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <vector>

using namespace rt;

static uint64_t rng_state;
static uint32_t rnd() {  // xorshift64*
  rng_state ^= rng_state >> 12;
  rng_state ^= rng_state << 25;
  rng_state ^= rng_state >> 27;
  return (uint32_t)((rng_state * 2685821657736338717ull) >> 32);
}

struct Chain {
  int32_t pix;
  uint32_t seg;
  Pcg32 g;
  uint32_t s, tc, st;
  f3 acc;
  int start_at;  // scheduling step before which it does not run
  bool done;
};

// one sample of pixel (i, j) from the chain's rng state (Camera_render's loop body)
static f3 sample(const DScene &S, int pix, Pcg32 &g) {
  const rt_camera &cam = S.cam;
  const int i = pix % cam.width, j = pix / cam.width;
  const f3 du = ld3(cam.delta_u), dv = ld3(cam.delta_v), lf = ld3(cam.origin);
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
  const f3 d = add(add(add(pixel_pos, scale(du, px)), scale(dv, py)), neg(o));
  return path_color<kFeatBook1>(S, o, d, g);
}

int main(int argc, char **argv) {
  if (argc < 11) {
    fprintf(stderr, "usage: chain_sim <scene> <width> <spp> <depth> <out.rgb> <seed> <kmin> <kmax> <margin> <slack>\n");
    return 2;
  }
  rt_flat_scene *s = rt_scene_preset(atoi(argv[1]), atoi(argv[2]), atoi(argv[3]), atoi(argv[4]));
  if (!s || (s->features & ~kFeatBook1) != 0) {
    fprintf(stderr, "needs a Book-1 scene\n");
    return 1;
  }
  rng_state = 0x9e3779b97f4a7c15ull ^ (uint64_t)atoll(argv[6]);
  const int kmin = atoi(argv[7]), kmax = atoi(argv[8]);
  const float margin = (float)atof(argv[9]);
  const uint32_t slack = (uint32_t)atoi(argv[10]);
  const double pad = argc > 11 ? atof(argv[11]) : 1.0;
  const int pre = argc > 12 ? atoi(argv[12]) : 0;
  const void *arrays[13] = {s->bvh,        s->spheres,  s->quads,     s->lists,  s->list_items,
                            s->translates, s->rotates,  s->media,     s->materials, s->textures,
                            s->images,     s->perlins,  s->image_bytes};
  const DScene view = make_view(*s, arrays);
  const int W = s->camera.width, H = s->camera.height, spp = s->camera.spp;
  const int npix = W * H;
  std::vector<uint8_t> img((size_t)npix * 3, 0);
  // plan: K per pixel, a deliberately noisy stream-length estimate (a 4-sample pre-pass x [0.5, 2])
  std::vector<b1::ChainPx> px(npix);
  std::vector<uint64_t> seg;
  std::vector<float4> col;
  std::vector<float4> acc0(npix);
  std::vector<uint32_t> split;
  // the pre-pass (kMode 1): the pixel's first samples from offset 0, as the cost kernel leaves them
  std::vector<float4> pre_state(npix, make_float4(0.0f, 0.0f, 0.0f, 0.0f));
  b1::Book1View PV;
  memset(&PV, 0, sizeof PV);
  PV.pre_state = pre > 0 ? pre_state.data() : nullptr;
  for (int p = 0; pre > 0 && p < npix; p++) {
    Pcg32 g;
    g.seed((uint64_t)(17 + p / W), (uint64_t)(23 + p % W));
    const int n = (rnd() % 4u) == 0 ? (int)(rnd() % (uint32_t)(pre + 1)) : pre;
    f3 a = mk(0.0f, 0.0f, 0.0f);
    for (int q = 0; q < n; q++) a = add(a, sample(view, p, g));
    pre_state[p] = make_float4(a.x, a.y, a.z, b1::u2f(b1::pre_word(g.n, (uint32_t)n)));
  }
  std::vector<Chain> chains;
  uint32_t rec = 0;
  for (int p = 0; p < npix; p++) {
    int K = kmin + (int)(rnd() % (uint32_t)(kmax - kmin + 1));
    if (K > spp) K = spp;
    Pcg32 g;
    g.seed((uint64_t)(17 + p / W), (uint64_t)(23 + p % W));
    for (int q = 0; q < 4; q++) (void)sample(view, p, g);
    const double est = (double)g.n / 4.0 * spp * (0.5 + 1.5 * (rnd() % 1000) / 1000.0) * (pad > 1.0 ? pad : 1.0);
    uint32_t seg_len = ((uint32_t)(est / K) + 1u) & ~1u;
    if (seg_len < 2) K = 1;
    if (K > 1) {
      b1::ChainPx &P = px[p];
      P.K = (uint32_t)K;
      P.seg_len = seg_len;
      P.cap = (uint32_t)ceilf(fminf(margin, (float)K) * (float)spp / (float)K) + slack;  // (as chain_plan_kernel)
      P.cap_last = (rnd() & 1) ? P.cap : (uint32_t)spp + slack;  // (the planner's, or a short one)
      P.rec0 = rec;
      rec += (uint32_t)(K - 2) * P.cap + P.cap_last;
      P.end0 = (uint32_t)seg.size();
      P.check = (uint32_t)(3 * (spp / K) / 4);
      P.pad = 0u;
      for (uint32_t k = 0; k < (uint32_t)K; k++) seg.push_back(0ull);
      split.push_back((uint32_t)p);
    }
    for (int k = 0; k < K; k++) {
      Chain c;
      c.pix = p;
      c.seg = K == 1 ? b1::kItemUnsplit : (uint32_t)k;
      c.g.seed((uint64_t)(17 + p / W), (uint64_t)(23 + p % W));
      c.s = 0;
      c.tc = b1::kNoTarget;
      c.st = 0;
      c.acc = mk(0.0f, 0.0f, 0.0f);
      if (K > 1) {
        c.g.skip((uint32_t)k * seg_len);
        if (k + 1 < K) c.tc = (uint32_t)(k + 1) << 24, c.st = (uint32_t)(k + 1) * seg_len;
      }
      b1::pre_resume(PV, p, c.seg, c.g, c.s, c.acc);
      c.start_at = (int)(rnd() % 64u);
      c.done = false;
      chains.push_back(c);
    }
  }
  col.assign(rec, make_float4(0, 0, 0, b1::u2f(b1::kRecFill)));  // (end word kRecFill: a clean arena)
  std::vector<uint32_t> mig(b1::kMigWords, 0u);
  b1::Book1View V;
  memset(&V, 0, sizeof V);
  V.S = view;
  V.ch_px = px.data();
  V.ch_seg = seg.data();
  V.ch_col = col.data();
  V.ch_acc0 = acc0.data();
  V.mig = mig.data();
  V.mig_epoch = 1u;
  V.walk_mask = 3u;  // (the product's default: a segment past its check walks every 4 samples)
  // interleaved execution: a random live chain takes one step (boundary, then one sample)
  std::vector<int> live;
  for (int c = 0; c < (int)chains.size(); c++) live.push_back(c);
  long step = 0, samples = 0;
  while (!live.empty()) {
    const int at = (int)(rnd() % (uint32_t)live.size());
    Chain &c = chains[live[at]];
    step++;
    if (c.start_at > 0) {
      c.start_at--;
      continue;
    }
    if (b1::chain_boundary(V, c.pix, c.seg, c.g.n, c.s, c.acc, c.tc, c.st, img.data(), true)) {
      c.done = true;
      live[at] = live.back();
      live.pop_back();
      continue;
    }
    const f3 color = sample(view, c.pix, c.g);
    samples++;
    if (!(c.seg & b1::kItemUnsplit) && c.seg > 0)
      b1::chain_record(V, c.pix, c.seg, c.s, color, c.g.n);
    else
      c.acc = add(c.acc, color);
    c.s++;
  }
  // the fold (chain_fold_kernel) and the continuations
  int n_cont = 0;
  for (uint32_t p : split) {
    const b1::ChainPx &P = px[p];
    uint64_t w = seg[P.end0];
    if ((w & b1::kEndEnded) && (w & b1::kEndNoLink)) continue;
    if (!(w & b1::kEndEnded)) {
      fprintf(stderr, "pixel %u: segment 0 never ended\n", p);
      return 3;
    }
    // the links must reach forward through ended segments (a protocol bug otherwise)
    for (uint32_t t = b1::end_t(w), it = 0; !(w & b1::kEndNoLink) && it < P.K; it++) {
      if (t == 0 || t >= P.K) {
        fprintf(stderr, "pixel %u: bad link %u\n", p, t);
        return 3;
      }
      w = seg[P.end0 + t];
      if (!(w & b1::kEndEnded)) {
        fprintf(stderr, "pixel %u: segment %u never ended\n", p, t);
        return 3;
      }
      t = b1::end_t(w);
    }
    b1::ChainCont q;  // the kernel's fold (chain_fold_kernel: chain_fold_px) into the image
    if (b1::chain_fold_px(V, p, img.data(), q)) continue;
    n_cont++;  // continuation: the true chain from (o, s, acc)
    f3 acc = mk(q.acc[0], q.acc[1], q.acc[2]);
    Pcg32 g;
    g.seed((uint64_t)(17 + p / W), (uint64_t)(23 + p % W));
    g.skip(q.o);
    for (uint32_t total = q.s; total < (uint32_t)spp; total++) acc = add(acc, sample(view, (int)p, g));
    b1::write_pixel(&img[(size_t)p * 3], acc, spp);
  }
  FILE *f = fopen(argv[5], "wb");
  fwrite(img.data(), 1, img.size(), f);
  fclose(f);
  printf("%d %d split=%zu chains=%zu samples=%ld (x%.3f) continuations=%d\n", W, H, split.size(),
         chains.size(), samples, (double)samples / ((double)npix * spp), n_cont);
  rt_flat_free(s);
  return 0;
}
