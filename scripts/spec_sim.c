/* spec_sim.c — CPU study of stream-split (speculative) rendering of one pixel.
 *
 * A pixel's samples share one pcg32 stream; sample s starts at the stream offset o_s and consumes
 * D(o_s) draws, so o_{s+1} = o_s + D(o_s).  D(o) and the sample colour are pure functions of the
 * offset o, so samples can be evaluated at offsets before the chain reaches them.  This tool
 * evaluates D(o) (and rays(o)) at every offset of a pixel's stream with the oracle restatement and
 * simulates "segment" speculation: the stream is cut at offset boundaries B_k = k*L; segment k>0
 * starts one chain at every offset of [B_k, B_k+w) and chains stop when they reach an offset another
 * chain has already visited (coalescence).  Reports the extra samples evaluated and the longest
 * chain (in rays) per segment, i.e. the overhead and the latency of the split.
 *
 *   gcc -O2 -fopenmp -Iinclude scripts/spec_sim.c -o /tmp/spec_sim -lm \
 *       ray-tracing-c_amd/librtc_amd.so  (for rt_scene_preset)
 *   /tmp/spec_sim I J SPP SEGMENTS WINDOW
 */
#define ORACLE_COUNT 1
#include "../oracle/oracle.c"
#include "rt_hip.h"

#include <stdlib.h>
#include <string.h>

/* One sample of pixel (i, j) from rng state g (same arithmetic as pixel() in oracle.c). */
static void one_sample(const rt_flat_scene *S, int i, int j, Rng *g) {
  const rt_camera *c = &S->camera;
  V du = vl(c->delta_u), dv = vl(c->delta_v), lf = vl(c->origin);
  V pos = vadd(vadd(vl(c->pixel00), vscale(du, (float)i)), vscale(dv, (float)j));
  float px = rng_between(g, -0.5f, 0.5f);
  float py = rng_between(g, -0.5f, 0.5f);
  Ray r;
  if (c->dof_angle > 0.0f) {
    float a, b;
    for (;;) {
      a = rng_between(g, -1.0f, 1.0f);
      b = rng_between(g, -1.0f, 1.0f);
      if (a * a + b * b < 1.0f) break;
    }
    r.o = vadd(vadd(lf, vscale(vl(c->disc_u), a)), vscale(vl(c->disc_v), b));
  } else {
    r.o = lf;
  }
  r.d = vadd(vadd(vadd(pos, vscale(du, px)), vscale(dv, py)), vneg(r.o));
  (void)ray_color(S, &r, c->max_depth, g);
}

int main(int argc, char **argv) {
  if (argc < 6) return 2;
  const int I = atoi(argv[1]), J = atoi(argv[2]), spp = atoi(argv[3]);
  const int nseg = atoi(argv[4]), w = atoi(argv[5]);
  rt_flat_scene *S = rt_scene_preset(1, 1200, spp, 50);
  /* true chain */
  Rng g0;
  rng_seed(&g0, 17 + J, 23 + I);
  const Rng start = g0;
  long total = 0;
  {
    Rng g = g0;
    for (int s = 0; s < spp; s++) {
      cnt_draw = 0;
      one_sample(S, I, J, &g);
      total += cnt_draw;
    }
  }
  const long n = total + 4096;
  int *D = malloc(sizeof(int) * n), *R = malloc(sizeof(int) * n);
#pragma omp parallel for schedule(dynamic, 64)
  for (long o = 0; o < n; o++) {
    Rng g = start;
    /* advance o steps (slow but simple: jump by squaring) */
    uint64_t am = 6364136223846793005ULL, ac = g.inc, mul = 1, add = 0;
    for (long k = o; k; k >>= 1) {
      if (k & 1) mul *= am, add = add * am + ac;
      ac = (am + 1) * ac, am *= am;
    }
    g.state = mul * g.state + add;
    cnt_draw = cnt_ray = 0;
    one_sample(S, I, J, &g);
    D[o] = (int)cnt_draw, R[o] = (int)cnt_ray;
  }
  /* chain */
  long chain_rays = 0;
  for (long o = 0; o < total;) chain_rays += R[o], o += D[o];
  printf("pixel %d %d spp %d total_draws %ld draws/sample %.1f chain_rays %ld\n", I, J, spp, total,
         (double)total / spp, chain_rays);
  /* segment speculation */
  const long L = (total + nseg - 1) / nseg;
  char *vis = calloc(n, 1);
  long extra_samples = 0, extra_rays = 0, worst_lat = 0, misses = 0;
  for (int k = 0; k < nseg; k++) {
    const long B = k * L, E = (k + 1) * L;
    long seg_lat = 0, seg_samples = 0;
    if (k == 0) {
      for (long o = 0; o < E && o < total; o += D[o]) seg_lat += R[o], seg_samples++;
      worst_lat = seg_lat;
      continue;
    }
    /* chains advance in lockstep (one step per round); a chain stops at a visited offset */
    long cur[4096];
    long lat[4096];
    int live = 0;
    for (int q = 0; q < w && B + q < total; q++) cur[live] = B + q, lat[live] = 0, live++;
    while (live) {
      int nl = 0;
      for (int q = 0; q < live; q++) {
        long o = cur[q];
        if (o >= E || o >= total || vis[o]) continue;
        vis[o] = 1;
        seg_samples++, extra_rays += R[o];
        lat[q] += R[o];
        if (lat[q] > seg_lat) seg_lat = lat[q];
        cur[nl] = o + D[o], lat[nl] = lat[q], nl++;
      }
      live = nl;
    }
    extra_samples += seg_samples;
    if (seg_lat > worst_lat) worst_lat = seg_lat;
  }
  /* check the true chain lands in each window */
  for (long o = 0; o < total; o += D[o]) {
    long k = o / L;
    if (k > 0 && o >= k * L && o < k * L + w) {
    }
  }
  for (int k = 1; k < nseg; k++) {
    long o = 0;
    while (o < k * L) o += D[o];
    if (o >= k * L + w) misses++;
  }
  printf("segments %d window %d: evaluated %ld samples (%.2fx spp), rays %.2fx chain, worst seg latency %ld rays "
         "(%.1f%% of chain), window misses %ld\n",
         nseg, w, extra_samples + (long)(spp / nseg), (double)(extra_samples + spp / nseg) / spp,
         (double)(extra_rays) / chain_rays, worst_lat, 100.0 * worst_lat / chain_rays, misses);
  return 0;
}
