/* couple_sim.c — CPU study of the chain render's coupling (rt_book1.h: ChainPx), DESIGN.md §5.
 *
 * A pixel's samples share one pcg32 stream; sample s starts at the stream offset o_s and consumes
 * D(o_s) draws, so o_{s+1} = o_s + D(o_s), and D(o) and the sample's colour are pure functions of
 * o.  A chain started at an arbitrary offset B samples the same D, so it lands on an offset of the
 * true chain after a few samples (the Kruskal count).  This tool evaluates D(o) at every offset of
 * one pixel's stream with the oracle restatement, cuts the stream into K segments at even offsets
 * B_k = k * total / K, and reports per cut the garbage samples the speculative chain computes before
 * it meets the true chain ("waste") and the true chain's samples past B_k until then ("overrun").
 *
 *   gcc -O2 -fopenmp -Iinclude scripts/couple_sim.c -o /tmp/couple_sim -lm \
 *       ray-tracing-c_amd/librtc_amd.so -Wl,-rpath,$PWD/ray-tracing-c_amd
 *   /tmp/couple_sim I J SPP          (Book-1 final scene, 1200 wide)
 * Measured (1000 spp): 1-15 samples of waste per cut, K = 2..16, on sky, ground, diffuse and the
 * heaviest glass pixels (777, 458): 85 draws / 22.6 rays per sample.
 */
#define ORACLE_COUNT 1
#include "../oracle/oracle.c"
#include "rt_hip.h"
#include <stdlib.h>
#include <string.h>
static void one_sample(const rt_flat_scene *S, int i, int j, Rng *g) {
  const rt_camera *c = &S->camera;
  V du = vl(c->delta_u), dv = vl(c->delta_v), lf = vl(c->origin);
  V pos = vadd(vadd(vl(c->pixel00), vscale(du, (float)i)), vscale(dv, (float)j));
  float px = rng_between(g, -0.5f, 0.5f);
  float py = rng_between(g, -0.5f, 0.5f);
  Ray r;
  if (c->dof_angle > 0.0f) {
    float a, b;
    for (;;) { a = rng_between(g, -1.0f, 1.0f); b = rng_between(g, -1.0f, 1.0f); if (a * a + b * b < 1.0f) break; }
    r.o = vadd(vadd(lf, vscale(vl(c->disc_u), a)), vscale(vl(c->disc_v), b));
  } else r.o = lf;
  r.d = vadd(vadd(vadd(pos, vscale(du, px)), vscale(dv, py)), vneg(r.o));
  (void)ray_color(S, &r, c->max_depth, g);
}
int main(int argc, char **argv) {
  const int I = atoi(argv[1]), J = atoi(argv[2]), spp = atoi(argv[3]);
  rt_flat_scene *S = rt_scene_preset(1, 1200, spp, 50);
  Rng g0; rng_seed(&g0, 17 + J, 23 + I);
  const Rng start = g0;
  long total = 0;
  { Rng g = g0; for (int s = 0; s < spp; s++) { cnt_draw = 0; one_sample(S, I, J, &g); total += cnt_draw; } }
  const long n = total + 20000;
  int *D = malloc(sizeof(int) * n), *R = malloc(sizeof(int) * n);
#pragma omp parallel for schedule(dynamic, 64)
  for (long o = 0; o < n; o++) {
    Rng g = start;
    uint64_t am = 6364136223846793005ULL, ac = g.inc, mul = 1, add = 0;
    for (long k = o; k; k >>= 1) { if (k & 1) mul *= am, add = add * am + ac; ac = (am + 1) * ac, am *= am; }
    g.state = mul * g.state + add;
    cnt_draw = cnt_ray = 0; one_sample(S, I, J, &g); D[o] = (int)cnt_draw; R[o] = (int)cnt_ray;
  }
  char *ontrue = calloc(n, 1);
  long chain_rays = 0; int odd = 0;
  for (long o = 0; o < total; o += D[o]) ontrue[o] = 1, chain_rays += R[o], odd += D[o] & 1;
  printf("pixel %d %d total_draws %ld mu %.1f rays/sample %.2f odd-D samples %d\n", I, J, total, (double)total / spp, (double)chain_rays / spp, odd);
  for (int K = 2; K <= 16; K *= 2) {
    double waste = 0, over = 0, wrays = 0; long worst = 0; int fail = 0;
    for (int k = 1; k < K; k++) {
      long B = (long)((double)k * total / K) & ~1L;
      long o = B, ws = 0, wr = 0;
      while (o < n - 1000 && !ontrue[o]) { ws++; wr += R[o]; o += D[o]; if (ws > 5000) break; }
      if (ws > 5000) { fail++; continue; }
      long t = 0; while (t < B) t += D[t];
      long ov = 0; while (t < o) { t += D[t]; ov++; }
      waste += ws; wrays += wr; over += ov; if (ov > worst) worst = ov;
    }
    printf("  K=%2d: per cut waste %.1f samples (%.1f rays), overrun %.1f samples (worst %ld), total waste %.1f%% fails %d\n",
           K, waste / (K - 1), wrays / (K - 1), over / (K - 1), worst, 100.0 * wrays / chain_rays, fail);
  }
  return 0;
}
