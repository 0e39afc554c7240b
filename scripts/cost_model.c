/* cost_model.c — CPU analysis of the per-pixel sequential chains of the headline frame.
 *
 * Renders a sample of pixels with the oracle restatement built with -DORACLE_COUNT and reports, per
 * pixel, the events of its whole spp-sample chain: pcg32 draws, rays, box tests, sphere tests.  These
 * are the quantities that bound a multi-GPU frame: a pixel's samples share one pcg32 stream, so its
 * chain is sequential; the rng offset of sample s+1 is the offset of sample s plus that sample's draw
 * count (what the stream-split render exploits).
 *
 *   make -C scripts cost_model && scripts/cost_model SCENE WIDTH SPP ROW_STEP COL_STEP > costs.tsv
 * Output: one line per pixel "i j draws rays boxes spheres" (totals over its spp samples), then
 * the per-sample draw-count histogram of the whole sample (# lines).
 */
#include <stdio.h>
#include <stdlib.h>

#include "rt_flat.h"
#include "rt_hip.h"

void oracle_count_pixel(const rt_flat_scene *S, int i, int j, long *trace);

int main(int argc, char **argv) {
  if (argc < 6) {
    fprintf(stderr, "usage: %s SCENE WIDTH SPP ROW_STEP COL_STEP\n", argv[0]);
    return 2;
  }
  const int scene = atoi(argv[1]), width = atoi(argv[2]), spp = atoi(argv[3]);
  const int rstep = atoi(argv[4]), cstep = atoi(argv[5]);
  rt_flat_scene *S = rt_scene_preset(scene, width, spp, 50);
  if (!S) return 1;
  const int W = S->camera.width, H = S->camera.height;
  const int nx = (W + cstep - 1) / cstep, ny = (H + rstep - 1) / rstep;
  long *res = calloc((size_t)nx * ny * 4, sizeof(long));
  enum { kHist = 256 };
  long hist[kHist] = {0};
#pragma omp parallel
  {
    long *tr = malloc(sizeof(long) * 4 * (size_t)spp);
    long h[kHist] = {0};
#pragma omp for schedule(dynamic, 4)
    for (long p = 0; p < (long)nx * ny; p++) {
      const int i = (int)(p % nx) * cstep, j = (int)(p / nx) * rstep;
      oracle_count_pixel(S, i, j, tr);
      long prev = 2;  // the seed's two draws
      for (int s = 0; s < spp; s++) {
        const long c = tr[4 * s] - prev;
        prev = tr[4 * s];
        h[c < kHist - 1 ? c : kHist - 1]++;
      }
      for (int q = 0; q < 4; q++) res[4 * p + q] = tr[4 * (spp - 1) + q] - (q == 0 ? 2 : 0);
    }
#pragma omp critical
    for (int k = 0; k < kHist; k++) hist[k] += h[k];
    free(tr);
  }
  for (long p = 0; p < (long)nx * ny; p++)
    printf("%d %d %ld %ld %ld %ld\n", (int)(p % nx) * cstep, (int)(p / nx) * rstep, res[4 * p], res[4 * p + 1],
           res[4 * p + 2], res[4 * p + 3]);
  for (int k = 0; k < kHist; k++)
    if (hist[k]) printf("# draws_per_sample %d %ld\n", k, hist[k]);
  return 0;
}
