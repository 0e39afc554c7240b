/* rt_main.c — the drop-in CLI: same arguments, defaults, scene numbering, stderr text and
 * output file as the reference driver (reference src/main.c:275-345), rendering on the GPU.
 *
 *   rt_main <scene 0-7> [width spp _]
 * Argument quirk kept on purpose: width is read only when argc > 3 and spp only when argc > 4
 * (src/main.c:289-292), so `rt_main 1 1200 1000 _` is the 1000-spp Book-1 render.
 * Extensions (environment only, defaults unchanged): RT_NUM_GPUS=<n> limits the GPUs used,
 * RT_MAX_DEPTH=<d> overrides max_depth (BASELINE config 1 uses depth 10), RT_OUTPUT=<path>
 * changes the output file name.
 */
#include "rt_internal.h"

#include <stdio.h>
#include <stdlib.h>
#include <time.h>

int main(int argc, char *argv[]) {
  if (argc <= 1) {
    fprintf(stderr, "usage: %s <scene 0-7> [width spp _]\n", argv[0]);
    return 1;
  }
  World world = {0};
  Camera camera;
  rt_camera_defaults(&camera);
  if (argc > 3) camera.img_width = (int)strtol(argv[2], NULL, 10);
  if (argc > 4) camera.samples_per_pixel = (int)strtol(argv[3], NULL, 10);

  const char *title = rt_build_scene((int)strtol(argv[1], NULL, 10), &world, &camera);
  fprintf(stderr, "%s\n", title);
  const char *depth_env = getenv("RT_MAX_DEPTH");
  if (depth_env && *depth_env) camera.max_depth = atoi(depth_env);
  Camera_init(&camera);

  uint8_t *image = my_malloc((size_t)camera.img_width * camera.img_height * 3);
  time_t start, stop;
  time(&start);
  Camera_render(&camera, &world, image);
  time(&stop);
  fprintf(stderr, "Took %ld seconds\n", (long)(stop - start));

  const char *path = getenv("RT_OUTPUT");
  FILE *f = fopen(path && *path ? path : "output.tiff", "wb");
  if (f == NULL) {
    fprintf(stderr, "rt: cannot open output file\n");
    return 1;
  }
  write_tiff(f, camera.img_width, camera.img_height, 3, image);
  fclose(f);
  free(image);
  return 0;
}
