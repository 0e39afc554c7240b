// kernel_host_check — TEST INFRASTRUCTURE.  Runs the gfx950 kernel's per-pixel code
// (ray-tracing-c_amd/csrc/rt_device.h: render_pixel) on the CPU, built with AddressSanitizer, over
// a small frame of a reference scene, and writes raw RGB.  tests/test_kernel_logic.py compares the
// output with the oracle: this catches out-of-bounds indexing and traversal / fold logic errors
// before a kernel is ever launched on a GPU (a GPU fault can take down the whole node).
// It is not part of the product and is never linked into librtc_amd.so.
//   kernel_host_check <scene> <width> <spp> <depth> <out.rgb> [variant: book1|all]
#include "../../ray-tracing-c_amd/csrc/rt_device.h"
#include "../../include/rt_hip.h"

#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <vector>

int main(int argc, char **argv) {
  if (argc < 6) {
    fprintf(stderr, "usage: kernel_host_check <scene> <width> <spp> <depth> <out.rgb> [book1|all]\n");
    return 2;
  }
  rt_flat_scene *s = rt_scene_preset(atoi(argv[1]), atoi(argv[2]), atoi(argv[3]), atoi(argv[4]));
  if (!s) {
    fprintf(stderr, "preset failed: %s\n", rt_last_error());
    return 1;
  }
  const bool use_pre = argc > 6 && !strcmp(argv[6], "pre");  // preorder trace (trace_pre)
  const bool force_all = argc > 6 && (!strcmp(argv[6], "all") || use_pre);
  const bool book1 = !force_all && (s->features & ~rt::kFeatBook1) == 0;
  if (s->stack_needed > rt::kStackMax || s->camera.max_depth > rt::kMaxDepth) {
    fprintf(stderr, "scene exceeds kernel limits\n");
    return 1;
  }
  const void *arrays[13] = {s->bvh,        s->spheres,  s->quads,     s->lists,  s->list_items,
                            s->translates, s->rotates,  s->media,     s->materials, s->textures,
                            s->images,     s->perlins,  s->image_bytes};
  rt::DScene view = rt::make_view(*s, arrays);
  std::vector<float4> pre;
  if (use_pre) {
    rt::build_preorder(*s, pre);
    view.pre = pre.data();
    view.n_pre = (int32_t)(pre.size() / 2);
  }
  const int W = s->camera.width, H = s->camera.height;
  std::vector<uint8_t> img((size_t)W * H * 3);
#pragma omp parallel for schedule(dynamic, 16)
  for (int p = 0; p < W * H; p++) {
    if (book1)
      rt::render_pixel<rt::kFeatBook1>(view, p % W, p / W, &img[(size_t)p * 3]);
    else
      rt::render_pixel<rt::kFeatAll>(view, p % W, p / W, &img[(size_t)p * 3]);
  }
  FILE *f = fopen(argv[5], "wb");
  fwrite(img.data(), 1, img.size(), f);
  fclose(f);
  printf("%d %d %s\n", W, H, book1 ? "book1" : use_pre ? "pre" : "all");
  rt_flat_free(s);
  return 0;
}
