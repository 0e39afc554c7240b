/* texture.h — drop-in for ray-tracing-c include/texture.h (reference include/texture.h:1-51).
 *
 * Textures keep the reference's function-pointer interface.  The `value` pointer identifies the
 * texture kind to the flattener; the values themselves are evaluated on the GPU
 * (rt_device.h, rt_texture_value), so calling `value` on the host aborts.
 *
 * Image textures: the reference decodes files with the (un-vendored) stb_image submodule.  This
 * library reads binary PPM (P6) — the format is taken from the file's content, as stb_image does —
 * and, like the reference's assert (src/texture.c:38-42), aborts on a file it cannot read.  The
 * reference's `earthmap.jpg` is not distributed; tests and benches use the documented substitute
 * picture written as a PPM under that name (rtc/earth.py).
 * Unlike the reference header this one has an include guard.
 */
#ifndef RT_TEXTURE_H
#define RT_TEXTURE_H

#include "pcg32.h"
#include "vec3.h"
#include <stdint.h>

typedef struct Texture Texture;
struct Texture {
  Vec3 (*value)(const Texture *self, float u, float v, Vec3 p);
};

typedef struct Solid {
  Texture texture;
  Vec3 color;
} Solid;

void Solid_init(Solid *self, Vec3 color);
Texture *Solid_new(Vec3 color);

/* alternates `even`/`odd` on floor(u/scale) + floor(v/scale) (reference src/texture.c:12-22) */
typedef struct Checker {
  Texture texture;
  float scale;
  Texture *even;
  Texture *odd;
} Checker;

void Checker_init(Checker *self, float scale, Texture *even, Texture *odd);
Texture *Checker_new(float scale, Texture *even, Texture *odd);

/* nearest-neighbour RGB8 lookup (reference src/texture.c:28-37) */
typedef struct Image {
  Texture texture;
  int width;
  int height;
  uint8_t *buffer;
} Image;

void Image_init(Image *self, char *filename);
Texture *Image_new(char *filename);

#define N_PERLIN 256

/* marble: 0.5 * (1 + sin(p.z + 10 * turbulence(p)))  (reference src/texture.c:47-114) */
typedef struct Perlin {
  Texture texture;
  float scale;
  int depth;
  Vec3 grad_field[N_PERLIN];
  int perm_x[N_PERLIN];
  int perm_y[N_PERLIN];
  int perm_z[N_PERLIN];
} Perlin;

void Perlin_init(Perlin *self, float scale, int depth, PCG32 *rng);
Texture *Perlin_new(float scale, int depth, PCG32 *rng);

#endif /* RT_TEXTURE_H */
