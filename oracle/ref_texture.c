/* ref_texture.c — TEST INFRASTRUCTURE (oracle).  Never linked into the product.
 *
 * Restatement of the reference's src/texture.c for the reference build in oracle/_ref/.
 * Why it exists: reference src/texture.c:5-6 includes "stb_image.h" from the `stb` git submodule,
 * which is empty in /root/reference (.gitmodules:1-3), so that one file cannot be compiled here.
 * The other eight reference sources compile from where they lie (oracle/Makefile); this file
 * supplies the texture API they link against, written against the REFERENCE headers
 * (/root/reference/include/texture.h) and following src/texture.c line by line:
 *   Solid_value  src/texture.c:8        Checker_value  src/texture.c:12-22
 *   Image_value  src/texture.c:28-37    Perlin_*       src/texture.c:45-114
 * Image_init: stbi_load is unavailable, so every image is the documented substitute image
 * (DESIGN.md §"Substitute earth image"); the product library uses the identical generator.
 * Scenes 0, 1 and 6 use only Solid textures: for them the reference build contains no
 * restated arithmetic at all.
 */
#include "texture.h"
#include "utils.h"
#include "vec3.h"

#include <math.h>
#include <stdint.h>
#include <stdlib.h>

static Vec3 Solid_value(const Texture *self_, float u, float v, Vec3 p) {
  (void)u, (void)v, (void)p;
  return ((const Solid *)self_)->color;
}
void Solid_init(Solid *self, Vec3 color) {
  self->texture.value = Solid_value;
  self->color = color;
}
Texture *Solid_new(Vec3 color) {
  Solid *t = my_malloc(sizeof(Solid));
  Solid_init(t, color);
  return (Texture *)t;
}

static Vec3 Checker_value(const Texture *self_, float u, float v, Vec3 p) {
  const Checker *self = (const Checker *)self_;
  int iu = (int)floorf(u / self->scale);
  int iv = (int)floorf(v / self->scale);
  Texture *pick = ((iu + iv) % 2) ? self->odd : self->even;
  return pick->value(pick, u, v, p);
}
void Checker_init(Checker *self, float scale, Texture *even, Texture *odd) {
  self->texture.value = Checker_value;
  self->scale = scale;
  self->even = even;
  self->odd = odd;
}
Texture *Checker_new(float scale, Texture *even, Texture *odd) {
  Checker *t = my_malloc(sizeof(Checker));
  Checker_init(t, scale, even, odd);
  return (Texture *)t;
}

static Vec3 Image_value(const Texture *self_, float u, float v, Vec3 p) {
  (void)p;
  const Image *self = (const Image *)self_;
  int i = (int)roundf(u * (float)(self->width - 1));
  int j = (int)roundf((1.0f - v) * (float)(self->height - 1));
  int at = ((j * self->width) + i) * 3;
  return vec3((float)self->buffer[at] / 255.0f, (float)self->buffer[at + 1] / 255.0f,
              (float)self->buffer[at + 2] / 255.0f);
}
void Image_init(Image *image, char *filename) {
  (void)filename;
  const int w = 1024, h = 512; /* substitute image: same formula as rt_substitute_image() */
  uint8_t *px = my_malloc((size_t)w * h * 3);
  for (int j = 0; j < h; j++)
    for (int i = 0; i < w; i++) {
      uint8_t *q = px + ((size_t)j * w + i) * 3;
      q[0] = (uint8_t)((i * 255) / (w - 1));
      q[1] = (uint8_t)((j * 255) / (h - 1));
      q[2] = (uint8_t)((i ^ j) & 255);
    }
  image->texture.value = Image_value;
  image->width = w;
  image->height = h;
  image->buffer = px;
}
Texture *Image_new(char *filename) {
  Image *t = my_malloc(sizeof(Image));
  Image_init(t, filename);
  return (Texture *)t;
}

static float smooth(float t) { return t * t * (3.0f - 2.0f * t); }

static float noise(const Perlin *P, Vec3 p) {
  int i = (int)floorf(p.x), j = (int)floorf(p.y), k = (int)floorf(p.z);
  float t1 = p.x - (float)i, t2 = p.y - (float)j, t3 = p.z - (float)k;
  float s1 = smooth(t1), s2 = smooth(t2), s3 = smooth(t3);
  float acc = 0;
  for (int di = 0; di < 2; di++)
    for (int dj = 0; dj < 2; dj++)
      for (int dk = 0; dk < 2; dk++) {
        Vec3 g = P->grad_field[P->perm_x[(i + di) & 255] ^ P->perm_y[(j + dj) & 255] ^ P->perm_z[(k + dk) & 255]];
        Vec3 wv = vec3(t1 - di, t2 - dj, t3 - dk);
        acc += vec3_dot(g, wv) * (di * s1 + (1 - di) * (1.0f - s1)) * (dj * s2 + (1 - dj) * (1.0f - s2)) *
               (dk * s3 + (1 - dk) * (1.0f - s3));
      }
  return acc;
}

static float turbulence(const Perlin *P, Vec3 p) {
  float acc = 0.0f, w = 1.0f;
  for (int o = 0; o < P->depth; o++) {
    acc += w * noise(P, p);
    w *= 0.5f;
    p = vec3_mul(p, 2.0f);
  }
  return fabsf(acc);
}

static Vec3 Perlin_value(const Texture *self_, float u, float v, Vec3 p) {
  (void)u, (void)v;
  const Perlin *self = (const Perlin *)self_;
  p = vec3_mul(p, self->scale);
  float m = 0.5f * (1.0f + sinf(p.z + 10.0f * turbulence(self, p)));
  return vec3(m, m, m);
}

static void shuffle(int perm[N_PERLIN], PCG32 *rng) {
  for (int i = 0; i < N_PERLIN; i++) perm[i] = i;
  for (int i = N_PERLIN - 1; i > 0; i--) {
    uint32_t t = pcg32_u32_between(rng, 0, i + 1);
    int x = perm[i];
    perm[i] = perm[t];
    perm[t] = x;
  }
}

void Perlin_init(Perlin *perlin, float scale, int depth, PCG32 *rng) {
  perlin->texture.value = Perlin_value;
  perlin->scale = scale;
  perlin->depth = depth;
  for (int i = 0; i < N_PERLIN; i++) perlin->grad_field[i] = vec3_rand_unit_vector(rng);
  shuffle(perlin->perm_x, rng);
  shuffle(perlin->perm_y, rng);
  shuffle(perlin->perm_z, rng);
}
Texture *Perlin_new(float scale, int depth, PCG32 *rng) {
  Perlin *t = my_malloc(sizeof(Perlin));
  Perlin_init(t, scale, depth, rng);
  return (Texture *)t;
}
