/* stb_image.h — TEST INFRASTRUCTURE (oracle).  Never linked into the product.
 *
 * What this is: a restatement of the part of a THIRD-PARTY dependency that the reference's
 * src/texture.c uses.  The reference includes "stb_image.h" from the `stb` git submodule
 * (nothings/stb, /root/reference/.gitmodules:1-3), which is un-vendored (the directory is empty and
 * its pinned commit is not recoverable from the mount).  Only the reference's own sources are
 * compiled by oracle/Makefile; this header stands in for the submodule so that src/texture.c builds
 * UNCHANGED where it lies.
 *
 * Restated API (stb_image's published interface, stb_image.h "PRIMARY API"):
 *   unsigned char *stbi_load(char const *filename, int *x, int *y, int *channels_in_file,
 *                            int desired_channels);
 *     - opens `filename` in binary mode; returns NULL when it cannot be opened or decoded
 *       (the reference then asserts "Unable to read image", src/texture.c:38-42);
 *     - the format is detected from the file's CONTENT (magic), never from its name;
 *     - returns x*y*desired_channels bytes, rows top to bottom, channels interleaved, 8 bit.
 *   void stbi_image_free(void *retval_from_stbi_load);
 * Formats restated: PNM only (stb_image's "PNM (PPM and PGM binary only)" loader): "P6" (RGB) and
 * "P5" (grey), maxval <= 255, '#' comments and whitespace in the header, a single whitespace byte
 * after maxval.  Grey expands to RGB as (g, g, g), as stbi__convert_format does.  JPEG/PNG/... are
 * not restated: the earth-texture scenes (3, 7) are run with the documented substitute picture
 * stored as a binary PPM file named earthmap.jpg (rtc/earth.py writes it).
 */
#ifndef ORACLE_STB_IMAGE_H
#define ORACLE_STB_IMAGE_H

/* the real header's implementation section includes these (texture.c relies on math.h via it) */
#include <math.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#ifdef STB_IMAGE_IMPLEMENTATION
static int stbi_oracle_skip_ws(FILE *f) {
  int c = fgetc(f);
  for (;;) {
    while (c == ' ' || c == '\t' || c == '\n' || c == '\r' || c == '\v' || c == '\f') c = fgetc(f);
    if (c != '#') return c;
    while (c != EOF && c != '\n' && c != '\r') c = fgetc(f);
  }
}

static int stbi_oracle_int(FILE *f, int *out) {
  int c = stbi_oracle_skip_ws(f), v = 0, n = 0;
  while (c >= '0' && c <= '9' && v < (1 << 24)) v = v * 10 + (c - '0'), n++, c = fgetc(f);
  *out = v;
  return n > 0 && (c == ' ' || c == '\t' || c == '\n' || c == '\r' || c == '\v' || c == '\f');
}

static unsigned char *stbi_load(char const *filename, int *x, int *y, int *comp, int req_comp) {
  FILE *f = fopen(filename, "rb");
  if (!f) return NULL;
  unsigned char *out = NULL;
  int w = 0, h = 0, maxv = 0;
  const int m0 = fgetc(f), m1 = fgetc(f);
  const int src_n = (m0 == 'P' && m1 == '6') ? 3 : (m0 == 'P' && m1 == '5') ? 1 : 0;
  if (src_n && stbi_oracle_int(f, &w) && stbi_oracle_int(f, &h) && stbi_oracle_int(f, &maxv) && w > 0 && h > 0 &&
      maxv > 0 && maxv <= 255) {
    const int n = req_comp ? req_comp : src_n;
    const size_t npx = (size_t)w * (size_t)h;
    unsigned char *raw = (unsigned char *)malloc(npx * src_n);
    out = raw ? (unsigned char *)malloc(npx * n) : NULL;
    if (out && fread(raw, 1, npx * src_n, f) == npx * src_n) {
      for (size_t p = 0; p < npx; p++)
        for (int k = 0; k < n; k++) {  /* stbi__convert_format: grey -> (g,g,g), alpha = 255 */
          const int alpha = (n == 2 && k == 1) || (n == 4 && k == 3);
          out[p * n + k] = alpha ? 255 : src_n == 3 ? raw[p * 3 + k] : raw[p];
        }
      if (x) *x = w;
      if (y) *y = h;
      if (comp) *comp = src_n;
    } else {
      free(out);
      out = NULL;
    }
    free(raw);
  }
  fclose(f);
  return out;
}

static void stbi_image_free(void *p) { free(p); }
#endif /* STB_IMAGE_IMPLEMENTATION */

#endif /* ORACLE_STB_IMAGE_H */
