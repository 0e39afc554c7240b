/* rt_jpeg.c — baseline JPEG decoding for Image_new (host side, once per scene).
 *
 * The reference's Image_init (src/texture.c:38-42) loads its picture with stb_image's
 * stbi_load(filename, &w, &h, NULL, 3) from the un-vendored `stb` submodule (.gitmodules:1-3).  This
 * is a restatement of stb_image's published JPEG decoding arithmetic, so that a real earthmap.jpg
 * renders instead of failing:
 *   - baseline / extended Huffman frames (SOF0, SOF1), 8-bit samples, 1 or 3 components, any
 *     sampling factors up to 4x4, restart intervals; progressive and arithmetic-coded frames are
 *     reported as unsupported (NULL);
 *   - dequantised coefficients stored as 16-bit integers, the 12-bit fixed-point separable integer
 *     IDCT with its column shortcut and rounding (+512 >> 10, then +65536 + (128 << 17) >> 17);
 *   - chroma upsampling by stb's filters: h2v1 and h1v2 triangle (3*near + far + 2) >> 2, h2v2
 *     (3*near + far per column, then (3*a + b + 8) >> 4), nearest for other factors;
 *   - YCbCr -> RGB in 20-bit fixed point (float2fixed(x) = (int)(x * 4096 + 0.5) << 8, the Cb term
 *     of green masked to its upper 16 bits), clamped; an Adobe transform-0 three-component frame is
 *     RGB already; a grey frame expands to (y, y, y).
 * Parity with the reference for a real JPEG is unpinned (no stb and no JPEG asset exist in this
 * environment; tests/test_host_library.py checks the decoder against an independent JPEG codec
 * within a small tolerance).  The hot path never sees this: Image texels reach the GPU as bytes.
 */
#include "rt_internal.h"

#include <stdio.h>
#include <stdlib.h>
#include <string.h>

typedef struct {
  uint8_t bits[16];
  uint8_t vals[256];
  int n;
  /* canonical decode: per length L (1..16), the first code of that length, the index of its first
   * value, and the largest code of that length (-1: none) */
  int first[17], index[17], maxcode[18];
} Huff;

typedef struct {
  int id, h, v, tq, td, ta;
  int bw, bh;     /* blocks per line / column in the padded MCU grid */
  uint8_t *data;  /* decoded samples, bw*8 x bh*8 */
  int dc;
} Comp;

typedef struct {
  const uint8_t *p, *end;
  uint32_t acc;
  int nbits;
  int marker;  /* a marker met inside entropy-coded data (then zeros are fed) */
  uint16_t q[4][64];
  Huff hd[4], ha[4];
  Comp c[3];
  int nc, w, h, hmax, vmax, restart, adobe, transform, jfif;
} Jpeg;

static const uint8_t kZigzag[64 + 15] = {
    0,  1,  8,  16, 9,  2,  3,  10, 17, 24, 32, 25, 18, 11, 4,  5,  12, 19, 26, 33, 40, 48,
    41, 34, 27, 20, 13, 6,  7,  14, 21, 28, 35, 42, 49, 56, 57, 50, 43, 36, 29, 22, 15, 23,
    30, 37, 44, 51, 58, 59, 52, 45, 38, 31, 39, 46, 53, 60, 61, 54, 47, 55, 62, 63,
    63, 63, 63, 63, 63, 63, 63, 63, 63, 63, 63, 63, 63, 63, 63}; /* (padding: a bad run stays in range) */

static int rd16(const uint8_t *p) { return (p[0] << 8) | p[1]; }

static int huff_build(Huff *t) {
  int code = 0, k = 0;
  for (int len = 1; len <= 16; len++) {
    t->first[len] = code;
    t->index[len] = k;
    code += t->bits[len - 1];
    k += t->bits[len - 1];
    t->maxcode[len] = t->bits[len - 1] ? code - 1 : -1;
    if (code > (1 << len)) return 0; /* over-subscribed */
    code <<= 1;
  }
  t->maxcode[17] = 0x7fffffff;
  return k == t->n;
}

/* entropy-coded bits, with 0xFF00 stuffing; a marker stops the input (zeros follow) */
static void fill(Jpeg *j) {
  while (j->nbits <= 24) {
    int b = 0;
    if (!j->marker && j->p < j->end) {
      b = *j->p++;
      if (b == 0xff) {
        int c = j->p < j->end ? *j->p : 0;
        while (c == 0xff && j->p + 1 < j->end) c = *++j->p; /* fill bytes */
        if (c != 0) {
          j->marker = c;  /* (j->p moves past the marker's code) */
          j->p++;
          b = 0;
        } else {
          j->p++;
        }
      }
    }
    j->acc |= (uint32_t)b << (24 - j->nbits);
    j->nbits += 8;
  }
}
static int getbits(Jpeg *j, int n) {
  if (n == 0) return 0;
  fill(j);
  const int v = (int)(j->acc >> (32 - n));
  j->acc <<= n;
  j->nbits -= n;
  return v;
}
static int decode_huff(Jpeg *j, const Huff *t) {
  fill(j);
  int code = 0;
  for (int len = 1; len <= 16; len++) {
    code = (code << 1) | (int)(j->acc >> 31);
    j->acc <<= 1;
    j->nbits--;
    if (t->maxcode[len] >= 0 && code <= t->maxcode[len]) return t->vals[t->index[len] + code - t->first[len]];
  }
  return -1;
}
/* the JPEG sign extension of an n-bit magnitude category */
static int extend(int v, int n) { return n == 0 ? 0 : (v < (1 << (n - 1)) ? v - (1 << n) + 1 : v); }

static int decode_block(Jpeg *j, Comp *c, short out[64]) {
  memset(out, 0, 64 * sizeof(short));
  const uint16_t *dq = j->q[c->tq];
  const int t = decode_huff(j, &j->hd[c->td]);
  if (t < 0 || t > 15) return 0;
  const int diff = extend(getbits(j, t), t);
  c->dc += diff;
  out[0] = (short)(c->dc * dq[0]);
  for (int k = 1; k < 64;) {
    const int rs = decode_huff(j, &j->ha[c->ta]);
    if (rs < 0) return 0;
    const int r = rs >> 4, s = rs & 15;
    if (s == 0) {
      if (r != 15) break; /* end of block */
      k += 16;
      continue;
    }
    k += r;
    if (k > 63) return 0;
    out[kZigzag[k]] = (short)(extend(getbits(j, s), s) * dq[k]);
    k++;
  }
  return 1;
}

/* 12-bit fixed-point separable IDCT (the integer IDCT stb_image uses) */
#define F2F(x) ((int)((x) * 4096 + 0.5))
#define FSH(x) ((x) * 4096)
#define IDCT_1D(s0, s1, s2, s3, s4, s5, s6, s7)                                                    \
  int t0, t1, t2, t3, p1, p2, p3, p4, p5, x0, x1, x2, x3;                                        \
  p2 = s2;                                                                                       \
  p3 = s6;                                                                                       \
  p1 = (p2 + p3) * F2F(0.5411961f);                                                              \
  t2 = p1 + p3 * F2F(-1.847759065f);                                                             \
  t3 = p1 + p2 * F2F(0.765366865f);                                                              \
  p2 = s0;                                                                                       \
  p3 = s4;                                                                                       \
  t0 = FSH(p2 + p3);                                                                             \
  t1 = FSH(p2 - p3);                                                                             \
  x0 = t0 + t3;                                                                                  \
  x3 = t0 - t3;                                                                                  \
  x1 = t1 + t2;                                                                                  \
  x2 = t1 - t2;                                                                                  \
  t0 = s7;                                                                                       \
  t1 = s5;                                                                                       \
  t2 = s3;                                                                                       \
  t3 = s1;                                                                                       \
  p3 = t0 + t2;                                                                                  \
  p4 = t1 + t3;                                                                                  \
  p1 = t0 + t3;                                                                                  \
  p2 = t1 + t2;                                                                                  \
  p5 = (p3 + p4) * F2F(1.175875602f);                                                            \
  t0 = t0 * F2F(0.298631336f);                                                                   \
  t1 = t1 * F2F(2.053119869f);                                                                   \
  t2 = t2 * F2F(3.072711026f);                                                                   \
  t3 = t3 * F2F(1.501321110f);                                                                   \
  p1 = p5 + p1 * F2F(-0.899976223f);                                                             \
  p2 = p5 + p2 * F2F(-2.562915447f);                                                             \
  p3 = p3 * F2F(-1.961570560f);                                                                  \
  p4 = p4 * F2F(-0.390180644f);                                                                  \
  t3 += p1 + p4;                                                                                 \
  t2 += p2 + p3;                                                                                 \
  t1 += p2 + p4;                                                                                 \
  t0 += p1 + p3;

static uint8_t clamp8(int x) { return (unsigned)x > 255 ? (x < 0 ? 0 : 255) : (uint8_t)x; }

static void idct_block(uint8_t *out, int stride, const short in[64]) {
  int val[64];
  for (int i = 0; i < 8; i++) { /* columns */
    const short *d = in + i;
    int *v = val + i;
    if (d[8] == 0 && d[16] == 0 && d[24] == 0 && d[32] == 0 && d[40] == 0 && d[48] == 0 && d[56] == 0) {
      const int dc = d[0] * 4;
      v[0] = v[8] = v[16] = v[24] = v[32] = v[40] = v[48] = v[56] = dc;
    } else {
      IDCT_1D(d[0], d[8], d[16], d[24], d[32], d[40], d[48], d[56])
      x0 += 512, x1 += 512, x2 += 512, x3 += 512;
      v[0] = (x0 + t3) >> 10;
      v[56] = (x0 - t3) >> 10;
      v[8] = (x1 + t2) >> 10;
      v[48] = (x1 - t2) >> 10;
      v[16] = (x2 + t1) >> 10;
      v[40] = (x2 - t1) >> 10;
      v[24] = (x3 + t0) >> 10;
      v[32] = (x3 - t0) >> 10;
    }
  }
  for (int i = 0; i < 8; i++) { /* rows: the 1 << 17 scale removed with rounding, and the +128 level shift */
    const int *v = val + 8 * i;
    uint8_t *o = out + i * stride;
    IDCT_1D(v[0], v[1], v[2], v[3], v[4], v[5], v[6], v[7])
    x0 += 65536 + (128 << 17);
    x1 += 65536 + (128 << 17);
    x2 += 65536 + (128 << 17);
    x3 += 65536 + (128 << 17);
    o[0] = clamp8((x0 + t3) >> 17);
    o[7] = clamp8((x0 - t3) >> 17);
    o[1] = clamp8((x1 + t2) >> 17);
    o[6] = clamp8((x1 - t2) >> 17);
    o[2] = clamp8((x2 + t1) >> 17);
    o[5] = clamp8((x2 - t1) >> 17);
    o[3] = clamp8((x3 + t0) >> 17);
    o[4] = clamp8((x3 - t0) >> 17);
  }
}

/* between restart intervals: the RSTn marker (the rest of the bit buffer is padding) */
static int restart(Jpeg *j) {
  if (!j->marker)
    for (; j->p + 1 < j->end; j->p++)
      if (j->p[0] == 0xff && j->p[1] != 0 && j->p[1] != 0xff) {
        j->marker = j->p[1];
        j->p += 2;
        break;
      }
  if (j->marker < 0xd0 || j->marker > 0xd7) return 0;
  j->marker = 0, j->acc = 0, j->nbits = 0;
  for (int k = 0; k < j->nc; k++) j->c[k].dc = 0;
  return 1;
}

static int decode_scan(Jpeg *j, const int *order, int ns) {
  const int mw = (j->w + 8 * j->hmax - 1) / (8 * j->hmax), mh = (j->h + 8 * j->vmax - 1) / (8 * j->vmax);
  short blk[64];
  int todo = j->restart ? j->restart : 0x7fffffff;
  if (ns == 1) { /* non-interleaved: the component's own block grid, only its real blocks */
    Comp *c = &j->c[order[0]];
    const int cw = (j->w * c->h + j->hmax - 1) / j->hmax, ch = (j->h * c->v + j->vmax - 1) / j->vmax;
    const int nbw = (cw + 7) / 8, nbh = (ch + 7) / 8;
    for (int by = 0; by < nbh; by++)
      for (int bx = 0; bx < nbw; bx++) {
        if (!decode_block(j, c, blk)) return 0;
        idct_block(c->data + (size_t)by * 8 * c->bw * 8 + bx * 8, c->bw * 8, blk);
        if (--todo <= 0 && !(by == nbh - 1 && bx == nbw - 1)) {
          if (!restart(j)) return 0;
          todo = j->restart;
        }
      }
    return 1;
  }
  for (int my = 0; my < mh; my++)
    for (int mx = 0; mx < mw; mx++) {
      for (int q = 0; q < ns; q++) {
        Comp *c = &j->c[order[q]];
        for (int y = 0; y < c->v; y++)
          for (int x = 0; x < c->h; x++) {
            if (!decode_block(j, c, blk)) return 0;
            const int bx = mx * c->h + x, by = my * c->v + y;
            idct_block(c->data + (size_t)by * 8 * c->bw * 8 + bx * 8, c->bw * 8, blk);
          }
      }
      if (--todo <= 0 && !(my == mh - 1 && mx == mw - 1)) { /* restart marker: reset the predictors */
        if (!restart(j)) return 0;
        todo = j->restart;
      }
    }
  return 1;
}

/* one output row of a component, upsampled to full width (stb_image's resamplers) */
static void upsample_row(const Comp *c, int hs, int vs, int y, int w_lo, int rows, uint8_t *out) {
  const int stride = c->bw * 8;
  if (hs == 1 && vs == 1) {
    memcpy(out, c->data + (size_t)y * stride, (size_t)w_lo);
    return;
  }
  if (hs == 2 && vs == 2) {
    const int near = y >> 1;
    int far = (y & 1) ? near + 1 : near - 1;
    if (far < 0) far = 0;
    if (far > rows - 1) far = rows - 1;
    const uint8_t *a = c->data + (size_t)near * stride, *b = c->data + (size_t)far * stride;
    if (w_lo == 1) {
      out[0] = out[1] = (uint8_t)((3 * a[0] + b[0] + 2) >> 2);
      return;
    }
    int t1 = 3 * a[0] + b[0], t0;
    out[0] = (uint8_t)((t1 + 2) >> 2);
    for (int i = 1; i < w_lo; i++) {
      t0 = t1;
      t1 = 3 * a[i] + b[i];
      out[i * 2 - 1] = (uint8_t)((3 * t0 + t1 + 8) >> 4);
      out[i * 2] = (uint8_t)((3 * t1 + t0 + 8) >> 4);
    }
    out[w_lo * 2 - 1] = (uint8_t)((t1 + 2) >> 2);
    return;
  }
  if (hs == 2 && vs == 1) {
    const uint8_t *in = c->data + (size_t)y * stride;
    if (w_lo == 1) {
      out[0] = out[1] = in[0];
      return;
    }
    out[0] = in[0];
    out[1] = (uint8_t)((in[0] * 3 + in[1] + 2) >> 2);
    int i;
    for (i = 1; i < w_lo - 1; i++) {
      const int n = 3 * in[i] + 2;
      out[i * 2] = (uint8_t)((n + in[i - 1]) >> 2);
      out[i * 2 + 1] = (uint8_t)((n + in[i + 1]) >> 2);
    }
    out[i * 2] = (uint8_t)((in[w_lo - 2] * 3 + in[w_lo - 1] + 2) >> 2);
    out[i * 2 + 1] = in[w_lo - 1];
    return;
  }
  if (hs == 1 && vs == 2) {
    const int near = y >> 1;
    int far = (y & 1) ? near + 1 : near - 1;
    if (far < 0) far = 0;
    if (far > rows - 1) far = rows - 1;
    const uint8_t *a = c->data + (size_t)near * stride, *b = c->data + (size_t)far * stride;
    for (int i = 0; i < w_lo; i++) out[i] = (uint8_t)((3 * a[i] + b[i] + 2) >> 2);
    return;
  }
  const uint8_t *in = c->data + (size_t)(y / vs) * stride; /* other factors: nearest */
  for (int i = 0; i < w_lo; i++)
    for (int k = 0; k < hs; k++) out[i * hs + k] = in[i];
}

static int fixed20(float x) { return ((int)(x * 4096.0f + 0.5f)) << 8; }

uint8_t *rt_jpeg_decode(const uint8_t *buf, size_t len, int *width, int *height, char *err, size_t err_len) {
  Jpeg *j = calloc(1, sizeof *j);
  uint8_t *rgb = NULL, *rows = NULL;
  const char *why = "not a JPEG file";
  if (!j) return NULL;
  const uint8_t *p = buf, *end = buf + len;
  int have_frame = 0, decoded = 0; /* decoded: bit k set once component k's scan is done */
  if (len < 4 || p[0] != 0xff || p[1] != 0xd8) goto fail;
  p += 2;
  for (;;) {
    while (p < end && *p != 0xff) p++; /* (garbage between segments) */
    while (p < end && *p == 0xff) p++;
    if (p >= end) {
      why = "truncated JPEG (no image data)";
      goto fail;
    }
    const int m = *p++;
    if (m == 0xd9) { /* EOI: an image whose components came in separate scans is complete here */
      if (have_frame && decoded == (1 << j->nc) - 1) break;
      why = decoded ? "JPEG ends before every component was scanned" : "JPEG without a scan";
      goto fail;
    }
    if (m >= 0xd0 && m <= 0xd7) continue;
    if (p + 2 > end) goto fail;
    const int L = rd16(p);
    const uint8_t *seg = p + 2, *next = p + L;
    if (L < 2 || next > end) {
      why = "corrupt JPEG segment";
      goto fail;
    }
    /* every read below stays inside [seg, next): tables and headers are checked against L first */
    why = "corrupt JPEG segment";
    if (m == 0xdb) { /* DQT */
      for (const uint8_t *q = seg; q < next;) {
        const int pq = *q >> 4, tq = *q & 15;
        q++;
        if (tq > 3 || pq > 1 || q + (pq ? 128 : 64) > next) goto fail;
        for (int k = 0; k < 64; k++) j->q[tq][k] = (uint16_t)(pq ? rd16(q + 2 * k) : q[k]);
        q += pq ? 128 : 64;
      }
    } else if (m == 0xc4) { /* DHT */
      for (const uint8_t *q = seg; q < next;) {
        const int tc = *q >> 4, th = *q & 15;
        q++;
        if (tc > 1 || th > 3 || q + 16 > next) goto fail;
        Huff *t = tc ? &j->ha[th] : &j->hd[th];
        int n = 0;
        for (int k = 0; k < 16; k++) n += (t->bits[k] = q[k]);
        q += 16;
        if (n > 256 || q + n > next) goto fail;
        t->n = n;
        memcpy(t->vals, q, (size_t)n);
        q += n;
        if (!huff_build(t)) {
          why = "bad Huffman table";
          goto fail;
        }
      }
    } else if (m == 0xdd) { /* DRI */
      if (L < 4) goto fail;
      j->restart = rd16(seg);
    } else if (m == 0xe0 && L >= 7 && !memcmp(seg, "JFIF", 5)) { /* APP0 JFIF: YCbCr */
      j->jfif = 1;
    } else if (m == 0xee && L >= 14 && !memcmp(seg, "Adobe", 5)) { /* APP14: colour transform flag */
      j->adobe = 1;
      j->transform = seg[11];
    } else if (m == 0xc0 || m == 0xc1) { /* SOF0 / SOF1: baseline, extended Huffman */
      if (have_frame || L < 8) goto fail; /* (one frame per image) */
      if (seg[0] != 8) {
        why = "JPEG with other than 8-bit samples";
        goto fail;
      }
      j->h = rd16(seg + 1);
      j->w = rd16(seg + 3);
      j->nc = seg[5];
      if (j->w <= 0 || j->h <= 0 || (j->nc != 1 && j->nc != 3)) {
        why = "unsupported JPEG frame (size or component count)";
        goto fail;
      }
      if (L < 8 + 3 * j->nc) goto fail;
      j->hmax = j->vmax = 1;
      for (int k = 0; k < j->nc; k++) {
        Comp *c = &j->c[k];
        c->id = seg[6 + 3 * k];
        c->h = seg[7 + 3 * k] >> 4;
        c->v = seg[7 + 3 * k] & 15;
        c->tq = seg[8 + 3 * k];
        if (c->h < 1 || c->h > 4 || c->v < 1 || c->v > 4 || c->tq > 3) goto fail;
        if (c->h > j->hmax) j->hmax = c->h;
        if (c->v > j->vmax) j->vmax = c->v;
      }
      /* the upsamplers need whole ratios (stb_image rejects the others: "bad H" / "bad V") */
      for (int k = 0; k < j->nc; k++)
        if (j->hmax % j->c[k].h || j->vmax % j->c[k].v) {
          why = "unsupported JPEG sampling factors (not whole ratios)";
          goto fail;
        }
      const int mw = (j->w + 8 * j->hmax - 1) / (8 * j->hmax), mh = (j->h + 8 * j->vmax - 1) / (8 * j->vmax);
      for (int k = 0; k < j->nc; k++) {
        Comp *c = &j->c[k];
        c->bw = mw * c->h;
        c->bh = mh * c->v;
        c->data = calloc((size_t)c->bw * 8 * c->bh * 8, 1);
        if (!c->data) {
          why = "out of memory";
          goto fail;
        }
      }
      have_frame = 1;
    } else if (m >= 0xc2 && m <= 0xcf && m != 0xc4 && m != 0xc8 && m != 0xcc) {
      why = "unsupported JPEG coding (progressive, lossless or arithmetic)";
      goto fail;
    } else if (m == 0xda) { /* SOS */
      if (!have_frame || L < 3) goto fail;
      const int ns = seg[0];
      int order[3];
      if (ns < 1 || ns > j->nc || L < 6 + 2 * ns) goto fail;
      for (int q = 0; q < ns; q++) {
        const int id = seg[1 + 2 * q];
        int k = 0;
        while (k < j->nc && j->c[k].id != id) k++;
        if (k == j->nc) goto fail;
        order[q] = k;
        j->c[k].td = seg[2 + 2 * q] >> 4;
        j->c[k].ta = seg[2 + 2 * q] & 15;
        if (j->c[k].td > 3 || j->c[k].ta > 3) goto fail;
        j->c[k].dc = 0;
      }
      j->p = next;
      j->end = end;
      j->acc = 0, j->nbits = 0, j->marker = 0;
      if (!decode_scan(j, order, ns)) {
        why = "corrupt JPEG entropy-coded data";
        goto fail;
      }
      for (int q = 0; q < ns; q++) decoded |= 1 << order[q];
      if (decoded == (1 << j->nc) - 1) break; /* every component decoded: the image is complete */
      /* non-interleaved scans follow one another: resume the segment walk at the marker after this scan */
      p = j->marker ? j->p - 2 : j->p;
      while (p + 1 < end && !(p[0] == 0xff && p[1] != 0 && p[1] != 0xff && !(p[1] >= 0xd0 && p[1] <= 0xd7))) p++;
      continue;
    }
    p = next;
  }
  /* colour conversion of the full-size rows */
  {
    const int W = j->w, H = j->h;
    rgb = malloc((size_t)W * H * 3);
    rows = malloc((size_t)W * 4 * 3 + 64);
    if (!rgb || !rows) goto fail;
    uint8_t *line[3] = {rows, rows + W + 16, rows + 2 * (W + 16)};
    const int cr_r = fixed20(1.40200f), cr_g = -fixed20(0.71414f), cb_g = -fixed20(0.34414f), cb_b = fixed20(1.77200f);
    for (int y = 0; y < H; y++) {
      for (int k = 0; k < j->nc; k++) {
        const Comp *c = &j->c[k];
        const int hs = j->hmax / c->h, vs = j->vmax / c->v;
        const int w_lo = (W + hs - 1) / hs, rows_lo = (H + vs - 1) / vs;
        upsample_row(c, hs, vs, y, w_lo, rows_lo, line[k]);
      }
      uint8_t *o = rgb + (size_t)y * W * 3;
      if (j->nc == 1) {
        for (int x = 0; x < W; x++) o[3 * x] = o[3 * x + 1] = o[3 * x + 2] = line[0][x];
      } else if ((j->c[0].id == 'R' && j->c[1].id == 'G' && j->c[2].id == 'B') ||
                 (j->adobe && j->transform == 0 && !j->jfif)) { /* stored as RGB */
        for (int x = 0; x < W; x++) o[3 * x] = line[0][x], o[3 * x + 1] = line[1][x], o[3 * x + 2] = line[2][x];
      } else {
        for (int x = 0; x < W; x++) {
          const int yf = (line[0][x] << 20) + (1 << 19);
          const int cr = line[2][x] - 128, cb = line[1][x] - 128;
          const int r = (yf + cr * cr_r) >> 20;
          const int g = (yf + cr * cr_g + ((cb * cb_g) & -65536)) >> 20;
          const int b = (yf + cb * cb_b) >> 20;
          o[3 * x] = clamp8(r), o[3 * x + 1] = clamp8(g), o[3 * x + 2] = clamp8(b);
        }
      }
    }
    *width = W;
    *height = H;
  }
  free(rows);
  for (int k = 0; k < 3; k++) free(j->c[k].data);
  free(j);
  return rgb;
fail:
  if (err && err_len) snprintf(err, err_len, "%s", why);
  free(rgb);
  free(rows);
  for (int k = 0; k < 3; k++) free(j->c[k].data);
  free(j);
  return NULL;
}
