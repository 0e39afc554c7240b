/* rt_tiff.c — byte-identical re-implementation of the reference TIFF writer
 * (reference src/tiff.c:15-49).  Serialised explicitly little-endian, so the bytes do not depend
 * on host struct padding or endianness.
 *
 * Layout for n channels: "II*\0" + IFD@8 | u16 11 | 11 x 12-byte entries | u32 0 |
 *   n x u16 8 (bits per sample) | 72/1 | 72/1 | pixels.
 */
#include "rt_internal.h"

#include <string.h>

static void put16(uint8_t *p, uint16_t v) {
  p[0] = (uint8_t)(v & 0xff);
  p[1] = (uint8_t)(v >> 8);
}
static void put32(uint8_t *p, uint32_t v) {
  for (int i = 0; i < 4; i++) p[i] = (uint8_t)(v >> (8 * i));
}

int write_tiff(FILE *f, int width, int height, int n_channels, uint8_t *buffer) {
  if (n_channels != 1 && n_channels != 3) {
    /* the reference has already written its 10-byte preamble and the first three entries when
     * it bails out (src/tiff.c:17-33); keep that observable behaviour */
    uint8_t pre[10 + 3 * 12];
    memcpy(pre, "II\x2A\0\x8\0\0\0", 8);
    put16(pre + 8, 11);
    const uint32_t early[3][4] = {{0x100, 3, 1, (uint32_t)width}, {0x101, 3, 1, (uint32_t)height}, {0x103, 3, 1, 1}};
    for (int e = 0; e < 3; e++) {
      put16(pre + 10 + 12 * e, (uint16_t)early[e][0]);
      put16(pre + 12 + 12 * e, (uint16_t)early[e][1]);
      put32(pre + 14 + 12 * e, early[e][2]);
      put32(pre + 18 + 12 * e, early[e][3]);
    }
    fwrite(pre, 1, sizeof pre, f);
    return 1;
  }
  const uint32_t n_entries = 11;
  const uint32_t extra = 8 + 2 + n_entries * 12 + 4; /* = 146: where the out-of-line values start */
  const uint32_t bps_at = extra, xres_at = extra + 2 * n_channels, yres_at = xres_at + 8, data_at = yres_at + 8;
  const uint32_t entries[11][3] = {
      /* tag, type, count; value below */
      {0x100, 3, 1}, {0x101, 3, 1}, {0x103, 3, 1}, {0x102, 3, (uint32_t)n_channels}, {0x106, 3, 1},
      {0x111, 3, 1}, {0x115, 3, 1}, {0x116, 3, 1}, {0x117, 4, 1},   {0x11A, 5, 1},  {0x11B, 5, 1}};
  const uint32_t values[11] = {(uint32_t)width,
                               (uint32_t)height,
                               1,
                               n_channels == 3 ? bps_at : 8,
                               n_channels == 3 ? 2u : 1u,
                               data_at,
                               (uint32_t)n_channels,
                               (uint32_t)height,
                               (uint32_t)(width * height * n_channels),
                               xres_at,
                               yres_at};
  uint8_t head[168];
  size_t k = 0;
  memcpy(head, "II\x2A\0\x8\0\0\0", 8);
  k = 8;
  put16(head + k, (uint16_t)n_entries);
  k += 2;
  for (int e = 0; e < 11; e++, k += 12) {
    put16(head + k, (uint16_t)entries[e][0]);
    put16(head + k + 2, (uint16_t)entries[e][1]);
    put32(head + k + 4, entries[e][2]);
    put32(head + k + 8, values[e]);
  }
  put32(head + k, 0);
  k += 4;
  for (int c = 0; c < n_channels; c++, k += 2) put16(head + k, 8);
  for (int r = 0; r < 2; r++, k += 8) { /* x and y resolution: 72 / 1 */
    put32(head + k, 72);
    put32(head + k + 4, 1);
  }
  fwrite(head, 1, k, f);
  fwrite(buffer, 1, (size_t)width * height * n_channels, f);
  return 0;
}
