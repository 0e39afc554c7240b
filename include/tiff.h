/* tiff.h — drop-in for ray-tracing-c include/tiff.h (reference include/tiff.h:1-9).
 *
 * Baseline uncompressed little-endian TIFF, one strip, byte-identical to the reference writer
 * (reference src/tiff.c:15-49): 8-byte header, 11 IFD entries, 8-bit samples, 72/1 dpi, pixel data
 * at offset 146 + 2*n_channels + 16.  Returns 0, or 1 for channel counts other than 1 and 3.
 */
#ifndef RT_TIFF_H
#define RT_TIFF_H
#ifndef TIFF_H
#define TIFF_H
#endif

#include <stdint.h>
#include <stdio.h>

int write_tiff(FILE *f, int width, int height, int n_channels, uint8_t *buffer);

#endif /* RT_TIFF_H */
