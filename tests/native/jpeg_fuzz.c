/* TEST INFRASTRUCTURE: host/rt_jpeg.c built with AddressSanitizer, run over files given on the command
 * line (truncated / corrupted JPEGs from tests/test_host_library.py).  Every file must end in a decoded
 * image or a reported error -- never an out-of-bounds read, which ASan turns into a failing exit. */
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

uint8_t *rt_jpeg_decode(const uint8_t *buf, size_t len, int *width, int *height, char *err, size_t err_len);

int main(int argc, char **argv) {
  int ok = 0, bad = 0;
  for (int a = 1; a < argc; a++) {
    FILE *f = fopen(argv[a], "rb");
    if (!f) return 2;
    fseek(f, 0, SEEK_END);
    const long n = ftell(f);
    fseek(f, 0, SEEK_SET);
    /* exactly the file's bytes in a heap block of that size: a read past the end is caught */
    uint8_t *buf = malloc(n > 0 ? (size_t)n : 1);
    if (!buf || fread(buf, 1, (size_t)n, f) != (size_t)n) return 2;
    fclose(f);
    int w = 0, h = 0;
    char why[160] = "";
    uint8_t *rgb = rt_jpeg_decode(buf, (size_t)n, &w, &h, why, sizeof why);
    if (rgb) ok++; else bad++;
    if (argc == 2) printf("%s %d %d %s\n", rgb ? "ok" : "err", w, h, why);
    free(rgb);
    free(buf);
  }
  if (argc != 2) printf("decoded %d rejected %d\n", ok, bad);
  return 0;
}
