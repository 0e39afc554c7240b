/* glibc_ref.c — TEST INFRASTRUCTURE: host glibc evaluations used as the truth for the device libm
 * port (tests/test_libm_port.py).  Compiled with gcc -O2, so these are the very libm calls the
 * reference makes (src/material.c:27,73; src/hittable.c:172-173,413; src/texture.c:50). */
#include <math.h>
#include <stdint.h>
void ref_sincosf(const float *x, float *out, int64_t n) {
  for (int64_t i = 0; i < n; i++) { out[2 * i] = sinf(x[i]); out[2 * i + 1] = cosf(x[i]); }
}
void ref_pow5(const float *x, float *out, int64_t n) { for (int64_t i = 0; i < n; i++) out[i] = powf(x[i], 5.0f); }
void ref_logf(const float *x, float *out, int64_t n) { for (int64_t i = 0; i < n; i++) out[i] = logf(x[i]); }
void ref_sinf(const float *x, float *out, int64_t n) { for (int64_t i = 0; i < n; i++) out[i] = sinf(x[i]); }
void ref_atan2f(const float *yx, float *out, int64_t n_pairs) { for (int64_t i = 0; i < n_pairs; i++) out[i] = atan2f(yx[2 * i], yx[2 * i + 1]); }
void ref_acosf(const float *x, float *out, int64_t n) { for (int64_t i = 0; i < n; i++) out[i] = acosf(x[i]); }
