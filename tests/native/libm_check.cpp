// libm_check — exhaustive host-side check of ray-tracing-c_amd/csrc/rt_libm.h against the host
// glibc that the reference links (test infrastructure; see tests/test_libm_port.py).
// Usage: libm_check <fn> [lo_bits hi_bits]   fn in {sincos_phi, sincos_all, pow5, logf_f32, logf_all}
// Prints "<fn> checked=<n> mismatches=<m> hash=<fnv64 of glibc results>" and exits 1 on mismatch.
#include "../../ray-tracing-c_amd/csrc/rt_libm.h"
#include <math.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <omp.h>

static uint64_t fnv_mix(uint64_t h, uint32_t v) {
  for (int b = 0; b < 4; b++) { h ^= (v >> (8 * b)) & 0xff; h *= 0x100000001b3ULL; }
  return h;
}

int main(int argc, char **argv) {
  if (argc < 2) { fprintf(stderr, "usage\n"); return 2; }
  const char *fn = argv[1];
  uint64_t lo = 0, hi = 0;
  int mode = 0;
  if (!strcmp(fn, "sincos_phi")) { mode = 0; lo = 0; hi = 1ull << 24; }
  else if (!strcmp(fn, "sincos_all")) { mode = 1; lo = 0; hi = 1ull << 32; }
  else if (!strcmp(fn, "pow5")) { mode = 2; lo = 0; hi = 0x40000001ull; }
  else if (!strcmp(fn, "logf_f32")) { mode = 3; lo = 1; hi = 1ull << 24; }
  else if (!strcmp(fn, "logf_all")) { mode = 4; lo = 0; hi = 0x80000000ull; }
  else { fprintf(stderr, "unknown fn\n"); return 2; }
  if (argc >= 4) { lo = strtoull(argv[2], 0, 0); hi = strtoull(argv[3], 0, 0); }
  const int nt = omp_get_max_threads();
  uint64_t *bad = (uint64_t *)calloc(nt, 8);
  uint64_t *hash = (uint64_t *)calloc(nt, 8);
  long long first_bad = -1;
  const uint64_t chunk = (hi - lo + nt - 1) / nt;
#pragma omp parallel
  {
    const int t = omp_get_thread_num();
    uint64_t h = 0xcbf29ce484222325ULL, nb = 0;
    const uint64_t a = lo + t * chunk, b = (a + chunk < hi) ? a + chunk : hi;
    for (uint64_t k = a; k < b; k++) {
      float x, r0, r1, p0, p1;
      switch (mode) {
      case 0: x = (2.0f * (float)M_PI) * ((float)(uint32_t)k / (float)(1 << 24)); goto sc;
      case 1: x = rtm::u2f((uint32_t)k); if (isnan(x) || isinf(x)) continue;
      sc:
        r0 = sinf(x); r1 = cosf(x);
        rtm::sincosf(x, &p0, &p1);
        h = fnv_mix(fnv_mix(h, rtm::f2u(r0)), rtm::f2u(r1));
        if (rtm::f2u(r0) != rtm::f2u(p0) || rtm::f2u(r1) != rtm::f2u(p1) || rtm::f2u(rtm::sinf(x)) != rtm::f2u(r0)) {
          nb++;
#pragma omp critical
          if (first_bad < 0) first_bad = (long long)k;
        }
        break;
      case 2:
        x = rtm::u2f((uint32_t)k); r0 = powf(x, 5.0f); p0 = rtm::powf(x, 5.0f);
        h = fnv_mix(h, rtm::f2u(r0));
        if (rtm::f2u(r0) != rtm::f2u(p0) && !(isnan(r0) && isnan(p0))) { nb++;
#pragma omp critical
          if (first_bad < 0) first_bad = (long long)k; }
        break;
      case 3: x = (float)(uint32_t)k / (float)(1 << 24); goto lg;
      case 4: x = rtm::u2f((uint32_t)k);
      lg:
        r0 = logf(x); p0 = rtm::logf(x);
        h = fnv_mix(h, rtm::f2u(r0));
        if (rtm::f2u(r0) != rtm::f2u(p0) && !(isnan(r0) && isnan(p0))) { nb++;
#pragma omp critical
          if (first_bad < 0) first_bad = (long long)k; }
        break;
      }
    }
    bad[t] = nb; hash[t] = h;
  }
  uint64_t nb = 0, H = 0xcbf29ce484222325ULL;
  for (int t = 0; t < nt; t++) { nb += bad[t]; H = fnv_mix(fnv_mix(H, (uint32_t)hash[t]), (uint32_t)(hash[t] >> 32)); }
  printf("%s checked=%llu mismatches=%llu first_bad=%lld hash=%016llx threads=%d\n", fn,
         (unsigned long long)(hi - lo), (unsigned long long)nb, first_bad, (unsigned long long)H, nt);
  return nb ? 1 : 0;
}
