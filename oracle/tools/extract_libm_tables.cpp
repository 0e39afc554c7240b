// extract_libm_tables — BUILD/TEST INFRASTRUCTURE (not linked into the product).
//
// Provenance recipe for the table words of ray-tracing-c_amd/csrc/rt_libm.h, the bit-exact port of
// the glibc 2.35 single-precision routines on the reference's hot path (sincosf, powf, logf, atanf).
// glibc keeps these tables as hidden data in libm.so.6 (__sincosf_table, __inv_pio4,
// __powf_log2_data, __exp2f_data, __logf_data, and fdlibm's atanhi/atanlo in .rodata).  This tool
// locates each table in the host library by its first entries, dumps the whole table from there
// (C hex literals, in the port's layout) and compares every word with the port.  Exit status 0
// only if every table is found and equal word for word.
//
//   hipcc -x hip --offload-host-only -O1 -std=c++17 -I../include oracle/tools/extract_libm_tables.cpp -o /tmp/x
//   /tmp/x [/lib/x86_64-linux-gnu/libm.so.6]        (tests/test_libm_port.py runs it)
//
// The tables and the algorithms around them are glibc's (GNU LGPL v2.1 or later; the sincosf /
// powf / logf code is Szabolcs Nagy's ARM optimized-routines contribution, the atanf / acosf code
// fdlibm's, Sun Microsystems).  rt_libm.h is a derived work under the same licence: see its
// header and THIRD_PARTY.md.
#include "../../ray-tracing-c_amd/csrc/rt_libm.h"

#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <vector>

static std::vector<unsigned char> lib;

static void put(std::vector<unsigned char> &v, const void *p, size_t n) {
  const unsigned char *b = (const unsigned char *)p;
  v.insert(v.end(), b, b + n);
}

// find `want` in the library; print the table as found there and whether it equals the port
static bool check(const char *name, const std::vector<unsigned char> &want, size_t anchor_bytes, size_t word,
                  bool is_float) {
  const unsigned char *hit = nullptr;
  int hits = 0;
  for (size_t off = 0; off + want.size() <= lib.size(); off++)
    if (memcmp(&lib[off], want.data(), anchor_bytes) == 0) {
      if (!hit) hit = &lib[off];
      hits++;
    }
  if (!hit) {
    printf("%-28s NOT FOUND\n", name);
    return false;
  }
  const bool same = memcmp(hit, want.data(), want.size()) == 0;
  printf("%-28s offset 0x%zx (%d anchor hit%s), %zu words, %s\n  {", name, (size_t)(hit - lib.data()), hits,
         hits == 1 ? "" : "s", want.size() / word, same ? "IDENTICAL to rt_libm.h" : "DIFFERS from rt_libm.h");
  for (size_t k = 0; k < want.size() / word; k++) {
    if (word == 8) {
      uint64_t u;
      memcpy(&u, hit + 8 * k, 8);
      double d;
      memcpy(&d, &u, 8);
      if (is_float) printf("%s%a", k ? ", " : "", d);
      else printf("%s0x%016llx", k ? ", " : "", (unsigned long long)u);
    } else {
      uint32_t u;
      memcpy(&u, hit + 4 * k, 4);
      printf("%s0x%08x", k ? ", " : "", u);
    }
  }
  printf("}\n");
  return same;
}

int main(int argc, char **argv) {
  const char *path = argc > 1 ? argv[1] : "/lib/x86_64-linux-gnu/libm.so.6";
  FILE *f = fopen(path, "rb");
  if (!f) {
    perror(path);
    return 2;
  }
  fseek(f, 0, SEEK_END);
  lib.resize((size_t)ftell(f));
  fseek(f, 0, SEEK_SET);
  if (fread(lib.data(), 1, lib.size(), f) != lib.size()) return 2;
  fclose(f);
  bool ok = true;
  {  // __sincosf_table[2]: sincos_t {sign[4], hpi_inv, hpi, c0, c1, s1, c2, s2, c3, s3, c4}
    std::vector<unsigned char> v;
    for (int t = 0; t < 2; t++) put(v, &rtm::sincos_tab(t), sizeof(rtm::SinCosTab));
    ok &= check("__sincosf_table", v, 48, 8, true);
  }
  {  // __inv_pio4[24]
    std::vector<unsigned char> v;
    for (int i = 0; i < 24; i++) {
      const uint32_t u = rtm::inv_pio4(i);
      put(v, &u, 4);
    }
    ok &= check("__inv_pio4", v, 16, 4, false);
  }
  {  // __powf_log2_data.tab[16] = {invc, logc}
    std::vector<unsigned char> v;
    for (int i = 0; i < 16; i++) {
      const double a = rtm::powf_log2_invc(i), b = rtm::powf_log2_logc(i);
      put(v, &a, 8), put(v, &b, 8);
    }
    ok &= check("__powf_log2_data.tab", v, 32, 8, true);
  }
  {  // __exp2f_data.tab[32]
    std::vector<unsigned char> v;
    for (int i = 0; i < 32; i++) {
      const uint64_t u = rtm::exp2f_tab(i);
      put(v, &u, 8);
    }
    ok &= check("__exp2f_data.tab", v, 32, 8, false);
  }
  {  // __logf_data.tab[16] = {invc, logc} (invc shared with powf's table)
    std::vector<unsigned char> v;
    for (int i = 0; i < 16; i++) {
      const double a = rtm::powf_log2_invc(i), b = rtm::logf_logc(i);
      put(v, &a, 8), put(v, &b, 8);
    }
    ok &= check("__logf_data.tab", v, 32, 8, true);
  }
  {  // fdlibm s_atanf.c atanhi[4] / atanlo[4]: gcc spreads them over .rodata / immediates, so each
     // word is looked up on its own (the port's literals, rt_libm.h atanf)
    const uint32_t w[8] = {0x3eed6338, 0x3f490fda, 0x3f7b985e, 0x3fc90fda,
                           0x31ac3769, 0x33222168, 0x33140fb4, 0x33a22168};
    for (int k = 0; k < 8; k++) {
      int n = 0;
      for (size_t off = 0; off + 4 <= lib.size(); off++) n += memcmp(&lib[off], &w[k], 4) == 0;
      printf("atanf %s[%d] 0x%08x          %d occurrence%s\n", k < 4 ? "atanhi" : "atanlo", k & 3, w[k], n,
             n == 1 ? "" : "s");
      ok &= n > 0;
    }
  }
  printf("%s\n", ok ? "all tables identical to the host libm" : "MISMATCH");
  return ok ? 0 : 1;
}
