// stack_check — TEST INFRASTRUCTURE.  The general kernel's path record (ray-tracing-c_amd/csrc/
// rt_general.h: PathRecord -- run-length albedo codes, the explicit-albedo and weight register stacks
// that overflow into the thread's global slots, the weight-2.0f bits, the zero-tail shortcut) compiled
// for the HOST under AddressSanitizer, at every register-stack depth the RT_GEN_WREG / RT_GEN_XREG
// switches can select, against the recursion's fold over plain arrays (src/raytracing.c:57, :69-71):
//   c = tail;  for k = n-1 .. 0:  x = a_k (x) c;  if weighted: x = x * w_k;  c = 0 + x
// Random paths (1-64 bounces; solid / unit / explicit albedos; weights of 2.0f, other values, inf and
// NaN; zero, -0 and non-zero tails).  acc + c must match bit for bit (c itself may be +0 where the
// recursion gives -0: acc + (+0) == acc + (-0) for every acc the kernel can hold, never -0).
// Exit 0 when every case matches; prints the first mismatch otherwise.
//   stack_check [cases]
#include "../../ray-tracing-c_amd/csrc/rt_general.h"

#include <stdio.h>
#include <stdlib.h>
#include <string.h>

using namespace rt;
using namespace rt::gen;

namespace {

uint64_t g_state = 0x9e3779b97f4a7c15ull;
uint32_t rnd() {
  g_state ^= g_state << 13, g_state ^= g_state >> 7, g_state ^= g_state << 17;
  return (uint32_t)(g_state >> 16);
}
float frnd(float lo, float hi) { return lo + (hi - lo) * (float)(rnd() & 0xffffff) / 16777216.0f; }
uint32_t bits(float x) {
  uint32_t u;
  memcpy(&u, &x, 4);
  return u;
}

constexpr int kAlbedoBits = 4;  // scenes of <= 13 textures (GeneralView.code_bits)
f3 g_colors[16];

template <int kW, int kX>
bool check_one(long id) {
  const int n = 1 + (int)(rnd() % 64u);
  f3 a[64];
  float w[64];
  bool weighted[64];
  PathRecord<kW, kX> P;
  rec_init(P, kAlbedoBits);
  const uint32_t code_explicit = (1u << kAlbedoBits) - 1u, code_unit = code_explicit - 1u, code_weighted = 1u << kAlbedoBits;
  float4 xrec[kMaxDepth];  // the thread's slots (ASan: an index past them aborts)
  float xw[kMaxDepth];
  // runs of one code (a medium walk) as well as mixed codes
  uint32_t prev_code = 1u + rnd() % 13u;
  for (int k = 0; k < n; k++) {
    uint32_t code;
    const uint32_t pick = rnd() % 10u;
    if (pick < 4) code = prev_code;  // repeat: a run
    else if (pick < 7) code = 1u + rnd() % 13u;
    else if (pick < 8) code = code_unit;
    else code = code_explicit;
    prev_code = code == code_explicit ? prev_code : code;
    if (code == code_explicit) a[k] = mk(frnd(0.0f, 1.0f), frnd(0.0f, 1.0f), frnd(0.0f, 1.0f));
    else if (code == code_unit) a[k] = mk(1.0f, 1.0f, 1.0f);
    else a[k] = g_colors[code - 1u];
    if (code == code_explicit && rnd() % 97u == 0) a[k].y = rnd() & 1 ? __builtin_inff() : __builtin_nanf("");
    weighted[k] = rnd() % 5u != 0;
    w[k] = 1.0f;
    if (weighted[k]) {
      const uint32_t q = rnd() % 8u;
      w[k] = q < 4 ? 2.0f : q < 7 ? frnd(0.01f, 40.0f) : (rnd() % 13u == 0 ? __builtin_inff() : frnd(0.5f, 3.0f));
      code |= code_weighted;
    }
    rec_push(P, code, a[k], w[k], xrec, xw);
  }
  f3 tail;
  switch (rnd() % 4u) {
    case 0: tail = mk(0.0f, 0.0f, 0.0f); break;
    case 1: tail = mk(-0.0f, 0.0f, -0.0f); break;
    case 2: tail = mk(frnd(0.0f, 8.0f), frnd(0.0f, 8.0f), frnd(0.0f, 8.0f)); break;
    default: tail = mk(0.0f, frnd(0.0f, 2.0f), 0.0f); break;
  }
  const auto colors = [](uint32_t t) { return g_colors[t]; };
  const f3 c = rec_fold(P, tail, colors, xrec, xw);
  f3 r = tail;  // the recursion's fold
  for (int k = n - 1; k >= 0; k--) {
    f3 x = mul(a[k], r);
    if (weighted[k]) x = scale(x, w[k]);
    r = add(mk(0.0f, 0.0f, 0.0f), x);
  }
  const f3 accs[2] = {mk(0.0f, 0.0f, 0.0f), mk(frnd(0.0f, 50.0f), frnd(0.0f, 50.0f), frnd(0.0f, 50.0f))};
  for (const f3 &acc : accs) {
    const f3 u = add(acc, c), v = add(acc, r);
    if (bits(u.x) != bits(v.x) || bits(u.y) != bits(v.y) || bits(u.z) != bits(v.z)) {
      fprintf(stderr, "case %ld (wreg %d, xreg %d, %d bounces): acc+fold %08x %08x %08x, recursion %08x %08x %08x\n", id, kW,
              kX, n, bits(u.x), bits(u.y), bits(u.z), bits(v.x), bits(v.y), bits(v.z));
      return false;
    }
  }
  if (P.wst.n != 0 || P.xst.n != 0) {  // every entry pushed was popped (unless the fold was skipped)
    const bool skipped = tail.x == 0.0f && tail.y == 0.0f && tail.z == 0.0f && P.nonfin == 0u;
    if (!skipped) {
      fprintf(stderr, "case %ld: %d weights / %d albedos left on the stacks after the fold\n", id, P.wst.n, P.xst.n);
      return false;
    }
  }
  return true;
}

template <int kW, int kX>
bool check_depth(long cases) {
  for (long i = 0; i < cases; i++)
    if (!check_one<kW, kX>(i)) return false;
  printf("wreg %d xreg %d: %ld paths ok\n", kW, kX, cases);
  return true;
}

}  // namespace

int main(int argc, char **argv) {
  const long cases = argc > 1 ? atol(argv[1]) : 20000;
  for (int t = 0; t < 16; t++) g_colors[t] = mk(frnd(0.0f, 1.0f), frnd(0.0f, 1.0f), frnd(0.0f, 1.0f));
  g_colors[5].z = __builtin_inff();  // a solid colour can be non-finite through the public API
  const bool ok = check_depth<0, 0>(cases) && check_depth<1, 0>(cases) && check_depth<0, 1>(cases) &&
                  check_depth<1, 1>(cases) && check_depth<2, 1>(cases) && check_depth<4, 1>(cases) &&
                  check_depth<8, 2>(cases) && check_depth<4, 4>(cases);
  return ok ? 0 : 1;
}
