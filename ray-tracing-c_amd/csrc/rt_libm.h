// rt_libm.h — bit-exact restatement of the glibc 2.35 (x86-64, FMA ifunc) single-precision
// transcendentals that sit on the reference's hot path, compiled for BOTH gfx950 device code and
// the host (hipcc host pass) so one source can be checked exhaustively against the host glibc.
//
// Why: the reference (C11, gcc) calls libm inside the per-sample loop and a single differing bit
// in a decision value desyncs a pixel's sequential pcg32 stream.  glibc is not
// correctly rounded on these domains, so the GPU must reproduce glibc's algorithm, not the math.
//
// Call sites in the reference (ray-tracing-c @ v2):
//   sincosf  src/material.c:26-27 (rand_cosine_theta; gcc merges cosf+sinf into sincosf),
//            src/hittable.c:171-173 (Sphere_rand)
//   powf     src/material.c:73      (Dielectric Schlick term, y = 5)
//   logf     src/hittable.c:413     (ConstantMedium free-flight distance)
//   sinf     src/texture.c:50       (Perlin marble)
//   atan2f   src/hittable.c:146     (sphere u; glibc 2.35 e_atan2f.c + s_atanf.c, fdlibm)
//   acosf    src/hittable.c:147     (sphere v; glibc 2.35 e_acosf.c, fdlibm)
//
// Algorithm + tables: glibc sysdeps/ieee754/flt-32/{s_sincosf.c,sincosf.h,e_powf.c,e_logf.c,
// s_sinf.c} (ARM optimized-routines).  The FMA placement below is the one gcc emitted for the
// `*_fma` ifunc variants that glibc selects on FMA-capable x86-64 (read off the disassembly of
// /lib/x86_64-linux-gnu/libm.so.6, glibc 2.35-0ubuntu3.11); the table words were read from the
// same library: oracle/tools/extract_libm_tables.cpp locates every table there and checks it word
// for word against this file (tests/test_libm_port.py runs it).  tests/test_libm_port.py also checks
// every port against the host libm over the full domain the hot path can feed it.
//
// Licence: the algorithms, polynomial coefficients and tables below are glibc's, a derived work
// under the GNU Lesser General Public License v2.1 or later (sincosf / powf / logf: ARM
// optimized-routines, Copyright (c) 2017-2018 Arm Ltd; atanf / acosf: fdlibm, Copyright (C) 1993
// Sun Microsystems).  See THIRD_PARTY.md.
//
// Compile with -ffp-contract=off: every fused multiply-add below is an explicit fma().
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#define RT_HD __host__ __device__ __forceinline__

namespace rtm {

RT_HD uint32_t f2u(float f) { return __builtin_bit_cast(uint32_t, f); }
RT_HD float u2f(uint32_t u) { return __builtin_bit_cast(float, u); }
RT_HD uint64_t d2u(double d) { return __builtin_bit_cast(uint64_t, d); }
RT_HD double u2d(uint64_t u) { return __builtin_bit_cast(double, u); }
RT_HD double fmad(double a, double b, double c) { return __builtin_fma(a, b, c); }
// A double constant materialized at its use, by two v_mov_b32 of its halves inside a volatile asm
// (which the compiler cannot hoist): otherwise it hoists the constant addends of the polynomials
// below out of the render loops into VGPR pairs that live across the whole kernel and spill, since
// v_fmac_f64 overwrites its addend register.  KD(lo, hi): the constant's 32-bit halves.
#if defined(__HIP_DEVICE_COMPILE__)
#define KD(LO, HI)                                                                          \
  ({                                                                                        \
    uint32_t kd_lo_, kd_hi_;                                                                \
    asm volatile("v_mov_b32 %0, " #LO "\n\tv_mov_b32 %1, " #HI : "=v"(kd_lo_), "=v"(kd_hi_)); \
    __builtin_bit_cast(double, ((uint64_t)kd_hi_ << 32) | kd_lo_);                          \
  })
#else
#define KD(LO, HI) __builtin_bit_cast(double, ((uint64_t)(HI) << 32) | (uint64_t)(LO))
#endif

// ---------------------------------------------------------------- sincosf / sinf
// sincos_t layout: sign[4], hpi_inv, hpi, c0, c1, s1, c2, s2, c3, s3, c4  (14 doubles, 2 copies).
struct SinCosTab {
  double sign[4], hpi_inv, hpi, c0, c1, s1, c2, s2, c3, s3, c4;
};

RT_HD const SinCosTab &sincos_tab(int which) {
  static constexpr SinCosTab T[2] = {
      {{0x1p+0, -0x1p+0, -0x1p+0, 0x1p+0},
       0x1.45f306dc9c883p+23, 0x1.921fb54442d18p+0,
       0x1p+0, -0x1.ffffffd0c621cp-2, -0x1.555545995a603p-3, 0x1.55553e1068f19p-5,
       0x1.1107605230bc4p-7, -0x1.6c087e89a359dp-10, -0x1.994eb3774cf24p-13, 0x1.99343027bf8c3p-16},
      {{0x1p+0, -0x1p+0, -0x1p+0, 0x1p+0},
       0x1.45f306dc9c883p+23, 0x1.921fb54442d18p+0,
       -0x1p+0, 0x1.ffffffd0c621cp-2, -0x1.555545995a603p-3, -0x1.55553e1068f19p-5,
       0x1.1107605230bc4p-7, 0x1.6c087e89a359dp-10, -0x1.994eb3774cf24p-13, -0x1.99343027bf8c3p-16},
  };
  return T[which];
}

// __inv_pio4: 4/pi bits, used by the |x| >= 120 reduction.
RT_HD uint32_t inv_pio4(int i) {
  static constexpr uint32_t T[24] = {
      0x000000a2, 0x0000a2f9, 0x00a2f983, 0xa2f9836e, 0xf9836e4e, 0x836e4e44, 0x6e4e4415, 0x4e441529,
      0x441529fc, 0x1529fc27, 0x29fc2757, 0xfc2757d1, 0x2757d1f5, 0x57d1f534, 0xd1f534dd, 0xf534ddc0,
      0x34ddc0db, 0xddc0db62, 0xc0db6295, 0xdb629599, 0x6295993c, 0x95993c43, 0x993c4390, 0x3c439041};
  return T[i];
}

RT_HD uint32_t abstop12(float x) { return (f2u(x) >> 20) & 0x7ff; }

// sincosf_poly with the FMA contraction of __sincosf_fma: returns (sin, cos) of the reduced
// argument, already swapped for odd quadrants.  neg_c: table 1 (quadrants with n & 2), whose cos
// coefficients are table 0's negated -- every fma of the cos half then yields exactly the negated
// value (round-to-nearest is symmetric; no intermediate is zero: the reduced |x| <= pi/4), so the
// polynomial runs on table 0's constants, materialized at their use (KD), and cv is negated.
RT_HD void sincos_poly(double x, double x2, bool neg_c, int n, float *sinp, float *cosp) {
  const SinCosTab &p = sincos_tab(0);
  double x3 = x2 * x;
  double x4 = x2 * x2;
  double s1 = fmad(x2, p.s3, KD(0x05230bc4, 0x3f811076) /* s2 = 0x1.1107605230bc4p-7 */);
  double c2 = fmad(x2, p.c4, KD(0xe89a359d, 0xbf56c087) /* c3 = -0x1.6c087e89a359dp-10 */);
  double c1 = fmad(x2, p.c1, KD(0x0, 0x3ff00000) /* c0 = 1 */);
  double x5 = x3 * x2;
  double x6 = x4 * x2;
  double s = fmad(x3, p.s1, x);
  double c = fmad(x4, p.c2, c1);
  float sv = (float)fmad(s1, x5, s);
  double cd = fmad(c2, x6, c);
  float cv = (float)(neg_c ? -cd : cd);
  if (n & 1) { *sinp = cv; *cosp = sv; }
  else { *sinp = sv; *cosp = cv; }
}

// reduce_fast: x - n*pi/2 with n = round(x*2/pi) via the 2^24-scaled integer trick; the
// subtraction is one fused negative multiply-add in the FMA build.
RT_HD double reduce_fast(double x, const SinCosTab &p, int *np) {
  double r = x * p.hpi_inv;
  int n = ((int32_t)r + 0x800000) >> 24;
  *np = n;
  return fmad(-(double)n, p.hpi, x);
}

RT_HD double reduce_large(uint32_t xi, int *np) {
  const int base = (xi >> 26) & 15;
  const int shift = (xi >> 23) & 7;
  xi = (xi & 0xffffff) | 0x800000;
  xi <<= shift;
  uint64_t res0 = (uint32_t)(xi * inv_pio4(base + 0));
  uint64_t res1 = (uint64_t)xi * inv_pio4(base + 4);
  uint64_t res2 = (uint64_t)xi * inv_pio4(base + 8);
  res0 = (res2 >> 32) | (res0 << 32);
  res0 += res1;
  uint64_t n = (res0 + (1ULL << 61)) >> 62;
  res0 -= n << 62;
  double x = (double)(int64_t)res0;
  *np = (int)n;
  return x * 0x1.921fb54442d18p-62;
}

// glibc sincosf (finite inputs; NaN/inf return NaN like glibc, without errno).
RT_HD void sincosf(float y, float *sinp, float *cosp) {
  double x = y;
  int n;
  const uint32_t at = abstop12(y);
  if (at < 0x3f4) {                       // |y| < pi/4
    double x2 = x * x;
    if (at < 0x398) {                     // |y| < 2^-12
      *sinp = y;
      *cosp = 1.0f;
      return;
    }
    sincos_poly(x, x2, false, 0, sinp, cosp);
  } else if (at < 0x42f) {                // |y| < 120
    x = reduce_fast(x, sincos_tab(0), &n);
    const double s = sincos_tab(0).sign[n & 3];
    sincos_poly(x * s, x * x, (n & 2) != 0, n, sinp, cosp);
  } else if (at < 0x7f8) {                // finite
    const uint32_t xi = f2u(y);
    const int sign = xi >> 31;
    x = reduce_large(xi, &n);
    const double s = sincos_tab(0).sign[(n + sign) & 3];
    sincos_poly(x * s, x * x, ((n + sign) & 2) != 0, n, sinp, cosp);
  } else {
    *sinp = *cosp = y - y;
  }
}

// glibc sinf: the same reduction and the sin/cos halves of the same polynomial.
RT_HD float sinf(float y) {
  float s, c;
  sincosf(y, &s, &c);
  return s;
}

// ---------------------------------------------------------------- powf
RT_HD double powf_log2_invc(int i) {
  static constexpr double T[16] = {
      0x1.661ec79f8f3bep+0, 0x1.571ed4aaf883dp+0, 0x1.49539f0f010bp+0, 0x1.3c995b0b80385p+0,
      0x1.30d190c8864a5p+0, 0x1.25e227b0b8eap+0, 0x1.1bb4a4a1a343fp+0, 0x1.12358f08ae5bap+0,
      0x1.0953f419900a7p+0, 0x1p+0, 0x1.e608cfd9a47acp-1, 0x1.ca4b31f026aap-1,
      0x1.b2036576afce6p-1, 0x1.9c2d163a1aa2dp-1, 0x1.886e6037841edp-1, 0x1.767dcf5534862p-1};
  return T[i];
}
RT_HD double powf_log2_logc(int i) {
  static constexpr double T[16] = {
      -0x1.efec65b963019p-2, -0x1.b0b6832d4fca4p-2, -0x1.7418b0a1fb77bp-2, -0x1.39de91a6dcf7bp-2,
      -0x1.01d9bf3f2b631p-2, -0x1.97c1d1b3b7afp-3, -0x1.2f9e393af3c9fp-3, -0x1.960cbbf788d5cp-4,
      -0x1.a6f9db6475fcep-5, 0x0p+0, 0x1.338ca9f24f53dp-4, 0x1.476a9543891bap-3,
      0x1.e840b4ac4e4d2p-3, 0x1.40645f0c6651cp-2, 0x1.88e9c2c1b9ff8p-2, 0x1.ce0a44eb17bccp-2};
  return T[i];
}
RT_HD uint64_t exp2f_tab(int i) {
  static constexpr uint64_t T[32] = {
      0x3ff0000000000000, 0x3fefd9b0d3158574, 0x3fefb5586cf9890f, 0x3fef9301d0125b51,
      0x3fef72b83c7d517b, 0x3fef54873168b9aa, 0x3fef387a6e756238, 0x3fef1e9df51fdee1,
      0x3fef06fe0a31b715, 0x3feef1a7373aa9cb, 0x3feedea64c123422, 0x3feece086061892d,
      0x3feebfdad5362a27, 0x3feeb42b569d4f82, 0x3feeab07dd485429, 0x3feea47eb03a5585,
      0x3feea09e667f3bcd, 0x3fee9f75e8ec5f74, 0x3feea11473eb0187, 0x3feea589994cce13,
      0x3feeace5422aa0db, 0x3feeb737b0cdc5e5, 0x3feec49182a3f090, 0x3feed503b23e255d,
      0x3feee89f995ad3ad, 0x3feeff76f2fb5e47, 0x3fef199bdd85529c, 0x3fef3720dcef9069,
      0x3fef5818dcfba487, 0x3fef7c97337b9b5f, 0x3fefa4afa2a490da, 0x3fefd0765b6e4540};
  return T[i];
}

RT_HD bool zeroinfnan(uint32_t ix) { return 2 * ix - 1 >= 2u * 0x7f800000 - 1; }

// checkint: 0 = not an integer, 1 = odd integer, 2 = even integer.
RT_HD int checkint(uint32_t iy) {
  int e = (iy >> 23) & 0xff;
  if (e < 0x7f) return 0;
  if (e > 0x7f + 23) return 2;
  if (iy & ((1u << (0x7f + 23 - e)) - 1)) return 0;
  if (iy & (1u << (0x7f + 23 - e))) return 1;
  return 2;
}

RT_HD double powf_log2_inline(uint32_t ix) {
  const uint32_t tmp = ix - 0x3f330000;
  const int i = (tmp >> 19) % 16;
  const uint32_t top = tmp & 0xff800000;
  const uint32_t iz = ix - top;
  const int k = (int32_t)top >> 23;
  const double invc = powf_log2_invc(i), logc = powf_log2_logc(i);
  const double z = (double)u2f(iz);
  const double r = fmad(z, invc, -1.0);
  const double y0 = (double)k + logc;
  const double r2 = r * r;
  double y = fmad(0x1.27616c9496e0bp-2, r, KD(0xa075c67a, 0xbfd71969) /* -0x1.71969a075c67ap-2 */);
  const double p = fmad(0x1.ec70a6ca7baddp-2, r, KD(0x48bef6c8, 0xbfe71547) /* -0x1.7154748bef6c8p-1 */);
  const double r4 = r2 * r2;
  double q = fmad(0x1.71547652ab82bp+0, r, y0);
  q = fmad(p, r2, q);
  y = fmad(y, r4, q);
  return y;
}

RT_HD double powf_exp2_inline(double xd, uint32_t sign_bias) {
  const double shift = 0x1.8p+47;
  double kd = xd + shift;
  const uint64_t ki = d2u(kd);
  kd -= shift;
  const double r = xd - kd;
  uint64_t t = exp2f_tab((int)(ki % 32));
  const uint64_t ski = ki + sign_bias;
  t += ski << (52 - 5);
  const double s = u2d(t);
  const double z = fmad(0x1.c6af84b912394p-5, r, KD(0x50fac4f3, 0x3fcebfce) /* 0x1.ebfce50fac4f3p-3 */);
  const double r2 = r * r;
  double y = fmad(0x1.62e42ff0c52d6p-1, r, KD(0x0, 0x3ff00000) /* 1.0 */);
  y = fmad(z, r2, y);
  return y * s;
}

// glibc powf (round-to-nearest, errno-free).
RT_HD float powf(float x, float y) {
  uint32_t sign_bias = 0;
  uint32_t ix = f2u(x), iy = f2u(y);
  if (ix - 0x00800000 >= 0x7f800000 - 0x00800000 || zeroinfnan(iy)) {
    if (zeroinfnan(iy)) {
      if (2 * iy == 0) return 1.0f;
      if (ix == 0x3f800000) return 1.0f;
      if (2 * ix > 2u * 0x7f800000 || 2 * iy > 2u * 0x7f800000) return x + y;
      if (2 * ix == 2 * 0x3f800000) return 1.0f;
      if ((2 * ix < 2 * 0x3f800000) == !(iy & 0x80000000)) return 0.0f;
      return y * y;
    }
    if (zeroinfnan(ix)) {
      float x2 = x * x;
      if ((ix & 0x80000000) && checkint(iy) == 1) x2 = -x2;
      return (iy & 0x80000000) ? 1.0f / x2 : x2;
    }
    if (ix & 0x80000000) {
      const int yint = checkint(iy);
      if (yint == 0) return (x - x) / (x - x);
      if (yint == 1) sign_bias = 1u << (5 + 11);
      ix &= 0x7fffffff;
    }
    if (ix < 0x00800000) {
      ix = f2u(x * 0x1p23f);
      ix &= 0x7fffffff;
      ix -= 23u << 23;
    }
  }
  const double logx = powf_log2_inline(ix);
  const double ylogx = (double)y * logx;
  if (((d2u(ylogx) >> 47) & 0xffff) >= (d2u(126.0) >> 47)) {
    const float sgn = sign_bias ? -1.0f : 1.0f;
    if (ylogx > 0x1.fffffffd1d571p+6) return sgn * 0x1p97f * 0x1p97f;           // overflow
    // (0x1.fffffffa3aae2p+6 < ylogx only overflows in directed rounding modes: falls through.)
    if (ylogx <= -150.0) return sgn * 0x1p-95f * 0x1p-95f;                      // underflow
    if (ylogx < -149.0) return sgn * 0x1.4p-75f * 0x1.4p-75f;                   // may underflow
  }
  return (float)powf_exp2_inline(ylogx, sign_bias);
}

// ---------------------------------------------------------------- logf
RT_HD double logf_logc(int i) {
  static constexpr double T[16] = {
      -0x1.57bf7808caadep-2, -0x1.2bef0a7c06ddbp-2, -0x1.01eae7f513a67p-2, -0x1.b31d8a68224e9p-3,
      -0x1.6574f0ac07758p-3, -0x1.1aa2bc79c81p-3, -0x1.a4e76ce8c0e5ep-4, -0x1.1973c5a611cccp-4,
      -0x1.252f438e10c1ep-5, 0x0p+0, 0x1.aa5aa5df25984p-5, 0x1.c5e53aa362eb4p-4,
      0x1.526e57720db08p-3, 0x1.bc2860d22477p-3, 0x1.1058bc8a07ee1p-2, 0x1.4043057b6ee09p-2};
  return T[i];
}

// glibc logf (round-to-nearest, errno-free).
RT_HD float logf(float x) {
  uint32_t ix = f2u(x);
  if (ix == 0x3f800000) return 0.0f;
  if (ix - 0x00800000 >= 0x7f800000 - 0x00800000) {
    if (ix * 2 == 0) return -__builtin_inff();
    if (ix == 0x7f800000) return x;
    if ((ix & 0x80000000) || ix * 2 >= 0xff000000) return (x - x) / (x - x);
    ix = f2u(x * 0x1p23f);
    ix -= 23u << 23;
  }
  const uint32_t tmp = ix - 0x3f330000;
  const int i = (tmp >> 19) % 16;
  const int k = (int32_t)tmp >> 23;
  const uint32_t iz = ix - (tmp & 0xff800000u);
  const double invc = powf_log2_invc(i), logc = logf_logc(i);
  const double z = (double)u2f(iz);
  const double r = fmad(z, invc, -1.0);
  const double y0 = fmad((double)k, 0x1.62e42fefa39efp-1, logc);
  const double r2 = r * r;
  double y = fmad(0x1.5575b0be00b6ap-2, r, KD(0xf20a4123, 0xbfdffffe) /* -0x1.ffffef20a4123p-2 */);
  y = fmad(-0x1.00ea348b88334p-2, r2, y);
  y = fmad(y, r2, y0 + r);
  return (float)y;
}

// ---------------------------------------------------------------- atanf / atan2f / acosf
// fdlibm single precision as in glibc 2.35 sysdeps/ieee754/flt-32 (no multiarch variant: plain
// SSE float arithmetic).  Constants read from /lib/x86_64-linux-gnu/libm.so.6.
RT_HD float atanf(float x) {
  const float atanhi[4] = {u2f(0x3eed6338), u2f(0x3f490fda), u2f(0x3f7b985e), u2f(0x3fc90fda)};
  const float atanlo[4] = {u2f(0x31ac3769), u2f(0x33222168), u2f(0x33140fb4), u2f(0x33a22168)};
  const uint32_t hx = f2u(x), ix = hx & 0x7fffffff;
  int id;
  if (ix >= 0x4c000000) {  // |x| >= 2^25
    if (ix > 0x7f800000) return x + x;
    return ((int32_t)hx > 0) ? atanhi[3] + atanlo[3] : -atanhi[3] - atanlo[3];
  }
  if (ix < 0x3ee00000) {              // |x| < 0.4375
    if (ix < 0x31000000) return x;    // |x| < 2^-29
    id = -1;
  } else {
    x = fabsf(x);
    if (ix < 0x3f980000) {            // |x| < 1.1875
      if (ix < 0x3f300000) {          // 7/16 <= |x| < 11/16
        id = 0;
        x = (2.0f * x - 1.0f) / (2.0f + x);
      } else {                        // 11/16 <= |x| < 19/16
        id = 1;
        x = (x - 1.0f) / (x + 1.0f);
      }
    } else if (ix < 0x401c0000) {     // |x| < 2.4375
      id = 2;
      x = (x - 1.5f) / (1.0f + 1.5f * x);
    } else {                          // 2.4375 <= |x| < 2^25
      id = 3;
      x = -1.0f / x;
    }
  }
  const float z = x * x;
  const float w = z * z;
  // Horner exactly as fdlibm writes it: s1 = z*(aT0+w*(aT2+w*(aT4+w*(aT6+w*(aT8+w*aT10)))))
  const float t1 = z * (u2f(0x3eaaaaab) +
                        w * (u2f(0x3e124925) +
                             w * (u2f(0x3dba2e6e) + w * (u2f(0x3d886b35) + w * (u2f(0x3d4bda59) + w * u2f(0x3c8569d7))))));
  // s2 = w*(aT1+w*(aT3+w*(aT5+w*(aT7+w*aT9))))
  const float t2 = w * (u2f(0xbe4ccccd) +
                        w * (u2f(0xbde38e38) + w * (u2f(0xbd9d8795) + w * (u2f(0xbd6ef16b) + w * u2f(0xbd15a221)))));
  if (id < 0) return x - x * (t1 + t2);
  const float r = atanhi[id] - ((x * (t1 + t2) - atanlo[id]) - x);
  return ((int32_t)hx < 0) ? -r : r;
}

RT_HD float atan2f(float y, float x) {
  const float tiny = 1.0e-30f, pi_o_4 = u2f(0x3f490fdb), pi_o_2 = u2f(0x3fc90fdb), pi = u2f(0x40490fdb);
  const float pi_lo = u2f(0xb3bbbd2e);
  const uint32_t hx = f2u(x), hy = f2u(y);
  const uint32_t ix = hx & 0x7fffffff, iy = hy & 0x7fffffff;
  if (ix > 0x7f800000 || iy > 0x7f800000) return x + y;
  if (hx == 0x3f800000) return atanf(y);
  const int m = (int)(((hy >> 31) & 1) | ((hx >> 30) & 2));
  if (iy == 0) {
    if (m <= 1) return y;
    return m == 2 ? pi + tiny : -pi - tiny;
  }
  if (ix == 0) return ((int32_t)hy < 0) ? -pi_o_2 - tiny : pi_o_2 + tiny;
  if (ix == 0x7f800000) {
    if (iy == 0x7f800000) {
      switch (m) {
      case 0: return pi_o_4 + tiny;
      case 1: return -pi_o_4 - tiny;
      case 2: return 3.0f * pi_o_4 + tiny;
      default: return -3.0f * pi_o_4 - tiny;
      }
    }
    switch (m) {
    case 0: return 0.0f;
    case 1: return -0.0f;
    case 2: return pi + tiny;
    default: return -pi - tiny;
    }
  }
  if (iy == 0x7f800000) return ((int32_t)hy < 0) ? -pi_o_2 - tiny : pi_o_2 + tiny;
  const int32_t k = ((int32_t)iy - (int32_t)ix) >> 23;
  float z;
  if (k > 60) z = pi_o_2 + 0.5f * pi_lo;
  else if ((int32_t)hx < 0 && k < -60) z = 0.0f;
  else z = atanf(fabsf(y / x));
  switch (m) {
  case 0: return z;
  case 1: return u2f(f2u(z) ^ 0x80000000u);
  case 2: return pi - (z - pi_lo);
  default: return (z - pi_lo) - pi;
  }
}

RT_HD float acosf(float x) {
  const float pi = u2f(0x40490fda), pio2_hi = u2f(0x3fc90fda), pio2_lo = u2f(0x33a22168);
  const float pS0 = u2f(0x3e2aaaab), pS1 = u2f(0xbea6b090), pS2 = u2f(0x3e4e0aa8), pS3 = u2f(0xbd241146),
              pS4 = u2f(0x3a4f7f04), pS5 = u2f(0x3811ef08);
  const float qS1 = u2f(0xc019d139), qS2 = u2f(0x4001572d), qS3 = u2f(0xbf303361), qS4 = u2f(0x3d9dc62e);
  const uint32_t hx = f2u(x), ix = hx & 0x7fffffff;
  if (ix == 0x3f800000) return ((int32_t)hx > 0) ? 0.0f : pi + 2.0f * pio2_lo;
  if (ix > 0x3f800000) return (x - x) / (x - x);
  if (ix < 0x3f000000) {  // |x| < 0.5
    if (ix <= 0x32800000) return pio2_hi + pio2_lo;
    const float z = x * x;
    const float p = z * (pS0 + z * (pS1 + z * (pS2 + z * (pS3 + z * (pS4 + z * pS5)))));
    const float q = 1.0f + z * (qS1 + z * (qS2 + z * (qS3 + z * qS4)));
    const float r = p / q;
    return pio2_hi - (x - (pio2_lo - x * r));
  }
  if ((int32_t)hx < 0) {  // x < -0.5
    const float z = (1.0f + x) * 0.5f;
    const float p = z * (pS0 + z * (pS1 + z * (pS2 + z * (pS3 + z * (pS4 + z * pS5)))));
    const float q = 1.0f + z * (qS1 + z * (qS2 + z * (qS3 + z * qS4)));
    const float s = sqrtf(z);
    const float r = p / q;
    const float w = r * s - pio2_lo;
    return pi - 2.0f * (s + w);
  }
  const float z = (1.0f - x) * 0.5f;  // x > 0.5
  const float s = sqrtf(z);
  const float df = u2f(f2u(s) & 0xfffff000u);
  const float c = (z - df * df) / (s + df);
  const float p = z * (pS0 + z * (pS1 + z * (pS2 + z * (pS3 + z * (pS4 + z * pS5)))));
  const float q = 1.0f + z * (qS1 + z * (qS2 + z * (qS3 + z * qS4)));
  const float r = p / q;
  const float w = r * s + c;
  return 2.0f * (df + w);
}

}  // namespace rtm
