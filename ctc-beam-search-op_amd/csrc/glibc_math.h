// glibc_math.h — bit-exact device restatements of the three float libm
// functions the reference decoder depends on.
//
// The reference computes every log-space quantity through glibc's libm:
//   * softmax normaliser: Eigen::numext::exp / numext::log on T=float, i.e.
//     expf / logf   (ctc_ext_beam_search_decoder.h:72-80)
//   * LogSumExp: log1pf(expf(b - a)) — float libm even for T=double
//     (ctc_loss_util.h:29-41)
// Decoded labels are the result of thousands of float comparisons per frame,
// so the GPU must reproduce those functions bit for bit, not to within an ULP.
//
// What is restated (glibc 2.35, x86_64, the libm the reference links):
//   expf  — sysdeps/ieee754/flt-32/e_expf.c (ARM optimized-routines design,
//           32-entry 2^(i/32) table, cubic in double).  x86_64 dispatches to
//           the FMA ifunc variant on any AVX2+FMA host, where GCC contracted
//           the polynomial's multiply-adds; the contractions are written out
//           below as explicit fma() calls.
//   logf  — sysdeps/ieee754/flt-32/e_logf.c (16-entry {1/c, log c} table,
//           cubic in double), FMA ifunc variant likewise.
//   log1pf— sysdeps/ieee754/flt-32/s_log1pf.c (fdlibm, pure float
//           arithmetic; no ifunc variant, no contraction).
// Table values were read out of the host's libm.so.6 data section and are
// pinned by tools/check_glibc_math.cpp, which compares these functions with
// the host libm over ALL 2^32 float inputs (result recorded in DESIGN.md).
//
// Build contract: every translation unit that includes this header must be
// compiled with -ffp-contract=off (hipcc defaults to fast contraction for
// HIP), and f32 denormals must not be flushed.
#pragma once

#include <stdint.h>

#ifndef CTCX_HD
#define CTCX_HD __host__ __device__ __forceinline__
#endif

namespace ctcx {
namespace gm {

CTCX_HD uint32_t f2u(float x) { return __builtin_bit_cast(uint32_t, x); }
CTCX_HD float u2f(uint32_t u) { return __builtin_bit_cast(float, u); }
CTCX_HD uint64_t d2u(double x) { return __builtin_bit_cast(uint64_t, x); }
CTCX_HD double u2d(uint64_t u) { return __builtin_bit_cast(double, u); }

// ---- expf ------------------------------------------------------------------
// 2^(i/32) with the exponent bits of i/32 removed (table-driven scaling).
CTCX_HD uint64_t exp2f_tab(int i) {
  // A switch keeps the table in the instruction stream on the device (no
  // constant-memory object to load), and on the host it is a jump table.
  switch (i) {
    case 0: return 0x3ff0000000000000ull;  case 1: return 0x3fefd9b0d3158574ull;
    case 2: return 0x3fefb5586cf9890full;  case 3: return 0x3fef9301d0125b51ull;
    case 4: return 0x3fef72b83c7d517bull;  case 5: return 0x3fef54873168b9aaull;
    case 6: return 0x3fef387a6e756238ull;  case 7: return 0x3fef1e9df51fdee1ull;
    case 8: return 0x3fef06fe0a31b715ull;  case 9: return 0x3feef1a7373aa9cbull;
    case 10: return 0x3feedea64c123422ull; case 11: return 0x3feece086061892dull;
    case 12: return 0x3feebfdad5362a27ull; case 13: return 0x3feeb42b569d4f82ull;
    case 14: return 0x3feeab07dd485429ull; case 15: return 0x3feea47eb03a5585ull;
    case 16: return 0x3feea09e667f3bcdull; case 17: return 0x3fee9f75e8ec5f74ull;
    case 18: return 0x3feea11473eb0187ull; case 19: return 0x3feea589994cce13ull;
    case 20: return 0x3feeace5422aa0dbull; case 21: return 0x3feeb737b0cdc5e5ull;
    case 22: return 0x3feec49182a3f090ull; case 23: return 0x3feed503b23e255dull;
    case 24: return 0x3feee89f995ad3adull; case 25: return 0x3feeff76f2fb5e47ull;
    case 26: return 0x3fef199bdd85529cull; case 27: return 0x3fef3720dcef9069ull;
    case 28: return 0x3fef5818dcfba487ull; case 29: return 0x3fef7c97337b9b5full;
    case 30: return 0x3fefa4afa2a490daull; default: return 0x3fefd0765b6e4540ull;
  }
}

// Tab: i -> 2^(i/32) bits as exp2f_tab gives them.  expf uses the switch
// (no memory object); a caller whose lanes take divergent indices (a switch
// is then a branch per case) passes a copy of the table in LDS (expf_t).
template <class Tab>
CTCX_HD float expf_impl(float x, const Tab& tab) {
  const uint32_t ux = f2u(x);
  const uint32_t abstop = (ux >> 20) & 0x7ff;
  if (abstop >= 0x42bu) {                  // |x| >= 88 or nan
    if (ux == 0xff800000u) return 0.0f;    // exp(-inf) = 0
    if (abstop >= 0x7f8u) return x + x;    // inf or nan
    if (x > 0x1.62e42ep6f) return __builtin_inff();   // overflow
    if (x < -0x1.9fe368p6f) return 0.0f;               // underflow
  }
  const double xd = (double)x;
  const double InvLn2N = 0x1.71547652b82fep+5;   // 32 / ln 2
  const double Shift = 0x1.8p+52;
  // GCC fused the product InvLn2N*xd into BOTH of its consumers (it only
  // contracts when every use of a product is an add/sub), so z is never
  // rounded on its own.  Pinned by the exhaustive check: the unfused form
  // differs from libm on 2 of 2^32 inputs.
  double kd = __builtin_fma(InvLn2N, xd, Shift);
  const uint64_t ki = d2u(kd);
  kd -= Shift;
  const double r = __builtin_fma(InvLn2N, xd, -kd);
  uint64_t t = tab((int)(ki % 32));
  t += ki << 47;
  const double s = u2d(t);
  const double zc = __builtin_fma(0x1.c6af84b912394p-20, r, 0x1.ebfce50fac4f3p-13);
  const double r2 = r * r;
  double y = __builtin_fma(0x1.62e42ff0c52d6p-6, r, 1.0);
  y = __builtin_fma(zc, r2, y);
  y = y * s;
  return (float)y;
}
CTCX_HD float expf(float x) {
  return expf_impl(x, [](int i) { return exp2f_tab(i); });
}
template <class P>
CTCX_HD float expf_t(float x, P tab) {   // tab[i] == exp2f_tab(i), e.g. in LDS
  return expf_impl(x, [tab](int i) { return (uint64_t)tab[i]; });
}
// expf_t for x <= 0, -inf or NaN (a softmax term x_j - max), without branches:
// below -0x1.9fe368p6 (and at -inf) glibc returns 0, a NaN comes back as
// x + x, and every other x <= 0 takes expf_impl's core path (from -88 down
// to the underflow bound glibc falls through to it too); no overflow above.
template <class P>
CTCX_HD float expf_t_nonpos(float x, P tab) {
  const bool under = x < -0x1.9fe368p6f;
  const double xd = (double)(under ? 0.0f : x);   // (the core path's result is dropped then)
  const double InvLn2N = 0x1.71547652b82fep+5;
  const double Shift = 0x1.8p+52;
  double kd = __builtin_fma(InvLn2N, xd, Shift);
  const uint64_t ki = d2u(kd);
  kd -= Shift;
  const double r = __builtin_fma(InvLn2N, xd, -kd);
  uint64_t t = (uint64_t)tab[(int)(ki % 32)];
  t += ki << 47;
  const double s = u2d(t);
  const double zc = __builtin_fma(0x1.c6af84b912394p-20, r, 0x1.ebfce50fac4f3p-13);
  const double r2 = r * r;
  double y = __builtin_fma(0x1.62e42ff0c52d6p-6, r, 1.0);
  y = __builtin_fma(zc, r2, y);
  y = y * s;
  const float e = under ? 0.0f : (float)y;
  return x != x ? x + x : e;
}
// expf's core path alone: glibc's expf for -0x1.9fe368p6 <= x <= 0 (a
// caller that has checked the bound for a whole batch of terms)
template <class P>
CTCX_HD float expf_t_core(float x, P tab) {
  const double xd = (double)x;
  const double InvLn2N = 0x1.71547652b82fep+5;
  const double Shift = 0x1.8p+52;
  double kd = __builtin_fma(InvLn2N, xd, Shift);
  const uint64_t ki = d2u(kd);
  kd -= Shift;
  const double r = __builtin_fma(InvLn2N, xd, -kd);
  uint64_t t = (uint64_t)tab[(int)(ki % 32)];
  t += ki << 47;
  const double s = u2d(t);
  const double zc = __builtin_fma(0x1.c6af84b912394p-20, r, 0x1.ebfce50fac4f3p-13);
  const double r2 = r * r;
  double y = __builtin_fma(0x1.62e42ff0c52d6p-6, r, 1.0);
  y = __builtin_fma(zc, r2, y);
  y = y * s;
  return (float)y;
}
constexpr float kExpfUnder = -0x1.9fe368p6f;   // below it glibc's expf returns 0
// expf_t_nonpos for x <= 0 or -inf, never NaN (a term of a row whose maximum
// is finite and which holds no NaN / +inf): the core path runs on x as it is
// (at -inf or below the underflow bound its result, garbage or NaN, is
// dropped for glibc's 0), and no NaN select
template <class P>
CTCX_HD float expf_t_le0(float x, P tab) {
  const bool under = x < -0x1.9fe368p6f;
  const double xd = (double)x;
  const double InvLn2N = 0x1.71547652b82fep+5;
  const double Shift = 0x1.8p+52;
  double kd = __builtin_fma(InvLn2N, xd, Shift);
  const uint64_t ki = d2u(kd);
  kd -= Shift;
  const double r = __builtin_fma(InvLn2N, xd, -kd);
  uint64_t t = (uint64_t)tab[(int)(ki % 32)];
  t += ki << 47;
  const double s = u2d(t);
  const double zc = __builtin_fma(0x1.c6af84b912394p-20, r, 0x1.ebfce50fac4f3p-13);
  const double r2 = r * r;
  double y = __builtin_fma(0x1.62e42ff0c52d6p-6, r, 1.0);
  y = __builtin_fma(zc, r2, y);
  y = y * s;
  return under ? 0.0f : (float)y;
}

// ---- logf ------------------------------------------------------------------
CTCX_HD void logf_tab(int i, double& invc, double& logc) {
  switch (i) {
    case 0:  invc = 0x1.661ec79f8f3bep+0; logc = -0x1.57bf7808caadep-2; break;
    case 1:  invc = 0x1.571ed4aaf883dp+0; logc = -0x1.2bef0a7c06ddbp-2; break;
    case 2:  invc = 0x1.49539f0f010b0p+0; logc = -0x1.01eae7f513a67p-2; break;
    case 3:  invc = 0x1.3c995b0b80385p+0; logc = -0x1.b31d8a68224e9p-3; break;
    case 4:  invc = 0x1.30d190c8864a5p+0; logc = -0x1.6574f0ac07758p-3; break;
    case 5:  invc = 0x1.25e227b0b8ea0p+0; logc = -0x1.1aa2bc79c8100p-3; break;
    case 6:  invc = 0x1.1bb4a4a1a343fp+0; logc = -0x1.a4e76ce8c0e5ep-4; break;
    case 7:  invc = 0x1.12358f08ae5bap+0; logc = -0x1.1973c5a611cccp-4; break;
    case 8:  invc = 0x1.0953f419900a7p+0; logc = -0x1.252f438e10c1ep-5; break;
    case 9:  invc = 0x1.0000000000000p+0; logc = 0.0; break;
    case 10: invc = 0x1.e608cfd9a47acp-1; logc = 0x1.aa5aa5df25984p-5; break;
    case 11: invc = 0x1.ca4b31f026aa0p-1; logc = 0x1.c5e53aa362eb4p-4; break;
    case 12: invc = 0x1.b2036576afce6p-1; logc = 0x1.526e57720db08p-3; break;
    case 13: invc = 0x1.9c2d163a1aa2dp-1; logc = 0x1.bc2860d224770p-3; break;
    case 14: invc = 0x1.886e6037841edp-1; logc = 0x1.1058bc8a07ee1p-2; break;
    default: invc = 0x1.767dcf5534862p-1; logc = 0x1.4043057b6ee09p-2; break;
  }
}

CTCX_HD float logf(float x) {
  uint32_t ix = f2u(x);
  if (ix == 0x3f800000u) return 0.0f;
  if (ix - 0x00800000u >= 0x7f800000u - 0x00800000u) {
    if (ix * 2 == 0) return -__builtin_inff();            // log(+-0) = -inf
    if (ix == 0x7f800000u) return x;                      // log(inf) = inf
    if ((ix & 0x80000000u) || ix * 2 >= 0xff000000u)      // x < 0 or nan
      return __builtin_nanf("");
    ix = f2u(x * 0x1p23f);                                // subnormal
    ix -= 23u << 23;
  }
  const uint32_t tmp = ix - 0x3f330000u;
  const int i = (int)((tmp >> (23 - 4)) % 16);
  const int k = (int32_t)tmp >> 23;
  const uint32_t iz = ix - (tmp & (0x1ffu << 23));
  double invc, logc;
  logf_tab(i, invc, logc);
  const double z = (double)u2f(iz);
  const double Ln2 = 0x1.62e42fefa39efp-1;
  const double r = __builtin_fma(z, invc, -1.0);
  const double y0 = __builtin_fma((double)k, Ln2, logc);
  const double r2 = r * r;
  double y = __builtin_fma(0x1.5575b0be00b6ap-2, r, -0x1.ffffef20a4123p-2);
  y = __builtin_fma(-0x1.00ea348b88334p-2, r2, y);
  y = __builtin_fma(y, r2, y0 + r);
  return (float)y;
}

// ---- log1pf (fdlibm, float arithmetic throughout) ---------------------------
CTCX_HD float log1pf(float x) {
  const float ln2_hi = 6.9313812256e-01f, ln2_lo = 9.0580006145e-06f;
  const float Lp1 = 6.6666668653e-01f, Lp2 = 4.0000000596e-01f,
              Lp3 = 2.8571429849e-01f, Lp4 = 2.2222198546e-01f,
              Lp5 = 1.8183572590e-01f, Lp6 = 1.5313838422e-01f,
              Lp7 = 1.4798198640e-01f;
  float hfsq, f = 0.0f, c = 0.0f, s, z, R, u;
  int32_t k, hx, hu = 0, ax;
  hx = (int32_t)f2u(x);
  ax = hx & 0x7fffffff;
  k = 1;
  if (hx < 0x3ed413d7) {                       // x < 0.41422
    if (ax >= 0x3f800000) {                    // x <= -1.0
      if (x == -1.0f) return -__builtin_inff();
      return __builtin_nanf("");
    }
    if (ax < 0x31000000) {                     // |x| < 2**-29
      if (ax < 0x24800000) return x;           // |x| < 2**-54
      return x - x * x * 0.5f;
    }
    if (hx > 0 || hx <= (int32_t)0xbe95f61f) { k = 0; f = x; hu = 1; }
  } else if (hx >= 0x7f800000) {
    return x + x;
  }
  if (k != 0) {
    if (hx < 0x5a000000) {
      u = 1.0f + x;
      hu = (int32_t)f2u(u);
      k = (hu >> 23) - 127;
      c = (k > 0) ? 1.0f - (u - x) : x - (u - 1.0f);
      c /= u;
    } else {
      u = x;
      hu = (int32_t)f2u(u);
      k = (hu >> 23) - 127;
      c = 0;
    }
    hu &= 0x007fffff;
    if (hu < 0x3504f7) {
      u = u2f((uint32_t)(hu | 0x3f800000));
    } else {
      k += 1;
      u = u2f((uint32_t)(hu | 0x3f000000));
      hu = (0x00800000 - hu) >> 2;
    }
    f = u - 1.0f;
  }
  hfsq = 0.5f * f * f;
  if (hu == 0) {                               // |f| < 2**-20
    if (f == 0.0f) {
      if (k == 0) return 0.0f;
      c += k * ln2_lo;
      return k * ln2_hi + c;
    }
    R = hfsq * (1.0f - 0.66666666666666666f * f);
    if (k == 0) return f - R;
    return k * ln2_hi - ((R - (c + k * ln2_lo)) - f);
  }
  s = f / (2.0f + f);
  z = s * s;
  R = z * (Lp1 + z * (Lp2 + z * (Lp3 + z * (Lp4 + z * (Lp5 + z * (Lp6 + z * Lp7))))));
  if (k == 0) return f - (hfsq - s * (hfsq + R));
  return k * ln2_hi - ((hfsq - (s * (hfsq + R) + (c + k * ln2_lo))) - f);
}

}  // namespace gm
}  // namespace ctcx
