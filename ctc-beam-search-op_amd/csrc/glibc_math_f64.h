// glibc_math_f64.h — bit-exact device restatements of glibc 2.35's double
// exp and log, which the reference's softmax normaliser uses for T=double
// (Eigen::numext::exp / numext::log, ctc_ext_beam_search_decoder.h:72-80).
//
// Source design: sysdeps/ieee754/dbl-64/e_exp.c and e_log.c (ARM
// optimized-routines: 128-entry 2^(i/128) table + degree-5 polynomial; 128-
// entry {1/c, log c} table + degree-6 polynomial, separate degree-12
// polynomial near 1).  On an AVX2+FMA host exp/log dispatch to the FMA ifunc
// variants (__exp_fma at libm+0x76470, __log_fma at libm+0x76660), where GCC
// contracted multiply-adds; every fma() below is one vfmadd/vfnmadd of that
// machine code, in its order, and every other operation is a separately
// rounded IEEE double operation (compile with -ffp-contract=off).  Tables:
// glibc_math_f64_tables.h, read from the same libm.  Pinned by
// tools/check_glibc_math_f64.cpp against the host libm.
#pragma once

#include <stdint.h>

#include "glibc_math.h"
#include "glibc_math_f64_tables.h"

namespace ctcx {
namespace gm {

CTCX_HD double hd(uint64_t u) { return u2d(u); }

// ---- exp -------------------------------------------------------------------
// specialcase() of e_exp.c: the scale 2^k would over/underflow the exponent.
CTCX_HD double exp_special(double tmp, uint64_t sbits, uint64_t ki) {
  if ((ki & 0x80000000ull) == 0) {   // k > 0: the result may overflow
    sbits -= 1009ull << 52;
    const double scale = u2d(sbits);
    return __builtin_fma(scale, tmp, scale) * hd(0x7f00000000000000ull);   // * 0x1p1009
  }
  // k < 0: the result may be subnormal; round once, in the subnormal range
  sbits += 1022ull << 52;
  const double scale = u2d(sbits);
  const double st = tmp * scale;
  double y = scale + st;
  if (1.0 > y) {
    const double hi = y + 1.0;
    const double lo = (scale - y) + st;
    double t = ((1.0 - hi) + y) + lo;
    y = (t + hi) - 1.0;
    if (y == 0.0) return 0.0;
  }
  return y * hd(0x0010000000000000ull);   // * 0x1p-1022
}

CTCX_HD double exp(double x) {
  const uint64_t ix = d2u(x);
  uint32_t abstop = (uint32_t)(ix >> 52) & 0x7ffu;
  if (abstop - 0x3c9u > 0x3eu) {
    if ((int32_t)(abstop - 0x3c9u) < 0) return x + 1.0;   // |x| < 2^-54
    if (abstop > 0x408u) {                               // |x| >= 1024
      if (ix == 0xfff0000000000000ull) return 0.0;
      if (abstop == 0x7ffu) return x + 1.0;               // inf, nan
      return (ix >> 63) ? 0.0 : hd(0x7ff0000000000000ull);
    }
    abstop = 0;                                          // large |x|: specialcase below
  }
  const double kd0 = __builtin_fma(x, hd(kExpHdr[0]), hd(kExpHdr[1]));   // InvLn2N * x + Shift
  const uint64_t ki = d2u(kd0);
  const double kd = kd0 - hd(kExpHdr[1]);
  double r = __builtin_fma(kd, hd(kExpHdr[2]), x);       // + kd * NegLn2hiN
  r = __builtin_fma(kd, hd(kExpHdr[3]), r);              // + kd * NegLn2loN
  const int idx = 2 * (int)(ki & 127u);
  const uint64_t top = ki << 45;
  const double t1 = __builtin_fma(r, hd(kExpHdr[5]), hd(kExpHdr[4]));    // C2 + r C3
  const double tailr = r + hd(kExpTab[idx]);
  const uint64_t sbits = kExpTab[idx + 1] + top;
  const double r2 = r * r;
  const double t2 = __builtin_fma(r, hd(kExpHdr[7]), hd(kExpHdr[6]));    // C4 + r C5
  double tmp = __builtin_fma(t1, r2, tailr);
  const double r4 = r2 * r2;
  tmp = __builtin_fma(r4, t2, tmp);
  if (abstop == 0) return exp_special(tmp, sbits, ki);
  const double scale = u2d(sbits);
  return __builtin_fma(scale, tmp, scale);
}

// ---- log -------------------------------------------------------------------
CTCX_HD double log(double x) {
  uint64_t ix = d2u(x);
  const uint32_t top = (uint32_t)(ix >> 48);
  if (ix - 0x3fee000000000000ull <= 0x308ffffffffffull) {   // x in [1 - 2^-4, 1 + 0x1.09p-4)
    if (ix == 0x3ff0000000000000ull) return 0.0;
    const double r = x - 1.0;
#define LB(i) hd(kLogHdr[7 + (i)])
    double b12 = __builtin_fma(r, LB(2), LB(1));
    double b45 = __builtin_fma(r, LB(5), LB(4));
    const double r2 = r * r;
    const double b78 = __builtin_fma(r, LB(8), LB(7));
    b12 = __builtin_fma(r2, LB(3), b12);
    b45 = __builtin_fma(r2, LB(6), b45);
    const double r3 = r * r2;
    double p3 = __builtin_fma(r2, LB(9), b78);
    p3 = __builtin_fma(r3, LB(10), p3);
    const double p2 = __builtin_fma(p3, r3, b45);
    const double p1 = __builtin_fma(p2, r3, b12);
    // rhi = r + w - w with w = r * 0x1p27, both sums fused with the product
    const double rw = __builtin_fma(r, hd(0x41a0000000000000ull), r);
    const double rhi = __builtin_fma(-hd(0x41a0000000000000ull), r, rw);
    const double rr = rhi * rhi;
    const double rlo = r - rhi;
    const double hi = __builtin_fma(rr, LB(0), r);        // r + rhi^2 * B0
    const double rmh = r - hi;
    const double rpr = r + rhi;
    double lo = __builtin_fma(rr, LB(0), rmh);
    const double t = LB(0) * rlo;
    lo = __builtin_fma(t, rpr, lo);
    const double y = __builtin_fma(p1, r3, lo);
#undef LB
    return hi + y;
  }
  if (top - 0x10u > 0x7fdfu) {                 // x < 0x1p-1022 or inf or nan
    if ((ix << 1) == 0) return -hd(0x7ff0000000000000ull);   // log(+-0) = -inf
    if (ix == 0x7ff0000000000000ull) return x;                // log(inf) = inf
    if ((top & 0x8000u) || (top & 0x7ff0u) == 0x7ff0u) return (x - x) / (x - x);
    ix = d2u(x * hd(0x4330000000000000ull)) - (52ull << 52);  // subnormal: normalise
  }
  const uint64_t tmp = ix - 0x3fe6000000000000ull;
  const int i = (int)((tmp >> 45) & 127u);
  const int k = (int)((int64_t)tmp >> 52);
  const uint64_t iz = ix - (tmp & 0xfff0000000000000ull);
  const double invc = hd(kLogTab[2 * i]), logc = hd(kLogTab[2 * i + 1]);
  const double z = u2d(iz);
  const double kd = (double)k;
#define LA(i) hd(kLogHdr[2 + (i)])
  const double r = __builtin_fma(z, invc, -1.0);
  const double w = __builtin_fma(kd, hd(kLogHdr[0]), logc);   // kd * Ln2hi + logc
  const double a12 = __builtin_fma(r, LA(2), LA(1));
  const double hi = r + w;
  const double r2 = r * r;
  double lo = (w - hi) + r;
  lo = __builtin_fma(kd, hd(kLogHdr[1]), lo);                 // + kd * Ln2lo
  const double r3 = r * r2;
  const double a34 = __builtin_fma(r, LA(4), LA(3));
  const double lo2 = __builtin_fma(r2, LA(0), lo);
  const double p = __builtin_fma(a34, r2, a12);
  const double y = __builtin_fma(r3, p, lo2);
#undef LA
  return y + hi;
}

}  // namespace gm
}  // namespace ctcx
