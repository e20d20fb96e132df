// glibc_math.h — device pow() that returns glibc's bits.
//
// The reference calls f64::powf, i.e. glibc's pow.  On x86-64 with FMA+AVX2 (every
// machine the reference plausibly runs on, including this image and the GPU boxes),
// glibc 2.35 dispatches pow to __pow_fma: the ARM optimized-routines algorithm,
//
//   log(x) = k ln2 + log(c) + log1p(z/c - 1)   (128-entry table, degree-8 polynomial,
//                                                double-double result hi + lo)
//   x^y    = exp(y * (hi + lo))                 (2^(i/128) table, degree-5 polynomial)
//
// compiled with FMA contraction.  pow_fast() below restates that code path operation
// by operation, with an explicit fma() exactly where __pow_fma executes vfmadd/vfmsub
// (decoded from its disassembly; tools/gen_glibc_tables.py extracts the tables), so
// the device result is bit-identical to glibc wherever the fast path applies:
//
//   x normal, positive, finite;  2^-65 <= |y| < 2^63;  2^-54 <= |y log x| < 512.
//
// Outside that domain (x <= 0, subnormal, inf/nan, results near under/overflow) the
// caller falls back to OCML's pow.  The step controller's argument eps/err lies in
// (1e-300, 1800) and y = 0.2, always on the fast path.  tests/test_glibc_math.py
// compiles this file for the host and checks it against glibc pow, bit for bit.
#pragma once
#include <stdint.h>
#include <string.h>

#if defined(__HIPCC__)
#define GRT_GLIBC_TABLE __device__ __constant__ static const
#define GRT_GLIBC_FN __device__ static inline
#else
#include <cmath>
#define GRT_GLIBC_TABLE static const
#define GRT_GLIBC_FN static inline
#endif

#include "glibc_tables.h"

namespace grt {
namespace glibc {

GRT_GLIBC_FN uint64_t as_u64(double x) {
  uint64_t u;
  memcpy(&u, &x, 8);
  return u;
}
GRT_GLIBC_FN double as_f64(uint64_t u) {
  double x;
  memcpy(&x, &u, 8);
  return x;
}
#if defined(__HIPCC__)
GRT_GLIBC_FN double fma_(double a, double b, double c) { return __builtin_fma(a, b, c); }
#else
GRT_GLIBC_FN double fma_(double a, double b, double c) { return std::fma(a, b, c); }
#endif

// Returns true and x^y in *out when (x, y) is on __pow_fma's fast path.
GRT_GLIBC_FN bool pow_fast(double x, double y, double* out) {
  const uint64_t ix = as_u64(x), iy = as_u64(y);
  const uint32_t topx = (uint32_t)(ix >> 52), topy = (uint32_t)(iy >> 52);
  if (topx - 1u > 0x7fdu) return false;                 // x <= 0, subnormal, inf, nan, or sign set
  if (((topy & 0x7ffu) - 0x3beu) > 0x7fu) return false;  // |y| < 2^-65 or >= 2^63 (or inf/nan)

  // ---- log_inline: hi + lo = log(x) ----
  const uint64_t tmp = ix - 0x3fe6955500000000ull;
  const int i = (int)((tmp >> 45) & 127u);
  const int32_t k = (int32_t)((int64_t)tmp >> 52);
  const uint64_t iz = ix - (tmp & 0xfff0000000000000ull);
  const double z = as_f64(iz);
  const double kd = (double)k;
  const double invc = POW_LOG_TAB[i][0], logc = POW_LOG_TAB[i][1], logctail = POW_LOG_TAB[i][2];
  const double t1 = fma_(kd, POW_LN2HI, logc);
  const double r = fma_(z, invc, -1.0);
  const double ar = r * POW_A[0];
  const double lo1 = fma_(kd, POW_LN2LO, logctail);
  const double q12 = fma_(r, POW_A[2], POW_A[1]);
  const double q34 = fma_(r, POW_A[4], POW_A[3]);
  const double t2 = r + t1;
  const double ar2 = r * ar;
  const double lo2 = (t1 - t2) + r;
  const double ar3 = r * ar2;
  const double lo3 = fma_(ar, r, -ar2);
  const double q56 = fma_(r, POW_A[6], POW_A[5]);
  const double hi = t2 + ar2;
  const double lo4 = (t2 - hi) + ar2;
  const double q = fma_(ar2, fma_(q56, ar2, q34), q12);
  const double lo = fma_(ar3, q, ((lo1 + lo2) + lo3) + lo4);
  const double lhi = hi + lo;
  const double llo = (hi - lhi) + lo;

  // ---- y * log(x) as ehi + elo ----
  const double ehi = y * lhi;
  const double elo = fma_(y, llo, fma_(lhi, y, -ehi));
  const uint32_t abstop = (uint32_t)(as_u64(ehi) >> 52) & 0x7ffu;
  if (abstop - 0x3c9u > 0x3eu) return false;  // |ehi| < 2^-54 or >= 512: special cases

  // ---- exp_inline(ehi, elo), sign_bias = 0 ----
  const double kd2 = fma_(ehi, EXP_INVLN2N, EXP_SHIFT);
  const uint64_t ki = as_u64(kd2);
  const double kn = kd2 - EXP_SHIFT;
  double re = fma_(kn, EXP_NEGLN2HIN, ehi);
  re = fma_(kn, EXP_NEGLN2LON, re);
  const uint32_t idx = (uint32_t)(ki & 127u) * 2u;
  const uint64_t top = ki << 45;
  const double tail = as_f64(EXP_TAB[idx]);
  const uint64_t sbits = EXP_TAB[idx + 1] + top;
  re = elo + re;
  const double p23 = fma_(re, EXP_C3, EXP_C2);
  const double tr = re + tail;
  const double r2 = re * re;
  const double p45 = fma_(re, EXP_C5, EXP_C4);
  const double t = fma_(p45, r2 * r2, fma_(p23, r2, tr));
  const double scale = as_f64(sbits);
  *out = fma_(t, scale, scale);
  return true;
}

}  // namespace glibc
}  // namespace grt
