// glibc_math.h — device pow(), sin(), cos(), sincos() that return glibc's bits.
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

// Table access.  On the device the lookups are per-lane gathers; from __constant__
// memory they go through L1/L2 and their latency stalls the two resident waves, so a
// kernel can stage the tables in LDS once per workgroup (tables_to_lds) and build with
// GRT_GLIBC_LDS.  Same values either way.
#if defined(__HIPCC__) && defined(GRT_GLIBC_LDS) && GRT_GLIBC_LDS
__shared__ double lds_sincos[440];
__shared__ double lds_powlog[128 * 3];
__shared__ uint64_t lds_exp[256];
#define GRT_SINCOS(k) lds_sincos[k]
#define GRT_POWLOG(i, j) lds_powlog[(i) * 3 + (j)]
#define GRT_EXPTAB(k) lds_exp[k]
// every thread of the block must call this before any lookup
__device__ static inline void tables_to_lds() {
  for (unsigned i = threadIdx.x; i < 440u; i += blockDim.x) lds_sincos[i] = SINCOS_TAB[i];
  for (unsigned i = threadIdx.x; i < 384u; i += blockDim.x) lds_powlog[i] = POW_LOG_TAB[i / 3][i % 3];
  for (unsigned i = threadIdx.x; i < 256u; i += blockDim.x) lds_exp[i] = EXP_TAB[i];
  __syncthreads();
}
#else
#define GRT_SINCOS(k) SINCOS_TAB[k]
#define GRT_POWLOG(i, j) POW_LOG_TAB[i][j]
#define GRT_EXPTAB(k) EXP_TAB[k]
#if defined(__HIPCC__)
__device__ static inline void tables_to_lds() {}
#endif
#endif

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
  const double invc = GRT_POWLOG(i, 0), logc = GRT_POWLOG(i, 1), logctail = GRT_POWLOG(i, 2);
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
  const double tail = as_f64(GRT_EXPTAB(idx));
  const uint64_t sbits = GRT_EXPTAB(idx + 1) + top;
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

// ---------------------------------------------------------------------- exp ----
// glibc 2.35 __exp_fma (sysdeps/ieee754/dbl-64/e_exp.c, ARM optimized routines, the
// FMA ifunc build): x = k ln2/128 + r, exp(x) = 2^(k/128) exp(r) with the same
// __exp_data table and polynomial as pow's exp_inline above.  Every fma_() below is
// one vfmadd of the disassembled __exp_fma; specialcase() follows its k > 0 (scale
// 2^1009) and k < 0 (subnormal rounding) branches.  Defined for every input
// (tests/test_glibc_math.py checks it against glibc exp, bit for bit).
GRT_GLIBC_FN double exp_special(double tmp, uint64_t sbits, uint64_t ki) {
  if ((ki & 0x80000000ull) == 0) {  // k > 0: the exponent of scale may have overflowed
    const double scale = as_f64(sbits - (1009ull << 52));
    return fma_(scale, tmp, scale) * 0x1p1009;
  }
  const double scale = as_f64(sbits + (1022ull << 52));  // k < 0: subnormal range
  const double st = tmp * scale;
  double y = scale + st;
  if (y < 1.0) {  // round y before scaling it into the subnormal range
    const double hi = y + 1.0;
    double lo = (scale - y) + st;
    const double one_minus_hi = 1.0 - hi;
    y = (((one_minus_hi + y) + lo) + hi) - 1.0;
    if (y == 0.0) return 0.0;
  }
  return y * 0x1p-1022;
}

GRT_GLIBC_FN double exp_(double x) {
  uint32_t abstop = (uint32_t)(as_u64(x) >> 52) & 0x7ffu;
  if (abstop - 0x3c9u > 0x3eu) {        // |x| < 2^-54 or |x| >= 512 (or inf / nan)
    if ((int32_t)(abstop - 0x3c9u) < 0) return 1.0 + x;  // tiny |x|
    if (abstop > 0x408u) {              // |x| >= 1024
      if (as_u64(x) == 0xfff0000000000000ull) return 0.0;
      if (abstop == 0x7ffu) return 1.0 + x;  // inf / nan
      return (as_u64(x) >> 63) ? 0.0 : __builtin_inf();  // __math_uflow / __math_oflow
    }
    abstop = 0;                         // 512 <= |x| < 1024: specialcase below
  }
  const double kd = fma_(x, EXP_INVLN2N, EXP_SHIFT);
  const uint64_t ki = as_u64(kd);
  const double kn = kd - EXP_SHIFT;
  double r = fma_(kn, EXP_NEGLN2HIN, x);
  r = fma_(kn, EXP_NEGLN2LON, r);
  const uint32_t idx = (uint32_t)(ki & 127u) * 2u;
  const uint64_t top = ki << 45;
  const double tail = as_f64(GRT_EXPTAB(idx));
  const uint64_t sbits = GRT_EXPTAB(idx + 1) + top;
  const double p23 = fma_(r, EXP_C3, EXP_C2);
  const double tr = r + tail;
  const double r2 = r * r;
  const double p45 = fma_(r, EXP_C5, EXP_C4);
  const double tmp = fma_(r2 * r2, p45, fma_(p23, r2, tr));
  if (abstop == 0) return exp_special(tmp, sbits, ki);
  const double scale = as_f64(sbits);
  return fma_(scale, tmp, scale);
}

// ---------------------------------------------------------------- sin / cos ----
// glibc 2.35 __sin_fma / __cos_fma (sysdeps/ieee754/dbl-64/s_sin.c, the IBM accurate
// mathematical library, built with FMA contraction).  do_sin / do_cos / TAYLOR_SIN /
// reduce_sincos below follow the disassembled FMA variant: each fma_() is one
// vfmadd/vfnmadd/vfmsub of __sin_fma / __cos_fma.  Covers |x| < 105414350 (the range
// before glibc's __branred large-argument reduction); the caller falls back beyond.

GRT_GLIBC_FN double copysign_(double mag, double sgn) {
  return as_f64((as_u64(mag) & 0x7fffffffffffffffull) | (as_u64(sgn) & 0x8000000000000000ull));
}
GRT_GLIBC_FN double fabs_(double x) { return as_f64(as_u64(x) & 0x7fffffffffffffffull); }

// TAYLOR_SIN (xx = a*a): a + ((POLY(xx) * a - 0.5 * da) * xx + da)
GRT_GLIBC_FN double taylor_sin(double a, double da) {
  const double xx = a * a;
  const double poly = fma_(fma_(fma_(fma_(S5, xx, S4), xx, S3), xx, S2), xx, S1);
  const double t = fma_(xx, fma_(poly, a, -(0.5 * da)), da);
  return a + t;
}

// do_sin (x, dx): sin(x + dx)
GRT_GLIBC_FN double do_sin(double x, double dx) {
  if (fabs_(x) < TAYLOR_MAX) return taylor_sin(x, dx);
  if (!(x > 0.0)) dx = -dx;
  const double u = BIG + fabs_(x);
  const double xr = fabs_(x) - (u - BIG);
  const int k = (int)((uint32_t)as_u64(u) << 2);
  const double sn = GRT_SINCOS(k), ssn = GRT_SINCOS(k + 1), cs = GRT_SINCOS(k + 2), ccs = GRT_SINCOS(k + 3);
  const double xx = xr * xr;
  const double s = xr + fma_(xr * xx, fma_(xx, SN5, SN3), dx);
  const double c = fma_(xr, dx, xx * fma_(xx, fma_(xx, CS6, CS4), CS2));
  const double cor = fma_(s, cs, fma_(-c, sn, fma_(s, ccs, ssn)));
  return copysign_(sn + cor, x);
}

// do_cos (x, dx): cos(x + dx)
GRT_GLIBC_FN double do_cos(double x, double dx) {
  if (x < 0.0) dx = -dx;
  const double u = BIG + fabs_(x);
  const double xr = (fabs_(x) - (u - BIG)) + dx;
  const int k = (int)((uint32_t)as_u64(u) << 2);
  const double sn = GRT_SINCOS(k), ssn = GRT_SINCOS(k + 1), cs = GRT_SINCOS(k + 2), ccs = GRT_SINCOS(k + 3);
  const double xx = xr * xr;
  const double s = fma_(xr * xx, fma_(xx, SN5, SN3), xr);
  const double c = xx * fma_(xx, fma_(xx, CS6, CS4), CS2);
  const double cor = fma_(-s, sn, fma_(-c, cs, fma_(-s, ssn, ccs)));
  return cs + cor;
}

// reduce_sincos: x = n * pi/2 + (a + da), |x| < 105414350
GRT_GLIBC_FN int reduce_sincos(double x, double* a, double* da) {
  const double t = fma_(x, HPINV, TOINT);
  const double xn = t - TOINT;
  const double y = fma_(-xn, MP2, fma_(-xn, MP1, x));
  const int n = (int)((uint32_t)as_u64(t) & 3u);
  const double t2 = fma_(-xn, PP3, y);
  double db = fma_(-PP3, xn, y - t2);
  const double b = fma_(-xn, PP4, t2);
  db = db + fma_(-xn, PP4, t2 - b);
  *a = b;
  *da = db;
  return n;
}

GRT_GLIBC_FN double do_sincos(double a, double da, int n) {
  const double r = (n & 1) ? do_cos(a, da) : do_sin(a, da);
  return (n & 2) ? -r : r;
}

// Returns true and sin(x) in *out for |x| < 105414350 (glibc's bits).
GRT_GLIBC_FN bool sin_fast(double x, double* out) {
  const uint32_t k = (uint32_t)(as_u64(x) >> 32) & 0x7fffffffu;
  if (k < 0x3e500000u) {
    *out = x;
  } else if (k < 0x3feb6000u) {
    *out = do_sin(x, 0.0);
  } else if (k < 0x400368fdu) {
    const double t = HP0 - fabs_(x);
    *out = copysign_(do_cos(t, HP1), x);
  } else if (k < 0x419921fbu) {
    double a, da;
    const int n = reduce_sincos(x, &a, &da);
    *out = do_sincos(a, da, n);
  } else {
    return false;
  }
  return true;
}

// Returns true and cos(x) in *out for |x| < 105414350 (glibc's bits).
GRT_GLIBC_FN bool cos_fast(double x, double* out) {
  const uint32_t k = (uint32_t)(as_u64(x) >> 32) & 0x7fffffffu;
  if (k < 0x3e400000u) {
    *out = 1.0;
  } else if (k < 0x3feb6000u) {
    *out = do_cos(x, 0.0);
  } else if (k < 0x400368fdu) {
    const double y = HP0 - fabs_(x);
    const double a = y + HP1;
    const double da = (y - a) + HP1;
    *out = do_sin(a, da);
  } else if (k < 0x419921fbu) {
    double a, da;
    const int n = reduce_sincos(x, &a, &da);
    *out = do_sincos(a, da, n + 1);
  } else {
    return false;
  }
  return true;
}

// ------------------------------------------------------------------- sincos ----
// glibc 2.35 __sincos (sysdeps/ieee754/dbl-64/s_sincos.c).  It has no ifunc: the
// baseline x86-64 build runs, i.e. the same IBM routines as sin/cos but WITHOUT FMA
// contraction.  Compilers fuse sin(x) and cos(x) of one operand into this call (LLVM's
// sincos libcall combine in the reference's Rust build, GCC's cse_sincos in the
// oracle), so wherever the reference evaluates both, the device must call this one.
// The *_nf helpers are s_sin.c's inline functions evaluated as written (device code is
// compiled with -ffp-contract=off).

GRT_GLIBC_FN double taylor_sin_nf(double a, double da) {
  const double xx = a * a;
  const double poly = (((S5 * xx + S4) * xx + S3) * xx + S2) * xx + S1;
  const double t = ((poly * a - 0.5 * da) * xx + da);
  return a + t;
}

GRT_GLIBC_FN double do_sin_nf(double x, double dx) {
#if defined(GRT_GLIBC_BRANCHLESS) && GRT_GLIBC_BRANCHLESS
  // both of glibc's forms, then a select: the same value as the branch, without the
  // divergent branch when a wave mixes |x| < 0.126 and |x| >= 0.126 lanes
  const double taylor = taylor_sin_nf(x, dx);
#else
  if (fabs_(x) < TAYLOR_MAX) return taylor_sin_nf(x, dx);
#endif
  if (x <= 0.0) dx = -dx;
  const double u = BIG + fabs_(x);
  const double xr = fabs_(x) - (u - BIG);
  const int k = (int)((uint32_t)as_u64(u) << 2);
  const double sn = GRT_SINCOS(k), ssn = GRT_SINCOS(k + 1), cs = GRT_SINCOS(k + 2), ccs = GRT_SINCOS(k + 3);
  const double xx = xr * xr;
  const double s = xr + (dx + xr * xx * (SN3 + xx * SN5));
  const double c = xr * dx + xx * (CS2 + xx * (CS4 + xx * CS6));
  const double cor = (ssn + s * ccs - sn * c) + cs * s;
#if defined(GRT_GLIBC_BRANCHLESS) && GRT_GLIBC_BRANCHLESS
  return fabs_(x) < TAYLOR_MAX ? taylor : copysign_(sn + cor, x);
#else
  return copysign_(sn + cor, x);
#endif
}

GRT_GLIBC_FN double do_cos_nf(double x, double dx) {
  if (x < 0.0) dx = -dx;
  const double u = BIG + fabs_(x);
  const double xr = fabs_(x) - (u - BIG) + dx;
  const int k = (int)((uint32_t)as_u64(u) << 2);
  const double sn = GRT_SINCOS(k), ssn = GRT_SINCOS(k + 1), cs = GRT_SINCOS(k + 2), ccs = GRT_SINCOS(k + 3);
  const double xx = xr * xr;
  const double s = xr + xr * xx * (SN3 + xx * SN5);
  const double c = xx * (CS2 + xx * (CS4 + xx * CS6));
  const double cor = (ccs - s * ssn - cs * c) - sn * s;
  return cs + cor;
}

GRT_GLIBC_FN int reduce_sincos_nf(double x, double* a, double* da) {
  const double t = (x * HPINV + TOINT);
  const double xn = t - TOINT;
  const double y = (x - xn * MP1) - xn * MP2;
  const int n = (int)((uint32_t)as_u64(t) & 3u);
  double t1 = xn * PP3;
  const double t2 = y - t1;
  double db = (y - t2) - t1;
  t1 = xn * PP4;
  const double b = t2 - t1;
  db += (t2 - b) - t1;
  *a = b;
  *da = db;
  return n;
}

GRT_GLIBC_FN double do_sincos_nf(double a, double da, int n) {
  const double r = (n & 1) ? do_cos_nf(a, da) : do_sin_nf(a, da);
  return (n & 2) ? -r : r;
}

// Returns true and (sin x, cos x) for |x| < 105414350 (glibc sincos's bits).
GRT_GLIBC_FN bool sincos_fast(double x, double* sinx, double* cosx) {
  const uint32_t k = (uint32_t)(as_u64(x) >> 32) & 0x7fffffffu;
  if (k < 0x400368fdu) {
    if (k < 0x3e400000u) {
      *sinx = x;
      *cosx = 1.0;
    } else if (k < 0x3feb6000u) {
      *sinx = do_sin_nf(x, 0.0);
      *cosx = do_cos_nf(x, 0.0);
    } else {
      const double y = HP0 - fabs_(x);
      const double a = y + HP1;
      const double da = (y - a) + HP1;
      *sinx = copysign_(do_cos_nf(y, HP1), x);
      *cosx = do_sin_nf(a, da);
    }
    return true;
  }
  if (k < 0x419921fbu) {
    double a, da;
    const int n = reduce_sincos_nf(x, &a, &da);
    *sinx = do_sincos_nf(a, da, n);
    *cosx = do_sincos_nf(a, da, n + 1);
    return true;
  }
  return false;
}

// The commonest case of sincos_fast for a polar angle near the equator, as straight-line
// code: region B (0.855469 <= |x| < 2.426265, where sin x = +-do_cos(pi/2 - |x|) and
// cos x = do_sin(a, da)) with do_sin's table path (|a| >= TAYLOR_MAX).  sincos_b_table_ok
// says whether x is in that case; sincos_b_table then returns sincos_fast's bits.
GRT_GLIBC_FN bool sincos_b_table_ok(double x) {
  const uint32_t k = (uint32_t)(as_u64(x) >> 32) & 0x7fffffffu;
  const double y = HP0 - fabs_(x);
  const double a = y + HP1;
  return k >= 0x3feb6000u && k < 0x400368fdu && !(fabs_(a) < TAYLOR_MAX);
}
GRT_GLIBC_FN void sincos_b_table(double x, double* sinx, double* cosx) {
  const double y = HP0 - fabs_(x);
  const double a = y + HP1;
  double da = (y - a) + HP1;
  *sinx = copysign_(do_cos_nf(y, HP1), x);
  // do_sin_nf(a, da) past its Taylor branch
  if (a <= 0.0) da = -da;
  const double u = BIG + fabs_(a);
  const double xr = fabs_(a) - (u - BIG);
  const int k = (int)((uint32_t)as_u64(u) << 2);
  const double sn = GRT_SINCOS(k), ssn = GRT_SINCOS(k + 1), cs = GRT_SINCOS(k + 2), ccs = GRT_SINCOS(k + 3);
  const double xx = xr * xr;
  const double s = xr + (da + xr * xx * (SN3 + xx * SN5));
  const double c = xr * da + xx * (CS2 + xx * (CS4 + xx * CS6));
  const double cor = (ssn + s * ccs - sn * c) + cs * s;
  *cosx = copysign_(sn + cor, a);
}

// Region B with do_sin's Taylor branch (|a| < TAYLOR_MAX: x within ~7 degrees of pi/2).
GRT_GLIBC_FN bool sincos_b_taylor_ok(double x) {
  const uint32_t k = (uint32_t)(as_u64(x) >> 32) & 0x7fffffffu;
  const double y = HP0 - fabs_(x);
  const double a = y + HP1;
  return k >= 0x3feb6000u && k < 0x400368fdu && fabs_(a) < TAYLOR_MAX;
}
GRT_GLIBC_FN void sincos_b_taylor(double x, double* sinx, double* cosx) {
  const double y = HP0 - fabs_(x);
  const double a = y + HP1;
  const double da = (y - a) + HP1;
  *sinx = copysign_(do_cos_nf(y, HP1), x);
  *cosx = taylor_sin_nf(a, da);
}

// sincos_fast without the region branches, for angles spread over (-pi, pi] within a
// wave (the VolumetricDisc's in-plane angle): every region of sincos_fast evaluates one
// do_sin_nf and one do_cos_nf, so the arguments are selected per lane, both are
// evaluated once (do_sin_nf's Taylor branch as a select too), and the results are
// routed and signed per region.  The same operations on the same operands as
// sincos_fast, hence the same bits (tests/test_glibc_math.py).
GRT_GLIBC_FN double do_sin_nf_sel(double x, double dx) {
  const double taylor = taylor_sin_nf(x, dx);
  if (x <= 0.0) dx = -dx;
  const double u = BIG + fabs_(x);
  const double xr = fabs_(x) - (u - BIG);
  const int k = (int)((uint32_t)as_u64(u) << 2);  // |x| < 0.855469 in every region: in the table
  const double sn = GRT_SINCOS(k), ssn = GRT_SINCOS(k + 1), cs = GRT_SINCOS(k + 2), ccs = GRT_SINCOS(k + 3);
  const double xx = xr * xr;
  const double s = xr + (dx + xr * xx * (SN3 + xx * SN5));
  const double c = xr * dx + xx * (CS2 + xx * (CS4 + xx * CS6));
  const double cor = (ssn + s * ccs - sn * c) + cs * s;
  return fabs_(x) < TAYLOR_MAX ? taylor : copysign_(sn + cor, x);
}

GRT_GLIBC_FN bool sincos_fast_uniform(double x, double* sinx, double* cosx) {
  const uint32_t k = (uint32_t)(as_u64(x) >> 32) & 0x7fffffffu;
  if (k >= 0x419921fbu) return false;
  const bool ra = k < 0x3feb6000u;                    // |x| < 0.855469: do_sin(x, 0), do_cos(x, 0)
  const bool rb = !ra && k < 0x400368fdu;             // |x| < 2.426265: pi/2 - |x| forms
  const double y = HP0 - fabs_(x);                    // region B
  const double ab = y + HP1;
  const double dab = (y - ab) + HP1;
  double ac, dac;                                     // region C: x = n pi/2 + (a + da)
  const int n = reduce_sincos_nf(x, &ac, &dac);
  const double s_x = ra ? x : (rb ? ab : ac);
  const double s_dx = ra ? 0.0 : (rb ? dab : dac);
  const double c_x = ra ? x : (rb ? y : ac);
  const double c_dx = ra ? 0.0 : (rb ? HP1 : dac);
  const double DS = do_sin_nf_sel(s_x, s_dx);
  const double DC = do_cos_nf(c_x, c_dx);
  double s, c;
  if (ra) {
    s = DS;
    c = DC;
  } else if (rb) {
    s = copysign_(DC, x);
    c = DS;
  } else {  // do_sincos_nf(a, da, n) and (.., n + 1)
    const double rs = (n & 1) ? DC : DS;
    const double rc = (n & 1) ? DS : DC;
    s = (n & 2) ? -rs : rs;
    c = ((n + 1) & 2) ? -rc : rc;
  }
  if (k < 0x3e400000u) {
    s = x;
    c = 1.0;
  }
  *sinx = s;
  *cosx = c;
  return true;
}

}  // namespace glibc
}  // namespace grt
