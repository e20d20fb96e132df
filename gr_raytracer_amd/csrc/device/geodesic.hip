// geodesic.hip — gfx950 kernels for the per-pixel geodesic hot path.
//
// One lane traces one camera ray from creation to final colour, entirely in VGPRs:
//   camera ray (camera.rs:214-254) -> RKF45 attempts (runge_kutta.rs:86-182)
//   -> for every accepted step: chord window test against every object
//      (objects.rs:65-120, disc.rs:41-88, sphere.rs:37-128), emitter redshift +
//      temperature + texture (redshift.rs, temperature.rs, texture.rs), then the
//      stop test (integrator.rs:203-268)
//   -> terminal colour + back-to-front blend (scene.rs:153-219).
// The reference stores the whole trajectory (Vec<Step>, 112 B/step) and runs the
// window pass afterwards; here the window test is fused into the step loop, which
// visits exactly the same windows in the same order, so no trajectory ever leaves
// the register file.
//
// The grid is persistent: each wave claims work items from one global
// counter, and whenever lanes finish their ray a wave ballot hands them the next
// items (lane refill), so long (near-photon-sphere) and short (captured) rays never
// leave lanes idle until the queue is empty.
//
// Floating point follows the reference's evaluation order (Rust, no contraction);
// the library is compiled with -ffp-contract=off.  Per-frame constants that need
// libm (sin/cos of the camera position, tan(alpha/2), LUTs) are evaluated on the
// host.  pow() is glibc's own algorithm restated bit-exactly (glibc_math.h); the
// remaining per-step transcendentals (sin/cos/atan2/acos) use the device libm (OCML).
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "grt_api.h"
#include "dev_scene.h"
#ifndef GRT_GLIBC_LDS
#define GRT_GLIBC_LDS 1  // glibc tables staged in LDS per workgroup (measured -1..2%)
#endif
#include "glibc_math.h"
#include "kernels.h"

// GRT_FUSED: this file compiled a second time, by geodesic_fused.hip, with FMA contraction
// (-ffp-contract=fast) into namespace grt::fused: the trace kernels of the light charts
// for grt_set_arithmetic(1).  Only launch_trace is defined there (Kerr-Schild excluded).
#ifndef GRT_FUSED
#define GRT_FUSED 0
#endif
// GRT_KERR_BL_TU: this file compiled a second time, by geodesic_kerr_bl.hip, without the
// machine-level loop-invariant code motion, into namespace grt::kerr_bl: the KerrBL trace
// kernels (launch_trace for GRT_GEOM_KERR_BL only; the exact build leaves them out).
#ifndef GRT_KERR_BL_TU
#define GRT_KERR_BL_TU 0
#endif
#define GRT_MAIN_TU (!GRT_FUSED && !GRT_KERR_BL_TU)

namespace grt {
#if GRT_FUSED
namespace fused {
#elif GRT_KERR_BL_TU
namespace kerr_bl {
#endif

#ifndef GDEV
#define GDEV __device__ __forceinline__
#endif

#ifndef GRT_SHARED_DIV
#define GRT_SHARED_DIV 1
#endif
#ifndef GRT_UNIT_H
#define GRT_UNIT_H 1  // far-field attempts of a wave with h == 1 everywhere skip h * o
#endif
#ifndef GRT_KLDS_GEOMS
#define GRT_KLDS_GEOMS (1 << GRT_GEOM_KERR)  // integrate kernels whose RKF stages k1..k4 live in LDS
#endif
#ifndef GRT_SINCOS_B
#define GRT_SINCOS_B 1  // Schwarzschild / KerrBL RHS: wave-uniform straight-line sincos (region B)
#endif
#ifndef GRT_FAST_DIV
#define GRT_FAST_DIV 1  // Schwarzschild / KerrBL region-B RHS: divisions without range steps when the operands allow
#endif
#ifndef GRT_FAST_DIV_KS
#define GRT_FAST_DIV_KS 1  // Kerr-Schild RHS: metric quotients without v_div_scale when the state allows
#endif
#ifndef GRT_FAST_SQRT_KS
#define GRT_FAST_SQRT_KS 1  // and its square roots without the range steps (sqrt_fx)
#endif
#ifndef GRT_FAST_DIV_BL
// KerrBL too: C3 is no faster with it (165-172 ms either way), but its 3-wave kernel's
// spills land elsewhere: 1.71 GB written per frame with it, 20.9 GB without
// (profiles/r04n_c3_pmc.json, r04o_c3_pmc.json)
#define GRT_FAST_DIV_BL 1
#endif
#ifndef GRT_QUICK_STEP
#define GRT_QUICK_STEP 1  // Schwarzschild: the far-field accepted step as one straight-line block
#endif
#ifndef GRT_KL_STAGES
#define GRT_KL_STAGES 4  // how many leading stages (k1, k2, ...) those kernels park in LDS
#endif
#ifndef GRT_TAIL_PRIO
#define GRT_TAIL_PRIO 1  // light charts: issue priority by steps left once the queue drains (C5 -1.2%, profiles/r05i)
#endif
#ifndef GRT_RAY_TIMES
#define GRT_RAY_TIMES 0  // diagnostic builds only: per-ray schedule record (tools/c4_ray_times.py)
#endif

// The OCML fallbacks below run outside glibc's fast paths only (never for the angles and
// controller ratios of a render): out of line, so their code stays out of the hot loops.
#ifndef GRT_SLOW_NOINLINE
#define GRT_SLOW_NOINLINE 1
#endif
#if GRT_SLOW_NOINLINE
#define GRT_SLOW __device__ __attribute__((noinline, cold))
#else
#define GRT_SLOW GDEV
#endif
GRT_SLOW double ocml_pow(double x, double y) { return pow(x, y); }
// returned by value: a pointer into the caller's frame passed to an out-of-line call would
// keep the caller's (sin, cos) in scratch memory at every rsincos site, fast path included
struct SinCos {
  double s, c;
};
GRT_SLOW SinCos ocml_sincos(double x) {
  SinCos r;
  sincos(x, &r.s, &r.c);
  return r;
}
GRT_SLOW double ocml_sin(double x) { return sin(x); }
GRT_SLOW double ocml_cos(double x) { return cos(x); }

// f64::powf == glibc pow: bit-exact on glibc's fast path, OCML outside it.
GDEV double rpow(double x, double y) {
  double r;
  if (glibc::pow_fast(x, y, &r)) return r;
  return ocml_pow(x, y);
}
// f64::sin / f64::cos of one operand in one reference function: the compiler fuses
// them into glibc's sincos (glibc_math.h); a lone sin() stays glibc's sin.  Both are
// bit-exact for |x| < 105414350; OCML beyond (never reached by angles here).
GDEV void rsincos(double x, double* s, double* c) {
  double ss, cc;
  if (!glibc::sincos_fast(x, &ss, &cc)) {
    const SinCos r = ocml_sincos(x);
    ss = r.s;
    cc = r.c;
  }
  *s = ss;
  *c = cc;
}
GDEV double rsin(double x) {
  double r;
  if (glibc::sin_fast(x, &r)) return r;
  return ocml_sin(x);
}
GDEV double rcos(double x) {
  double r;
  if (glibc::cos_fast(x, &r)) return r;
  return ocml_cos(x);
}

// x1 / y and x2 / y with one reciprocal refinement.  This is the compiler's own IEEE f64
// division expansion (div_scale, rcp, 2 Newton steps, div_fmas, div_fixup -- identical
// instructions), with the y-only part shared.  The shared part is v_div_scale(y, y, x),
// whose result depends on x only when |x| is extreme (exponent gap >= 768, x/y
// denormal, or exp(x) <= 53); the host enables this (DevScene::div_share) only when
// both numerators are normal with |exponent| < 500, where it cannot.  Every quotient
// is therefore bit-identical to x / y.
GDEV void div2_same_den(double x1, double x2, double y, double* q1, double* q2) {
  bool f0, f1, f2;
  const double ds0 = __builtin_amdgcn_div_scale(x1, y, false, &f0);
  const double rcp = __builtin_amdgcn_rcp(ds0);
  const double fma0 = __builtin_fma(-ds0, rcp, 1.0);
  const double fma1 = __builtin_fma(rcp, fma0, rcp);
  const double fma2 = __builtin_fma(-ds0, fma1, 1.0);
  const double fma3 = __builtin_fma(fma1, fma2, fma1);
  const double n1 = __builtin_amdgcn_div_scale(x1, y, true, &f1);
  const double m1 = n1 * fma3;
  *q1 = __builtin_amdgcn_div_fixup(__builtin_amdgcn_div_fmas(__builtin_fma(-ds0, m1, n1), fma3, m1, f1), y, x1);
  const double n2 = __builtin_amdgcn_div_scale(x2, y, true, &f2);
  const double m2 = n2 * fma3;
  *q2 = __builtin_amdgcn_div_fixup(__builtin_amdgcn_div_fmas(__builtin_fma(-ds0, m2, n2), fma3, m2, f2), y, x2);
}

// x / y as that same expansion without its range steps, for operands the caller has
// shown to be normals with |x|, |y|, |x / y| all within 2^-600 .. 2^600: there
// v_div_scale returns its operand unchanged and raises no flag (the exponent gap is
// < 768, neither 1 / y nor x / y is denormal, exp(x) > 53), so v_div_fmas is a plain
// fma, and v_div_fixup, which only rewrites NaN / infinity / zero / overflow / underflow
// cases, passes the quotient through.
// The same instructions on the same values, hence x / y's bits.  Measured over the whole
// exponent plane, the exact region is larger (E: |y| normal below 2^1022, x of exponent
// >= -969, gap -1021 .. 1022; the gap >= 768 scaling is an identity there too), and the
// first failures are one exponent outside it (tests/test_gpu_arith.py
// ::test_range_free_arithmetic_map, profiles/r05a/arith_map.json).
// 8 VALU instead of 11; div2_inrange shares 1 / y: 11 instead of 16.
GDEV double div_inrange(double x, double y) {
  const double rcp = __builtin_amdgcn_rcp(y);
  const double fma0 = __builtin_fma(-y, rcp, 1.0);
  const double fma1 = __builtin_fma(rcp, fma0, rcp);
  const double fma2 = __builtin_fma(-y, fma1, 1.0);
  const double fma3 = __builtin_fma(fma1, fma2, fma1);
  const double m = x * fma3;
  return __builtin_fma(__builtin_fma(-y, m, x), fma3, m);
}
GDEV void div2_inrange(double x1, double x2, double y, double* q1, double* q2) {
  const double rcp = __builtin_amdgcn_rcp(y);
  const double fma0 = __builtin_fma(-y, rcp, 1.0);
  const double fma1 = __builtin_fma(rcp, fma0, rcp);
  const double fma2 = __builtin_fma(-y, fma1, 1.0);
  const double fma3 = __builtin_fma(fma1, fma2, fma1);
  const double m1 = x1 * fma3;
  *q1 = __builtin_fma(__builtin_fma(-y, m1, x1), fma3, m1);
  const double m2 = x2 * fma3;
  *q2 = __builtin_fma(__builtin_fma(-y, m2, x2), fma3, m2);
}
// |x| in (2^-300, 2^300), NaN excluded: two compares with the abs modifier
GDEV bool in_div_range(double x) { return fabs(x) > 0x1p-300 && fabs(x) < 0x1p300; }

// x / y as the compiler's expansion without its two v_div_scale steps but with
// v_div_fixup: exact (the same instructions on the same values) when y is a normal within
// 2^+-600 and x is 0 or a normal with |x|, |x / y| within 2^+-600 -- v_div_scale would
// return its operand unchanged with no flag (so v_div_fmas is a plain fma), and
// v_div_fixup rewrites the zero-numerator case from the operands alone (a -0 / y chain
// gives +0; the fixup returns the signed zero).  9 VALU instead of 11.
GDEV double div_fx(double x, double y) {
  const double rcp = __builtin_amdgcn_rcp(y);
  const double fma0 = __builtin_fma(-y, rcp, 1.0);
  const double fma1 = __builtin_fma(rcp, fma0, rcp);
  const double fma2 = __builtin_fma(-y, fma1, 1.0);
  const double fma3 = __builtin_fma(fma1, fma2, fma1);
  const double m = x * fma3;
  return __builtin_amdgcn_div_fixup(__builtin_fma(__builtin_fma(-y, m, x), fma3, m), y, x);
}

// Kerr-Schild metric quotients: the compiler's division, or div_fx (FD) where the caller
// has established ks_fd_ok for the state
template <bool FD>
GDEV double kdiv(double x, double y) {
  if constexpr (FD) return div_fx(x, y);
  else return x / y;
}
// sqrt(x) as the compiler's f64 expansion for gfx950 without its range steps: for a
// normal x >= 2^-767 the input scaling (ldexp by 0), the output rescaling and the
// zero / infinity select are identities, leaving v_rsq_f64 and the Newton steps on the
// same values, hence sqrt's bits (device check: tests/test_gpu_arith.py: exact for every
// x >= 2^-969, the first failure at 2^-971).  10 VALU instead of 17.
GDEV double sqrt_fx(double x) {
  const double r = __builtin_amdgcn_rsq(x);
  double g = x * r, h = r * 0.5;
  const double e = __builtin_fma(-h, g, 0.5);
  g = __builtin_fma(g, e, g);
  h = __builtin_fma(h, e, h);
  double d = __builtin_fma(-g, g, x);
  g = __builtin_fma(d, h, g);
  d = __builtin_fma(-g, g, x);
  return __builtin_fma(d, h, g);
}
template <bool FD>
GDEV double ksqrt(double x) {
  if constexpr (FD && GRT_FAST_SQRT_KS) return sqrt_fx(x);
  else return sqrt(x);
}

#if GRT_MAIN_TU
// Device check of div_inrange / div2_inrange / div_fx / sqrt_fx against the compiler's
// division and sqrt over the whole exponent plane (tests/test_gpu_parity.py
// ::test_range_free_arithmetic_map): thread (ex, ey), ex, ey biased exponents 0 .. 2046
// (0: subnormals), runs `samples` operand pairs x = +-m_x 2^(ex-1023), y = +-m_y 2^(ey-1023)
// -- the first four with extreme mantissas (0 / all ones), the rest splitmix64-random, and
// a second numerator x2 of the same exponent for div2_inrange -- and sets in map[ex][ey]:
//   1 div_inrange(x, y) != x / y      2 div2_inrange(x, x2, y) != (x / y, x2 / y)
//   4 div_fx(x, y) != x / y
// Threads with ex == 0 also set zmap[ey] |= 8 when div_fx(+-0, y) != +-0 / y, and threads
// with ey == 0 set smap[ex] |= 16 when sqrt_fx(x) != sqrt(x) for positive x of exponent ex.
__global__ void arith_map_kernel(uint32_t samples, uint64_t seed, uint8_t* map, uint8_t* zmap, uint8_t* smap) {
  const uint32_t cell = blockIdx.x * blockDim.x + threadIdx.x;
  if (cell >= 2047u * 2047u) return;
  const uint32_t ex = cell / 2047u, ey = cell % 2047u;
  auto mix = [](uint64_t z) {
    z += 0x9e3779b97f4a7c15ull;
    z = (z ^ (z >> 30)) * 0xbf58476d1ce4e5b9ull;
    z = (z ^ (z >> 27)) * 0x94d049bb133111ebull;
    return z ^ (z >> 31);
  };
  constexpr uint64_t MANT = 0x000fffffffffffffull;
  auto bits = [](double v) { return (uint64_t)__double_as_longlong(v); };
  auto make = [](uint64_t sign, uint64_t e, uint64_t m) {
    return __longlong_as_double((long long)((sign << 63) | (e << 52) | m));
  };
  uint32_t flags = 0, zflags = 0, sflags = 0;
  for (uint32_t k = 0; k < samples; ++k) {
    const uint64_t u = mix(seed ^ ((uint64_t)cell * 64 + 3 * k + 1)), v = mix(seed ^ ((uint64_t)cell * 64 + 3 * k + 2)),
                   w = mix(seed ^ ((uint64_t)cell * 64 + 3 * k + 3));
    const uint64_t mx = k < 4 ? ((k & 1) ? MANT : 0) : (u & MANT);
    const uint64_t my = k < 4 ? ((k & 2) ? MANT : 0) : (v & MANT);
    const double x = make(u >> 63, ex, mx), y = make(v >> 63, ey, my), x2 = make(w >> 63, ex, w & MANT);
    volatile double vx = x, vy = y, vx2 = x2;  // keep the reference divisions as divisions
    const double ref1 = vx / vy, ref2 = vx2 / vy;
    double q1, q2;
    div2_inrange(x, x2, y, &q1, &q2);
    if (bits(div_inrange(x, y)) != bits(ref1)) flags |= 1u;
    if (bits(q1) != bits(ref1) || bits(q2) != bits(ref2)) flags |= 2u;
    if (bits(div_fx(x, y)) != bits(ref1)) flags |= 4u;
    if (ex == 0) {
      const double z0 = (u >> 62) & 1 ? -0.0 : 0.0;
      volatile double vz = z0;
      if (bits(div_fx(z0, y)) != bits(vz / vy)) zflags |= 8u;
    }
    if (ey == 0) {
      const double sx = fabs(x);
      volatile double vsx = sx;
      if (bits(sqrt_fx(sx)) != bits(sqrt(vsx))) sflags |= 16u;
    }
  }
  map[cell] = (uint8_t)flags;
  if (ex == 0) zmap[ey] = (uint8_t)zflags;
  if (ey == 0) smap[ex] = (uint8_t)sflags;
}
#endif  // GRT_MAIN_TU

constexpr double PI = 3.14159265358979323846;
constexpr double TWO_PI = 2.0 * 3.14159265358979323846;

// runge_kutta.rs:16-84
constexpr double B21 = 2.0 / 9.0;
constexpr double B31 = 1.0 / 12.0, B32 = 1.0 / 4.0;
constexpr double B41 = 69.0 / 128.0, B42 = -243.0 / 128.0, B43 = 135.0 / 64.0;
constexpr double B51 = -17.0 / 12.0, B52 = 27.0 / 4.0, B53 = -27.0 / 5.0, B54 = 16.0 / 15.0;
constexpr double B61 = 65.0 / 432.0, B62 = -5.0 / 16.0, B63 = 13.0 / 16.0, B64 = 4.0 / 27.0,
                 B65 = 5.0 / 144.0;
constexpr double CH1 = 47.0 / 450.0, CH2 = 0.0, CH3 = 12.0 / 25.0, CH4 = 32.0 / 225.0,
                 CH5 = 1.0 / 30.0, CH6 = 6.0 / 25.0;
constexpr double CT1 = 1.0 / 150.0, CT2 = 0.0, CT3 = -3.0 / 100.0, CT4 = 16.0 / 75.0,
                 CT5 = 1.0 / 20.0, CT6 = -6.0 / 25.0;
constexpr double BETA = 0.9;
constexpr double INV_ORDER = 1.0 / 5.0;
constexpr double SMALL_ERR = 1e-5;
constexpr int MAX_RETRY = 100;
constexpr double H_MAX = 1.0, H_MIN = 1e-12, H_GROWTH = 4.0;
constexpr double POW_SATURATED = 1800.0;  // (H_GROWTH / BETA)^5 = 1734.1, plus margin

GDEV double rclamp(double v, double lo, double hi) {  // f64::clamp
  if (v < lo) v = lo;
  if (v > hi) v = hi;
  return v;
}
GDEV double rem_euclid(double x, double m) {
  double r = fmod(x, m);
  return r < 0.0 ? r + fabs(m) : r;
}
GDEV uint32_t sat_u32(double v) {
  if (!(v > 0.0)) return 0u;
  if (v >= 4294967296.0) return 0xffffffffu;
  return (uint32_t)v;
}
GDEV uint64_t sat_u64(double v) {
  if (!(v > 0.0)) return 0ull;
  if (v >= 18446744073709551616.0) return ~0ull;
  return (uint64_t)v;
}

struct XYZA {
  double x, y, z, a;
};

// color.rs:49-69  ("other over self")
GDEV XYZA blend(const XYZA& self, const XYZA& other) {
  double ab = rclamp(self.a, 0.0, 1.0);
  double af = rclamp(other.a, 0.0, 1.0);
  double ao = af + ab * (1.0 - af);
  if (ao <= 0.0) return XYZA{0.0, 0.0, 0.0, 0.0};
  XYZA r;
  r.x = (other.x * af + self.x * ab * (1.0 - af)) / ao;
  r.y = (other.y * af + self.y * ab * (1.0 - af)) / ao;
  r.z = (other.z * af + self.z * ab * (1.0 - af)) / ao;
  r.a = ao;
  return r;
}

// Per-ray constants: observer energy (redshift.rs:40-60) and, for KerrBL, the
// conserved E, L_z, Carter Q (kerr_bl.rs:505-577).
struct RayConst {
  double obs;
  double e, lz, q;
  double pt, pphi;  // RayFrequencyData p_t, p_phi (redshift.rs:45-60), volumetric scenes only
};

// =========================================================== geometry kernels ======
// ---- Kerr-Schild helpers (kerr.rs:31-110) ----
template <bool FD = false>
GDEV double ks_r_sqr(double a, double x, double y, double z) {
  double rho_sqr = x * x + y * y + z * z;
  return 0.5 * (rho_sqr - a * a + ksqrt<FD>((rho_sqr - a * a) * (rho_sqr - a * a) + 4.0 * a * a * z * z));
}
// metric(): symmetric by construction; returns the 10 distinct entries in g.
template <bool FD = false>
GDEV void ks_metric(double radius, double a, double x, double y, double z, double g[4][4]) {
  double r_sqr = ks_r_sqr<FD>(a, x, y, z);
  double r = ksqrt<FD>(r_sqr);
  double f = kdiv<FD>(r * r * r * radius, r * r * r * r + a * a * z * z);
  double k_0 = 1.0;
  double k_x = kdiv<FD>(r * x + a * y, r_sqr + a * a);
  double k_y = kdiv<FD>(r * y - a * x, r_sqr + a * a);
  double k_z = kdiv<FD>(z, r);
  g[0][0] = k_0 * k_0 * f - 1.0;
  g[0][1] = k_0 * k_x * f;
  g[0][2] = k_0 * k_y * f;
  g[0][3] = k_0 * k_z * f;
  g[1][1] = k_x * k_x * f + 1.0;
  g[1][2] = k_x * k_y * f;
  g[1][3] = k_x * k_z * f;
  g[2][2] = k_y * k_y * f + 1.0;
  g[2][3] = k_y * k_z * f;
  g[3][3] = k_z * k_z * f + 1.0;
  g[1][0] = g[0][1];
  g[2][0] = g[0][2];
  g[2][1] = g[1][2];
  g[3][0] = g[0][3];
  g[3][1] = g[1][3];
  g[3][2] = g[2][3];
}
template <bool FD = false>
GDEV void ks_metric_contra(double radius, double a, double x, double y, double z, double g[4][4]) {
  double r_sqr = ks_r_sqr<FD>(a, x, y, z);
  double r = ksqrt<FD>(r_sqr);
  double f = kdiv<FD>(r * r * r * radius, r * r * r * r + a * a * z * z);
  double kc[4];
  kc[0] = -1.0;
  kc[1] = kdiv<FD>(r * x + a * y, r_sqr + a * a);
  kc[2] = kdiv<FD>(r * y - a * x, r_sqr + a * a);
  kc[3] = kdiv<FD>(z, r);
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      double eta = (i == j) ? (i == 0 ? -1.0 : 1.0) : 0.0;
      g[i][j] = eta - f * kc[i] * kc[j];
    }
}
// nalgebra gemv order: y_i = A_i0 x_0; y_i = A_ik x_k + y_i
GDEV void mat_vec(const double A[4][4], const double* x, double* y) {
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    double s = A[i][0] * x[0];
#pragma unroll
    for (int k = 1; k < 4; ++k) s = A[i][k] * x[k] + s;
    y[i] = s;
  }
}
GDEV double quad_form(const double* v, const double M[4][4], const double* w) {
  double s = 0.0;
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    double r = v[0] * M[0][j];
#pragma unroll
    for (int k = 1; k < 4; ++k) r = v[k] * M[k][j] + r;
    s = (j == 0) ? r * w[0] : r * w[j] + s;
  }
  return s;
}

// kerr.rs:149-186 + :228-235: returns 0.5 * p^T (G dG_i G) p, which equals
// -0.5 * p^T d_matrix_contravariant(i) p exactly (negation commutes with rounding).
template <bool FD = false>
GDEV double ks_accel(double radius, double a, int index, double x, double y, double z,
                     const double G[4][4], const double* p) {
  double c = index == 1 ? x : (index == 2 ? y : z);
  double h = 1e-10 * fmax(fabs(c), 1.0);
  double dx = index == 1 ? h : 0.0, dy = index == 2 ? h : 0.0, dz = index == 3 ? h : 0.0;
  double mp[4][4], mm[4][4];
  ks_metric<FD>(radius, a, x + dx, y + dy, z + dz, mp);
  ks_metric<FD>(radius, a, x - dx, y - dy, z - dz, mm);
  double two_h = 2.0 * h;
  double D[4][4];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) D[i][j] = kdiv<FD>(mp[i][j] - mm[i][j], two_h);
  double GD[4][4];
#pragma unroll
  for (int j = 0; j < 4; ++j)
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      double s = G[i][0] * D[0][j];
#pragma unroll
      for (int k = 1; k < 4; ++k) s = G[i][k] * D[k][j] + s;
      GD[i][j] = s;
    }
  // stream the columns of (GD)G straight into the quadratic form
  double q = 0.0;
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    double col[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      double s = GD[i][0] * G[0][j];
#pragma unroll
      for (int k = 1; k < 4; ++k) s = GD[i][k] * G[k][j] + s;
      col[i] = s;
    }
    double r = p[0] * col[0];
#pragma unroll
    for (int k = 1; k < 4; ++k) r = p[k] * col[k] + r;
    q = (j == 0) ? r * p[0] : r * p[j] + q;
  }
  return 0.5 * q;
}

// ---- KerrBL helpers (kerr_bl.rs:62-118, :253-272) ----
GDEV double bl_delta(double r, double r_s, double a) { return r * r - r_s * r + a * a; }
GDEV void metric_bl(double r_s, double a, double r, double sin_t, double cos_t, double g[4][4]) {
  double sig = r * r + a * a * (cos_t * cos_t);
  double sin2 = sin_t * sin_t;
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) g[i][j] = 0.0;
  g[0][0] = -(1.0 - r_s * r / sig);
  g[1][1] = sig / bl_delta(r, r_s, a);
  g[2][2] = sig;
  g[3][3] = (r * r + a * a + a * a * r_s * r * sin2 / sig) * sin2;
  double g_tph = -a * r_s * r * sin2 / sig;
  g[0][3] = g_tph;
  g[3][0] = g_tph;
}

#ifndef GRT_PATH_COUNT
#define GRT_PATH_COUNT 0  // diagnostic builds only: count code paths per wave and per lane
#endif
#if GRT_PATH_COUNT
// Diagnostic counters of integrate_kernel, [k] wave-level executions (one lane counts each),
// [8 + k] the same in lanes.  Kerr-Schild RHS: 0 range-free form, 1 IEEE form.  Light
// charts' RHS: 0 region-B table with range-free divisions, 1 region-B Taylor with them,
// 2 region-B with the IEEE divisions, 3 general (branchy) sincos.  All: 4 near-field window
// pass, 5 accepted step, 6 attempt.
constexpr int NPATH = 8;
__shared__ unsigned long long path_lds[2 * NPATH];
__device__ unsigned long long g_path[2 * NPATH];
GDEV void path_count(int k) {
  const uint64_t m = __ballot(1);  // the lanes executing this path together
  if ((int)(threadIdx.x & 63) == __ffsll((long long)m) - 1) {
    atomicAdd(&path_lds[k], 1ull);
    atomicAdd(&path_lds[NPATH + k], (unsigned long long)__popcll(m));
  }
}
#define PATH_COUNT(k) path_count(k)
#else
#define PATH_COUNT(k) ((void)0)
#endif

// sincos(theta), then body(sin, cos, fast).  When every lane of the wave is in one of
// sincos's region-B cases (x near pi/2; glibc_math.h sincos_b_*), the sincos is the
// straight-line form of that case and body runs in the same basic block, so its own
// dependency chains (the divisions) interleave with the sincos polynomial; fast = true
// there (the caller passes fast_ok = whether body may then take its fast form).  The same
// bits as rsincos in every case (tests/test_glibc_math.py).
// div_ok (per lane): the body's divisions may drop their range steps (div_inrange) in the
// region-B cases; body's fourth argument says so at compile time (std::true_type), so
// each form is one basic block from the sincos through the body.
template <bool FDIV = false, class F>
GDEV void with_sincos(double theta, bool fast_ok, F&& body, bool div_ok = false) {
#if GRT_SINCOS_B
  if (fast_ok) {
    double st, ct;
    const bool tab = glibc::sincos_b_table_ok(theta), tay = glibc::sincos_b_taylor_ok(theta);
    if constexpr (FDIV) {
      if (__ballot(!(tab & div_ok)) == 0) {
        PATH_COUNT(0);
        glibc::sincos_b_table(theta, &st, &ct);
        body(st, ct, true, std::true_type{});
        return;
      }
      if (__ballot(!(tay & div_ok)) == 0) {
        PATH_COUNT(1);
        glibc::sincos_b_taylor(theta, &st, &ct);
        body(st, ct, true, std::true_type{});
        return;
      }
    }
    if (__ballot(!tab) == 0) {
      PATH_COUNT(2);
      glibc::sincos_b_table(theta, &st, &ct);
      body(st, ct, true, std::false_type{});
      return;
    }
    if (__ballot(!tay) == 0) {
      PATH_COUNT(2);
      glibc::sincos_b_taylor(theta, &st, &ct);
      body(st, ct, true, std::false_type{});
      return;
    }
  }
#endif
  PATH_COUNT(3);
  double st, ct;
  rsincos(theta, &st, &ct);
  body(st, ct, false, std::false_type{});
}

// Whether every quotient and square root of rhs<KERR> at state (x, y, z) is in the exact
// region of div_fx / sqrt_fx.  That region (measured over the whole exponent plane,
// tests/test_gpu_arith.py::test_range_free_arithmetic_map) is E: y normal with
// |y| < 2^1022, x = 0 or of exponent >= -969, exponent gap within -1021 .. 1022; sqrt_fx:
// x >= 2^-969.  Bound chain, with cap = S.ks_cap <= 2^32 (host: 2^ceil(log2(2 max_radius)),
// within 2^10 .. 2^32) and S.div_fast (radius within 2^+-20, a = 0 or within 2^+-20):
//  * the state: each coordinate 0 or 2^-100 <= |c| < cap; D = rho^2 - a^2 >= 2^-10 + 2^-31 rho^2.
//  * the finite-difference points of ks_accel move one coordinate by h = 1e-10 max(|c|, 1):
//    it stays 0 / >= 2^-86 / +-1e-10 and <= 2^32, and rho^2 moves by < 2^-32 (rho^2 + 1), so
//    D >= 2^-11 and rho^2 < 2^66 at every point the metric is evaluated.
//  * sqrt_fx arguments: D^2 + 4 a^2 z^2 in 2^-22 .. 2^133; r^2 = (D + sqrt(..)) / 2 in
//    2^-11 .. 2^66 (r^2 <= rho^2), so r in 2^-5.5 .. 2^33.
//  * f = r^3 radius / (r^4 + a^2 z^2): numerator 2^-36.5 .. 2^119, denominator 2^-22 .. 2^133.
//  * k_x, k_y: numerator r x + a y is 0, or a nonzero sum of terms >= 2^-120 (>= 2^-172, a
//    multiple of the smaller term's ulp), <= 2^66; denominator r^2 + a^2 in 2^-11 .. 2^67.
//    k_z = z / r: numerator 0 or >= 2^-100, denominator 2^-5.5 .. 2^33.  So every k is 0 or
//    within 2^-239 .. 2^76, f within 2^-170 .. 2^15, metric entries 0 or within 2^-648 .. 2^168.
//  * D_ij = (mp - mm) / 2h: numerator 0 or >= an ulp of the smaller entry (>= 2^-700), <= 2^169;
//    2h = 2e-10 max(|c|, 1) within 2^-33 .. 2^0.
// Every numerator is 0 or of exponent -700 .. 169, every denominator of exponent -33 .. 133:
// inside E, with the box |x|, |y|, |x / y| <= 2^+-600 of the earlier argument to spare.  The
// device check of the whole RHS against its IEEE form on states at these edges, cap 2^15 and
// 2^32: tests/test_gpu_arith.py::test_rhs_kerr_schild_fast_form_matches_ieee.
GDEV bool ks_fd_ok(double a, double x, double y, double z, double cap) {
  auto c_ok = [cap](double c) { return (c == 0.0) | ((fabs(c) >= 0x1p-100) & (fabs(c) < cap)); };
  const double rho2 = x * x + y * y + z * z;
  return c_ok(x) & c_ok(y) & c_ok(z) & (rho2 - a * a >= 0x1p-10 + 0x1p-31 * rho2);
}
// Region-B division predicates of the Schwarzschild and KerrBL RHS (see there)
GDEV bool schw_div_ok(const DevScene& S, double r) {
  return S.div_fast && (fabs(r) > 0x1p-100) & (fabs(r) < 0x1p100) & (fabs(r - S.radius) > S.radius * 0x1p-40);
}
GDEV bool bl_div_ok(const DevScene& S, double r, double del, double l_z) {
  return S.div_fast && (fabs(r) < 0x1p100) & in_div_range(del) & (fabs(l_z) > 0x1p-200) & (fabs(l_z) < 0x1p100);
}


// ---- the ODE right-hand sides ----
// MODE 0: the render's RHS.  MODE 1 / 2 (rhs_check_kernel only): region-B sincos (or no
// sincos: Kerr-Schild), then the range-free (1) or the IEEE (2) form of the body, whatever
// the predicates say -- the check compares the two where the predicate holds.
template <int G, int MODE = 0>
GDEV void rhs(const DevScene& S, const RayConst& rc, const double* y, double* o) {
  if constexpr (G == GRT_GEOM_SCHWARZSCHILD) {  // schwarzschild.rs:54-80
    double radius = S.radius;
    double r = y[1], theta = y[2];
    double v_t = y[4], v_r = y[5], v_theta = y[6], v_phi = y[7];
    auto body = [&](double st, double ct, bool fast, auto fdiv) {
      if constexpr (decltype(fdiv)::value) {
        double radius_over_r, two_over_r;
        div2_inrange(radius, 2.0, r, &radius_over_r, &two_over_r);
        double a = 1.0 - radius_over_r;
        double a_prime = div_inrange(radius, r * r);
        double aprime_over_a = div_inrange(a_prime, a);
        o[0] = v_t;
        o[1] = v_r;
        o[2] = v_theta;
        o[3] = v_phi;
        o[4] = -(aprime_over_a)*v_t * v_r;
        o[5] = -0.5 * a * a_prime * v_t * v_t + 0.5 * (aprime_over_a)*v_r * v_r +
               a * r * (v_theta * v_theta + v_phi * v_phi * st * st);
        o[6] = -(two_over_r)*v_r * v_theta + st * ct * v_phi * v_phi;
        o[7] = -(two_over_r)*v_phi * v_r - div_inrange(2.0 * ct, st) * v_theta * v_phi;
        return;
      }
      double radius_over_r, two_over_r;
#if GRT_SHARED_DIV
      if (fast || S.div_share) {
        div2_same_den(radius, 2.0, r, &radius_over_r, &two_over_r);
      } else
#endif
      {
        radius_over_r = radius / r;
        two_over_r = 2.0 / r;
      }
      double a = 1.0 - radius_over_r;
      double a_prime = radius / (r * r);
      double aprime_over_a = a_prime / a;
      o[0] = v_t;
      o[1] = v_r;
      o[2] = v_theta;
      o[3] = v_phi;
      o[4] = -(aprime_over_a)*v_t * v_r;
      o[5] = -0.5 * a * a_prime * v_t * v_t + 0.5 * (aprime_over_a)*v_r * v_r +
             a * r * (v_theta * v_theta + v_phi * v_phi * st * st);
      o[6] = -(two_over_r)*v_r * v_theta + st * ct * v_phi * v_phi;
      o[7] = -(two_over_r)*v_phi * v_r - 2.0 * ct / st * v_theta * v_phi;
    };
    // fast form: the shared reciprocal, decided with the wave-uniform case (S.div_share).
    // Divisions without range steps (div_inrange) in region B: there sin theta >= 0.75 and
    // 2^-55 < |cos theta| < 0.66, and with S.div_fast (0 < radius within 2^+-50),
    // 2^-100 < |r| < 2^100 and |r - radius| > 2^-40 radius (so |a| > 2^-42), every operand
    // and quotient of the five divisions is within 2^+-600 (schw_div_ok; device check of the
    // two forms at the predicate's edges: tests/test_gpu_arith.py
    // ::test_rhs_schwarzschild_fast_form_matches_ieee).
    if constexpr (MODE != 0) {
      double st, ct;
      if (glibc::sincos_b_table_ok(theta)) glibc::sincos_b_table(theta, &st, &ct);
      else glibc::sincos_b_taylor(theta, &st, &ct);
      if constexpr (MODE == 1) body(st, ct, true, std::true_type{});
      else body(st, ct, true, std::false_type{});
      return;
    }
    with_sincos<GRT_FAST_DIV>(theta, S.div_share, body, schw_div_ok(S, r));
  } else if constexpr (G == GRT_GEOM_EUCLIDEAN_SPHERICAL) {  // euclidean_spherical.rs:48-70
    double r = y[1], theta = y[2];
    double v_t = y[4], v_r = y[5], v_theta = y[6], v_phi = y[7];
    double st, ct;
    rsincos(theta, &st, &ct);
    o[0] = v_t;
    o[1] = v_r;
    o[2] = v_theta;
    o[3] = v_phi;
    o[4] = 0.0;
    o[5] = r * (v_theta * v_theta + v_phi * v_phi * st * st);
    o[6] = -(2.0 / r) * v_r * v_theta + st * ct * v_phi * v_phi;
    o[7] = -(2.0 / r) * v_phi * v_r - 2.0 * ct / st * v_theta * v_phi;
  } else if constexpr (G == GRT_GEOM_KERR_BL) {  // kerr_bl.rs:141-174
    double radius = S.radius, a = S.a, e = rc.e, l_z = rc.lz, q = rc.q;
    double r = y[1], theta = y[2];
    const double del = bl_delta(r, radius, a);
    auto body = [&](double st, double ct, bool, auto fdiv) {
      double r2a2 = r * r + a * a;
      double p_r = r2a2 * e - a * l_z;
      double sin2 = st * st;
      if constexpr (decltype(fdiv)::value) {
        double r2a2_del, a_del;
        div2_inrange(r2a2, a, del, &r2a2_del, &a_del);
        o[0] = r2a2_del * p_r + a * (l_z - a * e * sin2);
        o[1] = y[4];
        o[2] = y[5];
        o[3] = a_del * p_r + div_inrange(l_z, sin2) - a * e;
        double le = l_z - a * e;
        double carter = le * le + q;
        o[4] = (4.0 * r * e * p_r - (2.0 * r - radius) * carter) / 2.0;
        o[5] = (-2.0 * a * a * e * e * ct * st + div_inrange(2.0 * l_z * l_z * ct, st * (st * st))) / 2.0;
        o[6] = 0.0;
        o[7] = 0.0;
        return;
      }
      o[0] = r2a2 / del * p_r + a * (l_z - a * e * sin2);
      o[1] = y[4];
      o[2] = y[5];
      o[3] = a / del * p_r + l_z / sin2 - a * e;
      double le = l_z - a * e;
      double carter = le * le + q;
      o[4] = (4.0 * r * e * p_r - (2.0 * r - radius) * carter) / 2.0;
      o[5] = (-2.0 * a * a * e * e * ct * st + 2.0 * l_z * l_z * ct / (st * (st * st))) / 2.0;
      o[6] = 0.0;
      o[7] = 0.0;
    };
    // Divisions without range steps (div_inrange) in region B: there sin theta >= 0.75 and
    // 2^-55 < |cos theta| < 0.66, and with S.div_fast (radius, |a| within 2^+-50),
    // 2^-200 < |l_z| < 2^100, |r| < 2^100 and del within 2^+-300, every operand and
    // quotient of the four divisions is within 2^+-600 (bl_div_ok; device check:
    // tests/test_gpu_arith.py::test_rhs_kerr_bl_fast_form_matches_ieee).
    if constexpr (MODE != 0) {
      double st, ct;
      if (glibc::sincos_b_table_ok(theta)) glibc::sincos_b_table(theta, &st, &ct);
      else glibc::sincos_b_taylor(theta, &st, &ct);
      if constexpr (MODE == 1) body(st, ct, true, std::true_type{});
      else body(st, ct, true, std::false_type{});
      return;
    }
    with_sincos<GRT_FAST_DIV_BL>(theta, true, body, bl_div_ok(S, r, del, l_z));
  } else if constexpr (G == GRT_GEOM_KERR) {  // kerr.rs:200-241
    double radius = S.radius, a = S.a;
    double x = y[1], yy = y[2], z = y[3];
    double p[4] = {y[4], y[5], y[6], y[7]};
    auto body = [&](auto fd) {
      constexpr bool FD = decltype(fd)::value;
      double Gc[4][4];
      ks_metric_contra<FD>(radius, a, x, yy, z, Gc);
      double xdot[4];
      mat_vec(Gc, p, xdot);
      o[0] = xdot[0];
      o[1] = xdot[1];
      o[2] = xdot[2];
      o[3] = xdot[3];
      o[4] = 0.0;
      o[5] = ks_accel<FD>(radius, a, 1, x, yy, z, Gc, p);
      o[6] = ks_accel<FD>(radius, a, 2, x, yy, z, Gc, p);
      o[7] = ks_accel<FD>(radius, a, 3, x, yy, z, Gc, p);
    };
    if constexpr (MODE != 0) {
      if constexpr (MODE == 1) body(std::true_type{});
      else body(std::false_type{});
      return;
    }
#if GRT_FAST_DIV_KS
    // The metric quotients without v_div_scale (div_fx) when every lane's state passes
    // ks_fd_ok (wave-uniform, like the region-B forms above)
    if (S.div_fast && __ballot(!ks_fd_ok(a, x, yy, z, S.ks_cap)) == 0) {
      PATH_COUNT(0);
      body(std::true_type{});
      return;
    }
#endif
    PATH_COUNT(1);
    body(std::false_type{});
  } else {  // Euclidean, euclidean.rs:47-53
    o[0] = y[4];
    o[1] = y[5];
    o[2] = y[6];
    o[3] = y[7];
    o[4] = 0.0;
    o[5] = 0.0;
    o[6] = 0.0;
    o[7] = 0.0;
  }
}

// Lane K's value of v in every lane of its quad (DPP quad_perm [K,K,K,K], no LDS).
template <int K>
GDEV double quad_bcast(double v) {
  constexpr int ctrl = K | (K << 2) | (K << 4) | (K << 6);
  const int lo = __builtin_amdgcn_mov_dpp(__double2loint(v), ctrl, 0xf, 0xf, false);
  const int hi = __builtin_amdgcn_mov_dpp(__double2hiint(v), ctrl, 0xf, 0xf, false);
  return __hiloint2double(hi, lo);
}

// rhs<KERR> on the 4 lanes of a quad (tail_kernel): every lane forms the contravariant
// metric and xdot as rhs<KERR> does; lane `sub` < 3 evaluates acceleration component
// sub + 1 (lane 3 repeats component 3), and the three components are broadcast across
// the quad.  Every value comes out of the same operations as in rhs<KERR>, so o is
// bit-identical in all four lanes; the quad's lanes must be active together.
template <bool FD>
GDEV void rhs_ks_quad_form(const DevScene& S, const double* y, double* o, int sub) {
  const double radius = S.radius, a = S.a;
  const double x = y[1], yy = y[2], z = y[3];
  const double p[4] = {y[4], y[5], y[6], y[7]};
  double Gc[4][4];
  ks_metric_contra<FD>(radius, a, x, yy, z, Gc);
  double xdot[4];
  mat_vec(Gc, p, xdot);
  const double acc = ks_accel<FD>(radius, a, sub < 3 ? sub + 1 : 3, x, yy, z, Gc, p);
  o[0] = xdot[0];
  o[1] = xdot[1];
  o[2] = xdot[2];
  o[3] = xdot[3];
  o[4] = 0.0;
  o[5] = quad_bcast<0>(acc);
  o[6] = quad_bcast<1>(acc);
  o[7] = quad_bcast<2>(acc);
}
// with rhs<KERR>'s range-free metric quotients and square roots when every lane's state
// passes ks_fd_ok (the quad's four lanes hold the same state)
GDEV void rhs_ks_quad(const DevScene& S, const double* y, double* o, int sub) {
#if GRT_FAST_DIV_KS
  if (S.div_fast && __ballot(!ks_fd_ok(S.a, y[1], y[2], y[3], S.ks_cap)) == 0) {
    rhs_ks_quad_form<true>(S, y, o, sub);
    return;
  }
#endif
  rhs_ks_quad_form<false>(S, y, o, sub);
}

template <int G, bool QUAD>
GDEV void rhs_sel(const DevScene& S, const RayConst& rc, const double* y, double* o, int sub) {
  if constexpr (QUAD) {
    static_assert(G == GRT_GEOM_KERR, "the quad-split RHS is the Kerr-Schild one");
    rhs_ks_quad(S, y, o, sub);
  } else {
    rhs<G>(S, rc, y, o);
  }
}

// Number of state components that can be non-zero: KerrBL's y[6], y[7] are
// identically 0 (its RHS returns literal zeros), so every RKF term on them is an
// exact +-0 and the norm term a2 + a6 == a2; skipping them is bit-exact.
template <int G>
struct Dim {
  static constexpr int D = (G == GRT_GEOM_KERR_BL) ? 6 : 8;
};

// One rkf45_step (runge_kutta.rs:86-125).  Returns the SQUARED truncation error norm:
// the controller takes the (correctly rounded) sqrt only when the decision needs it.
// UNIT_H: every lane of the wave has h == 1.0 (H_MAX, the far field), where h * o is o
// itself (x * 1.0 == x for every finite and infinite x and keeps the sign of zero; a NaN
// stays a NaN, which stops the ray either way), so the eight products per stage go.
// Stage values k1..k4 parked in LDS (KLDS): slot j of component i of thread t at
// kl_buf[(j * 8 + i) * KL_STRIDE + t].  The Kerr-Schild attempt keeps 6 x 8 stage doubles
// live across RHS evaluations that need ~100 registers of their own; at 2 waves per SIMD
// (256 registers) the compiler spilled ~90 registers to scratch.  The reads take their
// offset through an empty asm that depends on the stage just computed, so the compiler
// neither forwards the stored registers (keeping them live) nor hoists the reads above
// that RHS evaluation.  Values are stored and re-read unchanged: the arithmetic is the same.
constexpr int KL_STRIDE = 256;
__shared__ double kl_buf[GRT_KL_STAGES * 8 * KL_STRIDE];  // 16 KB per stage, only in kernels that use it
GDEV void kl_put(int j, const double* k, int D, int skip = -1) {
#pragma unroll
  for (int i = 0; i < 8; ++i)
    if (i < D && i != skip) kl_buf[(j * 8 + i) * KL_STRIDE + (int)threadIdx.x] = k[i];
}
// threadIdx.x, opaque to the compiler and ordered after `dep`
GDEV int kl_slot_after(double dep) {
  int t = (int)threadIdx.x;
  __asm__ volatile("" : "+v"(t) : "v"(dep));
  return t;
}
GDEV double kl_get(int t, int j, int i) { return kl_buf[(j * 8 + i) * KL_STRIDE + t]; }

// State components the RHS reads (the others -- t, and phi where the metric does not
// depend on it -- only receive stage values, so their stage inputs are never formed).
template <int G>
GDEV constexpr bool rhs_reads(int i) {
  if (G == GRT_GEOM_EUCLIDEAN) return i >= 4;
  if (G == GRT_GEOM_KERR) return i >= 1;
  return i == 1 || i == 2 || i >= 4;  // Schwarzschild, EuclideanSpherical, KerrBL: r, theta, velocities
}

// The state component whose derivative the RHS sets to the constant 0.0, or -1: p_t in
// Kerr-Schild (kerr.rs:233-241, the metric does not depend on t).  Its stage values are
// k_j = h * 0.0 = kz for every stage j of an attempt (kz = +0 for h > 0), so each of
// rkf45_step's left-to-right sums for it, y + c_1 kz + ... + c_m kz, is a sum of signed
// zeros (or NaNs) onto y, and IEEE addition gives it in one step: y + kz when every
// coefficient is >= 0 (each term carries kz's sign), y + kz * kz when the signs are mixed
// (some term is +0, which makes any later zero sum +0; kz * kz is +0, or NaN for a NaN
// kz).  Its error term (a mixed sum, no y) squares to +0: kz * kz as well.  Same bits as
// the full sums for every y, signed zeros and NaN included.
template <int G>
GDEV constexpr int zero_k() {
  return G == GRT_GEOM_KERR ? 4 : -1;
}

// nalgebra norm(): 8-accumulator unrolled dot, ((a0+a4) + (a1+a5)) + (a2+a6) + (a3+a7)
// z >= 0: e[z] * e[z] is given as zz (zero_k)
template <int D>
GDEV double err_norm_sq(const double* e, int z = -1, double zz = 0.0) {
  double res;
  if constexpr (D == 8) {
    double sq[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) sq[i] = (i == z) ? zz : e[i] * e[i];
    res = sq[0] + sq[4];
    res += sq[1] + sq[5];
    res += sq[2] + sq[6];
    res += sq[3] + sq[7];
  } else {
    res = e[0] * e[0] + e[4] * e[4];
    res += e[1] * e[1] + e[5] * e[5];
    res += e[2] * e[2];
    res += e[3] * e[3];
  }
  return res;
}

#ifndef GRT_RK_FOLD
#define GRT_RK_FOLD 1  // running RKF sums (rkf_attempt_fold) for every chart but Kerr-Schild
#endif

// rkf45_step with every left-to-right sum of runge_kutta.rs:94-124 evaluated as a running
// sum as soon as its terms exist.  The sums are the reference's, term by term in the same
// order ((y + B61*k1) + B62*k2) + ..., so every value is bit-identical to rkf_attempt_full;
// what changes is how many stage values are live across an RHS evaluation:
//   - a component the RHS does not read (rhs_reads) folds k_j into y_new and the error
//     right away: 2 live values instead of up to 6;
//   - the others keep k1..k3 until k4 exists, then fold k1..k4 into the stage-5 input, the
//     stage-6 partial, y_new and the error: 3 live values across RHS 5 and 2 across RHS 6,
//     instead of 4 and 5.
template <int G, bool UNIT_H, bool QUAD, int NKL>
GDEV double rkf_attempt_fold(const DevScene& S, const RayConst& rc, const double* y, double h, double* yn,
                             int sub) {
  constexpr int D = Dim<G>::D;
  double k1[8], k2[8], k3[8], k4[8], k5[8], k6[8], tmp[8], o[8], p6[8], e[8];
  int t = 0;  // LDS slot, re-derived after each stage (kl_slot_after)
#define KV(j, i) (((j) <= NKL) ? kl_get(t, (j) - 1, (i)) : k##j[i])
#define STAGE(kj)                                                   \
  _Pragma("unroll") for (int i = 0; i < D; ++i) kj[i] = UNIT_H ? o[i] : h * o[i];
  rhs_sel<G, QUAD>(S, rc, y, o, sub);
  STAGE(k1)
#pragma unroll
  for (int i = 0; i < D; ++i)
    if (!rhs_reads<G>(i)) {
      yn[i] = y[i] + CH1 * k1[i];
      e[i] = CT1 * k1[i];
    }
  if (NKL >= 1) kl_put(0, k1, D);
#pragma unroll
  for (int i = 0; i < D; ++i) tmp[i] = y[i] + B21 * k1[i];
  if (D < 8) { tmp[6] = 0.0; tmp[7] = 0.0; }
  rhs_sel<G, QUAD>(S, rc, tmp, o, sub);
  STAGE(k2)
#pragma unroll
  for (int i = 0; i < D; ++i)
    if (!rhs_reads<G>(i)) {
      yn[i] = yn[i] + CH2 * k2[i];
      e[i] = e[i] + CT2 * k2[i];
    }
  if (NKL >= 2) kl_put(1, k2, D);
  if (NKL >= 1) t = kl_slot_after(k2[D - 1]);
#pragma unroll
  for (int i = 0; i < D; ++i) tmp[i] = y[i] + B31 * KV(1, i) + B32 * k2[i];
  rhs_sel<G, QUAD>(S, rc, tmp, o, sub);
  STAGE(k3)
#pragma unroll
  for (int i = 0; i < D; ++i)
    if (!rhs_reads<G>(i)) {
      yn[i] = yn[i] + CH3 * k3[i];
      e[i] = e[i] + CT3 * k3[i];
    }
  if (NKL >= 3) kl_put(2, k3, D);
  if (NKL >= 1) t = kl_slot_after(k3[D - 1]);
#pragma unroll
  for (int i = 0; i < D; ++i) tmp[i] = y[i] + B41 * KV(1, i) + B42 * KV(2, i) + B43 * k3[i];
  rhs_sel<G, QUAD>(S, rc, tmp, o, sub);
  STAGE(k4)
  if (NKL >= 1) t = kl_slot_after(k4[D - 1]);
#pragma unroll
  for (int i = 0; i < D; ++i) {
    if (!rhs_reads<G>(i)) {
      yn[i] = yn[i] + CH4 * k4[i];
      e[i] = e[i] + CT4 * k4[i];
    } else {
      const double a1 = KV(1, i), a2 = KV(2, i), a3 = KV(3, i), a4 = k4[i];
      tmp[i] = y[i] + B51 * a1 + B52 * a2 + B53 * a3 + B54 * a4;
      p6[i] = y[i] + B61 * a1 + B62 * a2 + B63 * a3 + B64 * a4;
      yn[i] = y[i] + CH1 * a1 + CH2 * a2 + CH3 * a3 + CH4 * a4;
      e[i] = CT1 * a1 + CT2 * a2 + CT3 * a3 + CT4 * a4;
    }
  }
  if (D < 8) { tmp[6] = 0.0; tmp[7] = 0.0; }
  rhs_sel<G, QUAD>(S, rc, tmp, o, sub);
  STAGE(k5)
#pragma unroll
  for (int i = 0; i < D; ++i) {
    if (rhs_reads<G>(i)) tmp[i] = p6[i] + B65 * k5[i];
    yn[i] = yn[i] + CH5 * k5[i];
    e[i] = e[i] + CT5 * k5[i];
  }
  rhs_sel<G, QUAD>(S, rc, tmp, o, sub);
  STAGE(k6)
#pragma unroll
  for (int i = 0; i < D; ++i) {
    yn[i] = yn[i] + CH6 * k6[i];
    e[i] = e[i] + CT6 * k6[i];
  }
#undef STAGE
#undef KV
  if (D < 8) {
    yn[6] = 0.0;
    yn[7] = 0.0;
  }
  return err_norm_sq<D>(e);
}

// QUAD: the Kerr-Schild RHS split over a quad (rhs_ks_quad), `sub` = lane & 3.
// NKL: stages k1..k_NKL kept in LDS (see kl_put), 0 = none.
template <int G, bool UNIT_H = false, bool QUAD = false, int NKL = 0>
GDEV double rkf_attempt(const DevScene& S, const RayConst& rc, const double* y, double h,
                        double* yn, int sub = 0) {
  // Kerr-Schild keeps the plain form: its stages k1..k4 sit in LDS (NKL), which frees
  // more registers than the running sums (measured: 17 -> 122 spilled VGPRs with them)
  if constexpr (GRT_RK_FOLD && G != GRT_GEOM_KERR) {
    return rkf_attempt_fold<G, UNIT_H, QUAD, NKL>(S, rc, y, h, yn, sub);
  }
  constexpr int D = Dim<G>::D;
  constexpr int Z = zero_k<G>();  // component with k_j = kz in every stage (zero_k)
  double k1[8], k2[8], k3[8], k4[8], k5[8], k6[8], tmp[8], o[8];
  int t = 0;  // LDS slot, re-derived after each stage (kl_slot_after)
  // stage j's value k_j[i] (from LDS when parked there)
#define KV(j, i) (((j) <= NKL) ? kl_get(t, (j) - 1, (i)) : k##j[i])
  rhs_sel<G, QUAD>(S, rc, y, o, sub);
  // signs: B21 > 0; B31, B32 > 0; B4x, B5x, B6x mixed; CH1..CH6 >= 0; CT mixed
  const double kz = Z < 0 ? 0.0 : (UNIT_H ? o[Z < 0 ? 0 : Z] : h * o[Z < 0 ? 0 : Z]);
  const double kzz = kz * kz;
#pragma unroll
  for (int i = 0; i < D; ++i) k1[i] = UNIT_H ? o[i] : h * o[i];
  if (NKL >= 1) kl_put(0, k1, D, Z);
#pragma unroll
  for (int i = 0; i < D; ++i) tmp[i] = (i == Z) ? y[i] + kz : y[i] + B21 * k1[i];
  if (D < 8) { tmp[6] = 0.0; tmp[7] = 0.0; }
  rhs_sel<G, QUAD>(S, rc, tmp, o, sub);
#pragma unroll
  for (int i = 0; i < D; ++i) k2[i] = UNIT_H ? o[i] : h * o[i];
  if (NKL >= 2) kl_put(1, k2, D, Z);
  if (NKL >= 1) t = kl_slot_after(k2[D - 1]);
#pragma unroll
  for (int i = 0; i < D; ++i) tmp[i] = (i == Z) ? y[i] + kz : y[i] + B31 * KV(1, i) + B32 * k2[i];
  rhs_sel<G, QUAD>(S, rc, tmp, o, sub);
#pragma unroll
  for (int i = 0; i < D; ++i) k3[i] = UNIT_H ? o[i] : h * o[i];
  if (NKL >= 3) kl_put(2, k3, D, Z);
  if (NKL >= 1) t = kl_slot_after(k3[D - 1]);
#pragma unroll
  for (int i = 0; i < D; ++i)
    tmp[i] = (i == Z) ? y[i] + kzz : y[i] + B41 * KV(1, i) + B42 * KV(2, i) + B43 * k3[i];
  rhs_sel<G, QUAD>(S, rc, tmp, o, sub);
#pragma unroll
  for (int i = 0; i < D; ++i) k4[i] = UNIT_H ? o[i] : h * o[i];
  if (NKL >= 4) kl_put(3, k4, D, Z);
  if (NKL >= 1) t = kl_slot_after(k4[D - 1]);
#pragma unroll
  for (int i = 0; i < D; ++i)
    tmp[i] = (i == Z) ? y[i] + kzz : y[i] + B51 * KV(1, i) + B52 * KV(2, i) + B53 * KV(3, i) + B54 * k4[i];
  rhs_sel<G, QUAD>(S, rc, tmp, o, sub);
#pragma unroll
  for (int i = 0; i < D; ++i) k5[i] = UNIT_H ? o[i] : h * o[i];
  if (NKL >= 1) t = kl_slot_after(k5[D - 1]);
#pragma unroll
  for (int i = 0; i < D; ++i)
    tmp[i] = (i == Z) ? y[i] + kzz
                      : y[i] + B61 * KV(1, i) + B62 * KV(2, i) + B63 * KV(3, i) + B64 * KV(4, i) + B65 * k5[i];
  rhs_sel<G, QUAD>(S, rc, tmp, o, sub);
#pragma unroll
  for (int i = 0; i < D; ++i) k6[i] = UNIT_H ? o[i] : h * o[i];
  if (NKL >= 1) t = kl_slot_after(k6[D - 1]);
  double e[8];
#pragma unroll
  for (int i = 0; i < D; ++i) {
    if (i == Z) {  // e[Z] only enters the norm as e[Z]^2 = kz * kz
      yn[i] = y[i] + kz;
      e[i] = 0.0;
      continue;
    }
    const double a1 = KV(1, i), a2 = KV(2, i), a3 = KV(3, i), a4 = KV(4, i);
    yn[i] = y[i] + CH1 * a1 + CH2 * a2 + CH3 * a3 + CH4 * a4 + CH5 * k5[i] + CH6 * k6[i];
    e[i] = CT1 * a1 + CT2 * a2 + CT3 * a3 + CT4 * a4 + CT5 * k5[i] + CT6 * k6[i];
  }
#undef KV
  if (D < 8) {
    yn[6] = 0.0;
    yn[7] = 0.0;
  }
  return err_norm_sq<D>(e, Z, kzz);
}

// ---- chart helpers ----
// Cartesian spatial position of a state (scene.rs:48-69 get_position / point.rs:125-154).
template <int G>
GDEV void to_cart(const DevScene& S, const double* y, double* c) {
  if constexpr (G == GRT_GEOM_SCHWARZSCHILD || G == GRT_GEOM_EUCLIDEAN_SPHERICAL) {
    double st, ct, sp, cp;
    rsincos(y[2], &st, &ct);
    rsincos(y[3], &sp, &cp);
    double r = y[1];
    c[0] = r * st * cp;
    c[1] = r * st * sp;
    c[2] = r * ct;
  } else if constexpr (G == GRT_GEOM_KERR_BL) {
    double a = S.a, r = y[1];
    double st, ct, sp, cp;
    rsincos(y[2], &st, &ct);
    rsincos(y[3], &sp, &cp);
    c[0] = (r * cp - a * sp) * st;
    c[1] = (r * sp + a * cp) * st;
    c[2] = r * ct;
  } else {
    c[0] = y[1];
    c[1] = y[2];
    c[2] = y[3];
  }
}

// cartesian_to_spherical (spherical_coordinates_helper.rs:5-26): r, theta, phi
GDEV void cart_to_sph(double x, double y, double z, double* r_o, double* th_o, double* ph_o) {
  double r = sqrt(x * x + y * y + z * z);
  if (r == 0.0) {
    *r_o = 0.0;
    *th_o = 0.0;
    *ph_o = 0.0;
    return;
  }
  *r_o = r;
  *th_o = acos(z / r);
  *ph_o = atan2(y, x);
}
// cartesian_to_boyer_lindquist (spherical_coordinates_helper.rs:44-61)
GDEV void cart_to_bl(double a, double x, double y, double z, double* r_o, double* th_o, double* ph_o) {
  double rho_sqr = x * x + y * y + z * z;
  double d = rho_sqr - a * a;
  double r_sqr = 0.5 * (rho_sqr - a * a + sqrt(d * d + 4.0 * a * a * z * z));
  double r = sqrt(r_sqr);
  *r_o = r;
  *th_o = (r == 0.0) ? 0.0 : acos(rclamp(z / r, -1.0, 1.0));
  *ph_o = atan2(r * y - a * x, r * x + a * y);
}

// momentum_from_state (geometry.rs:29-31; kerr_bl.rs:225-249; kerr.rs:262-273)
template <int G>
GDEV void momentum(const DevScene& S, const RayConst& rc, const double* y, double* p) {
  if constexpr (G == GRT_GEOM_KERR_BL) {
    double a = S.a, e = rc.e, l_z = rc.lz;
    double r = y[1], theta = y[2], v_r = y[4], v_theta = y[5];
    double st, ct;
    rsincos(theta, &st, &ct);
    double del = bl_delta(r, S.radius, a);
    double sig = r * r + a * a * (ct * ct);
    double sin2 = st * st;
    double p_r_term = (r * r + a * a) * e - a * l_z;
    double dt = (r * r + a * a) / del * p_r_term + a * (l_z - a * e * sin2);
    double dphi = a / del * p_r_term + l_z / sin2 - a * e;
    p[0] = dt / sig;
    p[1] = v_r / sig;
    p[2] = v_theta / sig;
    p[3] = dphi / sig;
  } else if constexpr (G == GRT_GEOM_KERR) {
    double Gc[4][4];
    ks_metric_contra(S.radius, S.a, y[1], y[2], y[3], Gc);
    mat_vec(Gc, y + 4, p);
  } else {
    p[0] = y[4];
    p[1] = y[5];
    p[2] = y[6];
    p[3] = y[7];
  }
}

// x unchanged, through an empty volatile asm: the compiler can neither hoist what is
// computed from the result out of the branch it sits in nor merge it with the same
// computation on x elsewhere.
GDEV double opaque(double x) {
  asm volatile("" : "+v"(x));
  return x;
}
// The window pass's lerped momentum of a hit, sw p(ya) + t p(yb) (objects.rs:27-44).
// KerrBL reads the momentum's inputs through opaque(): otherwise both momenta, invariant
// in the object loop, have their sincos-free parts computed before the loop for every
// near-field window and kept live across it, and the 3-wave kernel spills them (the
// scratch stores of C3: 1.75 GB written per frame).  Now they are computed only for a
// recorded hit (1.55M of 1.79e9 C3 steps), with the same operations on the same values.
// (An out-of-line function does the same for the spills, but the call makes the kernel
// rematerialise its SGPR constants around it: +20% scalar instructions, +1.5% time.)
template <int G>
GDEV void lerp_momentum(const DevScene& S, const RayConst& rc, const double* ya, const double* yb, double t,
                        double* ph) {
  double pa[4], pb[4];
  if constexpr (G == GRT_GEOM_KERR_BL) {
    const double a8[8] = {0.0, opaque(ya[1]), opaque(ya[2]), 0.0, opaque(ya[4]), opaque(ya[5]), 0.0, 0.0};
    const double b8[8] = {0.0, opaque(yb[1]), opaque(yb[2]), 0.0, opaque(yb[4]), opaque(yb[5]), 0.0, 0.0};
    momentum<G>(S, rc, a8, pa);
    momentum<G>(S, rc, b8, pb);
  } else {
    momentum<G>(S, rc, ya, pa);
    momentum<G>(S, rc, yb, pb);
  }
  const double sw = 1.0 - t;
#pragma unroll
  for (int q = 0; q < 4; ++q) ph[q] = sw * pa[q] + t * pb[q];
}

// inner_product at a native-chart point whose polar-angle sin/cos are given.
template <int G>
GDEV double inner(const DevScene& S, const double* pos, double st, double ct, const double* v,
                  const double* w) {
  if constexpr (G == GRT_GEOM_SCHWARZSCHILD) {  // schwarzschild.rs:90-102
    double r = pos[1];
    double a = 1.0 - S.radius / r;
    return a * v[0] * w[0] - v[1] * w[1] / a - r * r * v[2] * w[2] - r * r * st * st * v[3] * w[3];
  } else if constexpr (G == GRT_GEOM_EUCLIDEAN_SPHERICAL) {  // euclidean_spherical.rs:80-91
    double r = pos[1];
    return 1.0 * v[0] * w[0] - v[1] * w[1] - r * r * v[2] * w[2] - r * r * st * st * v[3] * w[3];
  } else if constexpr (G == GRT_GEOM_KERR_BL) {  // kerr_bl.rs:338-359
    double g[4][4];
    metric_bl(S.radius, S.a, pos[1], st, ct, g);
    double result = 0.0;
#pragma unroll
    for (int mu = 0; mu < 4; ++mu)
#pragma unroll
      for (int nu = 0; nu < 4; ++nu) result += g[mu][nu] * v[mu] * w[nu];
    return result;
  } else if constexpr (G == GRT_GEOM_KERR) {  // kerr.rs:283-287
    double g[4][4];
    ks_metric(S.radius, S.a, pos[1], pos[2], pos[3], g);
    return quad_form(v, g, w);
  } else {  // euclidean.rs:62-67
    return 1.0 * v[0] * w[0] + -v[1] * w[1] + -v[2] * w[2] + -v[3] * w[3];
  }
}
template <int G>
GDEV double signature0() {
  return (G == GRT_GEOM_KERR || G == GRT_GEOM_KERR_BL) ? -1.0 : 1.0;
}

// get_stationary_velocity_at (schwarzschild.rs:237-240; kerr.rs:449-455; kerr_bl.rs:362-371)
template <int G>
GDEV void stationary_velocity(const DevScene& S, const double* pos, double* u) {
  u[1] = 0.0;
  u[2] = 0.0;
  u[3] = 0.0;
  if constexpr (G == GRT_GEOM_SCHWARZSCHILD) {
    double a = 1.0 - S.radius / pos[1];
    u[0] = 1.0 / sqrt(a);
  } else if constexpr (G == GRT_GEOM_KERR_BL) {
    double r = pos[1];
    double ct = rcos(pos[2]);  // kerr_bl.rs:362-371 evaluates sigma alone: a lone cos()
    double sig = r * r + S.a * S.a * (ct * ct);
    u[0] = 1.0 / sqrt(1.0 - S.radius * r / sig);
  } else if constexpr (G == GRT_GEOM_KERR) {
    double a = S.a, z = pos[3];
    double r_sqr = ks_r_sqr(a, pos[1], pos[2], pos[3]);
    double r = sqrt(r_sqr);
    double f = (r * r * r * S.radius) / (r * r * r * r + a * a * z * z);
    u[0] = 1.0 / sqrt(1.0 - f);
  } else {
    u[0] = 1.0;
  }
}

// circular_orbit::killing_coefficients (circular_orbit.rs:76-108)
GDEV bool killing_coefficients(const DevScene& S, double r, double* u_t, double* u_phi) {
  double r_s = S.radius, a = S.a;
  double m = 0.5 * r_s;
  double sqrt_m = sqrt(m);
  double omega = sqrt_m / (rpow(r, 1.5) + a * sqrt_m);
  double c = S.cos_half_pi, s = S.sin_half_pi;
  double sig = r * r + a * a * (c * c);
  double sin2 = s * s;
  double g_tt = -(1.0 - r_s * r / sig);
  double g_tphi = -a * r_s * r * sin2 / sig;
  double g_phiphi = (r * r + a * a + a * a * r_s * r * sin2 / sig) * sin2;
  double ut_pre = g_tt + 2.0 * omega * g_tphi + omega * omega * g_phiphi;
  if (ut_pre >= 0.0) return false;
  double ut = 1.0 / sqrt(-ut_pre);
  *u_t = ut;
  *u_phi = omega * ut;
  return true;
}

// ============================================================== shading =========
GDEV XYZA texel(const DevScene& S, const DevTexture& t, uint32_t x, uint32_t y) {
  uint32_t px = t.rgba[(uint64_t)y * t.width + x];
  double r = S.srgb_lin[px & 0xffu];
  double g = S.srgb_lin[(px >> 8) & 0xffu];
  double b = S.srgb_lin[(px >> 16) & 0xffu];
  XYZA c;  // srgb_to_xyz (color.rs:310-332), nalgebra gemv order
  c.x = 0.4124564 * r;
  c.x = 0.3575761 * g + c.x;
  c.x = 0.1804375 * b + c.x;
  c.y = 0.2126729 * r;
  c.y = 0.7151522 * g + c.y;
  c.y = 0.0721750 * b + c.y;
  c.z = 0.0193339 * r;
  c.z = 0.1191920 * g + c.z;
  c.z = 0.9503041 * b + c.z;
  c.a = (double)(px >> 24) / 255.0;
  return c;
}

// The reference's table searches (binary search, then idx = partition point - 1) over a
// sorted table a[0..n) with a[0] < x < a[n - 1]: the last idx with a[idx] <= x.  Both
// tables are evenly spaced grids (host/setup.cpp: x0 + i * step), so the index is guessed
// from the spacing and corrected by comparisons against the table itself: the same idx
// for any sorted table (a poor guess only costs more steps), with two dependent loads
// instead of the ~10 of the bisection.
GDEV uint32_t lut_index(const double* a, uint32_t n, double a0, double a_last, double x) {
  const double g = (x - a0) * ((double)(n - 1) / (a_last - a0));
  uint32_t idx = g >= (double)(n - 2) ? n - 2 : (g > 0.0 ? (uint32_t)g : 0u);
  while (idx < n - 2 && a[idx + 1] <= x) ++idx;
  while (idx > 0 && a[idx] > x) --idx;
  return idx;
}

// texture.rs:149-195 over a (log10 T, XYZ) table in global memory or LDS
GDEV XYZA sample_blackbody_lut(const double* lt, const double* c, uint32_t n, double temperature) {
  double log_t = log10(fmax(temperature, 10.0));
  const double lt_first = lt[0], lt_last = lt[n - 1];
  if (!isfinite(log_t) || log_t <= lt_first) return XYZA{c[0], c[1], c[2], 1.0};
  if (log_t >= lt_last) return XYZA{c[3 * (n - 1)], c[3 * (n - 1) + 1], c[3 * (n - 1) + 2], 1.0};
  const uint32_t idx = lut_index(lt, n, lt_first, lt_last, log_t);
  double lt0 = lt[idx], lt1 = lt[idx + 1];
  const double* c0 = c + 3 * idx;
  const double* c1 = c + 3 * (idx + 1);
  double t = (log_t - lt0) / (lt1 - lt0);
  return XYZA{c0[0] + t * (c1[0] - c0[0]), c0[1] + t * (c1[1] - c0[1]), c0[2] + t * (c1[2] - c0[2]), 1.0};
}
GDEV XYZA sample_blackbody(const DevScene& S, double temperature) {
  return sample_blackbody_lut(S.bb_log_t, S.bb_xyz, S.bb_n, temperature);
}

// TextureMap::color_at_uv (texture.rs:93-257); bb_lt / bb_xyz: the blackbody table
// (S.bb_log_t / S.bb_xyz, or an LDS copy of it)
GDEV XYZA texture_color_lut(const DevScene& S, const DevTexture& t, double u, double v, double redshift,
                            double temperature, const double* bb_lt, const double* bb_xyz) {
  XYZA c;
  if (t.kind == GRT_TEX_BITMAP) {
    uint32_t width = t.width, height = t.height;
    double p_x = (double)width * u;
    double p_y = (double)height * v;
    uint32_t xf = min(sat_u32(floor(p_x)), width - 1);
    uint32_t yf = min(sat_u32(floor(p_y)), height - 1);
    uint32_t xc = min(sat_u32(ceil(p_x)), width - 1);
    uint32_t yc = min(sat_u32(ceil(p_y)), height - 1);
    XYZA c00 = texel(S, t, xf, yf), c01 = texel(S, t, xf, yc);
    XYZA c11 = texel(S, t, xc, yc), c10 = texel(S, t, xc, yf);
    double dx = p_x - (double)xf;
    double dy = p_y - (double)yf;
    double w00 = (1.0 - dx) * (1.0 - dy);
    double w01 = (1.0 - dx) * dy;
    double w10 = dx * (1.0 - dy);
    double w11 = dx * dy;
    c.x = w00 * c00.x + w10 * c10.x + w01 * c01.x + w11 * c11.x;
    c.y = w00 * c00.y + w10 * c10.y + w01 * c01.y + w11 * c11.y;
    c.z = w00 * c00.z + w10 * c10.z + w01 * c01.z + w11 * c11.z;
    c.a = w00 * c00.a + w10 * c10.a + w01 * c01.a + w11 * c11.a;
  } else if (t.kind == GRT_TEX_CHECKER) {
    uint64_t ut = sat_u64(floor(u * t.cw));
    uint64_t vt = sat_u64(floor(v * t.ch));
    const double* cc = ((ut + vt) % 2 == 0) ? t.c1 : t.c2;
    c = XYZA{cc[0], cc[1], cc[2], cc[3]};
  } else {
    c = sample_blackbody_lut(bb_lt, bb_xyz, S.bb_n, temperature * redshift);
  }
  // apply_beaming (color.rs:72-80): powf(redshift, e); pow(x, +-0) is 1 for every x (C99
  // F.9.4.4, glibc), so the stock scenes' exponent 0 skips the call
  double f = t.beaming == 0.0 ? 1.0 : rpow(redshift, t.beaming);
  return XYZA{c.x * f, c.y * f, c.z * f, c.a};
}
GDEV XYZA texture_color(const DevScene& S, const DevTexture& t, double u, double v, double redshift,
                        double temperature) {
  return texture_color_lut(S, t, u, v, redshift, temperature, S.bb_log_t, S.bb_xyz);
}

// KerrTemperatureComputer::compute_temperature (temperature.rs:198-253); lut_r / lut_t:
// the object's (r, T) table in global memory or an LDS copy
GDEV int compute_temperature_lut(const DevObject& o, const double* lut_r, const double* lut_t, double radius,
                                 double* out) {
  if (o.temp_kind == GRT_TEMP_CONSTANT) {
    *out = o.temp_constant;
    return GRT_OK;
  }
  if (!isfinite(radius)) return GRT_ERR_NON_FINITE_RADIUS;
  if (radius < o.r_isco) return GRT_ERR_BELOW_RISCO;
  uint32_t n = o.lut_n;
  const double r_first = lut_r[0], r_last = lut_r[n - 1];
  if (radius <= r_first) { *out = lut_t[0]; return GRT_OK; }
  if (radius >= r_last) { *out = lut_t[n - 1]; return GRT_OK; }
  const uint32_t idx = lut_index(lut_r, n, r_first, r_last, radius);
  double r0 = lut_r[idx], t0 = lut_t[idx], r1 = lut_r[idx + 1], t1 = lut_t[idx + 1];
  double t = (radius - r0) / (r1 - r0);
  *out = t0 + t * (t1 - t0);
  return GRT_OK;
}
GDEV int compute_temperature(const DevObject& o, double radius, double* out) {
  return compute_temperature_lut(o, o.lut_r, o.lut_t, radius, out);
}

#include "volumetric.h"


// ====================================================== window (chord) tests ======
// Geometry only: the integrate kernel decides hit / no hit, the chord parameter t and
// the hit point; everything that needs the emitter (energy, temperature, colour) is
// evaluated later by the shade kernel from the recorded point and momentum.

// disc.rs:41-88.  The sign / magnitude pre-filter only skips divisions whose quotient
// is provably outside [0, 1] (and cannot underflow to -0); every accepted t is the
// same correctly rounded p1 / p2 the reference computes.
GDEV bool disc_chord(const DevObject& o, const double* s, const double* e, double* t_out, double* ip) {
  double d0 = e[0] - s[0], d1 = e[1] - s[1], d2 = e[2] - s[2];
  double p1 = (0.0 - s[0]) * 0.0 + (0.0 - s[1]) * 0.0 + (0.0 - s[2]) * 1.0;
  double p2 = d0 * 0.0 + d1 * 0.0 + d2 * 1.0;
  double a1 = fabs(p1), a2 = fabs(p2);
  if (a1 > 1e-200 && a2 < 1e100 && ((p1 > 0.0 && p2 < 0.0) || (p1 < 0.0 && p2 > 0.0))) return false;  // t < 0
  if (a1 > 2.0 * a2) return false;                                                                    // t > 2
  double t = p1 / p2;
  if (!(0.0 <= t && t <= 1.0)) return false;
  double ix = s[0] + t * d0, iy = s[1] + t * d1, iz = s[2] + t * d2;
  double rr = ix * ix + iy * iy + iz * iz;
  if (!(rr >= o.rin2 && rr <= o.rout2)) return false;
  *t_out = t;
  ip[0] = ix;
  ip[1] = iy;
  ip[2] = iz;
  return true;
}

// sphere.rs:37-128; returns the hit point in the sphere's local frame.
GDEV bool sphere_chord(const DevObject& o, const double* s_w, const double* e_w, double* t_out, double* lp) {
  double s0 = s_w[0] + -o.cx, s1 = s_w[1] + -o.cy, s2 = s_w[2] + -o.cz;
  double e0 = e_w[0] + -o.cx, e1 = e_w[1] + -o.cy, e2 = e_w[2] + -o.cz;
  double r_start = s0 * s0 + s1 * s1 + s2 * s2;
  double r_end = e0 * e0 + e1 * e1 + e2 * e2;
  double R2 = o.R2;
  if (!((r_start >= R2 && r_end <= R2) || (r_start <= R2 && r_end >= R2))) return false;
  double d0 = e0 - s0, d1 = e1 - s1, d2 = e2 - s2;
  double a = d0 * d0 + d1 * d1 + d2 * d2;
  double b = 2.0 * (s0 * d0 + s1 * d1 + s2 * d2);
  double c = (s0 * s0 + s1 * s1 + s2 * s2) - o.radius * o.radius;
  double disc = b * b - 4.0 * a * c;
  if (disc < 0.0) return false;
  double sq = sqrt(disc);
  double t1 = (-b + sq) / (2.0 * a);
  double t2 = (-b - sq) / (2.0 * a);
  double t;
  if (0.0 <= t1 && t1 <= 1.0) t = t1;
  else if (0.0 <= t2 && t2 <= 1.0) t = t2;
  else return false;
  *t_out = t;
  lp[0] = s0 + t * d0;
  lp[1] = s1 + t * d1;
  lp[2] = s2 + t * d2;
  return true;
}

// ======================================================== integrate kernel =======
// camera.rs:214-232 get_direction_for, then momentum = direction - e_t (:243, :252)
GDEV void camera_momentum(const DevCamera& c, double row, double column, double* p) {
  double shifted_column = column + 1.0;
  double shifted_row = row + 1.0;
  double tha = c.tan_half_alpha;
  double i_prime = c.hand * (2.0 * tha / c.rows) * (shifted_column - (c.cols + 1.0) / 2.0);
  double j_prime = (2.0 * tha / c.rows) * (shifted_row - (c.rows + 1.0) / 2.0);
  double w_squared = c.sig_s * (1.0 + i_prime * i_prime + j_prime * j_prime);
  double denom = c.sig_s * w_squared;
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    double w = c.tet[3][k] + i_prime * c.tet[1][k] + j_prime * c.tet[2][k];
    double dir = -c.tet[3][k] + 2.0 * w / denom;
    p[k] = dir + (-c.tet[0][k]);
  }
}

// Initial ODE state of a ray at native-chart position `pos` with contravariant momentum
// `p` (integrator.rs:82-99 + the geometry's get_geodesic_solver / create_initial_state);
// st, ct = sin / cos of pos[2] (KerrBL only).  Fills the KerrBL constants E, L_z, Q.
template <int G>
GDEV void init_state(const DevScene& S, const double* pos, double st, double ct, const double* p, double* y,
                     RayConst& rc) {
  rc.e = 0.0;
  rc.lz = 0.0;
  rc.q = 0.0;
  if constexpr (G == GRT_GEOM_KERR_BL) {  // kerr_bl.rs:505-577, :176-223 (BL ray)
    double a = S.a, radius = S.radius;
    double r = pos[1];
    double g[4][4];
    metric_bl(radius, a, r, st, ct, g);
    double pc[4];
    mat_vec(g, p, pc);
    double e = -pc[0], l_z = pc[3], p_theta = pc[2];
    double sin2 = st * st;
    double q = p_theta * p_theta + ct * ct * (l_z * l_z / fmax(sin2, 1e-28) - a * a * e * e);
    rc.e = e;
    rc.lz = l_z;
    rc.q = q;
    double sign_r = p[1] >= 0.0 ? 1.0 : -1.0;
    double sign_theta = p[2] >= 0.0 ? 1.0 : -1.0;
    double del = bl_delta(r, radius, a);
    double p_r = (r * r + a * a) * e - a * l_z;
    double le = l_z - a * e;
    double r_pot = p_r * p_r - del * (le * le + q);
    double th_pot = q + a * a * e * e * ct * ct - l_z * l_z * ct * ct / (st * st);
    y[0] = pos[0];
    y[1] = r;
    y[2] = pos[2];
    y[3] = pos[3];
    y[4] = sign_r * sqrt(fmax(r_pot, 0.0));
    y[5] = sign_theta * sqrt(fmax(th_pot, 0.0));
    y[6] = 0.0;
    y[7] = 0.0;
  } else if constexpr (G == GRT_GEOM_KERR) {  // kerr.rs:243-260
    double g[4][4];
    ks_metric(S.radius, S.a, pos[1], pos[2], pos[3], g);
    double pc[4];
    mat_vec(g, p, pc);
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      y[k] = pos[k];
      y[4 + k] = pc[k];
    }
  } else {
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      y[k] = pos[k];
      y[4 + k] = p[k];
    }
  }
}

// The image coordinates of the ray in output slot idx of a work list: an offset list's
// jittered pixel (get_ray_for_offset, camera.rs:247-254), or the pixel of a rectangle /
// row-band shard (local row idx / cols, mapped to its frame row).
GDEV void ray_pixel(const WorkList& wl, uint64_t idx, double* row, double* col) {
  if (wl.pixel_index) {
    const uint32_t pix = wl.pixel_index[idx];
    const double r = (double)(wl.row0 + pix / wl.cols), cc = (double)(wl.col0 + pix % wl.cols);
    *row = r + (wl.dy[idx] - 0.5);
    *col = cc + (wl.dx[idx] - 0.5);
  } else {
    const uint32_t r = (uint32_t)(idx / wl.cols), cc = (uint32_t)(idx % wl.cols);
    *row = (double)(wl.row0 + shard_frame_row(wl.band_rows, wl.shard, wl.n_shards, r));
    *col = (double)(wl.col0 + cc);
  }
}

// Create a camera ray's state (camera.rs:234-254 + init_state); also the observer
// energy the redshift needs (redshift.rs:40-43).
template <int G, bool FREQ = false>
GDEV void init_ray(const DevScene& S, double row, double col, double* y, RayConst& rc) {
  const DevCamera& cam = S.cam;
  double p[4];
  camera_momentum(cam, row, col, p);
  init_state<G>(S, cam.pos, cam.sin_theta, cam.cos_theta, p, y, rc);
  rc.obs = inner<G>(S, cam.pos, cam.sin_theta, cam.cos_theta, cam.vel, p);  // = observer_energy
  rc.pt = 0.0;
  rc.pphi = 0.0;
  if constexpr (FREQ) {  // get_ray_frequency_data: <e_t, p> and <axial Killing vector, p>
    const double et[4] = {1.0, 0.0, 0.0, 0.0};
    double ax[4] = {0.0, 0.0, 0.0, 1.0};  // d_phi (schwarzschild.rs:256, kerr_bl.rs:394, ...)
    if constexpr (G == GRT_GEOM_EUCLIDEAN || G == GRT_GEOM_KERR) {  // (0, -y, x, 0), kerr.rs:482-485
      ax[1] = -cam.pos[2];
      ax[2] = cam.pos[1];
      ax[3] = 0.0;
    }
    rc.pt = inner<G>(S, cam.pos, cam.sin_theta, cam.cos_theta, et, p);
    rc.pphi = inner<G>(S, cam.pos, cam.sin_theta, cam.cos_theta, ax, p);
  }
}

// integrator.rs:203-268
template <int G>
GDEV int should_stop(const DevScene& S, const double* y, double* c, bool& c_valid, uint64_t i) {
  if (!(isfinite(y[0]) && isfinite(y[1]) && isfinite(y[2]) && isfinite(y[3]))) return GRT_STOP_NAN;
  bool last = (i == S.max_steps - 1);
  if constexpr (G == GRT_GEOM_SCHWARZSCHILD || G == GRT_GEOM_KERR_BL) {
    if (G == GRT_GEOM_SCHWARZSCHILD || S.has_horizon) {
      if (y[1] <= S.horizon_r) return GRT_STOP_HORIZON;
    }
    if (last && y[1] < S.trapped_radius) return GRT_STOP_CLOSED_ORBIT;
  } else if constexpr (G == GRT_GEOM_KERR) {
    double r = sqrt(ks_r_sqr(S.a, y[1], y[2], y[3]));
    if (S.has_horizon && r <= S.horizon_r) return GRT_STOP_HORIZON;
    if (last && r < S.trapped_radius) return GRT_STOP_CLOSED_ORBIT;
  }
  // celestial test |x_cart|^2 > max_radius^2 (integrator.rs:203-268).  |x_cart| lies in
  // [|r|, |r| + far_a] in the curvilinear charts, so away from the celestial shell the
  // answer follows from r and the conversion is skipped.
  bool escaped = false, decided = false;
  if constexpr (G == GRT_GEOM_SCHWARZSCHILD || G == GRT_GEOM_KERR_BL || G == GRT_GEOM_EUCLIDEAN_SPHERICAL) {
    if (!c_valid && S.far_ok) {
      double ar = fabs(y[1]), hi = ar + S.far_a;
      if (hi * hi < S.cel_lo2) decided = true;
      else if (ar * ar > S.cel_hi2) decided = escaped = true;
    }
  }
  if (!decided) {
    if (!c_valid) {
      to_cart<G>(S, y, c);
      c_valid = true;
    }
    escaped = c[0] * c[0] + c[1] * c[1] + c[2] * c[2] > S.max_radius_sq;
  }
  if (escaped) return GRT_STOP_CELESTIAL;
  if (!(isfinite(y[4]) && isfinite(y[5]) && isfinite(y[6]) && isfinite(y[7]))) return GRT_STOP_NAN;
  return GRT_STOP_NONE;
}

// Exact far-field window filter (curvilinear charts).  True when neither end of the
// window (ya -> yb) can produce a hit in the reference's chord tests, decided from r and
// theta alone, so the Cartesian conversion and the chord arithmetic can be skipped:
//  * Disc (disc.rs:41-88): z = r cos(theta) keeps one strict sign, with |z| >= 1e-9 r at
//    both ends and r_a / r_b within [1e-3, 1e3], so t = -z_a / (z_b - z_a) is outside
//    [0, 1] by a factor ~1e-12, far above rounding (theta within 1e-9 of a zero of cos,
//    or outside (-pi/2, 3pi/2), is always converted).
//  * Sphere (sphere.rs:37-128): a hit needs |x - c|^2 - R^2 to change sign over the
//    window; |x| in [r, r + far_a] outside the host's shell [shell_lo, shell_hi]
//    (1e-9 margins) keeps both ends strictly outside.
//  * VolumetricDisc (volumetric_disc.rs:442-494): every hit lies in the capture region
//    |x.axis| <= cap_h, |x x axis| <= rout.  Skipped when (1) the chord stays farther than
//    vol_far_r = 2 |capture corner| (1 + 1e-6) from the origin: |x| >= r at both ends and
//    the chord is no longer than the chart path, |dr| + (r_max + far_a)(|dtheta| + |dphi|)
//    (the map's partial derivatives are bounded by 1, r + |a|, r + |a|); or (2) for the z
//    axis, both ends in one hemisphere with |z| = r |cos theta| >= r (2/pi) x (Jordan's
//    inequality, x = distance of theta to the equator) beyond cap_h (1 + 1e-6): z is
//    linear along the chord, so it never enters the slab.  Only for radii below
//    vol_rmax = 1e6 cap_h, where the chord arithmetic's rounding is far below the margins.
GDEV bool vol_far(const DevScene& S, const DevObject& o, const double* ya, const double* yb) {
  const double ra = ya[1], rb = yb[1];
  if (!(ra > 0.0 && rb > 0.0)) return false;
  const double rmax = fmax(ra, rb);
  if (!(rmax < o.vol_rmax)) return false;
  const double L = fabs(rb - ra) + (rmax + S.far_a) * (fabs(yb[2] - ya[2]) + fabs(yb[3] - ya[3]));
  if (fmin(ra, rb) > o.vol_far_r + L * (1.0 + 1e-9)) return true;
  if (!o.vol_slab_ok) return false;
  constexpr double N_LO = -1.5707963257948966, N_HI = 1.5707963257948966;  // (-pi/2, pi/2) -/+ 1e-9
  constexpr double S_LO = 1.5707963277948966, S_HI = 4.7123889793846899;   // (pi/2, 3pi/2) +/- 1e-9
  constexpr double HALF_PI = 1.5707963267948966, TWO_OVER_PI = 0.63661977236758134;
  const double ta = ya[2], tb = yb[2];
  double xa, xb;
  if (ta > N_LO && ta < N_HI && tb > N_LO && tb < N_HI) {
    xa = HALF_PI - fabs(ta);
    xb = HALF_PI - fabs(tb);
  } else if (ta > S_LO && ta < S_HI && tb > S_LO && tb < S_HI) {
    xa = HALF_PI - fabs(ta - PI);
    xb = HALF_PI - fabs(tb - PI);
  } else {
    return false;
  }
  const double za = ra * TWO_OVER_PI * (xa - 1e-15) * (1.0 - 1e-9);
  const double zb = rb * TWO_OVER_PI * (xb - 1e-15) * (1.0 - 1e-9);
  return za > o.vol_slab_h && zb > o.vol_slab_h;
}

template <int G, bool VOL>
GDEV bool window_far(const DevScene& S, const double* ya, const double* yb) {
  if constexpr (G != GRT_GEOM_SCHWARZSCHILD && G != GRT_GEOM_KERR_BL && G != GRT_GEOM_EUCLIDEAN_SPHERICAL) {
    return false;
  } else {
    if (!S.far_ok) return false;
    const double ra = ya[1], rb = yb[1], ta = ya[2], tb = yb[2];
    constexpr double N_LO = -1.5707963257948966, N_HI = 1.5707963257948966;  // (-pi/2, pi/2) -/+ 1e-9
    constexpr double S_LO = 1.5707963277948966, S_HI = 4.7123889793846899;   // (pi/2, 3pi/2) +/- 1e-9
    for (uint32_t k = 0; k < S.n_objects; ++k) {
      const DevObject& o = S.obj[k];
      if (o.kind == GRT_OBJ_DISC) {
        bool north = ta > N_LO && ta < N_HI && tb > N_LO && tb < N_HI;
        bool south = ta > S_LO && ta < S_HI && tb > S_LO && tb < S_HI;
        if (!(north || south)) return false;
        if (!(ra >= 1e-3 * rb && rb >= 1e-3 * ra && ra > 0.0)) return false;
      } else if (VOL && o.kind == GRT_OBJ_VOLUMETRIC_DISC) {
        if (!vol_far(S, o, ya, yb)) return false;
      } else {
        bool out_a = ra > o.shell_hi || fabs(ra) + S.far_a < o.shell_lo;
        bool out_b = rb > o.shell_hi || fabs(rb) + S.far_a < o.shell_lo;
        if (!(out_a && out_b)) return false;
      }
    }
    return true;
  }
}

// The commonest accepted step of a curvilinear chart as one predicate, evaluated without
// branches over the lanes (integrate_kernel's quick step): step_control's first case
// (err_sq < tiny_err_sq: accepted, next h = clamp(4h)), window_far for every object (no
// chord test, c_valid = false) and should_stop's checks all passing on yn with the
// celestial test decided by r (finite, outside the horizon, inside the celestial shell,
// not the last step).  True only where the general path does exactly the quick step's
// updates; every other case takes the general path.
template <int G>
GDEV bool quick_step_ok(const DevScene& S, double err_sq, const double* y, const double* yn, uint64_t i_next) {
  static_assert(G == GRT_GEOM_SCHWARZSCHILD, "quick step: Schwarzschild only");
  constexpr double N_LO = -1.5707963257948966, N_HI = 1.5707963257948966;
  constexpr double S_LO = 1.5707963277948966, S_HI = 4.7123889793846899;
  const double ra = y[1], rb = yn[1], ta = y[2], tb = yn[2];
  bool ok = (err_sq < S.tiny_err_sq) & (S.far_ok != 0);
  const bool north = (ta > N_LO) & (ta < N_HI) & (tb > N_LO) & (tb < N_HI);
  const bool south = (ta > S_LO) & (ta < S_HI) & (tb > S_LO) & (tb < S_HI);
  const bool ratio = (ra >= 1e-3 * rb) & (rb >= 1e-3 * ra) & (ra > 0.0);
  for (uint32_t k = 0; k < S.n_objects; ++k) {
    const DevObject& o = S.obj[k];
    const bool out_a = (ra > o.shell_hi) | (fabs(ra) + S.far_a < o.shell_lo);
    const bool out_b = (rb > o.shell_hi) | (fabs(rb) + S.far_a < o.shell_lo);
    ok = ok & ((o.kind == GRT_OBJ_DISC) ? ((north | south) & ratio) : (out_a & out_b));
  }
  bool fin = true;
#pragma unroll
  for (int k = 0; k < 8; ++k) fin = fin & (bool)isfinite(yn[k]);
  const double ar = fabs(rb), hi = ar + S.far_a;
  return ok & fin & (rb > S.horizon_r) & (hi * hi < S.cel_lo2) & (i_next != S.max_steps - 1);
}

// The step-size controller of rkf45 (runge_kutta.rs:148-178) after one attempt with
// error norm `err` at step h_cur.  Accepted: h_next is the next step's h.  Rejected:
// h_cur is the retry's step (STEP_RETRY), or the 100th retry failed (STEP_FAILED,
// Err(MaxStepsReached)).
enum { STEP_ACCEPTED = 0, STEP_RETRY = 1, STEP_FAILED = 2 };
GDEV int step_control(const DevScene& S, double err_sq, double& h_cur, int& retries, double& h_next) {
  // err_sq < tiny_err_sq (host: min(pow_skip_err, small_lo)^2 * (1 - 1e-9)) proves
  // err = sqrt(err_sq) < both thresholds (and < eps): accepted with h_next = clamp(4h),
  // the outcome of every branch below, without the sqrt (the far-field steps)
  if (err_sq < S.tiny_err_sq) {
    h_next = rclamp(h_cur * H_GROWTH, H_MIN, H_MAX);
    return STEP_ACCEPTED;
  }
  const double err = sqrt(err_sq);
  // h_prop = err > 0 ? BETA*h*(eps/err)^(1/5) : 4h, then min(., 4h).  For eps/err >= 1800,
  // BETA*1800^(1/5) = 4.0308 > 4, so the min is 4h whatever pow's last ulp: pow is
  // skipped there (the far-field steps), which leaves every result bit-identical.
  // err < pow_skip_err (host: eps/1800 * (1 - 1e-9)) proves eps/err > 1800: the division
  // is skipped with the pow.
  double h_prop = h_cur * H_GROWTH;
  if (err > 0.0 && !(err < S.pow_skip_err)) {
    const double ratio = S.epsilon / err;
    if (ratio < POW_SATURATED) h_prop = BETA * h_cur * rpow(ratio, INV_ORDER);
  }
  h_prop = rclamp(fmin(h_prop, h_cur * H_GROWTH), H_MIN, H_MAX);
  if (err > S.epsilon) {
    if (h_cur <= H_MIN) {
      h_next = h_cur;
      return STEP_ACCEPTED;
    }
    h_cur = rclamp(h_prop / 2.0, H_MIN, H_MAX);
    return (++retries >= MAX_RETRY) ? STEP_FAILED : STEP_RETRY;
  }
  // err / eps < 1e-5, decided without the division away from the threshold (1e-9 margins)
  const bool small = err < S.small_lo || (!(err > S.small_hi) && err / S.epsilon < SMALL_ERR);
  h_next = small ? rclamp(h_cur * H_GROWTH, H_MIN, H_MAX) : h_prop;
  return STEP_ACCEPTED;
}

#if GRT_RAY_TIMES
// Per-ray schedule record of a diagnostic build, [6][n] words at output slot idx: start,
// hand-off and end (s_memrealtime, 100 MHz), the starting lane's hardware place
// (XCC_ID << 32 | HW_ID), attempts in the integrate kernel, attempts in the tail kernel.
__device__ unsigned long long* g_ray_times;
GDEV void ray_time(uint64_t n, uint64_t idx, int k, unsigned long long v) {
  if (g_ray_times) g_ray_times[(uint64_t)k * n + idx] = v;
}
GDEV unsigned long long hw_place() {
  const unsigned hw = __builtin_amdgcn_s_getreg(4 | (31 << 11));    // HW_REG_HW_ID
  const unsigned xcc = __builtin_amdgcn_s_getreg(20 | (31 << 11));  // HW_REG_XCC_ID
  return ((unsigned long long)xcc << 32) | hw;
}
#if GRT_MAIN_TU  // the KerrBL unit's kernels record too
hipError_t set_ray_times(unsigned long long* p) {
  hipError_t e = hipMemcpyToSymbol(HIP_SYMBOL(g_ray_times), &p, sizeof(p));
  return e != hipSuccess ? e : kerr_bl::set_ray_times(p);
}
#elif GRT_KERR_BL_TU
hipError_t set_ray_times(unsigned long long* p) { return hipMemcpyToSymbol(HIP_SYMBOL(g_ray_times), &p, sizeof(p)); }
#endif
#if GRT_KERR_BL_TU && GRT_PATH_COUNT
hipError_t path_read(unsigned long long* out, bool reset) {
  hipError_t e = hipMemcpyFromSymbol(out, HIP_SYMBOL(g_path), sizeof(g_path));
  if (e == hipSuccess && reset) {
    const unsigned long long z[2 * NPATH] = {};
    e = hipMemcpyToSymbol(HIP_SYMBOL(g_path), z, sizeof(z));
  }
  return e;
}
#endif
#define RAY_TIME(n, idx, k, v) ray_time(n, idx, k, v)
#else
#define RAY_TIME(n, idx, k, v) ((void)0)
#endif

// The observer energy of the camera ray in output slot idx (init_ray's rc.obs, recomputed
// by the shade kernels instead of stored).
template <int G>
GDEV double observer_energy(const DevScene& S, const WorkList& wl, uint64_t idx) {
  double row, col, p[4];
  ray_pixel(wl, idx, &row, &col);
  const DevCamera& cam = S.cam;
  camera_momentum(cam, row, col, p);
  return inner<G>(S, cam.pos, cam.sin_theta, cam.cos_theta, cam.vel, p);
}

// The record of a ray (Workspace::fin, 8 doubles = one 64-B line, written whole by the
// lane that ends it): what the shade kernel reads of the final state and the ray
// constants, and the ray's counts.
//   Schwarzschild, Kerr-Schild, flat charts: y[1..7] (y[0] is not read; Kerr-Schild's
//   momentum needs none of E, L_z, Q), then the candidate count (low 32 bits), stop
//   reason and status (bits 32-39, 40-47).  The observer energy is not stored: the shade
//   kernel recomputes it from the ray's pixel (observer_energy: init_ray's operations on
//   the same operands, hence the same bits), and the step count goes straight to the
//   optional per-pixel output (Workspace::steps).
//   KerrBL: r, theta, phi, v_r, v_theta, observer energy, E, L_z (y[6], y[7] are
//   identically 0, Q only drives the RHS), and the counts in a 16-B meta record.  The
//   one-record layout measured C3 +8% (its 3-wave kernel's spills moved into the
//   accepted-step path: profiles/r04r), so KerrBL keeps this one.
struct RayMeta {
  uint32_t nrec, steps;
  int stop, status;
};
template <int G>
GDEV void fin_put(const Workspace& ws, uint64_t idx, const double* y, const RayConst& rc, uint32_t nrec, int stop,
                  int status) {
  double v[8];
  if constexpr (G == GRT_GEOM_KERR_BL) {
#pragma unroll
    for (int k = 0; k < 5; ++k) v[k] = y[1 + k];
    v[5] = rc.obs;
    v[6] = rc.e;
    v[7] = rc.lz;
  } else {
#pragma unroll
    for (int k = 0; k < 7; ++k) v[k] = y[1 + k];
    v[7] = __hiloint2double((int)((uint32_t)(stop & 0xff) | ((uint32_t)(status & 0xff) << 8)), (int)nrec);
  }
  double2* d = reinterpret_cast<double2*>(ws.fin + idx * 8);
#pragma unroll
  for (int k = 0; k < 4; ++k) d[k] = make_double2(v[2 * k], v[2 * k + 1]);
}
// rc.obs: KerrBL's from the record, else 0 (the caller sets observer_energy)
template <int G>
GDEV RayMeta fin_get(const Workspace& ws, uint64_t idx, double* y, RayConst& rc) {
  const double2* d = reinterpret_cast<const double2*>(ws.fin + idx * 8);
  double v[8];
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    const double2 w = d[k];
    v[2 * k] = w.x;
    v[2 * k + 1] = w.y;
  }
  y[0] = 0.0;
  rc.q = 0.0;
  rc.pt = 0.0;
  rc.pphi = 0.0;
  if constexpr (G == GRT_GEOM_KERR_BL) {
#pragma unroll
    for (int k = 0; k < 5; ++k) y[1 + k] = v[k];
    y[6] = 0.0;
    y[7] = 0.0;
    rc.obs = v[5];
    rc.e = v[6];
    rc.lz = v[7];
    const uint4 m = reinterpret_cast<const uint4*>(ws.meta)[idx];
    return RayMeta{m.y, m.x, (int)(m.z & 0xffu), (int)((m.z >> 8) & 0xffu)};
  } else {
#pragma unroll
    for (int k = 0; k < 7; ++k) y[1 + k] = v[k];
    rc.obs = 0.0;
    rc.e = 0.0;
    rc.lz = 0.0;
    const uint64_t m = (uint64_t)__double_as_longlong(v[7]);
    return RayMeta{(uint32_t)m, 0u, (int)((m >> 32) & 0xffu), (int)((m >> 40) & 0xffu)};
  }
}

// End of a ray: its record goes to the workspace for the shade kernel.
template <int G>
GDEV void store_ray(const Workspace& ws, uint64_t idx, const double* y, const RayConst& rc, int stop, int status,
                    uint32_t nrec, uint32_t steps) {
  RAY_TIME(ws.n, idx, 2, __builtin_amdgcn_s_memrealtime());
  fin_put<G>(ws, idx, y, rc, nrec, stop, status);
  if constexpr (G == GRT_GEOM_KERR_BL) {
    reinterpret_cast<uint4*>(ws.meta)[idx] =
        make_uint4(steps, nrec, (uint32_t)(stop & 0xff) | ((uint32_t)(status & 0xff) << 8), 0u);
  } else {
    if (ws.steps) ws.steps[idx] = steps;
  }
}

// Candidate nrec >= GRT_WS_SLOTS of ray idx: one record appended to the hit pool and
// linked after the ray's previous one.  Once a record does not fit, the ray's list is
// marked lost (ovf_last = HIT_NIL) and nothing more is linked; the count keeps growing so
// that the host learns the size the trace needed.
GDEV void hit_append(const Workspace& ws, uint64_t idx, uint32_t nrec, uint32_t win, uint32_t obj,
                     const double* p, const double* pt, const double* dir) {
  const HitPool& hp = *ws.pool;
  const unsigned long long pos = atomicAdd(hp.count, 1ull);
  const bool first = nrec == GRT_WS_SLOTS;
  const uint32_t prev = first ? HIT_NIL : ws.pool->last[idx];
  if (pos >= hp.cap || (!first && prev == HIT_NIL)) {
    if (first) ws.pool->head[idx] = HIT_NIL;
    ws.pool->last[idx] = HIT_NIL;
    return;
  }
  const uint64_t m = hp.cap;
  hp.win[pos] = win;
  hp.obj[pos] = (uint8_t)obj;
#pragma unroll
  for (int q = 0; q < 4; ++q) hp.p[q * m + pos] = p[q];
#pragma unroll
  for (int q = 0; q < 3; ++q) hp.pt[q * m + pos] = pt[q];
  if (dir) {
#pragma unroll
    for (int q = 0; q < 3; ++q) hp.dir[q * m + pos] = dir[q];
  }
  if (first) ws.pool->head[idx] = (uint32_t)pos;
  else hp.next[prev] = (uint32_t)pos;
  ws.pool->last[idx] = (uint32_t)pos;
}

// The window (y -> yn) of accepted step i against every object in config order
// (objects.rs:81); a hit nearer than the current nearest (objects.rs:86-88) is recorded
// as candidate nrec: its object, window index, hit point and the lerped momentum
// (objects.rs:27-44).  `writer`: this lane stores the candidate (one lane of a quad in
// tail_kernel; every lane computes the same decisions).  c / c_valid follow yn.
template <int G, bool VOL>
GDEV void window_pass(const DevScene& S, const Workspace& ws, const RayConst& rc, uint64_t idx, const double* y,
                      const double* yn, double* c, bool& c_valid, uint64_t i, uint32_t& nrec, bool writer) {
  const uint64_t n = ws.n;
  if (!window_far<G, VOL>(S, y, yn)) {
    PATH_COUNT(4);
    if (!c_valid) to_cart<G>(S, y, c);
    double cn[3];
    to_cart<G>(S, yn, cn);
    double shortest = 1.7976931348623157e308;
    for (uint32_t k = 0; k < S.n_objects; ++k) {
      const DevObject& o = S.obj[k];
      double t, pt[3];
      bool hit;
      if (VOL && o.kind == GRT_OBJ_VOLUMETRIC_DISC) hit = vdisc_chord(o, c, cn, &t, pt);
      else hit = (o.kind == GRT_OBJ_DISC) ? disc_chord(o, c, cn, &t, pt) : sphere_chord(o, c, cn, &t, pt);
      if (!hit) continue;
      double wx = pt[0], wy = pt[1], wz = pt[2];
      if (o.kind == GRT_OBJ_SPHERE) {
        wx = pt[0] + o.cx;
        wy = pt[1] + o.cy;
        wz = pt[2] + o.cz;
      }
      double dx = wx - c[0], dy = wy - c[1], dz = wz - c[2];
      double distance = sqrt(dx * dx + dy * dy + dz * dz);
      if (!(distance < shortest)) continue;
      shortest = distance;
      double ph[4];
      if (writer) lerp_momentum<G>(S, rc, y, yn, t, ph);
      if (writer && nrec < GRT_WS_SLOTS) {
        const uint64_t slot = (uint64_t)nrec * n + idx;
        double2* d = reinterpret_cast<double2*>(ws.rec + slot);
        d[0] = make_double2(ph[0], ph[1]);
        d[1] = make_double2(ph[2], ph[3]);
        d[2] = make_double2(pt[0], pt[1]);
        d[3] = make_double2(pt[2], __hiloint2double((int)k, (int)(uint32_t)i));
        if constexpr (VOL) {  // chord direction for the raymarch (volumetric_disc.rs:576, :589-594)
          ws.rec_dir[slot] = cn[0] - c[0];
          ws.rec_dir[(uint64_t)GRT_WS_SLOTS * n + slot] = cn[1] - c[1];
          ws.rec_dir[(uint64_t)2 * GRT_WS_SLOTS * n + slot] = cn[2] - c[2];
        }
      } else if (writer) {  // beyond the workspace slots: the hit pool
        double dir[3] = {cn[0] - c[0], cn[1] - c[1], cn[2] - c[2]};
        hit_append(ws, idx, nrec, (uint32_t)i, k, ph, pt, VOL ? dir : nullptr);
      }
      nrec++;
    }
#pragma unroll
    for (int k = 0; k < 3; ++k) c[k] = cn[k];
    c_valid = true;
  } else {
    c_valid = false;
  }
}

// A ray's loop state at the top of integrate_kernel's loop, in entry e of the tail list.
struct LoopState {
  double y[8], c[3];
  double h, h_cur;
  uint64_t i, idx;
  uint32_t nrec;
  int retries;
  bool c_valid;
};
// Entry e of an entry arena `st` of m entries ([16][m] words: TailList::st).
GDEV void tail_save(unsigned long long* st, uint64_t m, uint64_t e, const LoopState& s) {
  unsigned long long* w = st + e;
#pragma unroll
  for (int k = 0; k < 8; ++k) w[k * m] = (unsigned long long)__double_as_longlong(s.y[k]);
#pragma unroll
  for (int k = 0; k < 3; ++k) w[(8 + k) * m] = (unsigned long long)__double_as_longlong(s.c[k]);
  w[11 * m] = (unsigned long long)__double_as_longlong(s.h);
  w[12 * m] = (unsigned long long)__double_as_longlong(s.h_cur);
  w[13 * m] = s.i;
  w[14 * m] = s.idx;
  w[15 * m] = (unsigned long long)s.nrec | ((unsigned long long)(uint32_t)s.retries << 32) |
              ((unsigned long long)(s.c_valid ? 1 : 0) << 48);
}
GDEV void tail_load(const unsigned long long* st, uint64_t m, uint64_t e, LoopState& s) {
  const unsigned long long* w = st + e;
#pragma unroll
  for (int k = 0; k < 8; ++k) s.y[k] = __longlong_as_double((long long)w[k * m]);
#pragma unroll
  for (int k = 0; k < 3; ++k) s.c[k] = __longlong_as_double((long long)w[(8 + k) * m]);
  s.h = __longlong_as_double((long long)w[11 * m]);
  s.h_cur = __longlong_as_double((long long)w[12 * m]);
  s.i = w[13 * m];
  s.idx = w[14 * m];
  const unsigned long long f = w[15 * m];
  s.nrec = (uint32_t)f;
  s.retries = (int)((f >> 32) & 0xffffu);
  s.c_valid = ((f >> 48) & 1u) != 0;
}
GDEV unsigned long long load_agent(const unsigned long long* p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
// Items claimed so far from the work counter (both ends of a two-ended queue).
GDEV uint64_t items_claimed(unsigned long long w, bool two_ended) {
  return two_ended ? (w & 0xffffffffull) + (w >> 32) : w;
}
// This wave's hardware slot on its SIMD (HW_REG_HW_ID bits 3:0, gfx9).
GDEV unsigned hw_wave_slot() { return __builtin_amdgcn_s_getreg(4 | (3 << 11)); }
// One lane integrates one ray at a time: RKF45 attempts, and after every accepted
// step the chord test of window (previous step, step) against every object in config
// order (objects.rs:81) and the stop test (window_pass, should_stop).
// Kerr-Schild with tl.cap != 0: once the tile queue is drained and at most tl.threshold
// rays are live, each wave hands its rays to tail_kernel (tail_save) and exits.
template <int G, bool VOL>
__global__ void __launch_bounds__(256, integrate_waves(G, VOL)) integrate_kernel(
    const DevScene* __restrict__ Sp, WorkList wl, Workspace ws, unsigned long long* __restrict__ counter,
    unsigned long long* __restrict__ stats, TailList tl) {
  const DevScene& S = *Sp;
  // items present: the capacity, or the count the adaptive pass decided on the device
  const uint64_t n_items = wl.n_live ? (uint64_t)min((unsigned long long)wl.n_items, *wl.n_live) : wl.n_items;
  if (n_items == 0) return;  // an empty chunk of a supersample pass
#if GRT_PATH_COUNT
  if (threadIdx.x < 2 * NPATH) path_lds[threadIdx.x] = 0;  // ordered before use by the tables' barrier
#endif
  glibc::tables_to_lds();  // whole block, before any lookup
  const int lane = threadIdx.x & 63;
  const uint64_t lanemask_lt = (lane == 0) ? 0ull : (~0ull >> (64 - lane));
  constexpr uint64_t CHUNK = 64;
  const uint64_t n = ws.n;
  constexpr bool TAIL = (G == GRT_GEOM_KERR);
  const bool tail_on = TAIL && tl.cap != 0;
  constexpr int NKL = (((GRT_KLDS_GEOMS) >> G) & 1) ? GRT_KL_STAGES : 0;
  if (tail_on && blockIdx.x == 0 && threadIdx.x == 0) tl.ctl[3] = __builtin_amdgcn_s_memrealtime();

  // Two-ended queue (WorkList::two_ended).  The issue arbiter of a SIMD serves the oldest
  // wave first: with two Kerr-Schild waves per SIMD the older one runs an attempt in
  // ~31 us and the younger one in ~130 us while both are busy (per-ray record of a C4
  // shard, profiles/r04a).  So one wave per SIMD (even hardware slot) takes the items
  // with the longest predicted rays from the front and holds the issue priority
  // explicitly (s_setprio), and the others take the shortest items from the back.  Both
  // ends advance one packed counter, so a claim sees every earlier claim of either end:
  // with (front, back) its snapshot, rank r is item front + r or n - 1 - (back + r), and
  // exists while front + back + r < n.
  const bool two_ended = wl.two_ended != 0;
  const bool from_back = two_ended && (hw_wave_slot() & 1u);
  if (two_ended && !from_back) __builtin_amdgcn_s_setprio(1);
  uint64_t chunk_next = 0, chunk_end = 0;  // wave-uniform work cursor
  bool active = false, done = false;
  bool started = false, ended = false;  // since the last live-count update (tail_on)
  uint32_t poll = 0;
  bool q_drained = false;  // this wave has seen the tile queue drained (it stays drained)
  uint64_t idx = 0;      // output slot of the current ray
  double y[8];           // state
  double c[3];           // Cartesian position of the last accepted step (when c_valid)
  bool c_valid = false;
  double h = 0.0, h_cur = 0.0;
  uint64_t i = 0;        // accepted step index
  int retries = 0;
  uint32_t nrec = 0;
  RayConst rc;
  // per-lane counters in 32 bits (one VGPR each): a lane integrates far fewer than 2^32
  // steps in one launch (C4 whole frame: ~5e6 per lane)
  uint32_t n_acc = 0, n_att = 0;
  uint64_t w_rays = 0;  // rays started by this wave: counted in wave-uniform control flow (an SGPR)
#if GRT_RAY_TIMES
  uint32_t ray_att = 0;
#endif

  while (true) {
    // ---------------- lane refill: ballot, one atomic per claim ------------------
    bool need = !active && !done;
    uint64_t need_mask = __ballot(need);
    if (need_mask) {
      bool fresh = false;  // this lane started a ray in this refill
      uint64_t cnt = __popcll(need_mask);
      uint64_t remaining = chunk_end - chunk_next;
      uint64_t new_base = 0;
      // Claims are exact: a wave takes exactly the items it starts now.  A wave holding
      // unstarted items of a 64-item chunk when the queue drains starts them one ray
      // lifetime late, on its own lanes, while other waves have emptied (C5's supersample
      // pass, ~2.5 sub-rays per lane: its last ray started at 0.375 s of a 0.47 s pass with
      // chunks, at 0.21 s of 0.39 s with exact claims; C2 -2.5%; profiles/r05d, r05e).
      // KerrBL claims 64-item chunks until its view of the counter is within two grids'
      // worth of lanes of the end: its 2.25M short rays end ~13M times a second, and an
      // atomic on one address per refill cost C3 +16% (profiles/r05l, r05m).
      const uint64_t grid_lanes = (uint64_t)gridDim.x * blockDim.x;
      const bool exact = TAIL || two_ended || G != GRT_GEOM_KERR_BL || chunk_end + 2 * grid_lanes >= n_items;
      const uint64_t take = exact ? cnt - remaining : CHUNK;
      if (cnt > remaining) {
        unsigned long long b = 0;
        if (lane == 0) b = atomicAdd(counter, from_back ? (unsigned long long)take << 32 : (unsigned long long)take);
        new_base = __shfl(b, 0);
      }
      if (need) {
        uint64_t rank = __popcll(need_mask & lanemask_lt);
        uint64_t item = rank < remaining ? chunk_next + rank : new_base + (rank - remaining);
        if (two_ended) {  // new_base is the counter's snapshot (front | back << 32)
          const uint64_t f = new_base & 0xffffffffull, bk = new_base >> 32;
          item = (f + bk + rank >= n_items) ? n_items : (from_back ? n_items - 1 - (bk + rank) : f + rank);
        }
        if (item >= n_items) {
          if (TAIL && tail_on && !done && tl.ctl[4] == 0ull)
            atomicCAS(&tl.ctl[4], 0ull, (unsigned long long)__builtin_amdgcn_s_memrealtime());
          done = true;
        } else {
          double row, col;
          bool valid = true;
          if (wl.pixel_index) {  // offset list (get_ray_for_offset, camera.rs:247-254)
            idx = item;
            ray_pixel(wl, idx, &row, &col);
          } else {  // 8x8 pixel tiles, row-major tiles: a wave starts on a compact patch
            uint64_t tile = item >> 6;
            if (wl.tile_order) tile = wl.tile_order[tile];  // longest-predicted tiles first
            uint32_t w = (uint32_t)(item & 63);
            uint32_t tr = (uint32_t)(tile / wl.tiles_x), tc = (uint32_t)(tile % wl.tiles_x);
            uint32_t r = tr * 8 + (w >> 3), cc = tc * 8 + (w & 7);
            valid = (r < wl.rows) && (cc < wl.cols);
            // ray_pixel's rectangle / shard case, from (r, cc) directly
            row = (double)(wl.row0 + shard_frame_row(wl.band_rows, wl.shard, wl.n_shards, r));
            col = (double)(wl.col0 + cc);
            idx = (uint64_t)r * wl.cols + cc;
          }
          if (valid) {
            init_ray<G, VOL>(S, row, col, y, rc);
            if constexpr (VOL) {  // the raymarch's frequency data (march_kernel)
              ws.rc[0 * n + idx] = rc.obs;
              ws.rc[1 * n + idx] = rc.e;
              ws.rc[2 * n + idx] = rc.lz;
              ws.rc[3 * n + idx] = rc.q;
              ws.rc[4 * n + idx] = rc.pt;
              ws.rc[5 * n + idx] = rc.pphi;
            }
            c_valid = false;
            h = S.step_size;
            h_cur = rclamp(h, H_MIN, H_MAX);
            i = 0;
            retries = 0;
            nrec = 0;
            active = true;
            started = true;
            fresh = true;
#if GRT_RAY_TIMES
            ray_att = 0;
            RAY_TIME(n, idx, 0, __builtin_amdgcn_s_memrealtime());
            RAY_TIME(n, idx, 3, hw_place());
#endif
            if (S.max_steps <= 1) {  // `for i in 1..max_steps` never runs
              store_ray<G>(ws, idx, y, rc, GRT_STOP_NONE, GRT_OK, 0, 0);
              active = false;
              ended = true;
            }
          }
        }
      }
      w_rays += __popcll(__ballot(fresh));
#if GRT_TAIL_PRIO
      // KerrBL's rays are all short: measured no gain there
      if constexpr (!TAIL && G != GRT_GEOM_KERR_BL) {
        // After the queue has drained for this wave (one of its lanes found no item), the
        // pass ends on the rays with the most steps left, so the waves holding them get the
        // SIMD's issue slots first (s_setprio; the arbiter otherwise serves the oldest wave):
        // the estimate of what is left is max_radius unit steps (a ray escapes after about
        // that many) minus the wave's fewest accepted steps.  Scheduling only, never results.
        if (!two_ended && __ballot(done) != 0) {
          uint32_t mi = active ? (uint32_t)i : 0xffffffffu;
#pragma unroll
          for (int off = 32; off > 0; off >>= 1) mi = min(mi, (uint32_t)__shfl_xor((int)mi, off));
          const double len = sqrt(S.max_radius_sq);
          const double left = len - (double)mi;
          if (left > 0.67 * len) __builtin_amdgcn_s_setprio(3);
          else if (left > 0.33 * len) __builtin_amdgcn_s_setprio(2);
          else __builtin_amdgcn_s_setprio(1);
        }
      }
#endif
      if (cnt > remaining) {
        chunk_next = new_base + (cnt - remaining);
        chunk_end = new_base + take;
      } else {
        chunk_next += cnt;
      }
    }
    if constexpr (TAIL) {
      if (tail_on) {
        // live-ray count: one atomic per wave when rays started or ended
        const uint64_t st_mask = __ballot(started), en_mask = __ballot(ended);
        started = ended = false;
        const long long d = (long long)__popcll(st_mask) - (long long)__popcll(en_mask);
        if (d != 0 && lane == 0) atomicAdd(&tl.ctl[0], (unsigned long long)d);
        // hand-off: queue drained (and nothing left in this wave's chunk), few rays left.
        // Kerr-Schild claims exactly what it starts, so its chunk is always used up: the
        // drained test (an agent-scope load, served beyond this XCD's L2) runs every 256
        // attempts until the wave has seen the queue drained, then the live count every 16
        if ((chunk_next >= chunk_end || chunk_next >= n_items) && ((++poll & (q_drained ? 15u : 255u)) == 0u) &&
            (q_drained || (q_drained = items_claimed(load_agent(counter), two_ended) >= n_items)) &&
            (long long)load_agent(&tl.ctl[0]) <= (long long)tl.threshold) {
          const uint64_t ev = __ballot(active);
          if (ev) {
            unsigned long long b = 0;
            if (lane == 0) {
              b = atomicAdd(&tl.ctl[1], (unsigned long long)__popcll(ev));
              if (b == 0) tl.ctl[5] = __builtin_amdgcn_s_memrealtime();
            }
            b = __shfl(b, 0);
            if (active) {
              const uint64_t e = b + __popcll(ev & lanemask_lt);
              if (e < tl.cap) {
                LoopState s;
#pragma unroll
                for (int k = 0; k < 8; ++k) s.y[k] = y[k];
#pragma unroll
                for (int k = 0; k < 3; ++k) s.c[k] = c[k];
                s.h = h;
                s.h_cur = h_cur;
                s.i = i;
                s.idx = idx;
                s.nrec = nrec;
                s.retries = retries;
                s.c_valid = c_valid;
                tail_save(tl.st, tl.cap, e, s);
                RAY_TIME(n, idx, 1, __builtin_amdgcn_s_memrealtime());
                RAY_TIME(n, idx, 4, ray_att);
                active = false;
                done = true;
              }
            }
          }
        }
      }
    }
    if (__ballot(!done) == 0) break;
    if (!active) continue;

    // ---------------- one RKF45 attempt (runge_kutta.rs:148-178) ----------------
    double yn[8];
    double err_sq;
    // Kerr-Schild: the RHS dwarfs the saved products, and a second copy of its attempt
    // (+80 KB of code) is not worth them
    constexpr bool UNIT_H_COPY = GRT_UNIT_H && G != GRT_GEOM_KERR;
    constexpr bool QUICK = GRT_QUICK_STEP && G == GRT_GEOM_SCHWARZSCHILD && !VOL;
    while (true) {
      err_sq = (UNIT_H_COPY && __ballot(active && h_cur != 1.0) == 0)
                   ? rkf_attempt<G, UNIT_H_COPY, false, NKL>(S, rc, y, h_cur, yn)
                   : rkf_attempt<G, false, false, NKL>(S, rc, y, h_cur, yn);
      n_att++;
      PATH_COUNT(6);
#if GRT_RAY_TIMES
      ray_att++;
#endif
      if constexpr (QUICK) {
        // every lane of the wave on the commonest accepted step (quick_step_ok): the
        // general path's updates in one straight-line block, then straight on to the next
        // attempt (no ray ended, so no lane needs a refill)
        if (__ballot(!quick_step_ok<G>(S, err_sq, y, yn, i + 1)) == 0) {
          h = rclamp(h_cur * H_GROWTH, H_MIN, H_MAX);
          i++;
          n_acc++;
          c_valid = false;
#pragma unroll
          for (int k = 0; k < 8; ++k) y[k] = yn[k];
          retries = 0;
          h_cur = rclamp(h, H_MIN, H_MAX);
          continue;
        }
      }
      break;
    }
    double h_next;
    const int ctl = step_control(S, err_sq, h_cur, retries, h_next);
    if (ctl != STEP_ACCEPTED) {
      if (ctl == STEP_FAILED) {  // Err(MaxStepsReached)
        store_ray<G>(ws, idx, y, rc, GRT_STOP_NONE, GRT_ERR_MAX_STEPS_REACHED, 0, (uint32_t)i);
        RAY_TIME(n, idx, 4, ray_att);
        active = false;
        ended = true;
      }
      continue;
    }

    // ---------------- accepted step i (integrator.rs:100-162) --------------------
    PATH_COUNT(5);
    h = h_next;
    i++;
    n_acc++;
    window_pass<G, VOL>(S, ws, rc, idx, y, yn, c, c_valid, i, nrec, true);
#pragma unroll
    for (int k = 0; k < 8; ++k) y[k] = yn[k];

    int stop = should_stop<G>(S, y, c, c_valid, i);
    if (stop != GRT_STOP_NONE || i == S.max_steps - 1) {
      store_ray<G>(ws, idx, y, rc, stop, GRT_OK, nrec, (uint32_t)i);
      RAY_TIME(n, idx, 4, ray_att);
      active = false;
      ended = true;
      continue;
    }
    retries = 0;
    h_cur = rclamp(h, H_MIN, H_MAX);
  }

  // per-wave reduction of the counters, one atomic per wave
  uint64_t w_acc = n_acc, w_att = n_att;
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) {
    w_acc += __shfl_down(w_acc, off);
    w_att += __shfl_down(w_att, off);
  }
  if (lane == 0) {
    atomicAdd(stats + 0, (unsigned long long)w_acc);
    atomicAdd(stats + 1, (unsigned long long)w_att);
    atomicAdd(stats + 2, (unsigned long long)w_rays);
  }
#if GRT_PATH_COUNT
  __syncthreads();  // every wave of the block has left its loop
  if (threadIdx.x < 2 * NPATH) atomicAdd(&g_path[threadIdx.x], path_lds[threadIdx.x]);
#endif
}

// ============================================================= tail kernel =======
// One attempt of a handed-off ray on the 4 lanes of its quad: the loop body of
// integrate_kernel with the RHS split over the quad (rhs_ks_quad); lane 0 of the quad
// writes.  Returns true when the ray has ended (its outputs are stored).
template <int G, bool VOL>
GDEV bool quad_attempt(const DevScene& S, const Workspace& ws, const RayConst& rc, LoopState& s, int sub,
                       bool writer, uint64_t& n_acc, uint64_t& n_att) {
  double yn[8];
  const double err_sq = rkf_attempt<G, false, true>(S, rc, s.y, s.h_cur, yn, sub);
  n_att++;
  double h_next;
  const int ctl = step_control(S, err_sq, s.h_cur, s.retries, h_next);
  if (ctl != STEP_ACCEPTED) {
    if (ctl == STEP_FAILED) {  // Err(MaxStepsReached)
      if (writer) store_ray<G>(ws, s.idx, s.y, rc, GRT_STOP_NONE, GRT_ERR_MAX_STEPS_REACHED, 0, (uint32_t)s.i);
      return true;
    }
    return false;
  }
  s.h = h_next;
  s.i++;
  n_acc++;
  window_pass<G, VOL>(S, ws, rc, s.idx, s.y, yn, s.c, s.c_valid, s.i, s.nrec, writer);
#pragma unroll
  for (int k = 0; k < 8; ++k) s.y[k] = yn[k];
  const int stop = should_stop<G>(S, s.y, s.c, s.c_valid, s.i);
  if (stop != GRT_STOP_NONE || s.i == S.max_steps - 1) {
    if (writer) store_ray<G>(ws, s.idx, s.y, rc, stop, GRT_OK, s.nrec, (uint32_t)s.i);
    return true;
  }
  s.retries = 0;
  s.h_cur = rclamp(s.h, H_MIN, H_MAX);
  return false;
}

// The rays integrate_kernel handed off (Kerr-Schild): the 4 lanes of a quad carry one
// ray, splitting each RHS evaluation (rhs_ks_quad), and repeat the rest of the loop of
// integrate_kernel in lockstep (identical values in all four lanes; lane 0 of the quad
// writes).  A quad claims the next handed-off ray when its ray ends.  With one wave per
// SIMD a long ray no longer shares issue slots with another wave.
template <int G, bool VOL>
__global__ void __launch_bounds__(256, GRT_TAIL_WAVES) tail_kernel(const DevScene* __restrict__ Sp, Workspace ws,
                                                                   TailList tl,
                                                                   unsigned long long* __restrict__ stats) {
  const DevScene& S = *Sp;
  glibc::tables_to_lds();  // whole block, before any lookup
  const int lane = threadIdx.x & 63;
  const int sub = lane & 3;
  const bool writer = sub == 0;
  const uint64_t below_quad = (lane < 4) ? 0ull : (~0ull >> (64 - (lane & ~3)));
  const uint64_t n = ws.n;
  const unsigned long long handed = load_agent(&tl.ctl[1]);
  const uint64_t n_tail = handed < tl.cap ? handed : tl.cap;  // final: integrate_kernel has ended

  bool active = false, done = false;
  LoopState s;
  RayConst rc;
  uint64_t n_acc = 0, n_att = 0;
#if GRT_RAY_TIMES
  uint64_t att0 = 0;
#endif

  while (true) {
    const bool need = !active && !done;  // uniform within a quad
    const uint64_t leaders = __ballot(need && writer);
    if (leaders) {
      unsigned long long b = 0;
      if (lane == 0) b = atomicAdd(&tl.ctl[2], (unsigned long long)__popcll(leaders));
      b = __shfl(b, 0);
      if (need) {
        const uint64_t e = b + __popcll(leaders & below_quad);
        if (e >= n_tail) {
          done = true;
        } else {
          tail_load(tl.st, tl.cap, e, s);
          rc.obs = 0.0;  // Kerr-Schild: the RHS, the momentum and fin_put read no ray constant
          rc.e = 0.0;
          rc.lz = 0.0;
          rc.q = 0.0;
          rc.pt = VOL ? ws.rc[4 * n + s.idx] : 0.0;
          rc.pphi = VOL ? ws.rc[5 * n + s.idx] : 0.0;
          active = true;
#if GRT_RAY_TIMES
          att0 = n_att;
#endif
        }
      }
    }
    if (__ballot(!done) == 0) break;
    if (!active) continue;
    if (quad_attempt<G, VOL>(S, ws, rc, s, sub, writer, n_acc, n_att)) {
      active = false;
#if GRT_RAY_TIMES
      if (writer) RAY_TIME(n, s.idx, 5, n_att - att0);
#endif
    }
  }

  if (lane == 0) atomicMax(&tl.ctl[6], (unsigned long long)__builtin_amdgcn_s_memrealtime());
  if (!writer) n_acc = n_att = 0;
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) {
    n_acc += __shfl_down(n_acc, off);
    n_att += __shfl_down(n_att, off);
  }
  if (lane == 0) {
    atomicAdd(stats + 0, (unsigned long long)n_acc);
    atomicAdd(stats + 1, (unsigned long long)n_att);
  }
}

#if GRT_MAIN_TU  // trajectories, monitors, probes and test hooks: exact build only
// ======================================================= trajectory kernel =======
// Integrator::integrate with the whole Vec<Step> kept (integrator.rs:78-174), the path
// of `render-ray` / `render-ray-at` (main.rs:117-171, ray.rs:35-54).  One lane per ray;
// step 0 is the initial state.  Each record is (t, x^0..x^3, p^0..p^3): the affine
// parameter, the native-chart position and momentum_from_state.  Steps beyond the
// caller's capacity are counted but not stored.
template <int G>
__global__ void __launch_bounds__(64) trajectory_kernel(const DevScene* __restrict__ Sp, TrajectoryList tl) {
  const DevScene& S = *Sp;
  glibc::tables_to_lds();  // whole block, before the early return
  const uint64_t r = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (r >= tl.n) return;
  double y[8];
  RayConst rc;
  if (tl.row) {
    init_ray<G>(S, tl.row[r], tl.col[r], y, rc);
  } else {
    double st = 0.0, ct = 0.0;
    if constexpr (G == GRT_GEOM_KERR_BL) rsincos(tl.pos[4 * r + 2], &st, &ct);
    init_state<G>(S, tl.pos + 4 * r, st, ct, tl.mom + 4 * r, y, rc);
  }
  uint64_t count = 0;
  auto record = [&](double t) {
    if (count < tl.cap) {
      double* o = tl.steps + (r * tl.cap + count) * 9;
      o[0] = t;
#pragma unroll
      for (int k = 0; k < 4; ++k) o[1 + k] = y[k];
      momentum<G>(S, rc, y, o + 5);
    }
    count++;
  };
  record(0.0);
  int stop = GRT_STOP_NONE, status = GRT_OK;
  double t = 0.0, h = S.step_size;
  for (uint64_t i = 1; i < S.max_steps; ++i) {
    double h_cur = rclamp(h, H_MIN, H_MAX), h_next = 0.0, yn[8];
    int retries = 0, ctl;
    do {
      const double err_sq = rkf_attempt<G>(S, rc, y, h_cur, yn);
      ctl = step_control(S, err_sq, h_cur, retries, h_next);
    } while (ctl == STEP_RETRY);
    if (ctl == STEP_FAILED) {
      status = GRT_ERR_MAX_STEPS_REACHED;
      break;
    }
    t += h_cur;
    h = h_next;
#pragma unroll
    for (int k = 0; k < 8; ++k) y[k] = yn[k];
    record(t);
    double c[3];
    bool c_valid = false;
    stop = should_stop<G>(S, y, c, c_valid, i);
    if (stop != GRT_STOP_NONE) break;
  }
  tl.n_steps[r] = count;
  tl.stop[r] = (uint8_t)stop;
  tl.status[r] = (uint8_t)status;
}

hipError_t launch_arith_map(uint32_t samples, uint64_t seed, uint8_t* d_map, uint8_t* d_zmap, uint8_t* d_smap,
                            hipStream_t stream) {
  hipLaunchKernelGGL(arith_map_kernel, dim3((2047u * 2047u + 255u) / 256u), dim3(256), 0, stream, samples, seed, d_map,
                     d_zmap, d_smap);
  return hipGetLastError();
}

// Device check of the range-free RHS forms (tests/test_gpu_parity.py
// ::test_rhs_fast_forms_match_ieee): for state i (y[8]; KerrBL: e, l_z, q in consts[3 i ..])
// out[16 i ..] = the range-free form (rhs MODE 1), out[16 i + 8 ..] = the IEEE form (MODE 2),
// pred[i] = whether the render's predicate admits the range-free form there.
template <int G>
__global__ void __launch_bounds__(64) rhs_check_kernel(const DevScene* __restrict__ Sp, const double* __restrict__ states,
                                                      const double* __restrict__ consts, uint64_t n, double* out,
                                                      uint8_t* pred) {
  const DevScene& S = *Sp;
  glibc::tables_to_lds();  // whole block, before the early return
  const uint64_t i = (uint64_t)blockIdx.x * 64 + threadIdx.x;
  if (i >= n) return;
  double y[8], of[8], oi[8];
#pragma unroll
  for (int k = 0; k < 8; ++k) y[k] = states[8 * i + k];
  RayConst rc{};
  if constexpr (G == GRT_GEOM_KERR_BL) {
    rc.e = consts[3 * i];
    rc.lz = consts[3 * i + 1];
    rc.q = consts[3 * i + 2];
  }
  rhs<G, 1>(S, rc, y, of);
  rhs<G, 2>(S, rc, y, oi);
#pragma unroll
  for (int k = 0; k < 8; ++k) {
    out[16 * i + k] = of[k];
    out[16 * i + 8 + k] = oi[k];
  }
  bool p = false;
  const bool region_b = glibc::sincos_b_table_ok(y[2]) || glibc::sincos_b_taylor_ok(y[2]);
  if constexpr (G == GRT_GEOM_SCHWARZSCHILD) p = S.div_share && region_b && schw_div_ok(S, y[1]);
  if constexpr (G == GRT_GEOM_KERR_BL) p = region_b && bl_div_ok(S, y[1], bl_delta(y[1], S.radius, S.a), rc.lz);
  if constexpr (G == GRT_GEOM_KERR) p = S.div_fast && ks_fd_ok(S.a, y[1], y[2], y[3], S.ks_cap);
  pred[i] = p ? 1 : 0;
}

hipError_t launch_rhs_check(int geometry, const DevScene* d_scene, const double* d_states, const double* d_consts,
                            uint64_t n, double* d_out, uint8_t* d_pred, hipStream_t stream) {
  const unsigned blocks = (unsigned)((n + 63) / 64);
  switch (geometry) {
    case GRT_GEOM_SCHWARZSCHILD:
      hipLaunchKernelGGL(rhs_check_kernel<GRT_GEOM_SCHWARZSCHILD>, dim3(blocks), dim3(64), 0, stream, d_scene, d_states,
                         d_consts, n, d_out, d_pred);
      break;
    case GRT_GEOM_KERR:
      hipLaunchKernelGGL(rhs_check_kernel<GRT_GEOM_KERR>, dim3(blocks), dim3(64), 0, stream, d_scene, d_states, d_consts,
                         n, d_out, d_pred);
      break;
    case GRT_GEOM_KERR_BL:
      hipLaunchKernelGGL(rhs_check_kernel<GRT_GEOM_KERR_BL>, dim3(blocks), dim3(64), 0, stream, d_scene, d_states,
                         d_consts, n, d_out, d_pred);
      break;
    default:
      return hipErrorInvalidValue;
  }
  return hipGetLastError();
}

#if GRT_PATH_COUNT
// this unit's counters plus the KerrBL unit's
hipError_t path_read(unsigned long long* out, bool reset) {
  hipError_t e = hipMemcpyFromSymbol(out, HIP_SYMBOL(g_path), sizeof(g_path));
  if (e == hipSuccess && reset) {
    const unsigned long long z[2 * NPATH] = {};
    e = hipMemcpyToSymbol(HIP_SYMBOL(g_path), z, sizeof(z));
  }
  unsigned long long bl[2 * NPATH];
  if (e == hipSuccess) e = kerr_bl::path_read(bl, reset);
  for (int k = 0; e == hipSuccess && k < 2 * NPATH; ++k) out[k] += bl[k];
  return e;
}
#endif

hipError_t launch_trajectories(int geometry, const DevScene* d_scene, const TrajectoryList& tl, hipStream_t stream) {
  if (tl.n == 0) return hipSuccess;
  const unsigned blocks = (unsigned)((tl.n + 63) / 64);
  switch (geometry) {
    case GRT_GEOM_EUCLIDEAN:
      hipLaunchKernelGGL(trajectory_kernel<GRT_GEOM_EUCLIDEAN>, dim3(blocks), dim3(64), 0, stream, d_scene, tl);
      break;
    case GRT_GEOM_SCHWARZSCHILD:
      hipLaunchKernelGGL(trajectory_kernel<GRT_GEOM_SCHWARZSCHILD>, dim3(blocks), dim3(64), 0, stream, d_scene, tl);
      break;
    case GRT_GEOM_KERR:
      hipLaunchKernelGGL(trajectory_kernel<GRT_GEOM_KERR>, dim3(blocks), dim3(64), 0, stream, d_scene, tl);
      break;
    case GRT_GEOM_KERR_BL:
      hipLaunchKernelGGL(trajectory_kernel<GRT_GEOM_KERR_BL>, dim3(blocks), dim3(64), 0, stream, d_scene, tl);
      break;
    case GRT_GEOM_EUCLIDEAN_SPHERICAL:
      hipLaunchKernelGGL(trajectory_kernel<GRT_GEOM_EUCLIDEAN_SPHERICAL>, dim3(blocks), dim3(64), 0, stream, d_scene,
                         tl);
      break;
    default:
      return hipErrorInvalidValue;
  }
  return hipGetLastError();
}

// ====================================================== invariant monitors =======
// The reference's per-ray health checks, off the render path:
//  * the null condition of the camera ray, |k.k| < 1e-10 (scene.rs:116-124, logged as an
//    error otherwise);
//  * in debug builds, the largest |k.k| over the accepted steps and the largest drift of
//    each constant of motion from its value at step 0, relative when |initial| > 1e-12
//    (integrator.rs:91-146), warned above 1e-4 (report_drifts, :176-201).  A ray whose
//    rkf45 fails returns Err before report_drifts: it reports no drift.
// health_kernel re-integrates the rays (one lane per ray) with these monitors.

// get_constants_of_motion at (x, p): E, L_z and, for KerrBL, Carter's Q.  Returns the count.
template <int G>
GDEV int constants_of_motion(const DevScene& S, const double* x, const double* p, double* c) {
  if constexpr (G == GRT_GEOM_EUCLIDEAN) {  // euclidean.rs:160-182
    const double p_x = -p[1], p_y = -p[2];
    c[0] = p[0];
    c[1] = x[1] * p_y - x[2] * p_x;
    return 2;
  } else if constexpr (G == GRT_GEOM_EUCLIDEAN_SPHERICAL) {  // euclidean_spherical.rs:147-166
    const double r = x[1], st = rsin(x[2]);
    c[0] = p[0];
    c[1] = -r * r * st * st * p[3];
    return 2;
  } else if constexpr (G == GRT_GEOM_SCHWARZSCHILD) {  // schwarzschild.rs:213-233
    const double r = x[1], st = rsin(x[2]);
    const double a = 1.0 - S.radius / r;
    c[0] = a * p[0];
    c[1] = -r * r * st * st * p[3];
    return 2;
  } else if constexpr (G == GRT_GEOM_KERR) {  // kerr.rs:421-445
    double g[4][4], pc[4];
    ks_metric(S.radius, S.a, x[1], x[2], x[3], g);
    mat_vec(g, p, pc);
    c[0] = -pc[0];
    c[1] = -x[2] * pc[1] + x[1] * pc[2];
    return 2;
  } else {  // KerrBL, kerr_bl.rs:596-625 (metric_bl's and this sin / cos of one theta: one sincos)
    double st, ct;
    rsincos(x[2], &st, &ct);
    double g[4][4], pc[4];
    metric_bl(S.radius, S.a, x[1], st, ct, g);
    mat_vec(g, p, pc);
    const double e = -pc[0], l_z = pc[3], p_theta = pc[2];
    const double sin2 = st * st;
    c[0] = e;
    c[1] = l_z;
    c[2] = p_theta * p_theta + ct * ct * (l_z * l_z / fmax(sin2, 1e-28) - S.a * S.a * e * e);
    return 3;
  }
}
// inner_product(x, v, v) at a native-chart point
template <int G>
GDEV double inner_at(const DevScene& S, const double* x, const double* v) {
  double st = 0.0, ct = 0.0;
  if constexpr (G == GRT_GEOM_SCHWARZSCHILD || G == GRT_GEOM_EUCLIDEAN_SPHERICAL) st = rsin(x[2]);
  else if constexpr (G == GRT_GEOM_KERR_BL) rsincos(x[2], &st, &ct);
  return inner<G>(S, x, st, ct, v, v);
}
GDEV double drift_of(double cur, double init) {  // integrator.rs:127-134
  return fabs(init) > 1e-12 ? fabs(cur - init) / fabs(init) : fabs(cur - init);
}

// Per ray k (pixel (row0 + k / cols, col0 + k % cols)): out[k * 5 + 0] |k.k| of the camera
// ray, [1] the largest |k.k| over the accepted steps, [2..4] the largest drift of E, L_z, Q;
// status[k] = GRT_ERR_MAX_STEPS_REACHED when rkf45 failed (no drift report).
template <int G>
__global__ void __launch_bounds__(64) health_kernel(const DevScene* __restrict__ Sp, WorkList wl, uint64_t n,
                                                    double* __restrict__ out, uint8_t* __restrict__ status) {
  const DevScene& S = *Sp;
  glibc::tables_to_lds();  // whole block, before the early return
  const uint64_t k = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (k >= n) return;
  const double row = (double)(wl.row0 + (uint32_t)(k / wl.cols)), col = (double)(wl.col0 + (uint32_t)(k % wl.cols));
  double pcam[4];
  camera_momentum(S.cam, row, col, pcam);
  const double null_kk = fabs(inner<G>(S, S.cam.pos, S.cam.sin_theta, S.cam.cos_theta, pcam, pcam));
  double y[8];
  RayConst rc;
  init_ray<G>(S, row, col, y, rc);
  double p[4], c0[3] = {0.0, 0.0, 0.0}, c1[3];
  momentum<G>(S, rc, y, p);
  const int nc = constants_of_motion<G>(S, y, p, c0);
  double max_kk = 0.0, max_d[3] = {0.0, 0.0, 0.0};
  int st_out = GRT_OK;
  double h = S.step_size;
  for (uint64_t i = 1; i < S.max_steps; ++i) {
    double h_cur = rclamp(h, H_MIN, H_MAX), h_next = 0.0, yn[8];
    int retries = 0, ctl;
    do {
      const double err_sq = rkf_attempt<G>(S, rc, y, h_cur, yn);
      ctl = step_control(S, err_sq, h_cur, retries, h_next);
    } while (ctl == STEP_RETRY);
    if (ctl == STEP_FAILED) {
      st_out = GRT_ERR_MAX_STEPS_REACHED;
      break;
    }
    h = h_next;
#pragma unroll
    for (int q = 0; q < 8; ++q) y[q] = yn[q];
    momentum<G>(S, rc, y, p);
    const double kk = fabs(inner_at<G>(S, y, p));
    if (kk > max_kk) max_kk = kk;
    constants_of_motion<G>(S, y, p, c1);
    for (int q = 0; q < nc; ++q) {
      const double d = drift_of(c1[q], c0[q]);
      if (d > max_d[q]) max_d[q] = d;
    }
    double c[3];
    bool c_valid = false;
    if (should_stop<G>(S, y, c, c_valid, i) != GRT_STOP_NONE) break;
  }
  double* o = out + k * 5;
  o[0] = null_kk;
  o[1] = max_kk;
  o[2] = max_d[0];
  o[3] = max_d[1];
  o[4] = max_d[2];
  status[k] = (uint8_t)st_out;
}

hipError_t launch_health(int geometry, const DevScene* d_scene, const WorkList& wl, uint64_t n, double* d_out,
                         uint8_t* d_status, hipStream_t stream) {
  if (n == 0) return hipSuccess;
  const unsigned blocks = (unsigned)((n + 63) / 64);
  switch (geometry) {
    case GRT_GEOM_EUCLIDEAN:
      hipLaunchKernelGGL(health_kernel<GRT_GEOM_EUCLIDEAN>, dim3(blocks), dim3(64), 0, stream, d_scene, wl, n, d_out,
                         d_status);
      break;
    case GRT_GEOM_SCHWARZSCHILD:
      hipLaunchKernelGGL(health_kernel<GRT_GEOM_SCHWARZSCHILD>, dim3(blocks), dim3(64), 0, stream, d_scene, wl, n,
                         d_out, d_status);
      break;
    case GRT_GEOM_KERR:
      hipLaunchKernelGGL(health_kernel<GRT_GEOM_KERR>, dim3(blocks), dim3(64), 0, stream, d_scene, wl, n, d_out,
                         d_status);
      break;
    case GRT_GEOM_KERR_BL:
      hipLaunchKernelGGL(health_kernel<GRT_GEOM_KERR_BL>, dim3(blocks), dim3(64), 0, stream, d_scene, wl, n, d_out,
                         d_status);
      break;
    case GRT_GEOM_EUCLIDEAN_SPHERICAL:
      hipLaunchKernelGGL(health_kernel<GRT_GEOM_EUCLIDEAN_SPHERICAL>, dim3(blocks), dim3(64), 0, stream, d_scene, wl,
                         n, d_out, d_status);
      break;
    default:
      return hipErrorInvalidValue;
  }
  return hipGetLastError();
}

// ============================================================ probe kernel =======
// Work-order probe (scheduling only, never an output): one ray per 8x8 tile, the
// tile's pixel (3, 3), integrated for at most `cap` accepted steps.  A frame's cost is
// heavy-tailed where rays spiral into the horizon or orbit near the photon sphere
// (C4: 6% of the rays carry 60% of the steps, up to max_steps each); with the counts
// the host queues the long tiles first, so the frame does not end on a lone ray that
// started late.  Writes the steps taken, or for a probe still going at the cap a key
// above every finished count: cap + 2^30 (r - r_stop) / r_stop, r its radial coordinate
// there and r_stop the horizon test's radius (cap alone without a horizon).  The capped
// probes of a C4 shard all creep towards the horizon with steps of ~1e-8, and the
// distance they have left predicts the ray's length (log-log correlation 0.98 with the
// probe pixel's own count; the 300 tiles with a ray past 8e5 steps are among the 311
// largest keys but 11; tools/c4_probe_features.py), so the longest tiles are queued first.
#ifndef GRT_PROBE_ESCAPE
#define GRT_PROBE_ESCAPE 1  // end an outward-bound Kerr-Schild probe far from the hole at once
#endif
// A Kerr-Schild probe moving outward beyond min(10 radius, max_radius / 2) escapes (no
// turning point outside the photon orbits); its key becomes cap - 1: below every capped
// probe's key (those rays are longer), above the rays that fell in early, and "finished"
// for the edge-tile rule (schedule.hip).  So the cap (api.hip probe_cap) need not outlast
// the escaping rays, and the pass ends sooner.  Scheduling only, never an output.
template <int G>
GDEV bool probe_escaped(const DevScene& S, const double* y, double& r_prev, uint32_t cap, uint32_t* key) {
  if constexpr (G != GRT_GEOM_KERR || !GRT_PROBE_ESCAPE) {
    return false;
  } else {
    const double r = sqrt(ks_r_sqr(S.a, y[1], y[2], y[3]));
    const bool out = r > fmin(10.0 * S.radius, 0.5 * sqrt(S.max_radius_sq)) && r > r_prev;
    r_prev = r;
    if (out) *key = cap - 1;
    return out;
  }
}

// The probe's radial coordinate at its initial state, so that the first accepted step's
// "moving outward" test compares against where the ray started (a camera far from the
// hole, beyond the escape radius, must not end its inward probes at step 1).
template <int G>
GDEV double probe_r0(const DevScene& S, const double* y) {
  if constexpr (G != GRT_GEOM_KERR || !GRT_PROBE_ESCAPE) {
    return 0.0;
  } else {
    return sqrt(ks_r_sqr(S.a, y[1], y[2], y[3]));
  }
}

template <int G>
__global__ void __launch_bounds__(64) probe_kernel(const DevScene* __restrict__ Sp, WorkList wl, uint32_t n_tiles,
                                                   uint32_t cap, uint32_t* __restrict__ steps_out) {
  const DevScene& S = *Sp;
  glibc::tables_to_lds();
  const uint32_t t = blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= n_tiles) return;
  const uint32_t tr = t / wl.tiles_x, tc = t % wl.tiles_x;
  const uint32_t r = min(tr * 8 + 3, wl.rows - 1), c = min(tc * 8 + 3, wl.cols - 1);
  double y[8];
  RayConst rc;
  init_ray<G>(S, (double)(wl.row0 + shard_frame_row(wl.band_rows, wl.shard, wl.n_shards, r)),
              (double)(wl.col0 + c), y, rc);
  const uint64_t end = S.max_steps < (uint64_t)cap ? S.max_steps : (uint64_t)cap;
  uint64_t i = 1;
  double h = S.step_size;
  double r_prev = probe_r0<G>(S, y);
  uint32_t key = 0;
  bool escaped = false;
  for (; i < end; ++i) {
    double h_cur = rclamp(h, H_MIN, H_MAX), h_next = 0.0, yn[8];
    int retries = 0, ctl;
    do {
      const double err_sq = rkf_attempt<G>(S, rc, y, h_cur, yn);
      ctl = step_control(S, err_sq, h_cur, retries, h_next);
    } while (ctl == STEP_RETRY);
    if (ctl == STEP_FAILED) break;
    h = h_next;
#pragma unroll
    for (int k = 0; k < 8; ++k) y[k] = yn[k];
    double cc[3];
    bool c_valid = false;
    if (should_stop<G>(S, y, cc, c_valid, i) != GRT_STOP_NONE) break;
    if ((escaped = probe_escaped<G>(S, y, r_prev, cap, &key))) break;
  }
  if (!escaped) key = (uint32_t)i;
  if (!escaped && i >= end) {
    key = cap;
    const bool horizon = G == GRT_GEOM_SCHWARZSCHILD || ((G == GRT_GEOM_KERR || G == GRT_GEOM_KERR_BL) && S.has_horizon);
    if (horizon && S.horizon_r > 0.0) {
      const double rad = (G == GRT_GEOM_KERR) ? sqrt(ks_r_sqr(S.a, y[1], y[2], y[3])) : y[1];
      const double d = (rad - S.horizon_r) / S.horizon_r * 1073741824.0;
      if (d > 0.0) key = cap + (uint32_t)fmin(d, (double)(0xffffffffu - cap));  // NaN: stays cap
    }
  }
  steps_out[t] = key;
}

// Work-order key of a Schwarzschild tile without integrating: the predicted steps of its
// probe pixel's ray from the impact parameter b = L / E of its initial momentum (E =
// (1 - r_s / r) dt/dl, L = r^2 sqrt((dtheta/dl)^2 + sin^2 theta (dphi/dl)^2)).  A ray with
// b above the photon orbit's b_c = (3 sqrt 3 / 2) r_s escapes to the celestial sphere
// (~max_radius unit steps), one below it falls in (a few hundred steps), and near b_c
// both wind round the photon sphere for ~ln(1 / |b / b_c - 1|) more turns.  Only the
// queue order depends on it, never a result.
__global__ void __launch_bounds__(64) impact_key_kernel(const DevScene* __restrict__ Sp, WorkList wl,
                                                        uint32_t n_tiles, uint32_t* __restrict__ keys_out) {
  const DevScene& S = *Sp;
  glibc::tables_to_lds();
  const uint32_t t = blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= n_tiles) return;
  const uint32_t tr = t / wl.tiles_x, tc = t % wl.tiles_x;
  const uint32_t r = min(tr * 8 + 3, wl.rows - 1), c = min(tc * 8 + 3, wl.cols - 1);
  double y[8];
  RayConst rc;
  init_ray<GRT_GEOM_SCHWARZSCHILD>(S, (double)(wl.row0 + shard_frame_row(wl.band_rows, wl.shard, wl.n_shards, r)),
                                   (double)(wl.col0 + c), y, rc);
  const double rs = S.radius, rr = y[1], sn = sin(y[2]);
  const double e = fabs((1.0 - rs / rr) * y[4]);
  const double l = rr * rr * sqrt(y[6] * y[6] + sn * sn * y[7] * y[7]);
  const double bc = 2.598076211353316 * rs;
  const double b = l / e;
  const double x = fmax(fabs(b - bc) / bc, 1e-12);
  const double len = (b > bc ? sqrt(S.max_radius_sq) : 300.0) + 700.0 * fmax(0.0, -log(x));
  keys_out[t] = (len > 0.0 && len < 4.0e9) ? (uint32_t)len : (len >= 4.0e9 ? 4000000000u : 0u);  // NaN: 0
}

hipError_t launch_impact_keys(const DevScene* d_scene, const WorkList& wl, uint32_t n_tiles, uint32_t* d_keys,
                              hipStream_t stream) {
  if (n_tiles == 0) return hipSuccess;
  hipLaunchKernelGGL(impact_key_kernel, dim3((n_tiles + 63) / 64), dim3(64), 0, stream, d_scene, wl, n_tiles, d_keys);
  return hipGetLastError();
}

// probe_kernel<KERR> with each probe ray on the 4 lanes of a quad (rhs_ks_quad, as in
// tail_kernel): the same operations on the same values, so the same keys (GPU test
// tests/test_gpu_schedule.py).  For a pass of few probe rays (a 1/8 row-band shard of
// C4: 32,768 tiles, 0.5 waves per SIMD as one lane each) the pass lasts as long as its
// capped probes take to run `cap` steps at one wave's latency; splitting each RHS over a
// quad cuts that latency, at 4x the lanes (2 waves per SIMD here).
__global__ void __launch_bounds__(256, 2) probe_quad_kernel(const DevScene* __restrict__ Sp, WorkList wl,
                                                            uint32_t n_tiles, uint32_t cap,
                                                            uint32_t* __restrict__ steps_out) {
  constexpr int G = GRT_GEOM_KERR;
  const DevScene& S = *Sp;
  glibc::tables_to_lds();
  const uint32_t t = (blockIdx.x * blockDim.x + threadIdx.x) >> 2;  // the quad's tile
  const int sub = threadIdx.x & 3;
  if (t >= n_tiles) return;  // the whole quad
  const uint32_t tr = t / wl.tiles_x, tc = t % wl.tiles_x;
  const uint32_t r = min(tr * 8 + 3, wl.rows - 1), c = min(tc * 8 + 3, wl.cols - 1);
  double y[8];
  RayConst rc;
  init_ray<G>(S, (double)(wl.row0 + shard_frame_row(wl.band_rows, wl.shard, wl.n_shards, r)),
              (double)(wl.col0 + c), y, rc);
  const uint64_t end = S.max_steps < (uint64_t)cap ? S.max_steps : (uint64_t)cap;
  uint64_t i = 1;
  double h = S.step_size;
  double r_prev = probe_r0<G>(S, y);
  uint32_t key = 0;
  bool escaped = false;
  for (; i < end; ++i) {  // identical decisions in the quad's four lanes
    double h_cur = rclamp(h, H_MIN, H_MAX), h_next = 0.0, yn[8];
    int retries = 0, ctl;
    do {
      const double err_sq = rkf_attempt<G, false, true>(S, rc, y, h_cur, yn, sub);
      ctl = step_control(S, err_sq, h_cur, retries, h_next);
    } while (ctl == STEP_RETRY);
    if (ctl == STEP_FAILED) break;
    h = h_next;
#pragma unroll
    for (int k = 0; k < 8; ++k) y[k] = yn[k];
    double cc[3];
    bool c_valid = false;
    if (should_stop<G>(S, y, cc, c_valid, i) != GRT_STOP_NONE) break;
    if ((escaped = probe_escaped<G>(S, y, r_prev, cap, &key))) break;
  }
  if (!escaped) key = (uint32_t)i;
  if (!escaped && i >= end) {
    key = cap;
    if (S.has_horizon && S.horizon_r > 0.0) {
      const double d = (sqrt(ks_r_sqr(S.a, y[1], y[2], y[3])) - S.horizon_r) / S.horizon_r * 1073741824.0;
      if (d > 0.0) key = cap + (uint32_t)fmin(d, (double)(0xffffffffu - cap));  // NaN: stays cap
    }
  }
  if (sub == 0) steps_out[t] = key;
}

hipError_t launch_probe(int geometry, const DevScene* d_scene, const WorkList& wl, uint32_t n_tiles, uint32_t cap,
                        uint32_t* d_steps, bool quad, hipStream_t stream) {
  if (n_tiles == 0) return hipSuccess;
  if (quad && geometry == GRT_GEOM_KERR) {
    hipLaunchKernelGGL(probe_quad_kernel, dim3((n_tiles * 4ull + 255) / 256), dim3(256), 0, stream, d_scene, wl,
                       n_tiles, cap, d_steps);
    return hipGetLastError();
  }
  const unsigned blocks = (n_tiles + 63) / 64;
  switch (geometry) {
    case GRT_GEOM_EUCLIDEAN:
      hipLaunchKernelGGL(probe_kernel<GRT_GEOM_EUCLIDEAN>, dim3(blocks), dim3(64), 0, stream, d_scene, wl, n_tiles,
                         cap, d_steps);
      break;
    case GRT_GEOM_SCHWARZSCHILD:
      hipLaunchKernelGGL(probe_kernel<GRT_GEOM_SCHWARZSCHILD>, dim3(blocks), dim3(64), 0, stream, d_scene, wl,
                         n_tiles, cap, d_steps);
      break;
    case GRT_GEOM_KERR:
      hipLaunchKernelGGL(probe_kernel<GRT_GEOM_KERR>, dim3(blocks), dim3(64), 0, stream, d_scene, wl, n_tiles, cap,
                         d_steps);
      break;
    case GRT_GEOM_KERR_BL:
      hipLaunchKernelGGL(probe_kernel<GRT_GEOM_KERR_BL>, dim3(blocks), dim3(64), 0, stream, d_scene, wl, n_tiles,
                         cap, d_steps);
      break;
    case GRT_GEOM_EUCLIDEAN_SPHERICAL:
      hipLaunchKernelGGL(probe_kernel<GRT_GEOM_EUCLIDEAN_SPHERICAL>, dim3(blocks), dim3(64), 0, stream, d_scene, wl,
                         n_tiles, cap, d_steps);
      break;
    default:
      return hipErrorInvalidValue;
  }
  return hipGetLastError();
}


#endif  // GRT_MAIN_TU
// ============================================================ shade kernel =======
// Evaluate one recorded candidate: the emitter step at the intersection
// (objects.rs:27-44 + :95-115), its redshift, temperature and texture colour.
// A VolumetricDisc candidate gets its energy and temperature (and their errors) here;
// its colour is the raymarch of march_kernel (volumetric_disc.rs:580-601), so *col is
// left untouched.  color = false: errors only (the job-gathering pass).
template <int G>
GDEV int shade_record(const DevScene& S, const RayConst& rc, const DevObject& o, const double* p,
                      const double* pt, XYZA* col, bool color = true) {
  double u_tex = 0.0, v_tex = 0.0, wx, wy, wz;
  if (o.kind == GRT_OBJ_VOLUMETRIC_DISC) {  // world hit point (its uv is not used for colour)
    wx = pt[0];
    wy = pt[1];
    wz = pt[2];
  } else if (o.kind == GRT_OBJ_DISC) {  // disc.rs:60-76 uv from the in-plane point
    wx = pt[0];
    wy = pt[1];
    wz = pt[2];
    double rr = wx * wx + wy * wy + wz * wz;
    double phi = atan2(wy - 0.0, wx - 0.0);
    double r = (sqrt(rr) - o.rin) / (o.rout - o.rin);
    double sp, cp;
    rsincos(phi, &sp, &cp);
    u_tex = 0.5 + 0.5 * r * cp;
    v_tex = 0.5 + 0.5 * r * sp;
  } else {  // sphere.rs:92-117 uv from the sphere-local point, world point for physics
    double rr, theta, phi;
    cart_to_sph(pt[0], pt[1], pt[2], &rr, &theta, &phi);
    double u = (PI + phi) / TWO_PI;
    u_tex = 1.0 - u;
    v_tex = theta / PI;
    wx = pt[0] + o.cx;
    wy = pt[1] + o.cy;
    wz = pt[2] + o.cz;
  }
  double x[4];  // step.x = intersection point converted to the native chart
  double st = 0.0, ct = 0.0;
  x[0] = 0.0;
  if constexpr (G == GRT_GEOM_SCHWARZSCHILD || G == GRT_GEOM_EUCLIDEAN_SPHERICAL) {
    cart_to_sph(wx, wy, wz, &x[1], &x[2], &x[3]);
    st = rsin(x[2]);  // the only trig of the spherical inner products (ct unused)
  } else if constexpr (G == GRT_GEOM_KERR_BL) {
    cart_to_bl(S.a, wx, wy, wz, &x[1], &x[2], &x[3]);
    rsincos(x[2], &st, &ct);
  } else {
    x[1] = wx;
    x[2] = wy;
    x[3] = wz;
  }
  double u[4];
  if (o.kind != GRT_OBJ_SPHERE) {  // disc.rs:101-110, volumetric_disc.rs:603-612: circular-orbit emitter
    if constexpr (G == GRT_GEOM_EUCLIDEAN || G == GRT_GEOM_EUCLIDEAN_SPHERICAL) {  // at rest in flat space
      u[0] = 1.0; u[1] = 0.0; u[2] = 0.0; u[3] = 0.0;
    } else {
      double r;
      if constexpr (G == GRT_GEOM_KERR) r = sqrt(ks_r_sqr(S.a, x[1], x[2], x[3]));
      else r = x[1];
      double ut, uphi;
      if (!killing_coefficients(S, r, &ut, &uphi)) return GRT_ERR_NO_CIRCULAR_ORBIT;
      if constexpr (G == GRT_GEOM_KERR) {
        double ax[4] = {0.0, -x[2], x[1], 0.0};
        double et[4] = {1.0, 0.0, 0.0, 0.0};
#pragma unroll
        for (int q = 0; q < 4; ++q) u[q] = ut * et[q] + uphi * ax[q];
      } else {
        u[0] = ut; u[1] = 0.0; u[2] = 0.0; u[3] = uphi;
      }
    }
  } else {  // sphere.rs:141-150: static emitter
    stationary_velocity<G>(S, x, u);
  }
  double em = inner<G>(S, x, st, ct, u, p);
  double sig0 = signature0<G>();
  double redshift = (sig0 * rc.obs) / (sig0 * em);  // redshift.rs:36-38
  double temperature;
  if (o.kind != GRT_OBJ_SPHERE) {  // disc.rs:112-120, volumetric_disc.rs:614-622
    double rad;  // get_radial_coordinate of the Cartesian intersection point
    if constexpr (G == GRT_GEOM_KERR || G == GRT_GEOM_KERR_BL) {
      rad = sqrt(ks_r_sqr(S.a, wx, wy, wz));
    } else {
      rad = sqrt(wx * wx + wy * wy + wz * wz);
    }
    int e = compute_temperature(o, rad, &temperature);
    if (e != GRT_OK) return e;
  } else {
    temperature = o.temperature;
  }
  if (color && o.kind != GRT_OBJ_VOLUMETRIC_DISC) *col = texture_color(S, o.tex, u_tex, v_tex, redshift, temperature);
  return GRT_OK;
}

// (the step count goes to out.steps from store_ray, KerrBL's from shade_kernel)
GDEV void write_out(const Outputs& out, uint64_t idx, const XYZA& c, int cls, int status, int stop, uint32_t hits) {
  if (out.hits) out.hits[idx] = hits;
  reinterpret_cast<float4*>(out.xyza)[idx] = make_float4((float)c.x, (float)c.y, (float)c.z, (float)c.a);
  out.cls[idx] = (uint8_t)cls;
  out.status[idx] = (uint8_t)status;
  if (out.xyza64) {
    double* d = out.xyza64 + 4 * idx;
    d[0] = c.x;
    d[1] = c.y;
    d[2] = c.z;
    d[3] = c.a;
  }
  if (out.stop) out.stop[idx] = (uint8_t)stop;
}

// ---- a ray's candidates in window order: workspace slots 0..GRT_WS_SLOTS-1, then the
// hit pool's list (HitPool).
struct RecRef {
  bool pool;
  uint64_t s;  // workspace slot j * n + idx, or pool record
};
// Candidates a ray can replay in order: all of them, unless its pool list was lost
// (the pool was full), in which case only the workspace slots (*lost = true).
GDEV uint32_t rec_count(const Workspace& ws, uint64_t idx, uint32_t nrec, bool* lost) {
  *lost = nrec > GRT_WS_SLOTS && ws.pool->last[idx] == HIT_NIL;
  return *lost ? GRT_WS_SLOTS : nrec;
}
// Candidate j, for j = 0, 1, 2, ... in turn (*pos carries the position in the pool list).
GDEV RecRef rec_at(const Workspace& ws, uint64_t idx, uint32_t j, uint32_t* pos) {
  if (j < GRT_WS_SLOTS) return RecRef{false, (uint64_t)j * ws.n + idx};
  *pos = (j == GRT_WS_SLOTS) ? ws.pool->head[idx] : ws.pool->next[*pos];
  return RecRef{true, *pos};
}
GDEV uint32_t rec_win(const Workspace& ws, const RecRef& r) { return r.pool ? ws.pool->win[r.s] : ws.rec[r.s].win; }
// The window of candidate j + 1 (which exists), given candidate j.
GDEV uint32_t rec_next_win(const Workspace& ws, uint64_t idx, uint32_t j, const RecRef& r) {
  if (j + 1 < GRT_WS_SLOTS) return ws.rec[r.s + ws.n].win;
  if (j + 1 == GRT_WS_SLOTS) return ws.pool->win[ws.pool->head[idx]];
  return ws.pool->win[ws.pool->next[r.s]];
}
GDEV uint32_t rec_read(const Workspace& ws, const RecRef& r, double* p, double* pt) {
  if (!r.pool) {
    const double2* d = reinterpret_cast<const double2*>(ws.rec + r.s);
    const double2 a = d[0], b = d[1], c = d[2], e = d[3];
    p[0] = a.x;
    p[1] = a.y;
    p[2] = b.x;
    p[3] = b.y;
    pt[0] = c.x;
    pt[1] = c.y;
    pt[2] = e.x;
    return (uint32_t)__double2hiint(e.y);
  }
  const uint64_t m = ws.pool->cap;
#pragma unroll
  for (int q = 0; q < 4; ++q) p[q] = ws.pool->p[q * m + r.s];
#pragma unroll
  for (int q = 0; q < 3; ++q) pt[q] = ws.pool->pt[q * m + r.s];
  return ws.pool->obj[r.s];
}

// Volumetric scenes, pass 1: the candidate slots whose raymarched colour the composite
// needs -- the window-nearest VolumetricDisc hits of a ray whose window pass raises no
// error (an error aborts the pixel, scene.rs:146, so its marches would be wasted).
// Workspace slots come back as a mask; pool records get their jobs appended here.
template <int G>
GDEV uint32_t march_slots(const DevScene& S, const WorkList& wl, const Workspace& ws, uint64_t idx) {
  RayConst rc;
  double y[8];
  const RayMeta mt = fin_get<G>(ws, idx, y, rc);
  if (mt.status != GRT_OK) return 0u;
  if constexpr (G != GRT_GEOM_KERR_BL) rc.obs = observer_energy<G>(S, wl, idx);
  bool lost;
  const uint32_t nr = rec_count(ws, idx, mt.nrec, &lost);
  uint32_t mask = 0u, pool_jobs = 0u, pos = HIT_NIL;
  for (uint32_t j = 0; j < nr; ++j) {
    const RecRef r = rec_at(ws, idx, j, &pos);
    const uint32_t win = rec_win(ws, r);
    double p[4], pt[3];
    const DevObject& o = S.obj[rec_read(ws, r, p, pt)];
    XYZA col;
    if (shade_record<G>(S, rc, o, p, pt, &col, false) != GRT_OK) return 0u;
    bool last_in_window = (j + 1 == nr) || (rec_next_win(ws, idx, j, r) != win);
    if (last_in_window && o.kind == GRT_OBJ_VOLUMETRIC_DISC) {
      if (!r.pool) mask |= 1u << j;
      else pool_jobs++;
    }
  }
  if (pool_jobs) {  // the rare rays with more than GRT_WS_SLOTS candidates: no error, append
    unsigned long long at = atomicAdd(ws.march, (unsigned long long)pool_jobs);
    pos = HIT_NIL;
    for (uint32_t j = GRT_WS_SLOTS; j < nr; ++j) {
      const RecRef r = rec_at(ws, idx, j, &pos);
      bool last_in_window = (j + 1 == nr) || (rec_next_win(ws, idx, j, r) != rec_win(ws, r));
      if (last_in_window && S.obj[ws.pool->obj[r.s]].kind == GRT_OBJ_VOLUMETRIC_DISC)
        ws.jobs[at++] = JOB_POOL | (idx << 31) | r.s;
    }
  }
  return mask;
}

// Scene::color_of_ray's window pass, terminal colour and composite (scene.rs:141-219),
// one lane per ray, over the candidates the integrate kernel recorded.
//   MODE 0: scenes without volumetric objects.
//   MODE 1: volumetric scenes, pass 1 -- append the raymarch jobs (wave-aggregated).
//   MODE 2: volumetric scenes, pass 3 -- composite with the raymarched colours (ws.vcol).
template <int G, int MODE>
__global__ void __launch_bounds__(256) shade_kernel(const DevScene* __restrict__ Sp, WorkList wl, Workspace ws,
                                                    Outputs out, unsigned long long* __restrict__ stats) {
  const DevScene& S = *Sp;
  const uint64_t n = ws.n;
  const uint64_t n_live = ws.n_live ? (uint64_t)min((unsigned long long)n, *ws.n_live) : n;
  // a block past the live rays (the empty chunks of a supersample pass) has nothing to do;
  // block 0 stays for the pool high-water mark below
  if (blockIdx.x != 0 && (uint64_t)blockIdx.x * blockDim.x >= n_live) return;
  glibc::tables_to_lds();  // whole block, before the early return
  const uint64_t idx = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if constexpr (MODE == 1) {
    const uint32_t mask = idx < n_live ? march_slots<G>(S, wl, ws, idx) : 0u;
    const int lane = threadIdx.x & 63;
    const uint32_t c = __popc(mask);
    uint32_t incl = c;  // inclusive wave prefix sum of the job counts
#pragma unroll
    for (int off = 1; off < 64; off <<= 1) {
      const uint32_t v = __shfl_up(incl, off);
      if (lane >= off) incl += v;
    }
    const uint32_t total = __shfl(incl, 63);
    unsigned long long base = 0;
    if (lane == 63 && total) base = atomicAdd(ws.march, (unsigned long long)total);
    base = __shfl(base, 63);
    uint64_t pos = base + incl - c;
    for (uint32_t m = mask; m; m &= m - 1u) ws.jobs[pos++] = (idx << 8) | (uint64_t)__ffs(m) - 1u;
    return;
  }
  if (blockIdx.x == 0 && threadIdx.x == 0) atomicMax(ws.pool->count + 1, *ws.pool->count);
  if (idx >= n_live) return;
  RayConst rc;
  double y[8];
  const RayMeta mt = fin_get<G>(ws, idx, y, rc);
  int status = mt.status;
  const int stop = mt.stop;
  if constexpr (G == GRT_GEOM_KERR_BL) {
    if (out.steps) out.steps[idx] = mt.steps;  // the other charts: written by store_ray
  }
  const XYZA fail{0.0, 0.0, 0.0, 1.0};
  if (status != GRT_OK) {  // integrate error: reference default pixel (raytracer.rs:204-210)
    write_out(out, idx, fail, GRT_CLASS_ESCAPED, status, stop, 0u);
    return;
  }
  if constexpr (G != GRT_GEOM_KERR_BL) rc.obs = observer_energy<G>(S, wl, idx);
  bool lost;
  const uint32_t nr = rec_count(ws, idx, mt.nrec, &lost);
  // window-nearest hits: the first ones in registers, the later ones (pool records of
  // rays with more than GRT_WS_SLOTS candidates) next to their record, linked backwards
  XYZA hits[GRT_WS_SLOTS];
  uint32_t nh = 0, n_pool_hits = 0, pos = HIT_NIL, last_pool_hit = HIT_NIL;
  double opacity = 0.0;
  for (uint32_t j = 0; j < nr; ++j) {
    const RecRef r = rec_at(ws, idx, j, &pos);
    const uint32_t win = rec_win(ws, r);
    double p[4], pt[3];
    const DevObject& o = S.obj[rec_read(ws, r, p, pt)];
    XYZA col{0.0, 0.0, 0.0, 0.0};
    int e = shade_record<G>(S, rc, o, p, pt, &col);
    if (e != GRT_OK) {  // any window error aborts the pixel (scene.rs:146, objects.rs:96-102)
      write_out(out, idx, fail, GRT_CLASS_ESCAPED, e | (lost ? GRT_FLAG_HIT_OVERFLOW : 0), stop, nh + n_pool_hits);
      if (lost) atomicAdd(stats + 3, 1ull);
      return;
    }
    bool last_in_window = (j + 1 == nr) || (rec_next_win(ws, idx, j, r) != win);
    if constexpr (MODE == 2) {
      if (last_in_window && o.kind == GRT_OBJ_VOLUMETRIC_DISC) {
        const double* vc = r.pool ? ws.pool->vcol : ws.vcol;
        const uint64_t m = r.pool ? ws.pool->cap : (uint64_t)GRT_WS_SLOTS * n;
        col = XYZA{vc[r.s], vc[m + r.s], vc[2 * m + r.s], vc[3 * m + r.s]};
      }
    }
    if (last_in_window) {  // the window's nearest hit
      if (!r.pool) {
        hits[nh++] = col;
      } else {
        const uint64_t m = ws.pool->cap;
        ws.pool->hcol[r.s] = col.x;
        ws.pool->hcol[m + r.s] = col.y;
        ws.pool->hcol[2 * m + r.s] = col.z;
        ws.pool->hcol[3 * m + r.s] = col.a;
        ws.pool->hprev[r.s] = last_pool_hit;
        last_pool_hit = (uint32_t)r.s;
        n_pool_hits++;
      }
      double alpha = rclamp(col.a, 0.0, 1.0);
      opacity = alpha + opacity * (1.0 - alpha);
    }
  }
  // terminal colour (scene.rs:157-205) and back-to-front blend (:206-210)
  XYZA result{0.0, 0.0, 0.0, 1.0};
  int cls = GRT_CLASS_CAPTURED;
  if (stop == GRT_STOP_HORIZON || stop == GRT_STOP_CLOSED_ORBIT) {
    result = blend(result, XYZA{0.0, 0.0, 0.0, 1.0});
  } else if (stop == GRT_STOP_CELESTIAL) {
    double th, ph;  // get_as_spherical (point.rs:172-188)
    double st = 0.0, ct = 0.0;
    if constexpr (G == GRT_GEOM_SCHWARZSCHILD || G == GRT_GEOM_KERR_BL || G == GRT_GEOM_EUCLIDEAN_SPHERICAL) {
      th = rem_euclid(y[2], PI);
      ph = rem_euclid(y[3] + PI, TWO_PI) - PI;
      if constexpr (G != GRT_GEOM_KERR_BL) st = rsin(y[2]);  // inner_product: sin only
      else rsincos(y[2], &st, &ct);
    } else {
      double rr;
      cart_to_sph(y[1], y[2], y[3], &rr, &th, &ph);
    }
    double u = (PI + ph) / TWO_PI;
    double v = th / PI;
    double vel[4], p[4];
    stationary_velocity<G>(S, y, vel);
    momentum<G>(S, rc, y, p);
    double em = inner<G>(S, y, st, ct, vel, p);
    double sig0 = signature0<G>();
    double redshift = (sig0 * rc.obs) / (sig0 * em);
    result = blend(result, texture_color(S, S.celestial, 1.0 - u, v, redshift, S.celestial_temperature));
    cls = GRT_CLASS_ESCAPED;
  }
  // back to front: the pool's hits (the farthest windows), then the first ones
  for (uint32_t q = last_pool_hit; q != HIT_NIL; q = ws.pool->hprev[q]) {
    const uint64_t m = ws.pool->cap;
    result = blend(result, XYZA{ws.pool->hcol[q], ws.pool->hcol[m + q], ws.pool->hcol[2 * m + q], ws.pool->hcol[3 * m + q]});
  }
  for (int k = (int)nh - 1; k >= 0; --k) result = blend(result, hits[k]);
  if (opacity >= S.hit_threshold) cls = GRT_CLASS_HIT;
  if (lost) {  // the pool was full: candidates past the workspace slots are missing
    status |= GRT_FLAG_HIT_OVERFLOW;
    atomicAdd(stats + 3, 1ull);
  }
  write_out(out, idx, result, cls, status, stop, nh + n_pool_hits);
}

// ------------------------------------------------------------------ launch -------
// Plain scenes: integrate [-> tail] -> shade.  Volumetric scenes: integrate [-> tail] ->
// gather raymarch jobs -> march (persistent, lane refill) -> composite; ws.march must be
// zeroed.  The tail (Kerr-Schild) continues the long rays the integrate kernel handed off.
template <int G>
static hipError_t launch_g(const DevScene* d_scene, const WorkList& wl, const Workspace& ws_in, const Outputs& out,
                           unsigned long long* d_counter, unsigned long long* d_stats, int blocks, int threads,
                           bool vol, const TailList& tl_in, int tail_blocks, hipStream_t stream) {
  const unsigned nb = (unsigned)((ws_in.n + 255) / 256);
  Workspace ws = ws_in;
  ws.steps = G == GRT_GEOM_KERR_BL ? nullptr : out.steps;  // store_ray writes the per-pixel step counts
  TailList tl = tl_in;
  if (G != GRT_GEOM_KERR || tail_blocks <= 0) tl.cap = 0;
  if (!vol) {
    hipLaunchKernelGGL((integrate_kernel<G, false>), dim3(blocks), dim3(threads), 0, stream, d_scene, wl, ws,
                       d_counter, d_stats, tl);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return e;
    if constexpr (G == GRT_GEOM_KERR) {
      if (tl.cap) {
        hipLaunchKernelGGL((tail_kernel<G, false>), dim3(tail_blocks), dim3(256), 0, stream, d_scene, ws, tl,
                           d_stats);
        if ((e = hipGetLastError()) != hipSuccess) return e;
      }
    }
    hipLaunchKernelGGL((shade_kernel<G, 0>), dim3(nb), dim3(256), 0, stream, d_scene, wl, ws, out, d_stats);
    return hipGetLastError();
  }
  if (!ws.rec_dir || !ws.vcol || !ws.jobs || !ws.march) return hipErrorInvalidValue;
  hipLaunchKernelGGL((integrate_kernel<G, true>), dim3(blocks), dim3(threads), 0, stream, d_scene, wl, ws,
                     d_counter, d_stats, tl);
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) return e;
  if constexpr (G == GRT_GEOM_KERR) {
    if (tl.cap) {
      hipLaunchKernelGGL((tail_kernel<G, true>), dim3(tail_blocks), dim3(256), 0, stream, d_scene, ws, tl, d_stats);
      if ((e = hipGetLastError()) != hipSuccess) return e;
    }
  }
  hipLaunchKernelGGL((shade_kernel<G, 1>), dim3(nb), dim3(256), 0, stream, d_scene, wl, ws, out, d_stats);
  if ((e = hipGetLastError()) != hipSuccess) return e;
  hipLaunchKernelGGL((march_kernel<G>), dim3(blocks), dim3(256), 0, stream, d_scene, ws);
  if ((e = hipGetLastError()) != hipSuccess) return e;
  hipLaunchKernelGGL((shade_kernel<G, 2>), dim3(nb), dim3(256), 0, stream, d_scene, wl, ws, out, d_stats);
  return hipGetLastError();
}

hipError_t launch_trace(int geometry, const DevScene* d_scene, const WorkList& wl, const Workspace& ws,
                        const Outputs& out, unsigned long long* d_counter, unsigned long long* d_stats, int blocks,
                        int threads, bool vol, const TailList& tl, int tail_blocks, hipStream_t stream) {
  if (ws.n == 0) return hipSuccess;
  switch (geometry) {
#if !GRT_KERR_BL_TU
    case GRT_GEOM_EUCLIDEAN:
      return launch_g<GRT_GEOM_EUCLIDEAN>(d_scene, wl, ws, out, d_counter, d_stats, blocks, threads, vol, tl,
                                          tail_blocks, stream);
    case GRT_GEOM_SCHWARZSCHILD:
      return launch_g<GRT_GEOM_SCHWARZSCHILD>(d_scene, wl, ws, out, d_counter, d_stats, blocks, threads, vol, tl,
                                              tail_blocks, stream);
#endif
#if GRT_MAIN_TU  // Kerr-Schild always runs exact (grt_set_arithmetic)
    case GRT_GEOM_KERR:
      return launch_g<GRT_GEOM_KERR>(d_scene, wl, ws, out, d_counter, d_stats, blocks, threads, vol, tl, tail_blocks,
                                     stream);
#endif
#if !GRT_MAIN_TU  // the exact KerrBL trace is grt::kerr_bl's
    case GRT_GEOM_KERR_BL:
      return launch_g<GRT_GEOM_KERR_BL>(d_scene, wl, ws, out, d_counter, d_stats, blocks, threads, vol, tl,
                                        tail_blocks, stream);
#endif
#if !GRT_KERR_BL_TU
    case GRT_GEOM_EUCLIDEAN_SPHERICAL:
      return launch_g<GRT_GEOM_EUCLIDEAN_SPHERICAL>(d_scene, wl, ws, out, d_counter, d_stats, blocks, threads, vol,
                                                    tl, tail_blocks, stream);
#endif
    default:
      return hipErrorInvalidValue;
  }
}

#if GRT_FUSED || GRT_KERR_BL_TU
}  // namespace fused / kerr_bl
#endif
}  // namespace grt
