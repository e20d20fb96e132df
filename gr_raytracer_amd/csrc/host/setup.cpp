// setup.cpp — per-frame host setup, the C++ replacement of the reference's Rust host
// (cli/shared.rs::create_scene and what it calls).  Runs once per frame on the CPU:
//   * Camera::new                       rendering/camera.rs:151-196
//     - get_tetrad_at / lorentz_transformation per geometry
//       (euclidean.rs:86-142, schwarzschild.rs:116-179, kerr.rs:297-380,
//        kerr_bl.rs:428-480), gram_schmidt.rs:6-34, TetradValidator tetrad.rs:60-131,
//       spatial_handedness camera.rs:83-148
//   * observer velocities               SupportQuantities (geometry.rs:49-81)
//   * KerrTemperatureComputer::new      rendering/temperature.rs:45-193
//   * BlackBodyMapper::new              rendering/texture.rs:120-138,
//                                       black_body_radiation.rs:3-45
//   * sRGB <-> XYZ, tone mapping        rendering/color.rs:172-332
// Every quantity here is evaluated with the host libm in the reference's order.
#include <cerrno>
#include <cmath>
#include <cstdint>
#include <cstring>
#include <thread>
#include <vector>

#include "grt_api.h"
#include "host_internal.h"

namespace grt_host {

static const double PI = 3.14159265358979323846;
static const double FRAC_PI_2 = 1.57079632679489661923;

struct V4 {
  double v[4];
  double& operator[](int i) { return v[i]; }
  double operator[](int i) const { return v[i]; }
};
static V4 add(const V4& a, const V4& b) {
  V4 r;
  for (int i = 0; i < 4; ++i) r[i] = a[i] + b[i];
  return r;
}
static V4 scale(double s, const V4& a) {
  V4 r;
  for (int i = 0; i < 4; ++i) r[i] = s * a[i];
  return r;
}
static V4 neg(const V4& a) {
  V4 r;
  for (int i = 0; i < 4; ++i) r[i] = -a[i];
  return r;
}
typedef double M4[4][4];

static void gemv(const M4 A, const V4& x, V4& y) {  // nalgebra gemv order
  for (int i = 0; i < 4; ++i) {
    double s = A[i][0] * x[0];
    for (int k = 1; k < 4; ++k) s = A[i][k] * x[k] + s;
    y[i] = s;
  }
}
static double quad(const V4& v, const M4 M, const V4& w) {
  double row[4];
  for (int j = 0; j < 4; ++j) {
    double s = v[0] * M[0][j];
    for (int k = 1; k < 4; ++k) s = v[k] * M[k][j] + s;
    row[j] = s;
  }
  double s = row[0] * w[0];
  for (int j = 1; j < 4; ++j) s = row[j] * w[j] + s;
  return s;
}
static double rclamp(double v, double lo, double hi) {
  if (v < lo) v = lo;
  if (v > hi) v = hi;
  return v;
}
double rclamp_pub(double v, double lo, double hi) { return rclamp(v, lo, hi); }
static double rem_euclid(double x, double m) {
  double r = std::fmod(x, m);
  return r < 0.0 ? r + std::fabs(m) : r;
}

// ------------------------------------------------------------------ metrics ------
static double ks_r_sqr(double a, double x, double y, double z) {
  double rho_sqr = x * x + y * y + z * z;
  return 0.5 * (rho_sqr - a * a + std::sqrt((rho_sqr - a * a) * (rho_sqr - a * a) + 4.0 * a * a * z * z));
}
static void ks_metric(double radius, double a, double x, double y, double z, M4 g) {  // kerr.rs:49-84
  double r_sqr = ks_r_sqr(a, x, y, z);
  double r = std::sqrt(r_sqr);
  double f = (r * r * r * radius) / (r * r * r * r + a * a * z * z);
  double k0 = 1.0, kx = (r * x + a * y) / (r_sqr + a * a), ky = (r * y - a * x) / (r_sqr + a * a), kz = z / r;
  g[0][0] = k0 * k0 * f - 1.0;
  g[0][1] = k0 * kx * f;
  g[0][2] = k0 * ky * f;
  g[0][3] = k0 * kz * f;
  g[1][0] = g[0][1];
  g[1][1] = kx * kx * f + 1.0;
  g[1][2] = kx * ky * f;
  g[1][3] = kx * kz * f;
  g[2][0] = g[0][2];
  g[2][1] = g[1][2];
  g[2][2] = ky * ky * f + 1.0;
  g[2][3] = ky * kz * f;
  g[3][0] = g[0][3];
  g[3][1] = g[1][3];
  g[3][2] = g[2][3];
  g[3][3] = kz * kz * f + 1.0;
}
static double bl_sigma(double r, double a, double theta) {
  double c = std::cos(theta);
  return r * r + a * a * (c * c);
}
static double bl_delta(double r, double r_s, double a) { return r * r - r_s * r + a * a; }
static void metric_bl(double r_s, double a, double r, double theta, M4 g) {  // kerr_bl.rs:253-272
  double sig = bl_sigma(r, a, theta);
  double st = std::sin(theta);
  double sin2 = st * st;
  std::memset(g, 0, sizeof(M4));
  g[0][0] = -(1.0 - r_s * r / sig);
  g[1][1] = sig / bl_delta(r, r_s, a);
  g[2][2] = sig;
  g[3][3] = (r * r + a * a + a * a * r_s * r * sin2 / sig) * sin2;
  double g_tph = -a * r_s * r * sin2 / sig;
  g[0][3] = g_tph;
  g[3][0] = g_tph;
}

struct Geo {
  int kind;
  double radius, a;
};

static double sig0(const Geo& g) {
  return (g.kind == GRT_GEOM_KERR || g.kind == GRT_GEOM_KERR_BL) ? -1.0 : 1.0;
}

static double inner_product(const Geo& g, const V4& pos, const V4& v, const V4& w) {
  switch (g.kind) {
    case GRT_GEOM_EUCLIDEAN:
      return 1.0 * v[0] * w[0] + -v[1] * w[1] + -v[2] * w[2] + -v[3] * w[3];
    case GRT_GEOM_SCHWARZSCHILD: {
      double r = pos[1], theta = pos[2];
      double a = 1.0 - g.radius / r;
      return a * v[0] * w[0] - v[1] * w[1] / a - r * r * v[2] * w[2] -
             r * r * std::sin(theta) * std::sin(theta) * v[3] * w[3];
    }
    case GRT_GEOM_EUCLIDEAN_SPHERICAL: {  // euclidean_spherical.rs:80-91
      double r = pos[1], theta = pos[2];
      return 1.0 * v[0] * w[0] - v[1] * w[1] - r * r * v[2] * w[2] -
             r * r * std::sin(theta) * std::sin(theta) * v[3] * w[3];
    }
    case GRT_GEOM_KERR: {
      M4 m;
      ks_metric(g.radius, g.a, pos[1], pos[2], pos[3], m);
      return quad(v, m, w);
    }
    default: {
      M4 m;
      metric_bl(g.radius, g.a, pos[1], pos[2], m);
      double result = 0.0;
      for (int mu = 0; mu < 4; ++mu)
        for (int nu = 0; nu < 4; ++nu) result += m[mu][nu] * v[mu] * w[nu];
      return result;
    }
  }
}

// circular_orbit.rs:39-72
static void metric_components_at(double r_s, double a, double r, double theta, double* g_tt, double* g_tphi,
                                 double* g_phiphi) {
  double c = std::cos(theta), s = std::sin(theta);
  double sig = r * r + a * a * (c * c);
  double sin2 = s * s;
  *g_tt = -(1.0 - r_s * r / sig);
  *g_tphi = -a * r_s * r * sin2 / sig;
  *g_phiphi = (r * r + a * a + a * a * r_s * r * sin2 / sig) * sin2;
}
static void zamo_killing(double r_s, double a, double r, double theta, double* u_t, double* u_phi) {
  double g_tt, g_tphi, g_phiphi;
  metric_components_at(r_s, a, r, theta, &g_tt, &g_tphi, &g_phiphi);
  double omega = -g_tphi / g_phiphi;
  double ut = std::sqrt(-1.0 / (g_tt + 2.0 * g_tphi * omega + g_phiphi * omega * omega));
  *u_t = ut;
  *u_phi = omega * ut;
}
static double angular_velocity(double r_s, double a, double r) {  // :76-80
  double m = 0.5 * r_s;
  double sqrt_m = std::sqrt(m);
  return sqrt_m / (std::pow(r, 1.5) + a * sqrt_m);
}
static bool killing_coefficients(double r_s, double a, double r, double* u_t, double* u_phi) {  // :84-108
  double omega = angular_velocity(r_s, a, r);
  double g_tt, g_tphi, g_phiphi;
  metric_components_at(r_s, a, r, FRAC_PI_2, &g_tt, &g_tphi, &g_phiphi);
  double ut_pre = g_tt + 2.0 * omega * g_tphi + omega * omega * g_phiphi;
  if (ut_pre >= 0.0) return false;
  double ut = 1.0 / std::sqrt(-ut_pre);
  *u_t = ut;
  *u_phi = omega * ut;
  return true;
}

static V4 stationary_velocity(const Geo& g, const V4& p) {
  V4 u{{0, 0, 0, 0}};
  switch (g.kind) {
    case GRT_GEOM_EUCLIDEAN:
    case GRT_GEOM_EUCLIDEAN_SPHERICAL:  // euclidean_spherical.rs:168-170
      u[0] = 1.0;
      break;
    case GRT_GEOM_SCHWARZSCHILD: {
      double a = 1.0 - g.radius / p[1];
      u[0] = 1.0 / std::sqrt(a);
      break;
    }
    case GRT_GEOM_KERR: {
      double z = p[3];
      double r_sqr = ks_r_sqr(g.a, p[1], p[2], p[3]);
      double r = std::sqrt(r_sqr);
      double f = (r * r * r * g.radius) / (r * r * r * r + g.a * g.a * z * z);
      u[0] = 1.0 / std::sqrt(1.0 - f);
      break;
    }
    default: {
      double sig = bl_sigma(p[1], g.a, p[2]);
      u[0] = 1.0 / std::sqrt(1.0 - g.radius * p[1] / sig);
      break;
    }
  }
  return u;
}

static V4 zamo_velocity(const Geo& g, const V4& p) {
  if (g.kind == GRT_GEOM_EUCLIDEAN || g.kind == GRT_GEOM_SCHWARZSCHILD || g.kind == GRT_GEOM_EUCLIDEAN_SPHERICAL)
    return stationary_velocity(g, p);
  if (g.kind == GRT_GEOM_KERR_BL) {  // kerr_bl.rs:373-382
    double ut, uphi;
    zamo_killing(g.radius, g.a, p[1], p[2], &ut, &uphi);
    return V4{{ut, 0.0, 0.0, uphi}};
  }
  // kerr.rs:457-468
  double x = p[1], y = p[2], z = p[3];
  double r = std::sqrt(ks_r_sqr(g.a, x, y, z));
  double theta = (r == 0.0) ? 0.0 : std::acos(rclamp(z / r, -1.0, 1.0));
  double ut, uphi;
  zamo_killing(g.radius, g.a, r, theta, &ut, &uphi);
  V4 et{{1.0, 0.0, 0.0, 0.0}}, ax{{0.0, -y, x, 0.0}};
  return add(scale(ut, et), scale(uphi, ax));
}

// ------------------------------------------------------------------ tetrads -------
struct Tetrad {
  V4 t, x, y, z;
};

static std::vector<V4> gram_schmidt(const Geo& g, const V4& pos, const std::vector<V4>& vectors) {
  std::vector<V4> out;  // gram_schmidt.rs:13-34
  for (const V4& v : vectors) {
    V4 w = v;
    for (const V4& u : out) {
      double p1 = inner_product(g, pos, w, u);
      double p2 = inner_product(g, pos, u, u);
      V4 projection = scale(p1 / p2, u);
      w = add(w, neg(projection));
    }
    double norm = std::sqrt(std::fabs(inner_product(g, pos, w, w)));
    out.push_back(scale(1.0 / norm, w));
  }
  return out;
}

static V4 cart_to_sph_v(const V4& c) {  // spherical_coordinates_helper.rs:5-26
  double t = c[0], x = c[1], y = c[2], z = c[3];
  double r = std::sqrt(x * x + y * y + z * z);
  if (r == 0.0) return V4{{t, 0.0, 0.0, 0.0}};
  return V4{{t, r, std::acos(z / r), std::atan2(y, x)}};
}

static Tetrad get_tetrad_at(const Geo& g, const V4& p) {
  Tetrad T;
  switch (g.kind) {
    case GRT_GEOM_EUCLIDEAN: {  // euclidean.rs:86-109
      V4 s = cart_to_sph_v(p);
      double theta = s[2], phi = s[3];
      V4 e_t{{1.0, 0.0, 0.0, 0.0}};
      V4 e_r{{0.0, std::sin(theta) * std::cos(phi), std::sin(theta) * std::sin(phi), std::cos(theta)}};
      V4 e_theta{{0.0, std::cos(theta) * std::cos(phi), std::cos(theta) * std::sin(phi), -std::sin(theta)}};
      V4 e_phi{{0.0, -std::sin(phi), std::cos(phi), 0.0}};
      T.t = e_t;
      T.x = e_phi;
      T.y = neg(e_theta);
      T.z = neg(e_r);
      break;
    }
    case GRT_GEOM_EUCLIDEAN_SPHERICAL: {  // euclidean_spherical.rs:100-112
      double r = p[1], theta = p[2];
      T.t = V4{{1.0, 0.0, 0.0, 0.0}};
      T.x = V4{{0.0, 0.0, 0.0, 1.0 / (r * std::sin(theta))}};
      T.y = neg(V4{{0.0, 0.0, 1.0 / r, 0.0}});
      T.z = neg(V4{{0.0, 1.0, 0.0, 0.0}});
      break;
    }
    case GRT_GEOM_SCHWARZSCHILD: {  // schwarzschild.rs:116-132
      double r = p[1], theta = p[2];
      double rr0 = g.radius / r;
      double a = 1.0 - rr0;
      T.t = V4{{1.0 / a, -std::sqrt(rr0), 0.0, 0.0}};
      T.x = V4{{0.0, 0.0, 0.0, 1.0 / (r * std::sin(theta))}};
      T.y = V4{{0.0, 0.0, 1.0 / r, 0.0}};
      T.z = V4{{-std::sqrt(rr0) / a, 1.0, 0.0, 0.0}};
      break;
    }
    case GRT_GEOM_KERR: {  // kerr.rs:297-331
      double x = p[1], y = p[2], z = p[3];
      double r_sqr = ks_r_sqr(g.a, x, y, z);
      double r = std::sqrt(r_sqr);
      double f = (r * r * r * g.radius) / (r * r * r * r + g.a * g.a * z * z);
      double kx = (r * x + g.a * y) / (r_sqr + g.a * g.a), ky = (r * y - g.a * x) / (r_sqr + g.a * g.a);
      double kz = z / r;
      double alpha = 1.0 / std::sqrt(1.0 + f);
      double bfac = f / (1.0 + f);
      double beta[3] = {bfac * kx, bfac * ky, bfac * kz};
      V4 e_t{{1.0 / alpha, -beta[0] / alpha, -beta[1] / alpha, -beta[2] / alpha}};
      std::vector<V4> b = gram_schmidt(g, p, {e_t, V4{{0, 1, 0, 0}}, V4{{0, 0, 1, 0}}, V4{{0, 0, 0, 1}}});
      T.t = b[0];
      T.x = b[1];
      T.y = b[2];
      T.z = b[3];
      break;
    }
    default: {  // kerr_bl.rs:428-450
      double ut, uphi;
      zamo_killing(g.radius, g.a, p[1], p[2], &ut, &uphi);
      double omega = uphi / ut;
      V4 e_t{{ut, 0.0, 0.0, ut * omega}};
      std::vector<V4> b =
          gram_schmidt(g, p, {e_t, V4{{0, 0, 0, 1}}, V4{{0, 0, 1, 0}}, V4{{0, 1, 0, 0}}});
      T.t = b[0];
      T.x = b[1];
      T.y = b[2];
      T.z = b[3];
      break;
    }
  }
  return T;
}

static void lorentz_transformation(const Geo& g, const V4& pos, const V4& vel, M4 L) {
  Tetrad T0 = get_tetrad_at(g, pos);
  const V4& tt = T0.t;
  switch (g.kind) {
    case GRT_GEOM_EUCLIDEAN: {  // euclidean.rs:111-142
      double gamma = tt[0] * vel[0] - tt[1] * vel[1] - tt[2] * vel[2] - tt[3] * vel[3];
      for (int i = 0; i < 4; ++i)
        for (int j = 0; j < 4; ++j) {
          double res = (i == j) ? 1.0 : 0.0;
          double gj = j == 0 ? 1.0 : -1.0;
          double a = -1.0 / (1.0 + gamma);
          double b = tt[i] + vel[i];
          double c = gj * (tt[j] + vel[j]);
          res += a * b * c;
          res += 2.0 * gj * tt[i] * vel[j];
          L[i][j] = res;
        }
      break;
    }
    case GRT_GEOM_EUCLIDEAN_SPHERICAL:  // euclidean_spherical.rs:114-122: identity
      for (int i = 0; i < 4; ++i)
        for (int j = 0; j < 4; ++j) L[i][j] = (i == j) ? 1.0 : 0.0;
      break;
    case GRT_GEOM_SCHWARZSCHILD: {  // schwarzschild.rs:134-179
      double r = pos[1], theta = pos[2];
      double a = 1.0 - g.radius / r;
      double md[4] = {a, -1.0 / a, -r * r, -r * r * std::sin(theta) * std::sin(theta)};
      double gamma = 0.0;
      for (int i = 0; i < 4; ++i) gamma += md[i] * vel[i] * tt[i];
      for (int mu = 0; mu < 4; ++mu)
        for (int nu = 0; nu < 4; ++nu) {
          double res = (mu == nu) ? 1.0 : 0.0;
          double aa = 1.0 / (1.0 + gamma);
          double b = tt[mu] + vel[mu];
          double c = md[nu] * (tt[nu] + vel[nu]);
          res -= aa * b * c;
          res += 2.0 * md[nu] * tt[nu] * vel[mu];
          L[mu][nu] = res;
        }
      break;
    }
    default: {  // kerr.rs:333-380, kerr_bl.rs:452-480
      M4 m;
      if (g.kind == GRT_GEOM_KERR) ks_metric(g.radius, g.a, pos[1], pos[2], pos[3], m);
      else metric_bl(g.radius, g.a, pos[1], pos[2], m);
      double gamma = -quad(tt, m, vel);
      V4 uv = add(tt, vel);
      V4 uv_lower;
      gemv(m, uv, uv_lower);
      V4 gt;
      gemv(m, tt, gt);
      for (int mu = 0; mu < 4; ++mu)
        for (int nu = 0; nu < 4; ++nu) {
          double res = (mu == nu) ? 1.0 : 0.0;
          double a = 1.0 / (1.0 + gamma);
          double b = uv[mu];
          double c = uv_lower[nu];
          res += a * b * c;
          res -= 2.0 * gt[nu] * vel[mu];
          L[mu][nu] = res;
        }
      break;
    }
  }
}

static bool validate_tetrad(const Geo& g, const V4& pos, const Tetrad& T) {  // tetrad.rs:60-131
  double tol = 1e-5;
  double s0 = sig0(g), ss = -s0;
  auto ok = [&](double v, double want) { return std::fabs(v - want) < tol; };
  return ok(inner_product(g, pos, T.t, T.t), s0) && ok(inner_product(g, pos, T.x, T.x), ss) &&
         ok(inner_product(g, pos, T.y, T.y), ss) && ok(inner_product(g, pos, T.z, T.z), ss) &&
         ok(inner_product(g, pos, T.t, T.x), 0.0) && ok(inner_product(g, pos, T.t, T.y), 0.0) &&
         ok(inner_product(g, pos, T.t, T.z), 0.0) && ok(inner_product(g, pos, T.x, T.y), 0.0) &&
         ok(inner_product(g, pos, T.x, T.z), 0.0) && ok(inner_product(g, pos, T.y, T.z), 0.0);
}

// camera.rs:83-132
static void spatial_cartesian(const Geo& g, const V4& pos, const V4& v, double out[3]) {
  if (g.kind == GRT_GEOM_EUCLIDEAN || g.kind == GRT_GEOM_KERR) {
    out[0] = v[1];
    out[1] = v[2];
    out[2] = v[3];
    return;
  }
  double r = pos[1], theta = rem_euclid(pos[2], PI), phi = rem_euclid(pos[3] + PI, 2.0 * PI) - PI;
  double dr = v[1], dtheta = v[2], dphi = v[3];
  if (g.kind == GRT_GEOM_SCHWARZSCHILD || g.kind == GRT_GEOM_EUCLIDEAN_SPHERICAL) {
    double st = std::sin(theta), ct = std::cos(theta), sp = std::sin(phi), cp = std::cos(phi);
    out[0] = st * cp * dr + r * ct * cp * dtheta - r * st * sp * dphi;
    out[1] = st * sp * dr + r * ct * sp * dtheta + r * st * cp * dphi;
    out[2] = ct * dr - r * st * dtheta;
  } else {
    double a = g.a;
    double st = std::sin(theta), ct = std::cos(theta), sp = std::sin(phi), cp = std::cos(phi);
    out[0] = st * cp * dr + (r * cp - a * sp) * ct * dtheta + (-r * sp - a * cp) * st * dphi;
    out[1] = st * sp * dr + (r * sp + a * cp) * ct * dtheta + (r * cp - a * sp) * st * dphi;
    out[2] = ct * dr - r * st * dtheta;
  }
}
static double spatial_handedness(const Geo& g, const V4& pos, const Tetrad& T) {  // :134-148
  double x[3], y[3], z[3];
  spatial_cartesian(g, pos, T.x, x);
  spatial_cartesian(g, pos, T.y, y);
  spatial_cartesian(g, pos, T.z, z);
  double c0 = y[1] * z[2] - y[2] * z[1];
  double c1 = y[2] * z[0] - y[0] * z[2];
  double c2 = y[0] * z[1] - y[1] * z[0];
  double triple = x[0] * c0 + x[1] * c1 + x[2] * c2;
  if (!std::isfinite(triple) || std::fabs(triple) <= 1e-12)
    return (g.kind == GRT_GEOM_SCHWARZSCHILD || g.kind == GRT_GEOM_KERR_BL || g.kind == GRT_GEOM_EUCLIDEAN_SPHERICAL)
               ? -1.0
               : 1.0;
  return triple >= 0.0 ? 1.0 : -1.0;
}

static void rotate(const V4& v1, const V4& v2, double angle, V4& r1, V4& r2) {  // camera.rs:76-81
  r1 = add(scale(std::cos(angle), v1), scale(std::sin(angle), v2));
  r2 = add(scale(-std::sin(angle), v1), scale(std::cos(angle), v2));
}

int camera_build(int geometry, double radius, double a, const double position[4], const double velocity[4],
                 double alpha, int64_t rows, int64_t cols, double phi, double theta, double psi,
                 grt_camera_desc* out) {
  Geo g{geometry, radius, a};
  V4 pos{{position[0], position[1], position[2], position[3]}};
  V4 vel{{velocity[0], velocity[1], velocity[2], velocity[3]}};
  Tetrad orig = get_tetrad_at(g, pos);
  if (!validate_tetrad(g, pos, orig)) return -EDOM;
  V4 a_prime, b_prime, z, a_two_prime, x, y;
  rotate(orig.x, orig.y, phi, a_prime, b_prime);
  rotate(orig.z, a_prime, theta, z, a_two_prime);
  rotate(a_two_prime, b_prime, psi, x, y);
  Tetrad rot{orig.t, x, y, z};
  M4 L;
  lorentz_transformation(g, pos, vel, L);
  Tetrad T;
  gemv(L, rot.t, T.t);
  gemv(L, rot.x, T.x);
  gemv(L, rot.y, T.y);
  gemv(L, rot.z, T.z);
  if (!validate_tetrad(g, pos, T)) return -EDOM;
  std::memset(out, 0, sizeof(*out));
  for (int k = 0; k < 4; ++k) {
    out->position[k] = pos[k];
    out->velocity[k] = vel[k];
    out->tetrad[0][k] = T.t[k];
    out->tetrad[1][k] = T.x[k];
    out->tetrad[2][k] = T.y[k];
    out->tetrad[3][k] = T.z[k];
  }
  out->alpha = alpha;
  out->tan_half_alpha = std::tan(alpha / 2.0);
  out->rows = rows;
  out->cols = cols;
  out->spatial_signature = -sig0(g);  // signature[3]
  out->spatial_handedness = spatial_handedness(g, pos, T);
  // the KerrBL per-ray constants use sin and cos of this one theta (kerr_bl.rs:505-577):
  // the reference's compiled code evaluates them with one glibc sincos() call
  ::sincos(pos[2], &out->sin_theta, &out->cos_theta);
  return 0;
}

// cli/shared.rs:23-41 assert_directed (expected_sign = +1)
bool future_directed(int geometry, double radius, double a, const double position[4], const double v[4]) {
  Geo g{geometry, radius, a};
  V4 pos{{position[0], position[1], position[2], position[3]}};
  V4 vv{{v[0], v[1], v[2], v[3]}};
  Tetrad T = get_tetrad_at(g, pos);
  double orientation = sig0(g) * inner_product(g, pos, T.t, vv);
  return std::isfinite(vv[0]) && orientation > 0.0;
}
// The momentum `render-ray-at` integrates (cli/{euclidean,schwarzschild,kerr,kerr_bl}.rs
// render_ray_at): a unit spatial direction in the local observer's tetrad at a Cartesian
// position.  Writes the ray's native-chart position and contravariant momentum.
int ray_at(int geometry, double radius, double a, const double position[3], const double direction[3],
           double pos_out[4], double mom_out[4], std::string& err) {
  Geo g{geometry, radius, a};
  V4 cart{{0.0, position[0], position[1], position[2]}};
  const double d1 = direction[0], d2 = direction[1], d3 = direction[2];
  V4 pos, mom;
  switch (geometry) {
    case GRT_GEOM_EUCLIDEAN: {  // cli/euclidean.rs:74-100
      double spatial_norm = std::sqrt(d1 * d1 + d2 * d2 + d3 * d3);
      if (!(std::isfinite(spatial_norm) && spatial_norm > 0.0)) {
        err = "render_ray_at direction must have a non-zero finite spatial part.";
        return -EINVAL;
      }
      pos = cart;
      mom = V4{{spatial_norm, d1, d2, d3}};
      break;
    }
    case GRT_GEOM_EUCLIDEAN_SPHERICAL: {  // cli/euclidean_spherical.rs:77-142
      pos = cart_to_sph_v(cart);
      const double r = pos[1], theta = pos[2], phi = pos[3];
      if (!(std::isfinite(r) && r > 0.0)) {
        err = "Euclidean-spherical render_ray_at requires r > 0, got r=" + rust_display_f64(r) + ".";
        return -EINVAL;
      }
      const double sin_theta = std::sin(theta);
      if (!(std::isfinite(sin_theta) && std::fabs(sin_theta) > 1e-12)) {
        err = "Euclidean-spherical render_ray_at is undefined on the polar axis (theta=" + rust_display_f64(theta) +
              ").";
        return -EINVAL;
      }
      const double spatial_norm = std::sqrt(d1 * d1 + d2 * d2 + d3 * d3);
      if (!(std::isfinite(spatial_norm) && spatial_norm > 0.0)) {
        err = "render_ray_at direction must have a non-zero finite spatial part.";
        return -EINVAL;
      }
      const double r_dot = sin_theta * std::cos(phi) * d1 + sin_theta * std::sin(phi) * d2 + std::cos(theta) * d3;
      const double theta_unit_dot =
          std::cos(theta) * std::cos(phi) * d1 + std::cos(theta) * std::sin(phi) * d2 - sin_theta * d3;
      const double phi_unit_dot = -std::sin(phi) * d1 + std::cos(phi) * d2;
      mom = V4{{spatial_norm, r_dot, theta_unit_dot / r, phi_unit_dot / (r * sin_theta)}};
      break;
    }
    case GRT_GEOM_SCHWARZSCHILD: {  // cli/schwarzschild.rs:89-121
      pos = cart_to_sph_v(cart);
      double theta = pos[2], phi = pos[3];
      double r_d = std::sin(theta) * std::cos(phi) * d1 + std::sin(theta) * std::sin(phi) * d2 + std::cos(theta) * d3;
      double theta_d =
          std::cos(theta) * std::cos(phi) * d1 + std::cos(theta) * std::sin(phi) * d2 - std::sin(theta) * d3;
      double phi_d = -std::sin(phi) * d1 + std::cos(phi) * d2;
      Tetrad T = get_tetrad_at(g, pos);
      mom = add(add(add(scale(1.0, T.t), scale(phi_d, T.x)), scale(-theta_d, T.y)), scale(-r_d, T.z));
      break;
    }
    default: {  // cli/kerr.rs:77-100 (Cartesian chart), cli/kerr_bl.rs:78-107 (BL chart)
      if (geometry == GRT_GEOM_KERR) {
        pos = cart;
      } else {
        double out[4];
        grt_cartesian_to_boyer_lindquist(a, cart.v, out);
        pos = V4{{out[0], out[1], out[2], out[3]}};
      }
      Tetrad T = get_tetrad_at(g, pos);
      V4 space = add(add(scale(d1, T.x), scale(d2, T.y)), scale(d3, T.z));
      double norm = std::sqrt(inner_product(g, pos, space, space));
      V4 m;
      for (int k = 0; k < 4; ++k)
        m[k] = ((T.t[k] * 1.0 + T.x[k] * d1 / norm) + T.y[k] * d2 / norm) + T.z[k] * d3 / norm;
      mom = m;
      break;
    }
  }
  if (!future_directed(geometry, radius, a, pos.v, mom.v)) {  // cli/shared.rs:79-86
    err = "render_ray_at momentum is not future-directed";
    return -EINVAL;
  }
  for (int k = 0; k < 4; ++k) {
    pos_out[k] = pos[k];
    mom_out[k] = mom[k];
  }
  return 0;
}

double inner(int geometry, double radius, double a, const double position[4], const double v[4], const double w[4]) {
  Geo g{geometry, radius, a};
  V4 pos{{position[0], position[1], position[2], position[3]}};
  V4 vv{{v[0], v[1], v[2], v[3]}}, ww{{w[0], w[1], w[2], w[3]}};
  return inner_product(g, pos, vv, ww);
}
double signature0(int geometry) {
  Geo g{geometry, 0, 0};
  return sig0(g);
}

// ------------------------------------------------------- temperature LUT --------
// circular_orbit.rs:110-136
static bool conserved_energy(double r_s, double a, double r, double* out) {
  double omega = angular_velocity(r_s, a, r);
  double g_tt, g_tphi, g_phiphi;
  metric_components_at(r_s, a, r, FRAC_PI_2, &g_tt, &g_tphi, &g_phiphi);
  double ut, uphi;
  if (!killing_coefficients(r_s, a, r, &ut, &uphi)) return false;
  *out = -(g_tt + g_tphi * omega) * ut;
  return true;
}
static bool conserved_angular_momentum(double r_s, double a, double r, double* out) {
  double omega = angular_velocity(r_s, a, r);
  double g_tt, g_tphi, g_phiphi;
  metric_components_at(r_s, a, r, FRAC_PI_2, &g_tt, &g_tphi, &g_phiphi);
  double ut, uphi;
  if (!killing_coefficients(r_s, a, r, &ut, &uphi)) return false;
  *out = (g_tphi + g_phiphi * omega) * ut;
  return true;
}
double r_isco(double r_s, double a) {
  double a_s = 2.0 * a / r_s;
  double z1 = 1.0 + std::pow(1.0 - a_s * a_s, 1.0 / 3.0) *
                        (std::pow(1.0 + a_s, 1.0 / 3.0) + std::pow(1.0 - a_s, 1.0 / 3.0));
  double z2 = std::sqrt(3.0 * a_s * a_s + z1 * z1);
  return (3.0 + z2 - std::sqrt((3.0 - z1) * (3.0 + z1 + 2.0 * z2))) * r_s / 2.0;
}

namespace {
struct KerrTemp {  // temperature.rs:29-193
  double a, radius, r_isco, m_dot;
  bool d_l_dr(double r, double* out) const {
    double h = 1e-6 * std::fmax(r, 1.0);
    double lp, lm, l0;
    if (r - h < r_isco) {
      if (!conserved_angular_momentum(radius, a, r + h, &lp) || !conserved_angular_momentum(radius, a, r, &l0))
        return false;
      *out = (lp - l0) / h;
    } else {
      if (!conserved_angular_momentum(radius, a, r + h, &lp) || !conserved_angular_momentum(radius, a, r - h, &lm))
        return false;
      *out = (lp - lm) / (2.0 * h);
    }
    return true;
  }
  double d_omega_dr(double r) const {
    double h = 1e-10;
    return (angular_velocity(radius, a, r + h) - angular_velocity(radius, a, r - h)) / (2.0 * h);
  }
  int compute_integral(double r, double* out) const {
    double dr = (r - r_isco) / (double)1000;
    double integral = 0.0;
    for (int i = 0; i < 1000; ++i) {
      double rp = r_isco + ((double)i + 0.5) * dr;
      double e, l, dl;
      if (!conserved_energy(radius, a, rp, &e)) return -ERANGE;
      if (!conserved_angular_momentum(radius, a, rp, &l)) return -ERANGE;
      double omega = angular_velocity(radius, a, rp);
      if (!d_l_dr(rp, &dl)) return -ERANGE;
      integral += (e - omega * l) * dl * dr;
    }
    *out = integral;
    return 0;
  }
  int compute_prefactor(double r, double* out) const {
    double e, l;
    if (!conserved_energy(radius, a, r, &e)) return -ERANGE;
    if (!conserved_angular_momentum(radius, a, r, &l)) return -ERANGE;
    double omega = angular_velocity(radius, a, r);
    double root = r * r;
    double eol = e - omega * l;
    double denominator = root * (eol * eol);
    if (std::fabs(denominator) < 1e-20) return -ERANGE;  // DenominatorCloseToZero
    *out = d_omega_dr(r) / denominator;
    return 0;
  }
  int compute_f(double r, double* out) const {
    double integral, pre;
    int rc;
    if ((rc = compute_integral(r, &integral))) return rc;
    if ((rc = compute_prefactor(r, &pre))) return rc;
    double coefficient = -m_dot / (PI * radius * radius);
    *out = coefficient * pre * integral;
    return 0;
  }
};
}  // namespace

int kerr_temperature_lut(double temperature, double outer_radius, double a, double radius, uint32_t n,
                         double* lut_r, double* lut_t, double* r_isco_out, std::string* log) {
  double a_abs = std::fabs(a);
  double ri = r_isco(radius, a_abs);
  double eff_outer = outer_radius;
  if (outer_radius <= ri) {
    eff_outer = ri + std::fmax(1e-6, std::fabs(ri) * 1e-9);
    if (log)
      *log += "outer_radius (" + rust_display_f64(outer_radius) + ") <= r_isco (" + rust_display_f64(ri) +
              "); clamping to " + rust_display_f64(eff_outer) + " for stable LUT construction.\n";
  }
  if (log)
    *log += "Computed r_isco: " + rust_display_f64(ri) + " from a: " + rust_display_f64(a_abs) +
            " and radius: " + rust_display_f64(radius) + "\n";
  KerrTemp kt{a_abs, radius, ri, 1.0};
  double max_f = 0.0, max_r = 0.0;
  double dr = (eff_outer - ri) / (double)10;
  for (int i = 0; i < 10; ++i) {
    double r = ri + ((double)i + 0.5) * dr;
    double f;
    int rc = kt.compute_f(r, &f);
    if (rc) return rc;
    if (max_f < f) {
      max_f = f;
      max_r = r;
    }
  }
  if (log) *log += "Max f: " + rust_display_f64(max_f) + " at radius: " + rust_display_f64(max_r) + "\n";
  double integral, pre;
  int rc;
  if ((rc = kt.compute_integral(max_r, &integral))) return rc;
  if ((rc = kt.compute_prefactor(max_r, &pre))) return rc;
  double coefficient = -1.0 / (PI * radius * radius);
  double sigma_sb = 1.0;
  double f = sigma_sb * std::pow(temperature, 4.0);
  kt.m_dot = f / (coefficient * pre * integral);
  if (log)
    *log += "Computed m_dot: " + rust_display_f64(kt.m_dot) + " for target temperature: " +
            rust_display_f64(temperature) + "\n";
  double step = (eff_outer - ri) / (double)(n - 1);
  // the entries are independent (each its own integral): host threads, the first failing
  // entry's error in index order, as the reference's sequential loop would return it
  std::vector<int> rcs(n, 0);
  parallel_for(n, [&](uint64_t i) {
    double r = ri + (double)i * step;
    double fv;
    if ((rcs[i] = kt.compute_f(r, &fv))) return;
    lut_r[i] = r;
    lut_t[i] = std::pow(std::fmax(fv / sigma_sb, 0.0), 0.25);
  });
  for (uint32_t i = 0; i < n; ++i)
    if (rcs[i]) return rcs[i];
  *r_isco_out = ri;
  return 0;
}

// ----------------------------------------------------------- blackbody LUT ------
static double g_cie(double lambda, double mu, double tau_left, double tau_right) {  // color.rs:173-177
  double tau = lambda < mu ? tau_left : tau_right;
  double t = (lambda - mu) * tau;
  return std::exp(-0.5 * t * t);
}
static double x_bar(double l) {
  return 1.056 * g_cie(l, 599.8, 0.0264, 0.0323) + 0.362 * g_cie(l, 442.0, 0.0624, 0.0374) -
         0.065 * g_cie(l, 501.1, 0.0490, 0.0382);
}
static double y_bar(double l) { return 0.821 * g_cie(l, 568.8, 0.0213, 0.0247) + 0.286 * g_cie(l, 530.9, 0.0613, 0.0322); }
static double z_bar(double l) { return 1.217 * g_cie(l, 437.0, 0.0845, 0.0278) + 0.681 * g_cie(l, 459.0, 0.0385, 0.0725); }
static double powi5(double x) { return x * ((x * x) * (x * x)); }  // llvm.powi(x, 5) expansion

void blackbody_xyz(double temperature, double redshift, double out[3]) {  // black_body_radiation.rs:18-41
  const double H = 6.62607015e-34, C = 299792458.0, KB = 1.380649e-23;
  const double MIN_WL = 380.0, MAX_WL = 830.0, NM = 1e-9;
  double interval = (MAX_WL - MIN_WL) * NM;
  double step = 1.0 * NM;
  uint64_t num_steps = (uint64_t)std::floor(interval / step);
  double xa = 0.0, ya = 0.0, za = 0.0;
  for (uint64_t i = 0; i < num_steps; ++i) {
    double lambda = MIN_WL * NM + ((double)i + 0.5) * step;
    double lz = lambda * redshift;
    double a = 2.0 * H * C * C;
    double b = H * C / (lz * KB * temperature);
    double radiance = a / (powi5(lz) * (std::exp(b) - 1.0));
    xa += radiance * x_bar(lambda / NM) * step;
    ya += radiance * y_bar(lambda / NM) * step;
    za += radiance * z_bar(lambda / NM) * step;
  }
  double boost = powi5(redshift);
  out[0] = xa * boost;
  out[1] = ya * boost;
  out[2] = za * boost;
}

// run_blackbody_spectrum (cli/blackbody.rs:27-95): a width x height image of the
// redshifted blackbody colour, temperature along x and redshift along y, through the
// output stage (exposure 1, the CLI's tone mapping), RGBA with alpha 255.  Host threads
// stand in for the reference's rayon loop; each pixel is independent.
int blackbody_spectrum(double t_min, double t_max, double z_min, double z_max, uint32_t w, uint32_t h, int tone,
                       uint8_t* rgba) {
  const size_t n = (size_t)w * h;
  std::vector<double> xyza(4 * n);
  unsigned nt = std::max(1u, std::min(16u, std::thread::hardware_concurrency()));
  std::vector<std::thread> pool;
  for (unsigned k = 0; k < nt; ++k)
    pool.emplace_back([&, k] {
      for (size_t i = k; i < n; i += nt) {
        const double x = (double)(i % w), y = (double)(i / w);
        const double temperature = t_min + x * (t_max - t_min) / ((double)w - 1.0);
        const double redshift = z_min + y * (z_max - z_min) / ((double)h - 1.0);
        blackbody_xyz(temperature, redshift, &xyza[4 * i]);
        xyza[4 * i + 3] = 1.0;
      }
    });
  for (auto& t : pool) t.join();
  std::vector<uint8_t> rgb(3 * n);
  int rc = xyz_to_srgb8(xyza.data(), n, tone, 1.0, rgb.data());
  if (rc) return rc;
  for (size_t i = 0; i < n; ++i) {
    rgba[4 * i] = rgb[3 * i];
    rgba[4 * i + 1] = rgb[3 * i + 1];
    rgba[4 * i + 2] = rgb[3 * i + 2];
    rgba[4 * i + 3] = 255;
  }
  return 0;
}

int blackbody_lut(uint32_t n, double* log_t, double* xyz) {  // texture.rs:121-138
  if (n < 2) return -EINVAL;
  double min_log = std::log10(10.0), max_log = std::log10(10000000.0);
  double step = (max_log - min_log) / (double)(n - 1);
  parallel_for(n, [&](uint64_t i) {  // independent entries
    double lt = min_log + (double)i * step;
    double t = std::pow(10.0, lt);
    log_t[i] = lt;
    blackbody_xyz(t, 1.0, xyz + 3 * i);
  });
  return 0;
}

// ---------------------------------------------------------------- colours -------
double inv_compand_srgb(double u) {  // color.rs:301-308
  if (u <= 0.04045) return u / 12.92;
  return std::pow((u + 0.055) / 1.055, 2.4);
}
void srgb_to_xyza(uint8_t r8, uint8_t g8, uint8_t b8, uint8_t a8, double out[4]) {
  double r = inv_compand_srgb((double)r8 / 255.0), g = inv_compand_srgb((double)g8 / 255.0),
         b = inv_compand_srgb((double)b8 / 255.0);
  static const double M[3][3] = {{0.4124564, 0.3575761, 0.1804375},
                                 {0.2126729, 0.7151522, 0.0721750},
                                 {0.0193339, 0.1191920, 0.9503041}};
  double v[3] = {r, g, b};
  for (int i = 0; i < 3; ++i) {
    double s = M[i][0] * v[0];
    s = M[i][1] * v[1] + s;
    s = M[i][2] * v[2] + s;
    out[i] = s;
  }
  out[3] = (double)a8 / 255.0;
}
static double compand_srgb(double linear) {  // color.rs:193-202
  double sign = linear < 0.0 ? -1.0 : 1.0;
  double a = std::fabs(linear);
  double enc = a <= 0.0031308 ? 12.92 * a : 1.055 * std::pow(a, 1.0 / 2.4) - 0.055;
  return rclamp(sign * enc, 0.0, 1.0);
}
static uint8_t to_u8(double v) {  // (x * 255.0).round() as u8 (saturating)
  double r = std::round(v * 255.0);
  if (!(r > 0.0)) return 0;
  if (r >= 255.0) return 255;
  return (uint8_t)r;
}
static void to_linear(const double* c, double* lin) {  // color.rs:208-223, nalgebra gemv order
  static const double M[3][3] = {{3.2406255, -1.5372080, -0.4986286},
                                 {-0.9689307, 1.8757561, 0.0415175},
                                 {0.0557101, -0.2040211, 1.0569959}};
  for (int k = 0; k < 3; ++k) {
    double s = M[k][0] * c[0];
    s = M[k][1] * c[1] + s;
    s = M[k][2] * c[2] + s;
    lin[k] = s;
  }
}
// GlobalLinear's per-channel fold(0.0, f64::max) of (linear * exposure) (color.rs:238-258)
void linear_max(const double* xyza, size_t n, double exposure, double* max3) {
  double m[3] = {0.0, 0.0, 0.0};
  for (size_t i = 0; i < n; ++i) {
    double lin[3];
    to_linear(xyza + 4 * i, lin);
    for (int k = 0; k < 3; ++k) m[k] = std::fmax(m[k], lin[k] * exposure);
  }
  for (int k = 0; k < 3; ++k) max3[k] = m[k];
}
int tonemap(const double* xyza, size_t n, int tone, double exposure, const double* max3, uint8_t* rgb) {
  if (tone != GRT_TONE_REINHARD && tone != GRT_TONE_GLOBAL_LINEAR) return -EINVAL;
  double sc = 1.0;
  if (tone == GRT_TONE_GLOBAL_LINEAR) {
    if (!max3) return -EINVAL;
    double mc = std::fmax(std::fmax(max3[0], max3[1]), max3[2]);
    sc = mc > 0.0 ? 1.0 / mc : 1.0;
  }
  for (size_t i = 0; i < n; ++i) {
    double c[3];
    to_linear(xyza + 4 * i, c);
    for (int k = 0; k < 3; ++k) c[k] = c[k] * exposure;
    if (tone == GRT_TONE_REINHARD) {
      double l_in = 0.2126 * c[0] + 0.7152 * c[1] + 0.0722 * c[2];
      if (l_in > 0.0) {
        double l_out = l_in / (1.0 + l_in);
        double f = l_out / l_in;
        for (int k = 0; k < 3; ++k) c[k] = c[k] * f;
      }
    } else {
      for (int k = 0; k < 3; ++k) c[k] = sc * c[k];
    }
    for (int k = 0; k < 3; ++k) rgb[3 * i + k] = to_u8(compand_srgb(std::fmax(c[k], 0.0)));
  }
  return 0;
}
// xyz_to_srgb (color.rs:225-241): one colour, linear sRGB * exposure, no tone mapping.
void xyz_to_srgb(const double* xyz, double exposure, uint8_t* rgb) {
  double lin[3];
  to_linear(xyz, lin);
  for (int k = 0; k < 3; ++k) rgb[k] = to_u8(compand_srgb(std::fmax(lin[k] * exposure, 0.0)));
}
int xyz_to_srgb8(const double* xyza, size_t n, int tone, double exposure, uint8_t* rgb) {
  double m[3] = {0.0, 0.0, 0.0};
  if (tone == GRT_TONE_GLOBAL_LINEAR) linear_max(xyza, n, exposure, m);
  return tonemap(xyza, n, tone, exposure, m, rgb);
}

int stationary(int geometry, double radius, double a, const double position[4], double out[4]) {
  Geo g{geometry, radius, a};
  V4 p{{position[0], position[1], position[2], position[3]}};
  V4 u = stationary_velocity(g, p);
  for (int k = 0; k < 4; ++k) out[k] = u[k];
  return 0;
}
int zamo(int geometry, double radius, double a, const double position[4], double out[4]) {
  Geo g{geometry, radius, a};
  V4 p{{position[0], position[1], position[2], position[3]}};
  V4 u = zamo_velocity(g, p);
  for (int k = 0; k < 4; ++k) out[k] = u[k];
  return 0;
}

}  // namespace grt_host

// ================================================================== C ABI ========
extern "C" {

int grt_camera_build(int32_t geometry, double radius, double a, const double position[4], const double velocity[4],
                     double alpha, int64_t rows, int64_t cols, double phi, double theta, double psi,
                     grt_camera_desc* out) {
  if (!out || !position || !velocity) return -EINVAL;
  return grt_host::camera_build(geometry, radius, a, position, velocity, alpha, rows, cols, phi, theta, psi, out);
}
int grt_stationary_velocity(int32_t geometry, double radius, double a, const double position[4], double out[4]) {
  return grt_host::stationary(geometry, radius, a, position, out);
}
int grt_zamo_velocity(int32_t geometry, double radius, double a, const double position[4], double out[4]) {
  return grt_host::zamo(geometry, radius, a, position, out);
}
void grt_cartesian_to_spherical(const double in[4], double out[4]) {
  double t = in[0], x = in[1], y = in[2], z = in[3];
  double r = std::sqrt(x * x + y * y + z * z);
  out[0] = t;
  if (r == 0.0) {
    out[1] = out[2] = out[3] = 0.0;
    return;
  }
  out[1] = r;
  out[2] = std::acos(z / r);
  out[3] = std::atan2(y, x);
}
void grt_cartesian_to_boyer_lindquist(double a, const double in[4], double out[4]) {
  double t = in[0], x = in[1], y = in[2], z = in[3];
  double rho_sqr = x * x + y * y + z * z;
  double d = rho_sqr - a * a;
  double r_sqr = 0.5 * (rho_sqr - a * a + std::sqrt(d * d + 4.0 * a * a * z * z));
  double r = std::sqrt(r_sqr);
  double theta = (r == 0.0) ? 0.0 : std::acos(grt_host::rclamp_pub(z / r, -1.0, 1.0));
  out[0] = t;
  out[1] = r;
  out[2] = theta;
  out[3] = std::atan2(r * y - a * x, r * x + a * y);
}
int grt_kerr_temperature_lut(double temperature, double outer_radius, double a, double radius, uint32_t n,
                             double* lut_r, double* lut_t, double* r_isco) {
  if (n < 2 || !lut_r || !lut_t || !r_isco) return -EINVAL;
  return grt_host::kerr_temperature_lut(temperature, outer_radius, a, radius, n, lut_r, lut_t, r_isco);
}
double grt_r_isco(double radius, double a) { return grt_host::r_isco(radius, a); }
int grt_blackbody_lut(uint32_t n, double* log_t, double* xyz) { return grt_host::blackbody_lut(n, log_t, xyz); }
void grt_blackbody_xyz(double temperature, double redshift, double out_xyz[3]) {
  grt_host::blackbody_xyz(temperature, redshift, out_xyz);
}
void grt_srgb_to_xyza(uint8_t r, uint8_t g, uint8_t b, uint8_t a, double out[4]) {
  grt_host::srgb_to_xyza(r, g, b, a, out);
}
int grt_ray_at(int32_t geometry, double radius, double a, const double position[3], const double direction[3],
               double position_out[4], double momentum_out[4]) {
  std::string err;
  int rc = grt_host::ray_at(geometry, radius, a, position, direction, position_out, momentum_out, err);
  if (rc) grt_host::set_error(err);
  return rc;
}
void grt_xyz_to_srgb(const double xyz[3], double exposure, uint8_t rgb_out[3]) {
  grt_host::xyz_to_srgb(xyz, exposure, rgb_out);
}
int grt_blackbody_spectrum(double min_temperature, double max_temperature, double min_redshift, double max_redshift,
                           uint32_t width, uint32_t height, int32_t tone_mapping, uint8_t* rgba_out) {
  if (!rgba_out && (size_t)width * height != 0) return -EINVAL;
  int rc = grt_host::blackbody_spectrum(min_temperature, max_temperature, min_redshift, max_redshift, width, height,
                                        tone_mapping, rgba_out);
  if (rc) grt_host::set_error("grt_blackbody_spectrum: unknown tone mapping");
  return rc;
}
void grt_linear_max(const double* xyza, size_t n, double exposure, double max3[3]) {
  grt_host::linear_max(xyza, n, exposure, max3);
}
int grt_tonemap(const double* xyza, size_t n, int32_t tone_mapping, double exposure, const double max3[3],
                uint8_t* rgb_out) {
  int rc = grt_host::tonemap(xyza, n, tone_mapping, exposure, max3, rgb_out);
  if (rc) grt_host::set_error("grt_tonemap: unknown tone mapping or missing maxima");
  return rc;
}
int grt_xyz_to_srgb8(const double* xyza, size_t n, int32_t tone_mapping, double exposure, uint8_t* rgb_out) {
  if (!xyza || !rgb_out) return -EINVAL;
  return grt_host::xyz_to_srgb8(xyza, n, tone_mapping, exposure, rgb_out);
}

}  // extern "C"
