// trajectory.cpp — CSV export of integrated rays, the output of `render-ray` and
// `render-ray-at` (IntegratedRay::save, src/rendering/ray.rs:35-54):
//
//   i,t,tau,x,y,z
//   <step>,<affine t>,<x^0>,<x^1>,<x^2>,<x^3>      (position converted to Cartesian)
//
// Numbers are printed the way Rust's `{}` prints an f64: the shortest decimal that
// round-trips, written positionally (never in exponent form), "NaN" / "inf" / "-inf",
// and "-0" for negative zero.
#include <cerrno>
#include <charconv>
#include <cmath>
#include <cstdio>
#include <cstring>
#include <string>

#include "grt_api.h"
#include "host_internal.h"

namespace grt_host {

std::string rust_display_f64(double v) {
  if (std::isnan(v)) return "NaN";
  if (std::isinf(v)) return v > 0 ? "inf" : "-inf";
  char buf[64];
  auto res = std::to_chars(buf, buf + sizeof(buf), v, std::chars_format::scientific);  // shortest digits
  std::string sci(buf, res.ptr);
  std::string out;
  size_t p = 0;
  if (sci[0] == '-') {
    out = "-";
    p = 1;
  }
  const size_t e = sci.find('e');
  std::string digits;
  for (size_t k = p; k < e; ++k)
    if (sci[k] != '.') digits += sci[k];
  const int exp10 = std::atoi(sci.c_str() + e + 1);
  if (digits == "0") return out + "0";
  const int point = exp10 + 1;  // digits before the decimal point
  const int n = (int)digits.size();
  if (point <= 0) return out + "0." + std::string(-point, '0') + digits;
  if (point >= n) return out + digits + std::string(point - n, '0');
  return out + digits.substr(0, point) + "." + digits.substr(point);
}

// Point::to_cartesian (point.rs:140-154, spherical_coordinates_helper.rs:28-39)
static void to_cartesian(int geometry, double a, const double* x, double* c) {
  const double t = x[0], r = x[1], theta = x[2], phi = x[3];
  c[0] = t;
  if (geometry == GRT_GEOM_SCHWARZSCHILD || geometry == GRT_GEOM_EUCLIDEAN_SPHERICAL) {
    c[1] = r * std::sin(theta) * std::cos(phi);
    c[2] = r * std::sin(theta) * std::sin(phi);
    c[3] = r * std::cos(theta);
  } else if (geometry == GRT_GEOM_KERR_BL) {
    c[1] = (r * std::cos(phi) - a * std::sin(phi)) * std::sin(theta);
    c[2] = (r * std::sin(phi) + a * std::cos(phi)) * std::sin(theta);
    c[3] = r * std::cos(theta);
  } else {
    c[1] = x[1];
    c[2] = x[2];
    c[3] = x[3];
  }
}

}  // namespace grt_host

extern "C" {

size_t grt_format_f64(double v, char* buf, size_t cap) {
  const std::string s = grt_host::rust_display_f64(v);
  if (buf && cap) {
    const size_t n = s.size() < cap - 1 ? s.size() : cap - 1;
    std::memcpy(buf, s.data(), n);
    buf[n] = 0;
  }
  return s.size();
}

int grt_write_trajectory_csv(const char* path, int32_t geometry, double a, const double* steps, uint64_t n) {
  if (!path || (n && !steps)) {
    grt_host::set_error("grt_write_trajectory_csv: null argument");
    return -EINVAL;
  }
  FILE* f = std::fopen(path, "wb");
  if (!f) {
    grt_host::set_error(std::string("cannot create ") + path + ": " + std::strerror(errno));
    return -EIO;
  }
  std::string line = "i,t,tau,x,y,z\n";
  bool ok = std::fwrite(line.data(), 1, line.size(), f) == line.size();
  for (uint64_t i = 0; i < n && ok; ++i) {
    const double* rec = steps + 9 * i;
    double c[4];
    grt_host::to_cartesian(geometry, a, rec + 1, c);
    line = std::to_string(i);
    line += ',' + grt_host::rust_display_f64(rec[0]);
    for (int k = 0; k < 4; ++k) line += ',' + grt_host::rust_display_f64(c[k]);
    line += '\n';
    ok = std::fwrite(line.data(), 1, line.size(), f) == line.size();
  }
  if (std::fclose(f) != 0) ok = false;
  if (!ok) {
    grt_host::set_error(std::string("write failed: ") + path);
    return -EIO;
  }
  return 0;
}

}  // extern "C"
