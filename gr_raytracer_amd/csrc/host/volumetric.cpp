// volumetric.cpp — host-side constants of a VolumetricDisc, built once per scene
// (VolumetricDisc::new, src/scene_objects/volumetric_disc.rs:43-95):
//   * the normalised axis and the in-plane unit vectors e1, e2 (:61-73), with
//     nalgebra 0.35's Vector3 arithmetic (cross: a.y*b.z - a.z*b.y, ...; norm:
//     sqrt(x*x + y*y + z*z); normalize: component / norm);
//   * Perlin::new(seed) of the `noise` crate 0.9.0 (:83).  The crate is not vendored
//     under /root/reference (Cargo.lock pins noise 0.9.0, rand 0.8.7, rand_xorshift
//     0.3.0); this restates their published algorithms:
//       PermutationTable::new(seed): seed bytes [1,0,0,0, s,s,s,s, s,s,s,s, s,s,s,s]
//         (s = seed little-endian) -> XorShiftRng::from_seed (words x, y, z, w)
//       rng.gen::<PermutationTable>(): values = 0..=255, then values.shuffle(rng)
//       SliceRandom::shuffle: for i in (1..256).rev() { swap(i, gen_range(0..i+1)) }
//       gen_range(0..n) for u32 (UniformInt::sample_single_inclusive(0, n-1)):
//         range = n; zone = (range << range.leading_zeros()) - 1;
//         loop { v = next_u32(); m = v as u64 * range; if (m as u32) <= zone { return m >> 32 } }
//   The device kernels only read the resulting table.
#include <cmath>
#include <cstdint>

#include "host_internal.h"

namespace {

struct XorShift {  // rand_xorshift 0.3.0 XorShiftRng
  uint32_t x, y, z, w;
  uint32_t next_u32() {
    uint32_t t = x ^ (x << 11);
    x = y;
    y = z;
    z = w;
    w = w ^ (w >> 19) ^ (t ^ (t >> 8));
    return w;
  }
};

uint32_t gen_index(XorShift& rng, uint32_t n) {  // rand 0.8 gen_range(0..n), n >= 1
  const uint32_t range = n;
  const uint32_t zone = (range << __builtin_clz(range)) - 1u;
  for (;;) {
    const uint64_t m = (uint64_t)rng.next_u32() * range;
    if ((uint32_t)m <= zone) return (uint32_t)(m >> 32);
  }
}

void cross(const double a[3], const double b[3], double out[3]) {
  out[0] = a[1] * b[2] - a[2] * b[1];
  out[1] = a[2] * b[0] - a[0] * b[2];
  out[2] = a[0] * b[1] - a[1] * b[0];
}
double norm_sq(const double v[3]) { return v[0] * v[0] + v[1] * v[1] + v[2] * v[2]; }
void normalize(const double v[3], double out[3]) {
  const double n = std::sqrt(norm_sq(v));
  for (int i = 0; i < 3; ++i) out[i] = v[i] / n;
}

}  // namespace

extern "C" {

void grt_perlin_permutation(uint32_t seed, uint8_t out[256]) {
  // from_seed reads four little-endian words; an all-zero seed cannot occur (x = 1)
  XorShift rng{1u, seed, seed, seed};
  for (int i = 0; i < 256; ++i) out[i] = (uint8_t)i;
  for (uint32_t i = 255; i >= 1; --i) {
    const uint32_t j = gen_index(rng, i + 1);
    const uint8_t t = out[i];
    out[i] = out[j];
    out[j] = t;
  }
}

void grt_volumetric_frame(const double axis_in[3], double axis[3], double e1[3], double e2[3]) {
  static const double F64_EPSILON = 2.220446049250313e-16;
  if (norm_sq(axis_in) <= F64_EPSILON) {
    axis[0] = 0.0;
    axis[1] = 0.0;
    axis[2] = 1.0;
  } else {
    normalize(axis_in, axis);
  }
  const double ex[3] = {1.0, 0.0, 0.0}, ey[3] = {0.0, 1.0, 0.0};
  double c[3];
  cross(std::fabs(axis[0]) > 0.9 ? ey : ex, axis, c);
  normalize(c, e1);
  cross(axis, e1, c);
  normalize(c, e2);
}

}  // extern "C"
