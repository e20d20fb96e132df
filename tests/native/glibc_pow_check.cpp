// Host build of gr_raytracer_amd/csrc/device/glibc_math.h checked against glibc pow,
// bit for bit (driven by tests/test_glibc_math.py).  Prints: samples fast mismatches.
#include <cinttypes>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <random>

#include "glibc_math.h"

int main(int argc, char** argv) {
  const int mode = atoi(argv[1]);
  const long n = atol(argv[2]);
  std::mt19937_64 rng(12345 + mode);
  std::uniform_real_distribution<double> u01(0.0, 1.0);
  long fast = 0, bad = 0;
  for (long k = 0; k < n; ++k) {
    double x, y;
    switch (mode) {
      case 0:  // the step controller: eps/err, y = 1/5
        x = std::exp(u01(rng) * 1400.0 - 700.0);
        y = 1.0 / 5.0;
        break;
      case 1:  // controller range, y = 1/5
        x = std::exp(u01(rng) * 30.0 - 20.0);
        y = 0.2;
        break;
      case 2:  // beaming exponents: redshift^beaming
        x = u01(rng) * 4.0;
        y = std::floor(u01(rng) * 8.0) * 0.5;
        break;
      case 3:  // x near 1
        x = 1.0 + (u01(rng) - 0.5) * 1e-6;
        y = (u01(rng) - 0.5) * 100.0;
        break;
      default: {  // random positive normal x, moderate y
        uint64_t bits = (rng() & 0x000fffffffffffffull) | ((uint64_t)(1 + rng() % 2046) << 52);
        memcpy(&x, &bits, 8);
        y = (u01(rng) - 0.5) * 4.0;
      }
    }
    double got;
    if (!grt::glibc::pow_fast(x, y, &got)) continue;
    ++fast;
    double want = std::pow(x, y);
    if (memcmp(&got, &want, 8) != 0) {
      if (bad < 5) printf("# mismatch x=%a y=%a got=%a want=%a\n", x, y, got, want);
      ++bad;
    }
  }
  printf("%ld %ld %ld\n", n, fast, bad);
  return 0;
}
