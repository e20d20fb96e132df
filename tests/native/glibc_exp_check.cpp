// Host build of gr_raytracer_amd/csrc/device/glibc_math.h exp_() checked against glibc
// exp, bit for bit (driven by tests/test_glibc_math.py).  Prints: samples fast mismatches
// ("fast" = all samples: exp_ is defined on the whole domain).
#include <cinttypes>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <random>

#include "glibc_math.h"

int main(int argc, char** argv) {
  const int mode = atoi(argv[1]);
  const long n = atol(argv[2]);
  std::mt19937_64 rng(777 + mode);
  std::uniform_real_distribution<double> u01(0.0, 1.0);
  long bad = 0;
  for (long k = 0; k < n; ++k) {
    double x;
    switch (mode) {
      case 0: {  // VolumetricDisc vertical falloff: -(h / thickness)^2
        double q = u01(rng) * 4.0;
        x = -(q * q);
        break;
      }
      case 1: {  // boundary falloff: -1 / max(d^2, 1e-4)
        double d = u01(rng) * 12.0;
        x = -1.0 / std::fmax(d * d, 0.0001);
        break;
      }
      case 2:  // sample attenuation -d_s * density * sigma, over many decades
        x = -std::exp(u01(rng) * 60.0 - 50.0);
        break;
      case 3:  // subnormal results and overflow edge
        x = (k & 1) ? -745.5 + u01(rng) * 45.0 : 700.0 + u01(rng) * 10.0;
        break;
      default: {  // random bit patterns (all exponents, both signs, inf / nan)
        uint64_t bits = rng();
        memcpy(&x, &bits, 8);
      }
    }
    double got = grt::glibc::exp_(x);
    double want = std::exp(x);
    bool same = memcmp(&got, &want, 8) == 0 || (std::isnan(got) && std::isnan(want));
    if (!same) {
      if (bad < 5) printf("# mismatch x=%a got=%a want=%a\n", x, got, want);
      ++bad;
    }
  }
  printf("%ld %ld %ld\n", n, n, bad);
  return 0;
}
