// Host build of glibc_math.h's sin_fast / cos_fast checked against glibc, bit for bit
// (driven by tests/test_glibc_math.py).  Prints: samples fast mismatches.
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
  long fast = 0, bad = 0;
  for (long k = 0; k < n; ++k) {
    double x;
    switch (mode) {
      case 0: x = (u01(rng) * 1.4 - 0.2) * 3.141592653589793; break;    // theta of a ray
      case 1: x = (u01(rng) - 0.5) * 40.0; break;                        // several periods
      case 2: x = std::ldexp(u01(rng) - 0.5, (int)(rng() % 60) - 40); break;  // magnitudes 2^-41..2^19
      case 3: x = 1.5707963267948966 + (u01(rng) - 0.5) * 1e-6; break;   // near pi/2
      default: x = (u01(rng) - 0.5) * 2e8;                               // up to the reduction limit
    }
    double gs, gc;
    bool fs = grt::glibc::sin_fast(x, &gs), fc = grt::glibc::cos_fast(x, &gc);
    if (fs) {
      ++fast;
      double w = std::sin(x);
      if (memcmp(&gs, &w, 8) != 0) {
        if (bad < 5) printf("# sin mismatch x=%a got=%a want=%a\n", x, gs, w);
        ++bad;
      }
    }
    if (fc) {
      double w = std::cos(x);
      if (memcmp(&gc, &w, 8) != 0) {
        if (bad < 5) printf("# cos mismatch x=%a got=%a want=%a\n", x, gc, w);
        ++bad;
      }
    }
  }
  printf("%ld %ld %ld\n", n, fast, bad);
  return 0;
}
