// Host build of glibc_math.h's sincos_fast (and its branch-free and region-B forms)
// checked against glibc sincos, bit for bit.
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <random>

#include "glibc_math.h"

extern "C" void sincos(double, double*, double*);

int main(int argc, char** argv) {
  const int mode = atoi(argv[1]);
  const long n = atol(argv[2]);
  std::mt19937_64 rng(4242 + mode);
  std::uniform_real_distribution<double> u01(0.0, 1.0);
  long fast = 0, bad = 0;
  for (long k = 0; k < n; ++k) {
    double x;
    switch (mode) {
      case 0: x = (u01(rng) * 1.4 - 0.2) * 3.141592653589793; break;
      case 1: x = (u01(rng) - 0.5) * 40.0; break;
      case 2: x = std::ldexp(u01(rng) - 0.5, (int)(rng() % 60) - 40); break;
      case 3: x = 1.5707963267948966 + (u01(rng) - 0.5) * 1e-6; break;
      case 6: x = 1.5707963267948966 + (u01(rng) - 0.5) * 0.3; break;  // both sides of TAYLOR_MAX
      case 5: x = (u01(rng) * 2.0 - 1.0) * 3.141592653589793; break;  // VolumetricDisc phi
      default: x = (u01(rng) - 0.5) * 2e8;
    }
    double gs, gc, ws, wc, us, uc;
    if (!grt::glibc::sincos_fast(x, &gs, &gc)) continue;
    ++fast;
    sincos(x, &ws, &wc);
    // the branch-free variant must return the same bits on the same domain
    const bool uok = grt::glibc::sincos_fast_uniform(x, &us, &uc);
    // and so must the straight-line region-B form wherever it claims the case
    double bs = ws, bc = wc;
    if (grt::glibc::sincos_b_table_ok(x)) grt::glibc::sincos_b_table(x, &bs, &bc);
    if (grt::glibc::sincos_b_taylor_ok(x)) grt::glibc::sincos_b_taylor(x, &bs, &bc);
    if (memcmp(&gs, &ws, 8) != 0 || memcmp(&gc, &wc, 8) != 0 || !uok || memcmp(&us, &ws, 8) != 0 ||
        memcmp(&uc, &wc, 8) != 0 || memcmp(&bs, &ws, 8) != 0 || memcmp(&bc, &wc, 8) != 0) {
      if (bad < 5) printf("# mismatch x=%a got=(%a,%a) uniform=(%a,%a) want=(%a,%a)\n", x, gs, gc, us, uc, ws, wc);
      ++bad;
    }
  }
  printf("%ld %ld %ld\n", n, fast, bad);
  return 0;
}
