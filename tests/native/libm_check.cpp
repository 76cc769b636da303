// Host build of the product's Tier-B libm (csrc/rtw_libm.hpp) against the
// oracle's independent restatement (oracle/ro_libm.h) — must agree bit for
// bit — and against glibc (must be within 1 ulp).  Inputs: random doubles
// over many magnitudes, the exact multiples/cancellation points of pi/2 that
// select the argument-reduction branches, and special values.
// Usage: libm_check N seed  -> "cases C mismatch M maxulp U"
#include <cinttypes>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <random>
#include <vector>

#include "ro_libm.h"
#include "rtw_libm.hpp"

static int64_t ulps(double a, double b) {
  if (std::isnan(a) && std::isnan(b)) return 0;
  int64_t ia, ib;
  std::memcpy(&ia, &a, 8);
  std::memcpy(&ib, &b, 8);
  if ((ia < 0) != (ib < 0)) return a == b ? 0 : INT64_MAX;
  return ia > ib ? ia - ib : ib - ia;
}
static bool same(double a, double b) {
  uint64_t x, y;
  std::memcpy(&x, &a, 8);
  std::memcpy(&y, &b, 8);
  return x == y || (std::isnan(a) && std::isnan(b));
}

int main(int argc, char** argv) {
  const long n = argc > 1 ? atol(argv[1]) : 1000000;
  std::mt19937_64 g(argc > 2 ? atol(argv[2]) : 1);
  std::uniform_real_distribution<double> U(-1.0, 1.0), E(-8.0, 6.5);
  std::vector<double> xs;
  for (long i = 0; i < n; ++i) xs.push_back(U(g) * std::pow(10.0, E(g)));
  const double pio2 = 1.57079632679489661923;
  for (int k = -64; k <= 64; ++k)  // branch points of __rem_pio2
    for (int d = -3; d <= 3; ++d) xs.push_back(std::nextafter(k * pio2, d < 0 ? -INFINITY : INFINITY) + d * 1e-16 * k);
  const double sp[] = {0.0, -0.0, 1.0, -1.0, 0.5, -0.5, 1e-300, -1e-300, 5e-324, INFINITY, -INFINITY, NAN,
                       0.4375, 1.1875, 2.4375, 0x1p66, 0x1p-27, 0x1p20 * pio2 * 0.999};
  for (double s : sp) xs.push_back(s);
  long cases = 0, mismatch = 0;
  int64_t maxulp = 0;
  auto chk = [&](double a, double b, double ref) {
    ++cases;
    if (!same(a, b)) {
      if (mismatch < 5) printf("mismatch %.17g %.17g\n", a, b);
      ++mismatch;
    }
    const int64_t u = ulps(a, ref);
    if (u > maxulp) maxulp = u;
  };
  for (size_t i = 0; i < xs.size(); ++i) {
    const double x = xs[i];
    chk(rtwl::sin(x), ro_sin(x), std::sin(x));
    chk(rtwl::cos(x), ro_cos(x), std::cos(x));
    const double y = xs[(i * 7919 + 13) % xs.size()];
    chk(rtwl::atan2(y, x), ro_atan2(y, x), std::atan2(y, x));
    const double c = std::fmod(x, 1.0);
    chk(rtwl::acos(c), ro_acos(c), std::acos(c));
  }
  printf("cases %ld mismatch %ld maxulp %" PRId64 "\n", cases, mismatch, maxulp);
  return mismatch == 0 && maxulp <= 1 ? 0 : 1;
}
