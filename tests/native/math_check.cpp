// Host check of csrc/rtw_math.hpp against the libm / IEEE operations it
// replaces (built and run by tests/test_math_host.py).
#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstring>
#include <random>

#include "rtw_math.hpp"

static int sgn(double v) { return (v > 0) - (v < 0); }
static uint64_t bits(double d) { uint64_t u; std::memcpy(&u, &d, 8); return u; }
static double from_bits(uint64_t u) { double d; std::memcpy(&d, &u, 8); return d; }

int main(int argc, char** argv) {
  const long N = argc > 1 ? std::atol(argv[1]) : 2000000;
  std::mt19937_64 g(12345);
  long bad_sin = 0, bad_div = 0, bad_divf = 0, n_sin = 0, n_div = 0;
  // constants
  if (bits(rtwm::kP1) != 0x400921FB54400000ULL || bits(rtwm::kP2) != 0x3DE0B4611A600000ULL ||
      bits(rtwm::kP3) != 0x3BB3198A2E000000ULL || bits(rtwm::kP4) != 0x398B839A252049C1ULL ||
      bits(rtwm::kInvPi) != 0x3FD45F306DC9C883ULL) {
    std::printf("constants wrong\n");
    return 1;
  }
  std::uniform_real_distribution<double> U(-20000.0, 20000.0);
  for (long i = 0; i < N; ++i) {  // random arguments
    const double a = U(g);
    n_sin++;
    if (rtwm::sin_sign(a) != sgn(std::sin(a))) bad_sin++;
  }
  for (long k = -200000; k <= 200000; ++k) {  // the doubles nearest k*pi, +-8 ulps
    const double c = (double)k * M_PI;
    for (int d = -8; d <= 8; ++d) {
      const double a = k == 0 ? d * 1e-300 : from_bits(bits(c) + d);
      n_sin++;
      if (rtwm::sin_sign(a) != sgn(std::sin(a))) bad_sin++;
    }
  }
  // division
  std::uniform_int_distribution<int> E(-60, 60);
  std::uniform_int_distribution<uint64_t> M(0, (1ULL << 52) - 1);
  for (long i = 0; i < N; ++i) {
    const double x = std::ldexp(1.0 + std::ldexp((double)M(g), -52), E(g)) * ((g() & 1) ? -1 : 1);
    double b = std::ldexp(1.0 + std::ldexp((double)M(g), -52), E(g));
    if ((i & 7) == 0) b = from_bits((bits(b) | 0x000FFFFFFFFFFFFFULL) - (g() & 3));  // near all-ones mantissas
    const double y = 1.0 / b;
    n_div++;
    if (bits(rtwm::div_rn(x, b, y)) != bits(x / b)) bad_div++;
    const float xf = (float)x, bf = (float)b;
    if (rtwm::div_rn(xf, bf, 1.0f / bf) != xf / bf) bad_divf++;
  }
  // small integers / typical operands of the kernel (W-1, radii, |d|^2)
  for (int w = 2; w < 5000; ++w) {
    const double b = w - 1.0, y = 1.0 / b;
    for (int t = 0; t < 200; ++t) {
      const double x = (double)(g() % 5000) + std::ldexp((double)M(g), -52);
      n_div++;
      if (bits(rtwm::div_rn(x, b, y)) != bits(x / b)) bad_div++;
    }
  }
  std::printf("sin_sign %ld/%ld bad; div_rn f64 %ld/%ld bad; div_rn f32 %ld bad\n", bad_sin, n_sin, bad_div, n_div,
              bad_divf);
  return (bad_sin || bad_div || bad_divf) ? 1 : 0;
}
