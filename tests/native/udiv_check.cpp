// rtwm::udiv (csrc/rtw_math.hpp, the work-unit decode's division by a
// per-render constant) == n / d: every divisor 1..4096, the unit-decode
// divisors 64 * n_chunks up to 2^24, random divisors, with edge and random
// dividends.  Prints "udiv bad K/N"; exit 1 on a mismatch.
#include <cstdint>
#include <cstdio>
#include <random>
#include <vector>

#include "rtw_math.hpp"

int main() {
  std::mt19937_64 g(7);
  std::vector<uint32_t> ds;
  for (uint32_t d = 1; d <= 4096; ++d) ds.push_back(d);
  for (uint32_t k = 1; k <= (1u << 18); k += 37) ds.push_back(64u * k);
  for (int i = 0; i < 20000; ++i) ds.push_back((uint32_t)(g() | 1u) >> (g() % 32));
  ds.push_back(0xFFFFFFFFu);
  long bad = 0, n = 0;
  for (uint32_t d : ds) {
    if (d == 0) continue;
    const rtwm::UDivMagic mg = rtwm::udiv_magic(d);
    const uint32_t edge[] = {0u, 1u, d - 1u, d, d + 1u, 2u * d - 1u, 0x7FFFFFFFu, 0x80000000u, 0xFFFFFFFEu, 0xFFFFFFFFu};
    for (uint32_t x : edge) {
      ++n;
      if (rtwm::udiv(x, mg.m, mg.sh) != x / d) ++bad;
    }
    for (int i = 0; i < 64; ++i) {
      const uint32_t x = (uint32_t)g();
      ++n;
      if (rtwm::udiv(x, mg.m, mg.sh) != x / d) ++bad;
    }
  }
  std::printf("udiv bad %ld/%ld\n", bad, n);
  return bad ? 1 : 0;
}
