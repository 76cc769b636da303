// rtw_math.hpp — exactness-preserving arithmetic shortcuts used by the
// kernel.  Plain C++ (also compiles with g++), so tests/test_math_host.py can
// check each routine against the libm / IEEE operation it replaces.
//
// 1. sin_sign(a): the sign of sin(a), exactly, without evaluating sin.
//    CheckerTexture.value (texture.zig:79-82) only uses the SIGN of
//    sin(10x)*sin(10y)*sin(10z).  With k = rint(a/pi), a - k*pi is computed
//    from a 4-part split of pi (fdlibm's pio2_1/2/3/3t, doubled) with FMAs:
//    the first step is exact (Sterbenz), later steps leave an error far below
//    the smallest |a - k*pi| a double in range can have, so
//    sign(sin(a)) = (-1)^k * sign(r) is exact for |a| < 2^19 (else: libm sin).
//    A faithful sin (glibc, ocml, musl in Zig) returns that same sign.
// 2. div_rn(x, b, y): RN(x / b) given y = RN(1 / b) (Markstein):
//    q = RN(x*y) is within 1 ulp; r = x - b*q is exact (FMA);
//    RN(q + r*y) = RN(x / b).  Outside the normal range it falls back to x/b.
#pragma once
#include <cmath>
#include <cstdint>

#if defined(__HIPCC__)
#define RTW_HD __host__ __device__ __forceinline__
#else
#define RTW_HD inline
#endif

namespace rtwm {

// pi = P1 + P2 + P3 + P4 (P1..P3 have 33 significant bits: k*Pi exact for k < 2^20)
constexpr double kInvPi = 0.318309886183790671538;     // 0x3FD45F306DC9C883
constexpr double kP1 = 3.14159265346825122833e+00;      // 2 * pio2_1  0x400921FB54400000
constexpr double kP2 = 1.21542010126079319532e-10;      // 2 * pio2_2  0x3DE0B4611A600000
constexpr double kP3 = 4.04453249742233291160e-21;      // 2 * pio2_3  0x3BB3198A2E000000
constexpr double kP4 = 1.69568553207377991399e-31;      // 2 * pio2_3t 0x398B839A252049C1
constexpr double kSinSignMax = 524288.0;                // 2^19

// Out-of-range arguments (|a| >= 2^19, not produced by the cover scene): libm.
// Kept out of line so its constants do not occupy registers of the kernel.
#if defined(__HIPCC__)
static __host__ __device__ __noinline__
#else
inline
#endif
int sin_sign_libm(double a) {
  const double s = std::sin(a);
  return (s > 0) - (s < 0);
}

// -1, 0 or +1: the sign of sin(a).
RTW_HD int sin_sign(double a) {
  if (a == 0.0) return 0;  // sin(+-0) = +-0: product == 0, "not < 0"
  if (__builtin_expect(!(std::fabs(a) < kSinSignMax), 0)) return sin_sign_libm(a);
  const double k = std::rint(a * kInvPi);
  double r = std::fma(-k, kP1, a);
  r = std::fma(-k, kP2, r);
  r = std::fma(-k, kP3, r);
  r = std::fma(-k, kP4, r);
  const int s = (r > 0) - (r < 0);
  return (((int64_t)k) & 1) ? -s : s;
}

// CheckerTexture.value's test `sin(10x)*sin(10y)*sin(10z) < 0` (odd colour).
RTW_HD bool checker_odd(double ax, double ay, double az) {
  return sin_sign(ax) * sin_sign(ay) * sin_sign(az) < 0;
}

// The fallback must stay a real branch: an empty volatile asm stops the
// compiler from if-converting it (it would otherwise compute the full IEEE
// division sequence unconditionally and select).
#if defined(__HIP_DEVICE_COMPILE__)
#define RTW_NO_SPECULATE() asm volatile("")
#else
#define RTW_NO_SPECULATE() ((void)0)
#endif

// RN(x / b) from y = RN(1 / b).
RTW_HD double div_rn(double x, double b, double y) {
  const double q = x * y;
  const double r = std::fma(-q, b, x);
  double q1 = std::fma(r, y, q);
  const double aq = std::fabs(q1);
  if (__builtin_expect(!(aq < 0x1p1000 && aq > 0x1p-960), 0)) {
    RTW_NO_SPECULATE();
    q1 = x / b;
  }
  return q1;
}
RTW_HD float div_rn(float x, float b, float y) {
  const float q = x * y;
  const float r = std::fma(-q, b, x);
  float q1 = std::fma(r, y, q);
  const float aq = std::fabs(q1);
  if (__builtin_expect(!(aq < 0x1p120f && aq > 0x1p-100f), 0)) {
    RTW_NO_SPECULATE();
    q1 = x / b;
  }
  return q1;
}

// 3. sqrt_rn(x): f64 sqrt exactly as the compiler lowers __builtin_sqrt for
//    gfx9 (LLVM AMDGPU lowerFSQRTF64: v_rsq_f64, then Goldschmidt refinement
//    and two FMA residual corrections) without the input scaling (the scale
//    is 2^0 for x >= 2^-767) and without the +0/+inf select (x finite,
//    non-zero): for x in [2^-767, DBL_MAX] the same operations on the same
//    values, hence the same bits (tests/native/gpu_math_check.hip checks it
//    on the GPU).  Other x take the full builtin.
RTW_HD double sqrt_rn(double x) {
#if !defined(__HIP_DEVICE_COMPILE__)
  return std::sqrt(x);  // host passes (the kernels' device code is what runs)
#else
  if (__builtin_expect(!(x >= 0x1p-767 && x <= 0x1.fffffffffffffp+1023), 0)) {
    RTW_NO_SPECULATE();
    return __builtin_sqrt(x);
  }
  const double y = __builtin_amdgcn_rsq(x);
  double g = x * y, h = y * 0.5;
  const double r = std::fma(-h, g, 0.5);
  h = std::fma(h, r, h);
  g = std::fma(g, r, g);
  double d = std::fma(-g, g, x);
  g = std::fma(d, h, g);
  d = std::fma(-g, g, x);
  return std::fma(d, h, g);
#endif
}

// 4. udiv(n, m, sh): n / d for every 32-bit n, given the (m, sh) of
//    udiv_magic(d) (Granlund-Montgomery round-up method, Hacker's Delight
//    10-8): l = ceil(log2 d), m = floor(2^32 (2^l - d) / d) + 1,
//    q = (t + ((n - t) >> 1)) >> (l - 1) with t = mulhi(m, n); d = 1 is
//    encoded sh = 32 (q = n).  Five integer ops instead of the ~15 of the
//    compiler's division by a runtime divisor (the divisors are per-render
//    constants: the work-unit decode).  tests/test_math_host.py checks it.
struct UDivMagic {
  uint32_t m, sh;
};
inline UDivMagic udiv_magic(uint32_t d) {  // host side, d >= 1
  if (d == 1) return {0u, 32u};
  uint32_t l = 0;
  while ((1ull << l) < d) ++l;
  const uint64_t m = (((1ull << l) - d) << 32) / d + 1;
  return {(uint32_t)m, l - 1};
}
RTW_HD uint32_t udiv(uint32_t n, uint32_t m, uint32_t sh) {
  const uint32_t t = (uint32_t)(((uint64_t)m * n) >> 32);
  const uint32_t q = (t + ((n - t) >> 1)) >> (sh & 31u);
  return sh == 32u ? n : q;
}

}  // namespace rtwm
