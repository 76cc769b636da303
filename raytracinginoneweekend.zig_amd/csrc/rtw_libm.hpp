// rtw_libm.hpp — the transcendental functions of the general-world path,
// host + device (gfx950), with results defined bit for bit: the musl
// (fdlibm-derived) algorithms that Zig 0.14's std.math / compiler_rt port —
// sin/cos (@sin in texture.zig:80 and :104; std.math.sin/cos in RotateY.init,
// hittable.zig:516-517) and atan2/acos (Sphere.getSphereUv, hittable.zig:145-150).
//
// The device's own libm (ocml) is faithful but not identical to musl: one
// ulp of atan2 moves a texel index floor(u * width), one ulp of sin moves a
// noise colour.  The world kernel and the Tier-B oracle (oracle/ro_libm.h,
// an independent C restatement of the same algorithms) therefore share this
// definition; tests/test_world_cpu.py::test_tierb_libm_product_equals_oracle_and_glibc
// (driving tests/native/libm_check.cpp) checks host builds of both against
// each other bit for bit and against glibc (<= 1 ulp).  Compiled with
// -ffp-contract=off: one IEEE operation per source operation.  sin/cos with
// |x| >= 2^20 * pi/2 (the Payne-Hanek range, never produced by the
// reference's scenes) return the platform libm's value.
#pragma once
#include <cmath>
#include <cstdint>
#include <cstring>

#if defined(__HIPCC__)
#define RTWL_HD __host__ __device__ __forceinline__
#else
#define RTWL_HD inline
#endif

namespace rtwl {

RTWL_HD uint64_t bits(double x) {
  uint64_t u;
  std::memcpy(&u, &x, 8);
  return u;
}
RTWL_HD double from_bits(uint64_t u) {
  double x;
  std::memcpy(&x, &u, 8);
  return x;
}
RTWL_HD uint32_t hi(double x) { return (uint32_t)(bits(x) >> 32); }
RTWL_HD uint32_t lo(double x) { return (uint32_t)bits(x); }

// __sin / __cos kernels on [-pi/4, pi/4] (x + y, |y| < ulp(x)/2).
RTWL_HD double k_sin(double x, double y, int iy) {
  constexpr double S1 = -1.66666666666666324348e-01, S2 = 8.33333333332248946124e-03,
                   S3 = -1.98412698298579493134e-04, S4 = 2.75573137070700676789e-06,
                   S5 = -2.50507602534068634195e-08, S6 = 1.58969099521155010221e-10;
  const double z = x * x, w = z * z;
  const double r = S2 + z * (S3 + z * S4) + z * w * (S5 + z * S6);
  const double v = z * x;
  if (iy == 0) return x + v * (S1 + z * r);
  return x - ((z * (0.5 * y - v * r) - y) - v * S1);
}
RTWL_HD double k_cos(double x, double y) {
  constexpr double C1 = 4.16666666666666019037e-02, C2 = -1.38888888888741095749e-03,
                   C3 = 2.48015872894767294178e-05, C4 = -2.75573143513906633035e-07,
                   C5 = 2.08757232129817482790e-09, C6 = -1.13596475577881948265e-11;
  const double z = x * x;
  const double w2 = z * z;
  const double r = z * (C1 + z * (C2 + z * C3)) + w2 * w2 * (C4 + z * (C5 + z * C6));
  const double hz = 0.5 * z;
  const double w = 1.0 - hz;
  return w + (((1.0 - w) - hz) + (z * r - x * y));
}

// x = n * pi/2 + (y0 + y1); false for |x| >= 2^20 * pi/2.
RTWL_HD bool rem_pio2(double x, double& y0, double& y1, int& n) {
  constexpr double toint = 6755399441055744.0;  // 1.5 / DBL_EPSILON
  constexpr double pio4 = 0x1.921fb54442d18p-1, invpio2 = 6.36619772367581382433e-01,
                   p1 = 1.57079632673412561417e+00, p1t = 6.07710050650619224932e-11,
                   p2 = 6.07710050630396597660e-11, p2t = 2.02226624879595063154e-21,
                   p3 = 2.02226624871116645580e-21, p3t = 8.47842766036889956997e-32;
  const uint64_t u = bits(x);
  const bool neg = (u >> 63) != 0;
  const uint32_t ix = (uint32_t)(u >> 32) & 0x7fffffffu;
  // Small multiples of pi/2 (|x| ~<= 9pi/4) away from the cancelling cases:
  // one subtraction of k * (pi/2 split in two).
  int k = 0;
  if (ix <= 0x400f6a7au) {
    if ((ix & 0xfffffu) != 0x921fbu) k = ix <= 0x4002d97cu ? 1 : 2;
  } else if (ix <= 0x401c463bu) {
    if (ix <= 0x4015fdbcu) {
      if (ix != 0x4012d97cu) k = 3;
    } else if (ix != 0x401921fbu) {
      k = 4;
    }
  }
  if (k != 0) {
    const double kd = (double)k;
    if (!neg) {
      const double z = x - kd * p1;
      y0 = z - kd * p1t;
      y1 = (z - y0) - kd * p1t;
      n = k;
    } else {
      const double z = x + kd * p1;
      y0 = z + kd * p1t;
      y1 = (z - y0) + kd * p1t;
      n = -k;
    }
    return true;
  }
  if (ix > 0x401c463bu && ix >= 0x413921fbu) return false;  // Payne-Hanek range
  double fn = (x * invpio2 + toint) - toint;                // rint(x / (pi/2))
  int nn = (int)fn;
  double r = x - fn * p1;
  double w = fn * p1t;
  if (r - w < -pio4) {
    nn--;
    fn--;
    r = x - fn * p1;
    w = fn * p1t;
  } else if (r - w > pio4) {
    nn++;
    fn++;
    r = x - fn * p1;
    w = fn * p1t;
  }
  y0 = r - w;
  const int ex = (int)(ix >> 20);
  if (ex - (int)((bits(y0) >> 52) & 0x7ff) > 16) {
    double t = r;
    w = fn * p2;
    r = t - w;
    w = fn * p2t - ((t - r) - w);
    y0 = r - w;
    if (ex - (int)((bits(y0) >> 52) & 0x7ff) > 49) {
      t = r;
      w = fn * p3;
      r = t - w;
      w = fn * p3t - ((t - r) - w);
      y0 = r - w;
    }
  }
  y1 = (r - y0) - w;
  n = nn;
  return true;
}

RTWL_HD double sin(double x) {
  const uint32_t ix = hi(x) & 0x7fffffffu;
  if (ix <= 0x3fe921fbu) return ix < 0x3e500000u ? x : k_sin(x, 0.0, 0);
  if (ix >= 0x7ff00000u) return x - x;
  double y0, y1;
  int n;
  if (!rem_pio2(x, y0, y1, n)) return ::sin(x);
  switch (n & 3) {
    case 0: return k_sin(y0, y1, 1);
    case 1: return k_cos(y0, y1);
    case 2: return -k_sin(y0, y1, 1);
    default: return -k_cos(y0, y1);
  }
}

RTWL_HD double cos(double x) {
  const uint32_t ix = hi(x) & 0x7fffffffu;
  if (ix <= 0x3fe921fbu) return ix < 0x3e46a09eu ? 1.0 : k_cos(x, 0.0);
  if (ix >= 0x7ff00000u) return x - x;
  double y0, y1;
  int n;
  if (!rem_pio2(x, y0, y1, n)) return ::cos(x);
  switch (n & 3) {
    case 0: return k_cos(y0, y1);
    case 1: return -k_sin(y0, y1, 1);
    case 2: return -k_cos(y0, y1);
    default: return k_sin(y0, y1, 1);
  }
}

RTWL_HD double atan(double x) {
  constexpr double hi_[4] = {4.63647609000806093515e-01, 7.85398163397448278999e-01, 9.82793723247329054082e-01,
                             1.57079632679489655800e+00};
  constexpr double lo_[4] = {2.26987774529616870924e-17, 3.06161699786838301793e-17, 1.39033110312309984516e-17,
                             6.12323399573676603587e-17};
  constexpr double T0 = 3.33333333333329318027e-01, T1 = -1.99999999998764832476e-01,
                   T2 = 1.42857142725034663711e-01, T3 = -1.11111104054623557880e-01,
                   T4 = 9.09088713343650656196e-02, T5 = -7.69187620504482999495e-02,
                   T6 = 6.66107313738753120669e-02, T7 = -5.83357013379057348645e-02,
                   T8 = 4.97687799461593236017e-02, T9 = -3.65315727442169155270e-02,
                   T10 = 1.62858201153657823623e-02;
  const uint32_t hx = hi(x);
  const bool neg = (hx >> 31) != 0;
  const uint32_t ix = hx & 0x7fffffffu;
  int id;
  if (ix >= 0x44100000u) {  // |x| >= 2^66
    if (x != x) return x;
    const double z = hi_[3] + 0x1p-120;
    return neg ? -z : z;
  }
  if (ix < 0x3fdc0000u) {   // |x| < 0.4375
    if (ix < 0x3e400000u) return x;
    id = -1;
  } else {
    x = std::fabs(x);
    if (ix < 0x3ff30000u) {
      if (ix < 0x3fe60000u) {
        id = 0;
        x = (2.0 * x - 1.0) / (2.0 + x);
      } else {
        id = 1;
        x = (x - 1.0) / (x + 1.0);
      }
    } else if (ix < 0x40038000u) {
      id = 2;
      x = (x - 1.5) / (1.0 + 1.5 * x);
    } else {
      id = 3;
      x = -1.0 / x;
    }
  }
  const double z = x * x, w = z * z;
  const double s1 = z * (T0 + w * (T2 + w * (T4 + w * (T6 + w * (T8 + w * T10)))));
  const double s2 = w * (T1 + w * (T3 + w * (T5 + w * (T7 + w * T9))));
  if (id < 0) return x - x * (s1 + s2);
  const double r = hi_[id] - (x * (s1 + s2) - lo_[id] - x);
  return neg ? -r : r;
}

RTWL_HD double atan2(double y, double x) {
  constexpr double pi = 3.1415926535897931160E+00, pi_lo = 1.2246467991473531772E-16;
  if (x != x || y != y) return x + y;
  uint32_t ix = hi(x), iy = hi(y);
  const uint32_t lx = lo(x), ly = lo(y);
  if (((ix - 0x3ff00000u) | lx) == 0) return atan(y);  // x == 1
  const uint32_t m = ((iy >> 31) & 1u) | ((ix >> 30) & 2u);
  ix &= 0x7fffffffu;
  iy &= 0x7fffffffu;
  if ((iy | ly) == 0) return m == 0 || m == 1 ? y : (m == 2 ? pi : -pi);
  if ((ix | lx) == 0) return (m & 1u) ? -pi / 2 : pi / 2;
  if (ix == 0x7ff00000u) {
    if (iy == 0x7ff00000u) {
      const double q[4] = {pi / 4, -pi / 4, 3 * pi / 4, -3 * pi / 4};
      return q[m];
    }
    const double q[4] = {0.0, -0.0, pi, -pi};
    return q[m];
  }
  if (ix + (64u << 20) < iy || iy == 0x7ff00000u) return (m & 1u) ? -pi / 2 : pi / 2;
  const double z = ((m & 2u) && iy + (64u << 20) < ix) ? 0.0 : atan(std::fabs(y / x));
  switch (m) {
    case 0: return z;
    case 1: return -z;
    case 2: return pi - (z - pi_lo);
    default: return (z - pi_lo) - pi;
  }
}

RTWL_HD double acos_r(double z) {
  constexpr double pS0 = 1.66666666666666657415e-01, pS1 = -3.25565818622400915405e-01,
                   pS2 = 2.01212532134862925881e-01, pS3 = -4.00555345006794114027e-02,
                   pS4 = 7.91534994289814532176e-04, pS5 = 3.47933107596021167570e-05,
                   qS1 = -2.40339491173441421878e+00, qS2 = 2.02094576023350569471e+00,
                   qS3 = -6.88283971605453293030e-01, qS4 = 7.70381505559019352791e-02;
  const double p = z * (pS0 + z * (pS1 + z * (pS2 + z * (pS3 + z * (pS4 + z * pS5)))));
  const double q = 1.0 + z * (qS1 + z * (qS2 + z * (qS3 + z * qS4)));
  return p / q;
}
RTWL_HD double acos(double x) {
  constexpr double pio2_hi = 1.57079632679489655800e+00, pio2_lo = 6.12323399573676603587e-17;
  const uint32_t hx = hi(x), ix = hx & 0x7fffffffu;
  if (ix >= 0x3ff00000u) {
    if (((ix - 0x3ff00000u) | lo(x)) == 0) return (hx >> 31) ? 2 * pio2_hi + 0x1p-120 : 0.0;
    return 0 / (x - x);
  }
  if (ix < 0x3fe00000u) {
    if (ix <= 0x3c600000u) return pio2_hi + 0x1p-120;
    return pio2_hi - (x - (pio2_lo - x * acos_r(x * x)));
  }
  if (hx >> 31) {
    const double z = (1.0 + x) * 0.5;
    const double s = std::sqrt(z);
    const double w = acos_r(z) * s - pio2_lo;
    return 2 * (pio2_hi - (s + w));
  }
  const double z = (1.0 - x) * 0.5;
  const double s = std::sqrt(z);
  const double df = from_bits(bits(s) & 0xFFFFFFFF00000000ull);
  const double c = (z - df * df) / (s + df);
  const double w = acos_r(z) * s + c;
  return 2 * (df + w);
}

}  // namespace rtwl
