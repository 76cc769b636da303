/*
 * ro_libm.h — TEST INFRASTRUCTURE ONLY (part of the CPU oracle).
 *
 * The transcendental functions the general-world path calls, restated from
 * musl libc's fdlibm-derived implementations, which Zig 0.14's std.math and
 * compiler_rt port function for function:
 *   sin, cos   — @sin/@cos (texture.zig:80 checker, :104 noise texture;
 *                RotateY.init hittable.zig:516-517 uses std.math.sin/cos)
 *   atan2, acos — Sphere.getSphereUv (hittable.zig:145-150)
 * (musl src/math/__sin.c, __cos.c, __rem_pio2.c (|x| < 2^20*pi/2 paths),
 * sin.c, cos.c, atan.c, atan2.c, acos.c.)
 *
 * Why restate instead of calling the host libm: the GPU path and the Tier-B
 * oracle must evaluate these with bit-identical results (a texel index
 * floor(u * width) flips with one ulp of atan2), so Tier B DEFINES them as
 * this algorithm; the product (raytracinginoneweekend.zig_amd/csrc/
 * rtw_libm.hpp) implements the same algorithm independently.  Each function
 * is within 1 ulp of glibc (tests/test_world_cpu.py::
 * test_tierb_libm_product_equals_oracle_and_glibc, tests/native/libm_check.cpp);
 * |x| >= 2^20*pi/2 for sin/cos
 * (never produced by the reference's scenes) falls back to the host libm.
 * Compiled with -ffp-contract=off: one IEEE operation per source operation.
 */
#ifndef RO_LIBM_H
#define RO_LIBM_H
#include <math.h>
#include <stdint.h>
#include <string.h>

static inline uint64_t rol_bits(double x) { uint64_t u; memcpy(&u, &x, 8); return u; }
static inline double rol_from(uint64_t u) { double x; memcpy(&x, &u, 8); return x; }
static inline uint32_t rol_hi(double x) { return (uint32_t)(rol_bits(x) >> 32); }
static inline uint32_t rol_lo(double x) { return (uint32_t)rol_bits(x); }

/* musl __sin.c */
static inline double rol_ksin(double x, double y, int iy) {
  const double S1 = -1.66666666666666324348e-01, S2 = 8.33333333332248946124e-03,
               S3 = -1.98412698298579493134e-04, S4 = 2.75573137070700676789e-06,
               S5 = -2.50507602534068634195e-08, S6 = 1.58969099521155010221e-10;
  const double z = x * x, w = z * z;
  const double r = S2 + z * (S3 + z * S4) + z * w * (S5 + z * S6);
  const double v = z * x;
  if (iy == 0) return x + v * (S1 + z * r);
  return x - ((z * (0.5 * y - v * r) - y) - v * S1);
}

/* musl __cos.c */
static inline double rol_kcos(double x, double y) {
  const double C1 = 4.16666666666666019037e-02, C2 = -1.38888888888741095749e-03,
               C3 = 2.48015872894767294178e-05, C4 = -2.75573143513906633035e-07,
               C5 = 2.08757232129817482790e-09, C6 = -1.13596475577881948265e-11;
  const double z = x * x;
  double w = z * z;
  const double r = z * (C1 + z * (C2 + z * C3)) + w * w * (C4 + z * (C5 + z * C6));
  const double hz = 0.5 * z;
  w = 1.0 - hz;
  return w + (((1.0 - w) - hz) + (z * r - x * y));
}

/* musl __rem_pio2.c for |x| < 2^20*pi/2; returns n, or INT32_MIN when the
 * argument needs the large-argument (Payne-Hanek) path. */
static inline int32_t rol_rem_pio2(double x, double *y) {
  const double toint = 1.5 / 2.220446049250313080847e-16, pio4 = 0x1.921fb54442d18p-1,
               invpio2 = 6.36619772367581382433e-01, pio2_1 = 1.57079632673412561417e+00,
               pio2_1t = 6.07710050650619224932e-11, pio2_2 = 6.07710050630396597660e-11,
               pio2_2t = 2.02226624879595063154e-21, pio2_3 = 2.02226624871116645580e-21,
               pio2_3t = 8.47842766036889956997e-32;
  const uint64_t ui = rol_bits(x);
  const int sign = (int)(ui >> 63);
  const uint32_t ix = (uint32_t)(ui >> 32) & 0x7fffffff;
  double z, w, t, r, fn;
  int32_t n;
  if (ix <= 0x400f6a7a) {               /* |x| ~<= 5pi/4 */
    if ((ix & 0xfffff) == 0x921fb) goto medium; /* |x| ~= pi/2 or 2pi/2 */
    if (ix <= 0x4002d97c) {             /* |x| ~<= 3pi/4 */
      if (!sign) {
        z = x - pio2_1;
        y[0] = z - pio2_1t;
        y[1] = (z - y[0]) - pio2_1t;
        return 1;
      }
      z = x + pio2_1;
      y[0] = z + pio2_1t;
      y[1] = (z - y[0]) + pio2_1t;
      return -1;
    }
    if (!sign) {
      z = x - 2 * pio2_1;
      y[0] = z - 2 * pio2_1t;
      y[1] = (z - y[0]) - 2 * pio2_1t;
      return 2;
    }
    z = x + 2 * pio2_1;
    y[0] = z + 2 * pio2_1t;
    y[1] = (z - y[0]) + 2 * pio2_1t;
    return -2;
  }
  if (ix <= 0x401c463b) {               /* |x| ~<= 9pi/4 */
    if (ix <= 0x4015fdbc) {             /* |x| ~<= 7pi/4 */
      if (ix == 0x4012d97c) goto medium; /* |x| ~= 3pi/2 */
      if (!sign) {
        z = x - 3 * pio2_1;
        y[0] = z - 3 * pio2_1t;
        y[1] = (z - y[0]) - 3 * pio2_1t;
        return 3;
      }
      z = x + 3 * pio2_1;
      y[0] = z + 3 * pio2_1t;
      y[1] = (z - y[0]) + 3 * pio2_1t;
      return -3;
    }
    if (ix == 0x401921fb) goto medium;  /* |x| ~= 4pi/2 */
    if (!sign) {
      z = x - 4 * pio2_1;
      y[0] = z - 4 * pio2_1t;
      y[1] = (z - y[0]) - 4 * pio2_1t;
      return 4;
    }
    z = x + 4 * pio2_1;
    y[0] = z + 4 * pio2_1t;
    y[1] = (z - y[0]) + 4 * pio2_1t;
    return -4;
  }
  if (ix >= 0x413921fb) return INT32_MIN; /* large argument */
medium:
  fn = (x * invpio2 + toint) - toint;     /* rint(x / (pi/2)) */
  n = (int32_t)fn;
  r = x - fn * pio2_1;
  w = fn * pio2_1t;                       /* 1st round, good to 85 bits */
  if (r - w < -pio4) {
    n--;
    fn--;
    r = x - fn * pio2_1;
    w = fn * pio2_1t;
  } else if (r - w > pio4) {
    n++;
    fn++;
    r = x - fn * pio2_1;
    w = fn * pio2_1t;
  }
  y[0] = r - w;
  {
    const uint32_t ey = (uint32_t)(rol_bits(y[0]) >> 52) & 0x7ff, ex = ix >> 20;
    if ((int)ex - (int)ey > 16) {         /* 2nd round, good to 118 bits */
      t = r;
      w = fn * pio2_2;
      r = t - w;
      w = fn * pio2_2t - ((t - r) - w);
      y[0] = r - w;
      const uint32_t ey2 = (uint32_t)(rol_bits(y[0]) >> 52) & 0x7ff;
      if ((int)ex - (int)ey2 > 49) {      /* 3rd round, good to 151 bits */
        t = r;
        w = fn * pio2_3;
        r = t - w;
        w = fn * pio2_3t - ((t - r) - w);
        y[0] = r - w;
      }
    }
  }
  y[1] = (r - y[0]) - w;
  return n;
}

/* musl sin.c */
static inline double ro_sin(double x) {
  const uint32_t ix = rol_hi(x) & 0x7fffffff;
  double y[2];
  if (ix <= 0x3fe921fb) {               /* |x| ~< pi/4 */
    if (ix < 0x3e500000) return x;      /* |x| < 2^-26 */
    return rol_ksin(x, 0.0, 0);
  }
  if (ix >= 0x7ff00000) return x - x;   /* Inf or NaN */
  const int32_t n = rol_rem_pio2(x, y);
  if (n == INT32_MIN) return sin(x);
  switch (n & 3) {
    case 0: return rol_ksin(y[0], y[1], 1);
    case 1: return rol_kcos(y[0], y[1]);
    case 2: return -rol_ksin(y[0], y[1], 1);
    default: return -rol_kcos(y[0], y[1]);
  }
}

/* musl cos.c */
static inline double ro_cos(double x) {
  const uint32_t ix = rol_hi(x) & 0x7fffffff;
  double y[2];
  if (ix <= 0x3fe921fb) {               /* |x| ~< pi/4 */
    if (ix < 0x3e46a09e) return 1.0;    /* |x| < 2^-27 * sqrt(2) */
    return rol_kcos(x, 0);
  }
  if (ix >= 0x7ff00000) return x - x;
  const int32_t n = rol_rem_pio2(x, y);
  if (n == INT32_MIN) return cos(x);
  switch (n & 3) {
    case 0: return rol_kcos(y[0], y[1]);
    case 1: return -rol_ksin(y[0], y[1], 1);
    case 2: return -rol_kcos(y[0], y[1]);
    default: return rol_ksin(y[0], y[1], 1);
  }
}

/* musl atan.c */
static inline double ro_atan(double x) {
  static const double atanhi[] = {4.63647609000806093515e-01, 7.85398163397448278999e-01,
                                  9.82793723247329054082e-01, 1.57079632679489655800e+00};
  static const double atanlo[] = {2.26987774529616870924e-17, 3.06161699786838301793e-17,
                                  1.39033110312309984516e-17, 6.12323399573676603587e-17};
  static const double aT[] = {3.33333333333329318027e-01,  -1.99999999998764832476e-01,
                              1.42857142725034663711e-01,  -1.11111104054623557880e-01,
                              9.09088713343650656196e-02,  -7.69187620504482999495e-02,
                              6.66107313738753120669e-02,  -5.83357013379057348645e-02,
                              4.97687799461593236017e-02,  -3.65315727442169155270e-02,
                              1.62858201153657823623e-02};
  uint32_t ix = rol_hi(x);
  const uint32_t sign = ix >> 31;
  int id;
  ix &= 0x7fffffff;
  if (ix >= 0x44100000) {               /* |x| >= 2^66 */
    if (isnan(x)) return x;
    const double z = atanhi[3] + 0x1p-120;
    return sign ? -z : z;
  }
  if (ix < 0x3fdc0000) {                /* |x| < 0.4375 */
    if (ix < 0x3e400000) return x;      /* |x| < 2^-27 */
    id = -1;
  } else {
    x = fabs(x);
    if (ix < 0x3ff30000) {              /* |x| < 1.1875 */
      if (ix < 0x3fe60000) {            /* 7/16 <= |x| < 11/16 */
        id = 0;
        x = (2.0 * x - 1.0) / (2.0 + x);
      } else {                          /* 11/16 <= |x| < 19/16 */
        id = 1;
        x = (x - 1.0) / (x + 1.0);
      }
    } else {
      if (ix < 0x40038000) {            /* |x| < 2.4375 */
        id = 2;
        x = (x - 1.5) / (1.0 + 1.5 * x);
      } else {                          /* 2.4375 <= |x| < 2^66 */
        id = 3;
        x = -1.0 / x;
      }
    }
  }
  double z = x * x;
  const double w = z * z;
  const double s1 = z * (aT[0] + w * (aT[2] + w * (aT[4] + w * (aT[6] + w * (aT[8] + w * aT[10])))));
  const double s2 = w * (aT[1] + w * (aT[3] + w * (aT[5] + w * (aT[7] + w * aT[9]))));
  if (id < 0) return x - x * (s1 + s2);
  z = atanhi[id] - (x * (s1 + s2) - atanlo[id] - x);
  return sign ? -z : z;
}

/* musl atan2.c */
static inline double ro_atan2(double y, double x) {
  const double pi = 3.1415926535897931160E+00, pi_lo = 1.2246467991473531772E-16;
  if (isnan(x) || isnan(y)) return x + y;
  uint32_t ix = rol_hi(x), lx = rol_lo(x), iy = rol_hi(y), ly = rol_lo(y);
  if (((ix - 0x3ff00000) | lx) == 0) return ro_atan(y); /* x = 1.0 */
  const uint32_t m = ((iy >> 31) & 1) | ((ix >> 30) & 2);  /* 2*sign(x)+sign(y) */
  ix &= 0x7fffffff;
  iy &= 0x7fffffff;
  if ((iy | ly) == 0) {                 /* y = 0 */
    switch (m) {
      case 0:
      case 1: return y;
      case 2: return pi;
      default: return -pi;
    }
  }
  if ((ix | lx) == 0) return (m & 1) ? -pi / 2 : pi / 2; /* x = 0 */
  if (ix == 0x7ff00000) {               /* x = +-inf */
    if (iy == 0x7ff00000) {
      switch (m) {
        case 0: return pi / 4;
        case 1: return -pi / 4;
        case 2: return 3 * pi / 4;
        default: return -3 * pi / 4;
      }
    }
    switch (m) {
      case 0: return 0.0;
      case 1: return -0.0;
      case 2: return pi;
      default: return -pi;
    }
  }
  if (ix + (64 << 20) < iy || iy == 0x7ff00000) return (m & 1) ? -pi / 2 : pi / 2; /* |y/x| > 2^64 */
  double z;
  if ((m & 2) && iy + (64 << 20) < ix)  /* |y/x| < 2^-64, x < 0 */
    z = 0;
  else
    z = ro_atan(fabs(y / x));
  switch (m) {
    case 0: return z;
    case 1: return -z;
    case 2: return pi - (z - pi_lo);
    default: return (z - pi_lo) - pi;
  }
}

/* musl acos.c */
static inline double rol_acos_R(double z) {
  const double pS0 = 1.66666666666666657415e-01, pS1 = -3.25565818622400915405e-01,
               pS2 = 2.01212532134862925881e-01, pS3 = -4.00555345006794114027e-02,
               pS4 = 7.91534994289814532176e-04, pS5 = 3.47933107596021167570e-05,
               qS1 = -2.40339491173441421878e+00, qS2 = 2.02094576023350569471e+00,
               qS3 = -6.88283971605453293030e-01, qS4 = 7.70381505559019352791e-02;
  const double p = z * (pS0 + z * (pS1 + z * (pS2 + z * (pS3 + z * (pS4 + z * pS5)))));
  const double q = 1.0 + z * (qS1 + z * (qS2 + z * (qS3 + z * qS4)));
  return p / q;
}
static inline double ro_acos(double x) {
  const double pio2_hi = 1.57079632679489655800e+00, pio2_lo = 6.12323399573676603587e-17;
  const uint32_t hx = rol_hi(x), ix = hx & 0x7fffffff;
  if (ix >= 0x3ff00000) {               /* |x| >= 1 or NaN */
    if (((ix - 0x3ff00000) | rol_lo(x)) == 0) {
      if (hx >> 31) return 2 * pio2_hi + 0x1p-120;
      return 0;
    }
    return 0 / (x - x);
  }
  if (ix < 0x3fe00000) {                /* |x| < 0.5 */
    if (ix <= 0x3c600000) return pio2_hi + 0x1p-120;
    return pio2_hi - (x - (pio2_lo - x * rol_acos_R(x * x)));
  }
  if (hx >> 31) {                       /* x < -0.5 */
    const double z = (1.0 + x) * 0.5;
    const double s = sqrt(z);
    const double w = rol_acos_R(z) * s - pio2_lo;
    return 2 * (pio2_hi - (s + w));
  }
  const double z = (1.0 - x) * 0.5;     /* x > 0.5 */
  const double s = sqrt(z);
  const double df = rol_from(rol_bits(s) & 0xFFFFFFFF00000000ULL);
  const double c = (z - df * df) / (s + df);
  const double w = rol_acos_R(z) * s + c;
  return 2 * (df + w);
}

#endif
