// rtw_cull.hpp — conservative f32 pretest for the closest-hit loop.
//
// Sphere.hit / MovingSphere.hit (hittable.zig:95-101, :165-171) reject a
// sphere when disc = half_b^2 - a*c < 0; ~97 % of (ray, sphere) tests end
// there.  The kernel first evaluates disc for two spheres at once in packed
// f32 (v_pk_fma_f32) and adds a margin M larger than the total error of that
// estimate; x = disc_f32 + M < 0 PROVES that the exact discriminant (f64, or
// f32 in precision 1) is negative, so the exact test of that sphere can be
// skipped without changing any result.  Survivors get the exact test.
//
// Error budget (P = |o - c|, D = |d|, e = absolute error of each component of
// o - c as computed here, u = 2^-24; first order, Cauchy-Schwarz |hb| <= PD):
//   |disc_f32 - disc| <= D^2 [4 sqrt(3) P e + 22 u P^2 + 5 u r^2 + 7 e^2]
//                     <= D^2 [(3.5 e + 22 u)(P^2 + 1) + 5 u r^2 + 7 e^2]
// and e <= 4u (|o|_inf + Cmax) with Cmax = max |c0|_inf + |c1 - c0|_inf over
// the narrow spheres.  The kernel uses M = alpha * (cc + rho) with
// alpha = a (16 e' + 100 u), e' = 8u (|o|_inf + Cmax) (a 4x-8x safety
// factor on every term), cc + rho = P^2 + r^2 + 1 (rho = 2 r^2 + 1).  The
// kernel uses rho_max (over the scene's narrow spheres) for every sphere, so
// x = hb^2 + alpha rho_max - (a - alpha) cc needs two packed ops past hb, cc,
// the same as disc alone.  Lanes
// with |o|_inf > 2^20 or a outside [2^-40, 2^40] (or non-finite values) do
// not use the pretest; scenes with Cmax > 2^20 do not either.
// tests/test_cull_host.py checks the bound on adversarial near-grazing cases.
#pragma once
#include <cmath>
#include <cstdint>

#if defined(__HIPCC__)
#define RTWC_HD __host__ __device__ __forceinline__
#else
#define RTWC_HD inline
#endif

namespace rtwc {

constexpr float kU = 0x1p-24f;
constexpr float kOriginMax = 0x1p20f;  // |o|_inf limit of a lane that uses the pretest
constexpr float kCmaxLimit = 0x1p20f;  // scene limit

struct LaneCull {
  float alpha;  // margin scale
  bool ok;      // lane may use the pretest
};

RTWC_HD LaneCull lane_cull(float ox, float oy, float oz, float a, float cmax) {
  const float om = std::fmax(std::fabs(ox), std::fmax(std::fabs(oy), std::fabs(oz)));
  const bool ok = (om <= kOriginMax) & (a >= 0x1p-40f) & (a <= 0x1p40f);
  const float e = (om + cmax) * (8.0f * kU);
  return {a * std::fma(16.0f, e, 100.0f * kU), ok};
}

// Per-lane constants of the pretest: na = -(a - alpha), k = alpha * rho_max.
struct LaneConst {
  float na, k;
};
RTWC_HD LaneConst lane_const(float a, float alpha, float rho_max) { return {-(a - alpha), alpha * rho_max}; }

// One sphere of a pretest record: c = f32(c0), ndc = -f32(c1 - c0),
// nr2 = -f32(r)^2.  frac = f32 estimate of (time - t0) / (t1 - t0) (any
// finite value for a static sphere, ndc = 0).  Returns x: x < 0 proves
// disc < 0.  Operation order = the kernel's packed code (rtw_trace.hip
// cull_pair), so host and device give the same bits.
RTWC_HD float cull_x(float ox, float oy, float oz, float dx, float dy, float dz, LaneConst lk, float frac, float cx,
                     float cy, float cz, float ndcx, float ndcy, float ndcz, float nr2, bool moving) {
  float ocx = ox - cx, ocy = oy - cy, ocz = oz - cz;
  if (moving) {  // (the kernel skips the updates whose ndc is 0: an exact no-op)
    if (ndcx != 0.0f) ocx = std::fma(ndcx, frac, ocx);
    ocy = std::fma(ndcy, frac, ocy);
    if (ndcz != 0.0f) ocz = std::fma(ndcz, frac, ocz);
  }
  const float hb = std::fma(ocz, dz, std::fma(ocy, dy, ocx * dx));
  const float cc = std::fma(ocz, ocz, std::fma(ocy, ocy, std::fma(ocx, ocx, nr2)));
  return std::fma(lk.na, cc, std::fma(hb, hb, lk.k));
}

// Bounding sphere of a cluster of n (possibly moving) narrow spheres for the
// clustered pretest (trace VAR kVarCluster; host only).  Member i: centre
// c0_i + f * dc_i for f in [0, 1] (the shutter inside its time group),
// radius |r_i|.  Centre cf = f32 of the centre of the members' swept box;
// radius R = max_i max(|c0_i - cf|, |c0_i + dc_i - cf|) + |r_i|, widened by
// 1e-4 (1 + R) and rounded up to f32.  A line whose f64 discriminant against
// (cf, rf) is negative passes each member's centre farther than |r_i| +
// ~1e-4 (1 + R): the member's own f64 discriminant (rounding ~1e-15 relative)
// is then negative too, so the cull_x proof for (cf, rf) proves every member
// missed.  tests/test_cull_host.py checks it on adversarial clusters.
inline void cluster_sphere(const double (*c0)[3], const double (*dc)[3], const double* r, int n, float cf[3],
                           float& rf) {
  double lo[3] = {INFINITY, INFINITY, INFINITY}, hi[3] = {-INFINITY, -INFINITY, -INFINITY};
  for (int i = 0; i < n; ++i)
    for (int k = 0; k < 3; ++k)
      for (int e = 0; e < 2; ++e) {
        const double c = c0[i][k] + (e ? dc[i][k] : 0.0);
        lo[k] = std::fmin(lo[k], c - std::fabs(r[i]));
        hi[k] = std::fmax(hi[k], c + std::fabs(r[i]));
      }
  for (int k = 0; k < 3; ++k) cf[k] = (float)(0.5 * (lo[k] + hi[k]));
  double R = 0.0;
  for (int i = 0; i < n; ++i) {
    double d0 = 0.0, d1 = 0.0;
    for (int k = 0; k < 3; ++k) {
      d0 += (c0[i][k] - cf[k]) * (c0[i][k] - cf[k]);
      d1 += (c0[i][k] + dc[i][k] - cf[k]) * (c0[i][k] + dc[i][k] - cf[k]);
    }
    R = std::fmax(R, std::sqrt(std::fmax(d0, d1)) + std::fabs(r[i]));
  }
  R = R + 1e-4 * (1.0 + R);
  rf = std::nextafter((float)R, INFINITY);
}

}  // namespace rtwc
