// cull_bound_check.cpp — adversarial check of the packed-f32 pretest bound
// (raytracinginoneweekend.zig_amd/csrc/rtw_cull.hpp).  For random and
// near-grazing (ray, sphere) pairs it evaluates the exact discriminant the
// kernel's closest-hit test computes (hittable.zig:96-101: f64, and the f32
// variant of precision 1) and the pretest x; x < 0 must imply disc < 0.
// Prints "cases N skipped S violations V".  Built and run by
// tests/test_cull_host.py (g++ -O2 -ffp-contract=off).
#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <random>

#include "rtw_cull.hpp"

struct V {
  double x, y, z;
};
static V sub(V a, V b) { return {a.x - b.x, a.y - b.y, a.z - b.z}; }
static V add(V a, V b) { return {a.x + b.x, a.y + b.y, a.z + b.z}; }
static V mul(V a, double t) { return {a.x * t, a.y * t, a.z * t}; }
static double dot(V a, V b) { return a.x * b.x + a.y * b.y + a.z * b.z; }
static V cross(V a, V b) { return {a.y * b.z - a.z * b.y, a.z * b.x - a.x * b.z, a.x * b.y - a.y * b.x}; }
static V unit(V a) { return mul(a, 1.0 / std::sqrt(dot(a, a))); }

int main(int argc, char** argv) {
  const long n = argc > 1 ? atol(argv[1]) : 4000000;
  std::mt19937_64 g(argc > 2 ? atol(argv[2]) : 12345);
  std::uniform_real_distribution<double> U(0.0, 1.0);
  auto lu = [&](double lo, double hi) { return std::exp(std::log(lo) + (std::log(hi) - std::log(lo)) * U(g)); };
  auto rv = [&](double s) { return V{(2 * U(g) - 1) * s, (2 * U(g) - 1) * s, (2 * U(g) - 1) * s}; };
  auto rdir = [&]() {
    V v;
    do v = rv(1.0);
    while (dot(v, v) > 1.0 || dot(v, v) < 1e-6);
    return unit(v);
  };
  long skipped = 0, viol = 0, cases = 0;
  for (long it = 0; it < n; ++it) {
    const double cs = std::pow(10.0, (double)(g() % 5));  // centre scale 1 .. 1e4
    const V c0 = rv(cs);
    const double r = lu(1e-3, 99.0);
    const bool moving = g() & 1;
    const V dc = moving ? rv(lu(1e-3, 2.0)) : V{0, 0, 0};
    const double time = U(g);
    const double frac = time;  // t0 = 0, t1 = 1: (time - t0) / (t1 - t0)
    const V c = moving ? add(c0, mul(dc, frac)) : c0;
    // origin: random box / on the surface / inside
    V o;
    const int om = g() % 4;
    if (om == 0) o = rv(std::pow(10.0, (double)(g() % 7)));  // up to 1e6
    else if (om == 1) o = add(c, mul(rdir(), r * (1.0 + (2 * U(g) - 1) * lu(1e-12, 1e-3))));
    else if (om == 2) o = add(c, mul(rdir(), r * U(g)));
    else o = add(c, mul(rdir(), r * lu(1.0, 1e4)));
    // direction: random, or grazing the silhouette
    V d;
    if (g() % 3 == 0) {
      d = rdir();
    } else {
      const V oc = sub(c, o);
      V w = cross(oc, rdir());
      if (dot(w, w) == 0) continue;
      w = unit(w);
      const double delta = (g() & 1 ? 1 : -1) * lu(1e-15, 1e-2);
      d = sub(add(c, mul(w, r * (1.0 + delta))), o);
      if (dot(d, d) == 0) continue;
    }
    d = mul(d, lu(1e-3, 1e3) / std::sqrt(dot(d, d)));
    ++cases;
    // exact f64 (kernel test lambda, -ffp-contract=off order)
    const double a = d.x * d.x + d.y * d.y + d.z * d.z;
    const V oc = sub(o, c);
    const double hb = oc.x * d.x + oc.y * d.y + oc.z * d.z;
    const double cc = (oc.x * oc.x + oc.y * oc.y + oc.z * oc.z) - r * r;
    const double disc64 = hb * hb - a * cc;
    // exact f32 (precision 1): f32 inputs, f32 ops
    const float rf = (float)r, fr = (float)time;
    const float c0f[3] = {(float)c0.x, (float)c0.y, (float)c0.z}, dcf[3] = {(float)dc.x, (float)dc.y, (float)dc.z};
    const float cf[3] = {moving ? c0f[0] + dcf[0] * fr : c0f[0], moving ? c0f[1] + dcf[1] * fr : c0f[1],
                         moving ? c0f[2] + dcf[2] * fr : c0f[2]};
    const float of[3] = {(float)o.x, (float)o.y, (float)o.z}, df[3] = {(float)d.x, (float)d.y, (float)d.z};
    const float af32 = df[0] * df[0] + df[1] * df[1] + df[2] * df[2];
    const float ocf[3] = {of[0] - cf[0], of[1] - cf[1], of[2] - cf[2]};
    const float hbf = ocf[0] * df[0] + ocf[1] * df[1] + ocf[2] * df[2];
    const float ccf = (ocf[0] * ocf[0] + ocf[1] * ocf[1] + ocf[2] * ocf[2]) - rf * rf;
    const float disc32 = hbf * hbf - af32 * ccf;
    // pretest, table values as rtw_capi.hip builds them
    const double cm = std::fmax(std::fabs(c0.x), std::fmax(std::fabs(c0.y), std::fabs(c0.z))) +
                      std::fmax(std::fabs(dc.x), std::fmax(std::fabs(dc.y), std::fabs(dc.z)));
    const float cmax = std::nextafter((float)cm, INFINITY);
    const float rho = std::nextafter((float)(2.0 * (r * r) + 1.0), INFINITY);
    bool bad = false;
    for (int prec = 0; prec < 2; ++prec) {
      const float aa = prec == 0 ? (float)a : af32;
      const rtwc::LaneCull lc = rtwc::lane_cull(of[0], of[1], of[2], aa, cmax);
      if (!lc.ok) continue;
      const float x = rtwc::cull_x(of[0], of[1], of[2], df[0], df[1], df[2], rtwc::lane_const(aa, lc.alpha, rho), fr,
                                   c0f[0], c0f[1], c0f[2], -dcf[0], -dcf[1], -dcf[2], -(rf * rf), moving);
      const bool exact_neg = prec == 0 ? (disc64 < 0) : (disc32 < 0);
      if (x < 0) {
        if (prec == 0) ++skipped;
        if (!exact_neg) bad = true;
      }
    }
    if (bad) {
      if (viol < 5)
        fprintf(stderr, "violation: o=(%g %g %g) d=(%g %g %g) c=(%g %g %g) r=%g disc64=%g disc32=%g\n", o.x, o.y,
                o.z, d.x, d.y, d.z, c.x, c.y, c.z, r, disc64, (double)disc32);
      ++viol;
    }
  }
  printf("cases %ld skipped %ld violations %ld\n", cases, skipped, viol);
  return viol ? 1 : 0;
}
