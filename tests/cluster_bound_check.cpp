// cluster_bound_check.cpp — adversarial check of the clustered pretest
// (raytracinginoneweekend.zig_amd/csrc/rtw_cull.hpp cluster_sphere + cull_x;
// trace VAR kVarCluster).  For random clusters of <= 8 static / moving
// spheres and rays grazing the cluster's bounding sphere, x < 0 for the
// cluster record must imply that every member's exact f64 discriminant
// (hittable.zig:96-101, the kernel's operation order) is negative at any
// time of the shutter.  argv: n seed [shrink]: shrink > 0 scales the bound
// radius by (1 - shrink) (the check must then find violations: teeth).
// Prints "cases N skipped S violations V".  Built and run by tests/test_cull_host.py.
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
  const long n = argc > 1 ? atol(argv[1]) : 1000000;
  std::mt19937_64 g(argc > 2 ? atol(argv[2]) : 12345);
  const double shrink = argc > 3 ? atof(argv[3]) : 0.0;
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
    const int m = 1 + (int)(g() % 8);
    const double cs = std::pow(10.0, (double)(g() % 4));  // cluster position scale 1 .. 1e3
    const V base = rv(cs);
    const double spread = lu(1e-2, 10.0);
    double c0[8][3], dc[8][3], r[8];
    double cm = 0.0;
    for (int i = 0; i < m; ++i) {
      const V c = add(base, rv(spread));
      const bool moving = g() & 1;
      const V d = moving ? (g() & 1 ? V{0, lu(1e-3, 2.0), 0} : rv(lu(1e-3, 2.0))) : V{0, 0, 0};
      c0[i][0] = c.x, c0[i][1] = c.y, c0[i][2] = c.z;
      dc[i][0] = d.x, dc[i][1] = d.y, dc[i][2] = d.z;
      r[i] = (g() % 8 == 0 ? -1.0 : 1.0) * lu(1e-3, 5.0);
      cm = std::fmax(cm, std::fmax(std::fabs(c.x), std::fmax(std::fabs(c.y), std::fabs(c.z))) +
                             std::fmax(std::fabs(d.x), std::fmax(std::fabs(d.y), std::fabs(d.z))));
    }
    float cf[3], rf;
    rtwc::cluster_sphere(c0, dc, r, m, cf, rf);
    if (shrink > 0) rf = (float)(rf * (1.0 - shrink));
    cm = std::fmax(cm, std::fmax(std::fabs(cf[0]), std::fmax(std::fabs(cf[1]), std::fabs(cf[2]))));
    const float cmax = std::nextafter((float)cm, INFINITY);
    const float rho = std::nextafter((float)(2.0 * (double)rf * (double)rf + 1.0), INFINITY);
    const V C{cf[0], cf[1], cf[2]};
    // ray: origin far / near the bound; direction grazing the bound or toward a member
    V o;
    const int om = g() % 3;
    if (om == 0) o = rv(std::pow(10.0, (double)(g() % 6)));
    else if (om == 1) o = add(C, mul(rdir(), rf * lu(1.0, 1e3)));
    else o = add(C, mul(rdir(), rf * U(g)));
    V d;
    const int dm = g() % 3;
    if (dm == 0) {
      d = rdir();
    } else {
      const V target = dm == 1 ? C : V{c0[0][0], c0[0][1], c0[0][2]};
      const double rad = dm == 1 ? rf : std::fabs(r[0]);
      const V oc = sub(target, o);
      V w = cross(oc, rdir());
      if (dot(w, w) == 0) continue;
      w = unit(w);
      d = sub(add(target, mul(w, rad * (1.0 + (g() & 1 ? 1 : -1) * lu(1e-12, 1e-2)))), o);
      if (dot(d, d) == 0) continue;
    }
    d = mul(d, lu(1e-3, 1e3) / std::sqrt(dot(d, d)));
    ++cases;
    const float of[3] = {(float)o.x, (float)o.y, (float)o.z}, df[3] = {(float)d.x, (float)d.y, (float)d.z};
    const double a = d.x * d.x + d.y * d.y + d.z * d.z;
    const rtwc::LaneCull lc = rtwc::lane_cull(of[0], of[1], of[2], (float)a, cmax);
    if (!lc.ok) continue;
    const float x = rtwc::cull_x(of[0], of[1], of[2], df[0], df[1], df[2], rtwc::lane_const((float)a, lc.alpha, rho),
                                 0.0f, cf[0], cf[1], cf[2], 0.0f, 0.0f, 0.0f, -(rf * rf), false);
    if (!(x < 0)) continue;
    ++skipped;
    bool bad = false;
    for (int i = 0; i < m && !bad; ++i) {
      for (int k = 0; k < 5; ++k) {  // shutter times incl. both ends
        const double f = k == 0 ? 0.0 : (k == 1 ? 1.0 : U(g));
        const V c{c0[i][0] + dc[i][0] * f, c0[i][1] + dc[i][1] * f, c0[i][2] + dc[i][2] * f};
        const V oc = sub(o, c);
        const double hb = oc.x * d.x + oc.y * d.y + oc.z * d.z;
        const double cc = (oc.x * oc.x + oc.y * oc.y + oc.z * oc.z) - r[i] * r[i];
        if (!(hb * hb - a * cc < 0)) {
          bad = true;
          break;
        }
      }
    }
    if (bad) ++viol;
  }
  printf("cases %ld skipped %ld violations %ld\n", cases, skipped, viol);
  return viol ? 1 : 0;
}
