/*
 * ro_cpu_port.c — the reference's CPU render loop as a PERFORMANCE port, for
 * bench.py's cpu_baseline leg only (TEST / MEASUREMENT INFRASTRUCTURE: never
 * on the product path; the GPU library neither links nor loads it).
 *
 * It computes exactly what oracle Tier A (rtw_oracle.c ro_render_tier_a)
 * computes — the reference's main.zig:378-402 loop over ONE sequential
 * DefaultPrng stream, recursive rayColor (main.zig:103-122), f64 — and its
 * image is bit-identical to Tier A's (tests/test_oracle_tier_a.py), but it is
 * written to be fast on one CPU core, so the GPU/CPU ratio in the bench line
 * is measured against a fair CPU program rather than the checker:
 *
 *  - HittableList.hit (hittable.zig:231-244) in two passes per segment:
 *    half_b and the discriminant of every sphere (hittable.zig:96-101) over
 *    SoA arrays (static spheres, then moving ones), loops the compiler
 *    vectorises (AVX2 / AVX-512 with -march=native); then the reference's
 *    sequential acceptance in list order, with the square root and the root
 *    divisions only for spheres whose discriminant is >= 0 (the values do
 *    not depend on `closest`, only the choice between the roots does, so
 *    every decision and value is the reference's);
 *  - per-segment invariants hoisted (|d|^2, r^2, c1 - c0, t1 - t0: the same
 *    IEEE operations on the same operands);
 *  - the hit record (hittable.zig:113-130, incl. getSphereUv's atan2 / acos)
 *    built once, for the winner, not for every accepted candidate (earlier
 *    candidates' records are overwritten unread in the reference).
 *
 * Build: bench.py compiles it on the timing host with
 * gcc -O3 -march=native -ffp-contract=off (oracle/Makefile builds a portable
 * -march=x86-64-v3 copy for the CPU tests).
 */
#include <math.h>
#include <stdint.h>
#include <string.h>

#include "rtw_oracle.h"

typedef struct { double x, y, z; } V3;
static inline V3 v3(double x, double y, double z) { V3 r = {x, y, z}; return r; }
static inline V3 vadd(V3 a, V3 b) { return v3(a.x + b.x, a.y + b.y, a.z + b.z); }
static inline V3 vsub(V3 a, V3 b) { return v3(a.x - b.x, a.y - b.y, a.z - b.z); }
static inline V3 vmul(V3 a, double t) { return v3(a.x * t, a.y * t, a.z * t); }
static inline V3 vmulv(V3 a, V3 b) { return v3(a.x * b.x, a.y * b.y, a.z * b.z); }
static inline V3 vdiv(V3 a, double t) { return v3(a.x / t, a.y / t, a.z / t); }
static inline double vdot(V3 a, V3 b) { return a.x * b.x + a.y * b.y + a.z * b.z; }
static inline double vnorm2(V3 a) { return a.x * a.x + a.y * a.y + a.z * a.z; }
static inline V3 vnormalized(V3 v) { /* vec.zig:32-39 */
  const double n = sqrt(vnorm2(v));
  return (n == 0.0) ? v : vdiv(v, n);
}
static inline V3 vload(const double p[3]) { return v3(p[0], p[1], p[2]); }

/* ---- Zig std.Random: Xoshiro256++ and Random.float(f64) (rtw_oracle.c) ---- */
typedef struct { uint64_t s0, s1, s2, s3; } Rng;
static inline uint64_t rotl(uint64_t x, unsigned k) { return (x << k) | (x >> (64 - k)); }
static inline uint64_t xnext(Rng *r) {
  const uint64_t out = rotl(r->s0 + r->s3, 23) + r->s0;
  const uint64_t t = r->s1 << 17;
  r->s2 ^= r->s0;
  r->s3 ^= r->s1;
  r->s1 ^= r->s2;
  r->s0 ^= r->s3;
  r->s2 ^= t;
  r->s3 = rotl(r->s3, 45);
  return out;
}
static inline double rand01(Rng *r) {
  const uint64_t rnd = xnext(r);
  uint64_t lz = rnd ? (uint64_t)__builtin_clzll(rnd) : 64u;
  if (__builtin_expect(lz >= 12, 0)) {
    lz = 12;
    for (;;) {
      const uint64_t w = xnext(r);
      const uint64_t addl = w ? (uint64_t)__builtin_clzll(w) : 64u;
      lz += addl;
      if (addl != 64) break;
      if (lz >= 1022) { lz = 1022; break; }
    }
  }
  const uint64_t bits = ((1022 - lz) << 52) | (rnd & ((1ULL << 52) - 1));
  double d;
  memcpy(&d, &bits, 8);
  return d;
}
static inline double rrange(Rng *r, double mn, double mx) { return mn + rand01(r) * (mx - mn); }
static inline V3 rand_in_unit_sphere(Rng *r) { /* rand.zig:22-28 */
  for (;;) {
    V3 p;
    p.x = rrange(r, -1.0, 1.0);
    p.y = rrange(r, -1.0, 1.0);
    p.z = rrange(r, -1.0, 1.0);
    if (sqrt(vnorm2(p)) >= 1) continue;
    return p;
  }
}
static inline V3 rand_in_unit_disk(Rng *r) { /* rand.zig:30-36 */
  for (;;) {
    V3 p;
    p.x = rrange(r, -1.0, 1.0);
    p.y = rrange(r, -1.0, 1.0);
    p.z = 0;
    if (sqrt(vnorm2(p)) >= 1) continue;
    return p;
  }
}

/* std/math/pow.zig's integer path for pow(1 - cos, 5.0) on [0, 2] (material.zig:90):
 * Go's repeated squaring of the frexp mantissa is exactly x*((x*x)*(x*x)) there
 * (rtw_oracle.c zig_pow_posint is the general restatement). */
static inline double pow5(double x) {
  if (x == 0 || x == 1) return x;
  int e;
  const double m = frexp(x, &e);
  double a1 = m, x1 = m * m;
  int ae = e, xe = 2 * e;
  if (x1 < 0.5) { x1 += x1; xe -= 1; }
  x1 *= x1;
  xe <<= 1;
  if (x1 < 0.5) { x1 += x1; xe -= 1; }
  a1 *= x1;
  ae += xe;
  return ldexp(a1, ae);
}

/* ---- scene in SoA form: static spheres at [0, ns), moving ones at [ns, n)
 * (each in list order); pos[i] = the SoA slot of list entry i ---- */
#define PORT_MAX RO_MAX_SPHERES
typedef struct {
  uint32_t n, ns, ng;
  uint32_t pos[PORT_MAX];
  double c0x[PORT_MAX], c0y[PORT_MAX], c0z[PORT_MAX];
  double dcx[PORT_MAX], dcy[PORT_MAX], dcz[PORT_MAX]; /* c1 - c0 (MovingSphere.center, hittable.zig:219-221) */
  double rr[PORT_MAX];                                /* radius * radius (hittable.zig:99) */
  uint32_t grp[PORT_MAX];                             /* time group of a moving slot */
  double gt0[PORT_MAX], gdt[PORT_MAX];                /* distinct (time0, time1 - time0) */
  /* per-segment scratch */
  double gf[PORT_MAX], f[PORT_MAX], hb[PORT_MAX], disc[PORT_MAX];
} SoA;

typedef struct {
  const ro_scene *sc;
  SoA *s;
  V3 bg;
  Rng rng;
} Ctx;

typedef struct { V3 origin, dir; double time; } Ray;

/* Closest hit of HittableList.hit (hittable.zig:231-244): index of the winner or -1. */
static int closest_hit(Ctx *cx, const Ray *r, double tmin, double *t_out) {
  SoA *s = cx->s;
  const uint32_t n = s->n, ns = s->ns;
  const double ox = r->origin.x, oy = r->origin.y, oz = r->origin.z;
  const double dx = r->dir.x, dy = r->dir.y, dz = r->dir.z, tm = r->time;
  const double a = dx * dx + dy * dy + dz * dz; /* r.direction.lengthSquared() */
  /* pass 1 (vectorised): half_b and the discriminant of every sphere; no
   * division or square root (pass 2 runs them for the few spheres whose
   * discriminant is >= 0) */
  for (uint32_t i = 0; i < ns; ++i) {
    const double ocx = ox - s->c0x[i], ocy = oy - s->c0y[i], ocz = oz - s->c0z[i];
    const double hb = ocx * dx + ocy * dy + ocz * dz;
    const double c = (ocx * ocx + ocy * ocy + ocz * ocz) - s->rr[i];
    s->hb[i] = hb;
    s->disc[i] = hb * hb - a * c;
  }
  if (n > ns) {
    /* MovingSphere.center's time fraction (hittable.zig:219-221): one division
     * per distinct (time0, time1) of the scene, not one per sphere */
    for (uint32_t g = 0; g < s->ng; ++g) s->gf[g] = (tm - s->gt0[g]) / s->gdt[g];
    if (s->ng == 1)
      for (uint32_t i = ns; i < n; ++i) s->f[i] = s->gf[0];
    else
      for (uint32_t i = ns; i < n; ++i) s->f[i] = s->gf[s->grp[i]];
    for (uint32_t i = ns; i < n; ++i) {
      const double f = s->f[i];
      const double ocx = ox - (s->c0x[i] + s->dcx[i] * f), ocy = oy - (s->c0y[i] + s->dcy[i] * f),
                   ocz = oz - (s->c0z[i] + s->dcz[i] * f);
      const double hb = ocx * dx + ocy * dy + ocz * dz;
      const double c = (ocx * ocx + ocy * ocy + ocz * ocz) - s->rr[i];
      s->hb[i] = hb;
      s->disc[i] = hb * hb - a * c;
    }
  }
  /* pass 2: the reference's sequential acceptance in list order
   * (hittable.zig:102-112, :236-242) */
  double closest = INFINITY;
  int hit = -1;
  for (uint32_t i = 0; i < n; ++i) {
    const uint32_t k = s->pos[i];
    const double disc = s->disc[k];
    if (disc < 0.0) continue;
    const double hb = s->hb[k], sq = sqrt(disc);
    double root = (-hb - sq) / a;
    if (root < tmin || closest < root) {
      root = (-hb + sq) / a;
      if (root < tmin || closest < root) continue;
    }
    closest = root;
    hit = (int)i;
  }
  *t_out = closest;
  return hit;
}

static V3 ray_color(Ctx *cx, const Ray *r, uint32_t depth) { /* main.zig:103-122 */
  if (depth == 0) return v3(0, 0, 0);
  double t;
  const int i = closest_hit(cx, r, 0.001, &t);
  if (i < 0) return cx->bg;
  const ro_sphere *sp = &cx->sc->spheres[i];
  /* the hit record (hittable.zig:113-130 / :183-200) */
  V3 center = vload(sp->c0);
  if (sp->moving) center = vadd(vload(sp->c0), vmul(vsub(vload(sp->c1), vload(sp->c0)), (r->time - sp->t0) / (sp->t1 - sp->t0)));
  const V3 p = vadd(r->origin, vmul(r->dir, t));
  const V3 outward = vdiv(vsub(p, center), sp->radius);
  const int front = vdot(outward, r->dir) < 0.0;
  const V3 normal = front ? outward : vmul(outward, -1.0);
  volatile double uv_sink;
  if (!sp->moving) { /* getSphereUv (hittable.zig:145-150): the reference computes it; nothing reads it */
    const double phi = atan2(-outward.z, outward.x) + M_PI;
    const double theta = acos(-outward.y);
    uv_sink = phi / (2.0 * M_PI) + theta / M_PI;
  }
  (void)uv_sink;
  const ro_material *m = &cx->sc->mats[sp->mat];
  Ray sc_;
  sc_.origin = p;
  sc_.time = r->time;
  V3 att;
  switch (m->kind) {
    case RO_LAMBERT_SOLID:
    case RO_LAMBERT_CHECKER: { /* material.zig:44-52 */
      const V3 b = rand_in_unit_sphere(&cx->rng);
      V3 dir = vadd(normal, vnormalized(b));
      if (fabs(dir.x) < 1e-8 && fabs(dir.y) < 1e-8 && fabs(dir.z) < 1e-8) dir = normal;
      sc_.dir = dir;
      att = vload(m->albedo);
      if (m->kind == RO_LAMBERT_CHECKER) { /* texture.zig:79-82 */
        const double sines = sin(10 * p.x) * sin(10 * p.y) * sin(10 * p.z);
        if (sines < 0) att = vload(m->albedo_odd);
      }
      break;
    }
    case RO_METAL: { /* material.zig:59-65 */
      const V3 ud = vnormalized(r->dir);
      const V3 refl = vsub(ud, vmul(normal, 2 * vdot(ud, normal)));
      sc_.dir = vadd(refl, vmul(rand_in_unit_sphere(&cx->rng), m->fuzz));
      if (!(vdot(refl, normal) > 0.0)) return v3(0, 0, 0); /* absorbed: emitted */
      att = vload(m->albedo);
      break;
    }
    default: { /* DielectricMaterial, material.zig:72-91 */
      const double ratio = front ? 1.0 / m->ir : m->ir;
      const V3 ud = vnormalized(r->dir);
      const double cos_theta = fmin(vdot(vmul(ud, -1.0), normal), 1.0);
      const double sin_theta = sqrt(1.0 - cos_theta * cos_theta);
      int refract = 0;
      if (ratio * sin_theta <= 1.0) {
        const double r0 = (1.0 - ratio) / (1.0 + ratio);
        const double r1 = r0 * r0;
        refract = r1 + (1.0 - r1) * pow5(1.0 - cos_theta) < rand01(&cx->rng);
      }
      if (refract) { /* material.zig:116-121 */
        const double ct = fmin(vdot(vmul(ud, -1.0), normal), 1.0);
        const V3 perp = vmul(vadd(ud, vmul(normal, ct)), ratio);
        const V3 par = vmul(normal, -sqrt(fabs(1.0 - vnorm2(perp))));
        sc_.dir = vadd(perp, par);
      } else {
        sc_.dir = vsub(ud, vmul(normal, 2 * vdot(ud, normal)));
      }
      att = v3(1.0, 1.0, 1.0);
      break;
    }
  }
  return vadd(v3(0, 0, 0), vmulv(att, ray_color(cx, &sc_, depth - 1))); /* emitted + att * rayColor(...) */
}

/* main.zig:395-400 (rtw_oracle.c ro_quantize) */
static inline uint8_t quantize(double c, double scale) {
  const double g = sqrt(c * scale);
  const double cl = fmax(0.0, fmin(g, 0.999));
  return (uint8_t)(256.0 * cl);
}

static SoA g_soa; /* (not re-entrant: measurement infrastructure) */

/* Tier A's render loop (main.zig:378-402), bit-identical output to
 * ro_render_tier_a.  rng: the stream after the scene build. */
void rp_render(const ro_scene *scene, const ro_camera *cam, const double bg[3], uint32_t W, uint32_t H, uint32_t spp,
               uint32_t depth, uint64_t rng[4], uint8_t *rgb, uint32_t rows) {
  SoA *s = &g_soa;
  s->n = scene->n_spheres;
  s->ns = 0;
  s->ng = 0;
  for (uint32_t i = 0; i < s->n; ++i) s->ns += !scene->spheres[i].moving;
  uint32_t ks = 0, km = s->ns;
  for (uint32_t i = 0; i < s->n; ++i) {
    const ro_sphere *sp = &scene->spheres[i];
    const uint32_t k = sp->moving ? km++ : ks++;
    s->pos[i] = k;
    s->c0x[k] = sp->c0[0], s->c0y[k] = sp->c0[1], s->c0z[k] = sp->c0[2];
    s->dcx[k] = sp->c1[0] - sp->c0[0], s->dcy[k] = sp->c1[1] - sp->c0[1], s->dcz[k] = sp->c1[2] - sp->c0[2];
    s->rr[k] = sp->radius * sp->radius;
    s->grp[k] = 0;
    if (sp->moving) {
      uint32_t g = 0;
      while (g < s->ng && !(s->gt0[g] == sp->t0 && s->gdt[g] == sp->t1 - sp->t0)) ++g;
      if (g == s->ng) {
        s->gt0[g] = sp->t0;
        s->gdt[g] = sp->t1 - sp->t0;
        ++s->ng;
      }
      s->grp[k] = g;
    }
  }
  Ctx cx;
  cx.sc = scene;
  cx.s = s;
  cx.bg = vload(bg);
  cx.rng.s0 = rng[0], cx.rng.s1 = rng[1], cx.rng.s2 = rng[2], cx.rng.s3 = rng[3];
  const V3 origin = vload(cam->origin), hor = vload(cam->horizontal), ver = vload(cam->vertical);
  const V3 llc = vload(cam->lower_left_corner), cu = vload(cam->u), cv = vload(cam->v);
  for (uint32_t j = 0; j < H && j < rows; ++j) {
    for (uint32_t i = 0; i < W; ++i) {
      V3 pc = v3(0, 0, 0);
      for (uint32_t k = 0; k < spp; ++k) {
        const double u = ((double)i + rand01(&cx.rng)) / ((double)W - 1.0);
        const double v = ((double)j + rand01(&cx.rng)) / ((double)H - 1.0);
        /* Camera.getRay, main.zig:91-100 */
        const V3 rd = vmul(rand_in_unit_disk(&cx.rng), cam->lens_radius);
        const V3 offset = vadd(vmul(cu, rd.x), vmul(cv, rd.y));
        Ray r;
        r.origin = vadd(origin, offset);
        r.dir = vsub(vsub(vadd(vadd(llc, vmul(hor, u)), vmul(ver, v)), origin), offset);
        r.time = rrange(&cx.rng, cam->time0, cam->time1);
        pc = vadd(pc, ray_color(&cx, &r, depth));
      }
      const double scale = 1.0 / (double)spp;
      const size_t o = ((size_t)i + (size_t)(H - j - 1) * W) * 3;
      rgb[o + 0] = quantize(pc.x, scale);
      rgb[o + 1] = quantize(pc.y, scale);
      rgb[o + 2] = quantize(pc.z, scale);
    }
  }
  rng[0] = cx.rng.s0, rng[1] = cx.rng.s1, rng[2] = cx.rng.s2, rng[3] = cx.rng.s3;
}
