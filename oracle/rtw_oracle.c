/*
 * rtw_oracle.c — CPU ORACLE (test infrastructure only; see rtw_oracle.h).
 *
 * Plain-C restatement of nsfisis/RayTracingInOneWeekend.zig's cover-scene
 * render path.  Every function cites the reference file:line it follows
 * (paths relative to the reference root, src/).  Compiled with
 * -ffp-contract=off so each Zig f64 operation is one IEEE operation here.
 *
 * Parity: unpinned against the Zig binary (no toolchain / no goldens in the
 * reference); pinned by RNG KATs and by an independent Python restatement.
 */
#include "rtw_oracle.h"

#include <math.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#ifdef _OPENMP
#include <omp.h>
#endif

/* ===================================================================== */
/* Zig 0.14 std.Random restatement                                        */
/* ===================================================================== */

/* std/Random/SplitMix64.zig: next() */
uint64_t ro_splitmix64_next(uint64_t *state) {
  *state += 0x9e3779b97f4a7c15ULL;
  uint64_t z = *state;
  z = (z ^ (z >> 30)) * 0xbf58476d1ce4e5b9ULL;
  z = (z ^ (z >> 27)) * 0x94d049bb133111ebULL;
  return z ^ (z >> 31);
}

/* std/Random/Xoshiro256.zig: seed() — four SplitMix64 outputs.
 * Call site: DefaultPrng.init(42), main.zig:300. */
void ro_xoshiro256_seed(uint64_t s[4], uint64_t seed) {
  uint64_t sm = seed;
  s[0] = ro_splitmix64_next(&sm);
  s[1] = ro_splitmix64_next(&sm);
  s[2] = ro_splitmix64_next(&sm);
  s[3] = ro_splitmix64_next(&sm);
}

static inline uint64_t rotl64(uint64_t x, unsigned k) { return (x << k) | (x >> (64 - k)); }

/* std/Random/Xoshiro256.zig: next() (xoshiro256++). Random.int(u64) == next(). */
uint64_t ro_xoshiro256_next(uint64_t s[4]) {
  const uint64_t r = rotl64(s[0] + s[3], 23) + s[0];
  const uint64_t t = s[1] << 17;
  s[2] ^= s[0];
  s[3] ^= s[1];
  s[1] ^= s[2];
  s[0] ^= s[3];
  s[2] ^= t;
  s[3] = rotl64(s[3], 45);
  return r;
}

static inline unsigned clz64(uint64_t x) { return x ? (unsigned)__builtin_clzll(x) : 64u; }

/* std/Random.zig: float(f64).  52 random mantissa bits; the exponent is
 * 1022 - (leading zeros), extended with further u64 draws when the first 12
 * bits are all zero.  Call site: randomReal01, rand.zig:13-15. */
double ro_random_f64(uint64_t s[4]) {
  const uint64_t rnd = ro_xoshiro256_next(s);
  uint64_t lz = clz64(rnd);
  if (lz >= 12) {
    lz = 12;
    for (;;) {
      const uint64_t addl = clz64(ro_xoshiro256_next(s));
      lz += addl;
      if (addl != 64) break;
      if (lz >= 1022) { lz = 1022; break; }
    }
  }
  const uint64_t mant = rnd & ((1ULL << 52) - 1);
  const uint64_t bits = ((1022 - lz) << 52) | mant;
  double d;
  memcpy(&d, &bits, 8);
  return d;
}

/* std/Random.zig: float(f32) — 23 mantissa bits, exponent from the leading
 * zeros of the same u64 (extended when >= 41).  Used by the f32-hybrid
 * precision mode of the Tier-B contract only. */
float ro_random_f32(uint64_t s[4]) {
  const uint64_t rnd = ro_xoshiro256_next(s);
  uint32_t lz = clz64(rnd);
  if (lz >= 41) {
    lz = 41 + clz64(ro_xoshiro256_next(s));
    if (lz == 41 + 64) {
      const uint32_t r32 = (uint32_t)ro_xoshiro256_next(s) | 0x7FFu;
      lz += (uint32_t)__builtin_clz(r32);
    }
  }
  const uint32_t mant = (uint32_t)rnd & ((1u << 23) - 1);
  const uint32_t bits = ((126u - lz) << 23) | mant;
  float f;
  memcpy(&f, &bits, 4);
  return f;
}

/* std/math/pow.zig (Go-derived): the integer-exponent branch used by
 * DielectricMaterial.reflectance (material.zig:90, pow(f64, 1-cos, 5.0)).
 * Restated for finite x >= 0 and positive integral y (the only call site). */
static double zig_pow_posint(double x, double y) {
  if (y == 0 || x == 1) return 1;
  if (isnan(x) || isnan(y)) return NAN;
  if (y == 1) return x;
  if (x == 0) {
    /* y > 0: odd integer -> x, else 0 */
    double ip;
    const int odd = (modf(y * 0.5, &ip) != 0.0);
    return odd ? x : 0.0;
  }
  double yi;
  modf(fabs(y), &yi);
  double a1 = 1.0;
  int ae = 0;
  int xe;
  double x1 = frexp(x, &xe);
  int64_t i = (int64_t)yi;
  while (i != 0) {
    const int overflow_shift = 11 + 1;
    if (xe < -(1 << overflow_shift) || (1 << overflow_shift) < xe) {
      ae += xe;
      break;
    }
    if ((i & 1) == 1) {
      a1 *= x1;
      ae += xe;
    }
    x1 *= x1;
    xe <<= 1;
    if (x1 < 0.5) {
      x1 += x1;
      xe -= 1;
    }
    i >>= 1;
  }
  if (y < 0) {
    a1 = 1 / a1;
    ae = -ae;
  }
  return ldexp(a1, ae);
}

double ro_zig_pow(double x, double y) { return zig_pow_posint(x, y); }

/* ===================================================================== */
/* Tier A: f64 value types (vec.zig, ray.zig, hit_record.zig)            */
/* ===================================================================== */

typedef struct { double x, y, z; } V3;
static inline V3 v3(double x, double y, double z) { V3 r = {x, y, z}; return r; }
static inline V3 vadd(V3 a, V3 b) { return v3(a.x + b.x, a.y + b.y, a.z + b.z); }  /* vec.zig:41-47 */
static inline V3 vsub(V3 a, V3 b) { return v3(a.x - b.x, a.y - b.y, a.z - b.z); }  /* vec.zig:49-55 */
static inline V3 vmul(V3 a, double t) { return v3(a.x * t, a.y * t, a.z * t); }    /* vec.zig:57-63 */
static inline V3 vmulv(V3 a, V3 b) { return v3(a.x * b.x, a.y * b.y, a.z * b.z); } /* vec.zig:65-71 */
static inline V3 vdiv(V3 a, double t) { return v3(a.x / t, a.y / t, a.z / t); }    /* vec.zig:73-79 */
static inline double vdot(V3 a, V3 b) { return a.x * b.x + a.y * b.y + a.z * b.z; } /* vec.zig:20-22 */
static inline double vnorm2(V3 a) { return a.x * a.x + a.y * a.y + a.z * a.z; }     /* vec.zig:16-18 */
static inline double vnorm(V3 a) { return sqrt(vnorm2(a)); }                        /* vec.zig:12-14 */
static inline V3 vcross(V3 u, V3 v) {                                               /* vec.zig:24-30 */
  return v3(u.y * v.z - u.z * v.y, u.z * v.x - u.x * v.z, u.x * v.y - u.y * v.x);
}
static inline V3 vnormalized(V3 v) { /* vec.zig:32-39: zero vector returned unchanged */
  const double n = vnorm(v);
  return (n == 0.0) ? v : vdiv(v, n);
}
static inline int vnear_zero(V3 v) { /* vec.zig:98-101 */
  const double e = 1e-8;
  return fabs(v.x) < e && fabs(v.y) < e && fabs(v.z) < e;
}
static inline V3 vload(const double p[3]) { return v3(p[0], p[1], p[2]); }
static inline void vstore(double p[3], V3 v) { p[0] = v.x; p[1] = v.y; p[2] = v.z; }

typedef struct { V3 origin, dir; double time; } RayA; /* ray.zig:5-9 */
static inline V3 ray_at(const RayA *r, double t) { return vadd(r->origin, vmul(r->dir, t)); } /* ray.zig:10-12 */

typedef struct { /* hit_record.zig:7-21 */
  V3 p, normal;
  uint32_t mat;
  double t, u, v;
  int front_face;
} HitA;

/* rand.zig:13-40 over the sequential stream */
static inline double rand01(uint64_t s[4]) { return ro_random_f64(s); }
static inline double rand_range(uint64_t s[4], double mn, double mx) { return mn + rand01(s) * (mx - mn); }
static V3 rand_in_unit_sphere(uint64_t s[4], uint64_t *draws) { /* rand.zig:22-28, vec.zig:88-96 */
  for (;;) {
    V3 p;
    p.x = rand_range(s, -1.0, 1.0);
    p.y = rand_range(s, -1.0, 1.0);
    p.z = rand_range(s, -1.0, 1.0);
    if (draws) *draws += 3;
    if (vnorm(p) >= 1) continue;
    return p;
  }
}
static V3 rand_in_unit_disk(uint64_t s[4], uint64_t *draws) { /* rand.zig:30-36 */
  for (;;) {
    V3 p;
    p.x = rand_range(s, -1.0, 1.0);
    p.y = rand_range(s, -1.0, 1.0);
    p.z = 0.0;
    if (draws) *draws += 2;
    if (vnorm(p) >= 1) continue;
    return p;
  }
}

/* ===================================================================== */
/* Host pieces: camera, image height, cover scene                          */
/* ===================================================================== */

/* Camera.init, main.zig:52-89 */
void ro_camera_init(ro_camera *cam, const double look_from[3], const double look_at[3],
                    const double vup_[3], double vfov, double aspect, double aperture,
                    double focus_dist, double time0, double time1) {
  const double theta = vfov * M_PI / 180.0; /* deg2rad, main.zig:36-38 */
  const double h = tan(theta / 2);
  const double viewport_height = 2.0 * h;
  const double viewport_width = aspect * viewport_height;
  const V3 lf = vload(look_from), la = vload(look_at), vup = vload(vup_);
  const V3 w = vnormalized(vsub(lf, la));
  const V3 u = vnormalized(vcross(vup, w));
  const V3 v = vcross(w, u);
  const V3 origin = lf;
  const V3 horizontal = vmul(u, viewport_width * focus_dist);
  const V3 vertical = vmul(v, viewport_height * focus_dist);
  const V3 llc = vsub(vsub(vsub(origin, vdiv(horizontal, 2.0)), vdiv(vertical, 2.0)), vmul(w, focus_dist));
  vstore(cam->origin, origin);
  vstore(cam->horizontal, horizontal);
  vstore(cam->vertical, vertical);
  vstore(cam->lower_left_corner, llc);
  vstore(cam->u, u);
  vstore(cam->v, v);
  vstore(cam->w, w);
  cam->lens_radius = aperture / 2.0;
  cam->time0 = time0;
  cam->time1 = time1;
}

/* main.zig:306: @intFromFloat(@divTrunc(@as(f64, W), aspect)) */
uint32_t ro_image_height(uint32_t width, double aspect) { return (uint32_t)trunc((double)width / aspect); }

static uint32_t add_mat(ro_scene *sc, uint32_t kind, V3 albedo, V3 odd, double fuzz, double ir) {
  ro_material *m = &sc->mats[sc->n_mats];
  memset(m, 0, sizeof(*m));
  m->kind = kind;
  vstore(m->albedo, albedo);
  vstore(m->albedo_odd, odd);
  m->fuzz = fuzz;
  m->ir = ir;
  return sc->n_mats++;
}
static void add_sphere(ro_scene *sc, V3 c0, V3 c1, double r, double t0, double t1, int moving, uint32_t mat) {
  ro_sphere *s = &sc->spheres[sc->n_spheres++];
  memset(s, 0, sizeof(*s));
  vstore(s->c0, c0);
  vstore(s->c1, c1);
  s->radius = r;
  s->t0 = t0;
  s->t1 = t1;
  s->moving = (uint32_t)moving;
  s->mat = mat;
}

/* generateRandomScene, main.zig:157-221.  Draw order: choose_mat, x jitter,
 * z jitter, then diffuse: 6 albedo draws + center1.y; metal: 3 albedo + fuzz;
 * glass: none. */
int ro_cover_scene(uint64_t rng[4], ro_scene *sc) {
  memset(sc, 0, sizeof(*sc));
  const V3 zero = v3(0, 0, 0);
  /* main.zig:160-175 */
  const uint32_t mat_ground = add_mat(sc, RO_LAMBERT_CHECKER, v3(0.9, 0.9, 0.9), v3(0.2, 0.3, 0.1), 0, 0);
  const uint32_t mat1 = add_mat(sc, RO_DIELECTRIC, zero, zero, 0, 1.5);
  const uint32_t mat2 = add_mat(sc, RO_LAMBERT_SOLID, v3(0.4, 0.2, 0.1), zero, 0, 0);
  const uint32_t mat3 = add_mat(sc, RO_METAL, v3(0.7, 0.6, 0.5), zero, 0.0, 0);
  add_sphere(sc, v3(0, -1000, 0), v3(0, -1000, 0), 1000, 0, 0, 0, mat_ground);
  add_sphere(sc, v3(0, 1, 0), v3(0, 1, 0), 1.0, 0, 0, 0, mat1);
  add_sphere(sc, v3(-4, 1, 0), v3(-4, 1, 0), 1.0, 0, 0, 0, mat2);
  add_sphere(sc, v3(4, 1, 0), v3(4, 1, 0), 1.0, 0, 0, 0, mat3);
  for (int a = -3; a < 3; ++a) {     /* main.zig:177-178 */
    for (int b = -3; b < 3; ++b) {   /* main.zig:179-180 */
      const double choose_mat = rand01(rng);
      V3 center;
      center.x = (double)a + 0.9 * rand01(rng);
      center.y = 0.2;
      center.z = (double)b + 0.9 * rand01(rng);
      if (vnorm(vsub(center, v3(4, 0.2, 0))) <= 0.9) continue; /* main.zig:188 */
      if (choose_mat < 0.8) {
        V3 a1, a2;
        a1.x = rand01(rng); a1.y = rand01(rng); a1.z = rand01(rng);
        a2.x = rand01(rng); a2.y = rand01(rng); a2.z = rand01(rng);
        const V3 albedo = vmulv(a1, a2);
        const uint32_t m = add_mat(sc, RO_LAMBERT_SOLID, albedo, zero, 0, 0);
        const V3 center1 = vadd(center, v3(0, rand_range(rng, 0, 0.5), 0));
        add_sphere(sc, center, center1, 0.2, 0, 1, 1, m);
      } else if (choose_mat < 0.95) {
        V3 albedo;
        albedo.x = rand_range(rng, 0.5, 1);
        albedo.y = rand_range(rng, 0.5, 1);
        albedo.z = rand_range(rng, 0.5, 1);
        const double fuzz = rand_range(rng, 0, 0.5);
        const uint32_t m = add_mat(sc, RO_METAL, albedo, zero, fuzz, 0);
        add_sphere(sc, center, center, 0.2, 0, 0, 0, m);
      } else {
        const uint32_t m = add_mat(sc, RO_DIELECTRIC, zero, zero, 0, 1.5);
        add_sphere(sc, center, center, 0.2, 0, 0, 0, m);
      }
    }
  }
  return (int)sc->n_spheres;
}

/* ===================================================================== */
/* Tier A: hit / scatter / rayColor / render loop                          */
/* ===================================================================== */

typedef struct {
  const ro_scene *scene;
  V3 bg;
  uint64_t *rng;
  ro_stats st;
  uint32_t flags; /* RO_BOOK1_* / RO_MUT_* (ro_render_tier_a_ex), 0 = the current main.zig */
} CtxA;

/* MovingSphere.center, hittable.zig:219-221 */
static inline V3 moving_center(const ro_sphere *s, double t) {
  const V3 c0 = vload(s->c0), c1 = vload(s->c1);
  return vadd(c0, vmul(vsub(c1, c0), (t - s->t0) / (s->t1 - s->t0)));
}

/* Sphere.hit (hittable.zig:95-131) and MovingSphere.hit (:165-201). */
static int sphere_hit(const ro_sphere *s, const RayA *r, double t_min, double t_max, HitA *rec) {
  const V3 center = s->moving ? moving_center(s, r->time) : vload(s->c0);
  const V3 oc = vsub(r->origin, center);
  const double a = vnorm2(r->dir);
  const double half_b = vdot(oc, r->dir);
  const double c = vnorm2(oc) - s->radius * s->radius;
  const double disc = half_b * half_b - a * c;
  if (disc < 0.0) return 0;
  const double sqrtd = sqrt(disc);
  double root = (-half_b - sqrtd) / a;
  if (root < t_min || t_max < root) {
    root = (-half_b + sqrtd) / a;
    if (root < t_min || t_max < root) return 0;
  }
  rec->t = root;
  rec->p = ray_at(r, root);
  const V3 outward = vdiv(vsub(rec->p, center), s->radius);
  rec->front_face = vdot(outward, r->dir) < 0.0;
  rec->normal = rec->front_face ? outward : vmul(outward, -1.0);
  if (!s->moving) { /* getSphereUv, hittable.zig:145-150 (MovingSphere leaves u,v undefined) */
    const double phi = atan2(-outward.z, outward.x) + M_PI;
    const double theta = acos(-outward.y);
    rec->u = phi / (2.0 * M_PI);
    rec->v = theta / M_PI;
  } else {
    rec->u = 0;
    rec->v = 0;
  }
  rec->mat = s->mat;
  return 1;
}

/* HittableList.hit, hittable.zig:231-244: linear closest hit, later wins ties. */
static int world_hit(CtxA *cx, const RayA *r, double t_min, double t_max, HitA *rec) {
  int hit_anything = 0;
  double closest = t_max;
  const ro_scene *sc = cx->scene;
  cx->st.segments++;
  for (uint32_t i = 0; i < sc->n_spheres; ++i) {
    HitA tmp;
    if (sc->spheres[i].moving) cx->st.moving_tests++; else cx->st.static_tests++;
    if (sphere_hit(&sc->spheres[i], r, t_min, closest, &tmp)) {
      hit_anything = 1;
      closest = tmp.t;
      *rec = tmp;
    }
  }
  return hit_anything;
}

/* Texture.value (texture.zig:36-55 solid, :79-82 checker) */
static V3 texture_value(const ro_material *m, V3 p) {
  if (m->kind == RO_LAMBERT_CHECKER) {
    const double sines = sin(10 * p.x) * sin(10 * p.y) * sin(10 * p.z);
    return sines < 0 ? vload(m->albedo_odd) : vload(m->albedo);
  }
  return vload(m->albedo);
}

/* material.zig:112-114 */
static inline V3 reflect(V3 v, V3 n) { return vsub(v, vmul(n, 2 * vdot(v, n))); }
/* material.zig:116-121 */
static inline V3 refract(V3 uv, V3 n, double etai_over_etat) {
  const double cos_theta = fmin(vdot(vmul(uv, -1.0), n), 1.0);
  const V3 perp = vmul(vadd(uv, vmul(n, cos_theta)), etai_over_etat);
  const V3 par = vmul(n, -sqrt(fabs(1.0 - vnorm2(perp))));
  return vadd(perp, par);
}
/* material.zig:87-91 */
static inline double reflectance(double cosine, double ref_idx) {
  const double r0 = (1.0 - ref_idx) / (1.0 + ref_idx);
  const double r1 = r0 * r0;
  return r1 + (1.0 - r1) * zig_pow_posint(1.0 - cosine, 5.0);
}

/* reflectance with another Schlick exponent: test control only (RO_MUT_SCHLICK_EXP) */
static inline double reflectance_exp(double cosine, double ref_idx, double e) {
  const double r0 = (1.0 - ref_idx) / (1.0 + ref_idx);
  const double r1 = r0 * r0;
  return r1 + (1.0 - r1) * pow(1.0 - cosine, e);
}

/* Material.scatter (material.zig:22-29) */
static int scatter_a(CtxA *cx, const RayA *r_in, const HitA *rec, V3 *att, RayA *scattered) {
  const ro_material *m = &cx->scene->mats[rec->mat];
  switch (m->kind) {
    case RO_LAMBERT_SOLID:
    case RO_LAMBERT_CHECKER: { /* material.zig:44-52 */
      const V3 b = rand_in_unit_sphere(cx->rng, &cx->st.draws);
      /* RO_MUT_LAMBERT_NONORM: test control only (tests/test_readme_image.py) */
      V3 dir = vadd(rec->normal, (cx->flags & RO_MUT_LAMBERT_NONORM) ? b : vnormalized(b));
      if (vnear_zero(dir)) dir = rec->normal;
      scattered->origin = rec->p;
      scattered->dir = dir;
      scattered->time = r_in->time;
      *att = texture_value(m, rec->p);
      return 1;
    }
    case RO_METAL: { /* material.zig:59-65 */
      const V3 reflected = reflect(vnormalized(r_in->dir), rec->normal);
      scattered->origin = rec->p;
      scattered->dir = vadd(reflected, vmul(rand_in_unit_sphere(cx->rng, &cx->st.draws), m->fuzz));
      scattered->time = r_in->time;
      *att = vload(m->albedo);
      if (cx->flags & RO_MUT_METAL_SCATTERED) return vdot(scattered->dir, rec->normal) > 0.0; /* test control */
      return vdot(reflected, rec->normal) > 0.0;
    }
    case RO_DIELECTRIC: { /* material.zig:72-85 */
      const double ratio = rec->front_face ? 1.0 / m->ir : m->ir;
      const V3 unit_dir = vnormalized(r_in->dir);
      const double cos_theta = fmin(vdot(vmul(unit_dir, -1.0), rec->normal), 1.0);
      const double sin_theta = sqrt(1.0 - cos_theta * cos_theta);
      const int can_refract = ratio * sin_theta <= 1.0;
      int do_refract = 0;
      if (cx->flags & RO_MUT_DIEL_ALWAYS_DRAW) { /* test control: no short circuit (draws on TIR too) */
        cx->st.draws++;
        const double r = rand01(cx->rng);
        do_refract = can_refract && reflectance(cos_theta, ratio) < r;
      } else if (can_refract) { /* short-circuit `and`: the draw happens only here */
        cx->st.draws++;
        const double refl = (cx->flags & RO_MUT_SCHLICK_EXP) ? reflectance_exp(cos_theta, ratio, 2.0)
                                                             : reflectance(cos_theta, ratio);
        do_refract = refl < rand01(cx->rng);
      }
      scattered->origin = rec->p;
      scattered->dir = do_refract ? refract(unit_dir, rec->normal, ratio) : reflect(unit_dir, rec->normal);
      scattered->time = r_in->time;
      *att = v3(1.0, 1.0, 1.0);
      return 1;
    }
  }
  return 0;
}

/* rayColor, main.zig:103-122 (recursive; emitted == 0 for these materials) */
static V3 ray_color_a(CtxA *cx, const RayA *r, uint32_t depth) {
  if (depth == 0) return v3(0.0, 0.0, 0.0);
  HitA rec = {{0, 0, 0}, {0, 0, 0}, 0, 0, 0, 0, 0}; /* (set by world_hit when it returns 1) */
  if (!world_hit(cx, r, 0.001, INFINITY, &rec)) {
    if (cx->flags & RO_BOOK1_SKY) { /* the Book-1 sky of the reference's README image (ro_render_tier_a_ex) */
      const V3 ud = vnormalized(r->dir);
      const double t = 0.5 * (ud.y + 1.0);
      return vadd(vmul(v3(1.0, 1.0, 1.0), 1.0 - t), vmul(v3(0.5, 0.7, 1.0), t));
    }
    return cx->bg;
  }
  RayA scattered;
  V3 att;
  const V3 emitted = v3(0, 0, 0); /* Material.emitted, material.zig:31-38 */
  if (scatter_a(cx, r, &rec, &att, &scattered))
    return vadd(emitted, vmulv(att, ray_color_a(cx, &scattered, depth - 1)));
  return emitted;
}

/* Camera.getRay, main.zig:91-100 */
static RayA get_ray_a(const ro_camera *cam, uint64_t rng[4], double s, double t, uint64_t *draws, int time_draw) {
  const V3 rd = vmul(rand_in_unit_disk(rng, draws), cam->lens_radius);
  const V3 offset = vadd(vmul(vload(cam->u), rd.x), vmul(vload(cam->v), rd.y));
  const V3 dir = vsub(vsub(vadd(vadd(vload(cam->lower_left_corner), vmul(vload(cam->horizontal), s)),
                               vmul(vload(cam->vertical), t)),
                          vload(cam->origin)),
                     offset);
  RayA r;
  r.origin = vadd(vload(cam->origin), offset);
  r.dir = dir;
  if (!time_draw) { /* Book-1 camera: no shutter time */
    r.time = cam->time0;
    return r;
  }
  r.time = rand_range(rng, cam->time0, cam->time1);
  if (draws) *draws += 1;
  return r;
}

/* main.zig:395-400 */
uint8_t ro_quantize(double c, double scale) {
  const double g = sqrt(c * scale);
  const double cl = fmax(0.0, fmin(g, 0.999)); /* std.math.clamp = @max(lo, @min(v, hi)) */
  return (uint8_t)(256.0 * cl);
}

/* Render loop, main.zig:378-402: j rows, i columns, s samples, one stream.
 * ro_render_tier_a_ex: the same loop over the first `rows` values of j only
 * (the stream of row j depends on rows < j alone), with `flags` selecting the
 * Book-1 variant of the README image (RO_BOOK1_SKY: the gradient sky of the
 * book's first volume instead of `bg`; RO_BOOK1_NO_TIME: Camera.getRay draws
 * no shutter time) — test infrastructure for tests/test_readme_image.py. */
void ro_render_tier_a_ex(const ro_scene *scene, const ro_camera *cam, const double bg[3],
                         uint32_t W, uint32_t H, uint32_t spp, uint32_t depth,
                         uint64_t rng[4], uint8_t *rgb, double *sum_out, ro_stats *stats,
                         uint32_t flags, uint32_t rows) {
  CtxA cx;
  memset(&cx, 0, sizeof(cx));
  cx.scene = scene;
  cx.bg = vload(bg);
  cx.rng = rng;
  cx.flags = flags;
  for (uint32_t j = 0; j < H && j < rows; ++j) {
    for (uint32_t i = 0; i < W; ++i) {
      V3 pc = v3(0.0, 0.0, 0.0);
      for (uint32_t s = 0; s < spp; ++s) {
        const double u = ((double)i + rand01(rng)) / ((double)W - 1.0);
        const double v = ((double)j + rand01(rng)) / ((double)H - 1.0);
        cx.st.draws += 2;
        const RayA r = get_ray_a(cam, rng, u, v, &cx.st.draws, !(flags & RO_BOOK1_NO_TIME));
        pc = vadd(pc, ray_color_a(&cx, &r, depth));
        cx.st.samples++;
      }
      const double scale = 1.0 / (double)spp;
      const size_t o = ((size_t)i + (size_t)(H - j - 1) * W) * 3;
      rgb[o + 0] = ro_quantize(pc.x, scale);
      rgb[o + 1] = ro_quantize(pc.y, scale);
      rgb[o + 2] = ro_quantize(pc.z, scale);
      if (sum_out) { sum_out[o + 0] = pc.x; sum_out[o + 1] = pc.y; sum_out[o + 2] = pc.z; }
    }
  }
  if (stats) *stats = cx.st;
}
/* Tier A's per-sample arithmetic (flags as ro_render_tier_a_ex) over image
 * loop rows j in [row0, row1), with one stream PER PIXEL: DefaultPrng seeded
 * with SplitMix64(seed + pixel) (pixel = j * W + i) instead of the reference's
 * single stream.  Test infrastructure for the README pin's matched-filter
 * statistic (tests/test_readme_image.py): renders of the same pixels with and
 * without a mutated rule then share their random numbers until the mutation
 * first changes a path (common random numbers), so their difference is the
 * rule's systematic effect, not render noise; row bands are independent, so
 * callers run them on several threads.  sum_out: W*H*3 f64 sums (layout of
 * ro_render_tier_a; only the bands' rows written). */
void ro_render_tier_a_pixel_streams(const ro_scene *scene, const ro_camera *cam, const double bg[3], uint32_t W,
                                    uint32_t H, uint32_t spp, uint32_t depth, uint64_t seed, double *sum_out,
                                    uint32_t flags, uint32_t row0, uint32_t row1) {
  CtxA cx;
  memset(&cx, 0, sizeof(cx));
  cx.scene = scene;
  cx.bg = vload(bg);
  cx.flags = flags;
  uint64_t rng[4];
  cx.rng = rng;
  for (uint32_t j = row0; j < H && j < row1; ++j) {
    for (uint32_t i = 0; i < W; ++i) {
      uint64_t sm = seed + (uint64_t)j * W + i;
      ro_xoshiro256_seed(rng, ro_splitmix64_next(&sm));
      V3 pc = v3(0.0, 0.0, 0.0);
      for (uint32_t s = 0; s < spp; ++s) {
        const double u = ((double)i + rand01(rng)) / ((double)W - 1.0);
        const double v = ((double)j + rand01(rng)) / ((double)H - 1.0);
        const RayA r = get_ray_a(cam, rng, u, v, NULL, !(flags & RO_BOOK1_NO_TIME));
        pc = vadd(pc, ray_color_a(&cx, &r, depth));
      }
      const size_t o = ((size_t)i + (size_t)(H - j - 1) * W) * 3;
      sum_out[o + 0] = pc.x;
      sum_out[o + 1] = pc.y;
      sum_out[o + 2] = pc.z;
    }
  }
}
void ro_render_tier_a(const ro_scene *scene, const ro_camera *cam, const double bg[3],
                      uint32_t W, uint32_t H, uint32_t spp, uint32_t depth,
                      uint64_t rng[4], uint8_t *rgb, double *sum_out, ro_stats *stats) {
  ro_render_tier_a_ex(scene, cam, bg, W, H, spp, depth, rng, rgb, sum_out, stats, 0u, H);
}

/* main(), main.zig:295-402 with scene == 1 and the given image parameters. */
void ro_main_cover(uint32_t W, double aspect, uint32_t spp, uint32_t depth, uint64_t seed,
                   uint8_t *rgb, ro_stats *stats) {
  uint64_t rng[4];
  ro_xoshiro256_seed(rng, seed);
  static ro_scene scene; /* large; not re-entrant (oracle is test infra) */
  ro_cover_scene(rng, &scene);
  const double bg[3] = {0.70, 0.80, 1.00};
  const double lf[3] = {13, 2, 3}, la[3] = {0, 0, 0}, vup[3] = {0, 1, 0};
  ro_camera cam;
  ro_camera_init(&cam, lf, la, vup, 20.0, aspect, 0.1, 10.0, 0, 1);
  const uint32_t H = ro_image_height(W, aspect);
  ro_render_tier_a(&scene, &cam, bg, W, H, spp, depth, rng, rgb, NULL, stats);
}

/* ===================================================================== */
/* Tier B: the GPU contract (per-sample counter-keyed Xoshiro256++)        */
/* ===================================================================== */

/* Tier-B RNG: a COUNTER-BASED generator over SplitMix64's Weyl sequence.
 * base = SplitMix64.init(seed).next() (std/Random/SplitMix64.zig, as
 * Tier A's seeding); sample (pixel p, sample s) owns the disjoint block of
 * 2^16 consecutive Weyl states starting at
 *   base + (((p << 24) | s) << 16) * gamma,
 * and its draws are ro_tb_mix of the next states: draw k of the sample is
 * ro_tb_mix(that state + (k + 1) * gamma).  Every draw of a frame is the mix
 * of a distinct element of ONE Weyl sequence (gamma is odd, so n -> n*gamma
 * is a bijection), any draw is computable from (p, s, k) alone, and
 * u64 -> f64/f32 is Zig's Random.float as in Tier A.
 *
 * The mixer (round 5; rounds 1-4 used SplitMix64's own output function,
 * ro_splitmix64_next's last three lines): four Feistel half-rounds on the
 * state's 32-bit words (hi, lo), each a 32x32 -> 64-bit product and one xor:
 *   t = hi * M0; lo ^= t >> 32; hi = (uint32)t;   then lo * M1 into hi,
 *   hi * M2 into lo, lo * M3 into hi.
 * It is a bijection of the 64-bit state.  The reference renders with ONE
 * sequential Xoshiro256++ stream (main.zig:300), which no parallel renderer
 * can reproduce, so Tier B's only requirement on the mixer is statistical:
 * tests/native/rng_stats.c (mixer 10) checks bit bias, byte uniformity,
 * lag-1/2/3 pairs and triples of one sample's draws, and every byte of the
 * draws of neighbouring samples and pixels over 2^32 draws laid out as a
 * render uses them (tests/test_rng_stats.py); Tier C checks
 * the image against Tier A's. */
uint64_t ro_tb_mix(uint64_t z) {
  static const uint32_t M[4] = {0xD2511F53u, 0xCD9E8D57u, 0x9E3779B1u, 0x85EBCA6Bu};
  uint32_t hi = (uint32_t)(z >> 32), lo = (uint32_t)z;
  uint64_t t;
  t = (uint64_t)hi * M[0];
  lo ^= (uint32_t)(t >> 32);
  hi = (uint32_t)t;
  t = (uint64_t)lo * M[1];
  hi ^= (uint32_t)(t >> 32);
  lo = (uint32_t)t;
  t = (uint64_t)hi * M[2];
  lo ^= (uint32_t)(t >> 32);
  hi = (uint32_t)t;
  t = (uint64_t)lo * M[3];
  hi ^= (uint32_t)(t >> 32);
  lo = (uint32_t)t;
  return ((uint64_t)hi << 32) | lo;
}
static inline uint64_t tb_next(uint64_t *st) {
  *st += 0x9e3779b97f4a7c15ULL;
  return ro_tb_mix(*st);
}

static inline uint64_t tierb_state(uint64_t seed, uint64_t pixel, uint64_t sample) {
  uint64_t sm = seed;
  const uint64_t base = ro_splitmix64_next(&sm);
  const uint64_t block = ((pixel << 24) | sample) << 16;
  return base + block * 0x9e3779b97f4a7c15ULL;
}

/* Tier-B reals: Zig's Random.float over the counter stream, with ONE rule
 * change that makes every draw exactly one Weyl step (so draw k of a sample is
 * random-access): when the draw's u64 has >= 12 (f64) / >= 41 (f32) leading
 * zeros, Zig takes further u64s from the same generator; here they come from
 * the draw's own extension stream: the Weyl sequence from state_of_draw ^
 * kTierBExt through the same mixer.  Probability 2^-12 / 2^-41 per draw; the
 * value distribution is unchanged. */
#define kTierBExt 0x5851F42D4C957F2DULL

double ro_sm_f64(uint64_t *st) {
  const uint64_t rnd = tb_next(st);
  uint64_t lz = clz64(rnd);
  if (lz >= 12) {
    uint64_t ext = *st ^ kTierBExt;
    lz = 12;
    for (;;) {
      const uint64_t addl = clz64(tb_next(&ext));
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

float ro_sm_f32(uint64_t *st) {
  const uint64_t rnd = tb_next(st);
  uint32_t lz = clz64(rnd);
  if (lz >= 41) {
    uint64_t ext = *st ^ kTierBExt;
    lz = 41 + clz64(tb_next(&ext));
    if (lz == 41 + 64) {
      const uint32_t r32 = (uint32_t)tb_next(&ext) | 0x7FFu;
      lz += (uint32_t)__builtin_clz(r32);
    }
  }
  const uint32_t bits = ((126u - lz) << 23) | ((uint32_t)rnd & ((1u << 23) - 1));
  float f;
  memcpy(&f, &bits, 4);
  return f;
}

uint64_t ro_tierb_state(uint64_t seed, uint64_t pixel, uint64_t sample) {
  return tierb_state(seed, pixel, sample);
}

int ro_tb_trace = 0; /* tierb_core.h: per-segment trace on stderr (diagnostics) */
#define TB_REAL double
#define TB_SUFFIX _f64
#define TB_IS_F32 0
#include "tierb_core.h"
#undef TB_REAL
#undef TB_SUFFIX
#undef TB_IS_F32

#define TB_REAL float
#define TB_SUFFIX _f32
#define TB_IS_F32 1
#include "tierb_core.h"
#undef TB_REAL
#undef TB_SUFFIX
#undef TB_IS_F32

void ro_render_tier_b(const ro_scene *scene, const ro_camera *cam, const ro_params *p,
                      uint8_t *rgb, float *mean_out, ro_stats *stats) {
  if (p->precision == 1)
    tierb_render_f32(scene, cam, p, rgb, mean_out, stats);
  else
    tierb_render_f64(scene, cam, p, rgb, mean_out, stats);
}

void ro_tierb_samples(const ro_scene *scene, const ro_camera *cam, const ro_params *p, uint32_t y, uint32_t x,
                      uint32_t s0, uint32_t n, double *out, int trace) {
  ro_tb_trace = trace;
  if (p->precision == 1)
    tierb_samples_f32(scene, cam, p, y, x, s0, n, out);
  else
    tierb_samples_f64(scene, cam, p, y, x, s0, n, out);
  ro_tb_trace = 0;
}
