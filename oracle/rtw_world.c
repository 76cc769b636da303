/*
 * rtw_world.c — CPU ORACLE for the general-world renders.  TEST
 * INFRASTRUCTURE ONLY (see rtw_world.h for the contract and the rules).
 * Every function cites the reference file:line it restates
 * (nsfisis/RayTracingInOneWeekend.zig, src/).
 */
#include "rtw_world.h"

#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>
#ifdef _OPENMP
#include <omp.h>
#endif

#include "ro_libm.h"

/* ------------------------------------------------------------ vec.zig -- */
typedef struct { double x, y, z; } V;
static inline V v3(double x, double y, double z) { V r = {x, y, z}; return r; }
static inline V vadd(V a, V b) { return v3(a.x + b.x, a.y + b.y, a.z + b.z); }
static inline V vsub(V a, V b) { return v3(a.x - b.x, a.y - b.y, a.z - b.z); }
static inline V vmul(V a, double t) { return v3(a.x * t, a.y * t, a.z * t); }
static inline V vmulv(V a, V b) { return v3(a.x * b.x, a.y * b.y, a.z * b.z); }
static inline V vdiv(V a, double t) { return v3(a.x / t, a.y / t, a.z / t); }
static inline double vdot(V a, V b) { return a.x * b.x + a.y * b.y + a.z * b.z; }
static inline double vnorm2(V a) { return a.x * a.x + a.y * a.y + a.z * a.z; }
static inline double vnorm(V a) { return sqrt(vnorm2(a)); }
static inline V vnormalized(V v) { const double n = vnorm(v); return n == 0.0 ? v : vdiv(v, n); } /* vec.zig:32-39 */
static inline int vnear_zero(V v) { return fabs(v.x) < 1e-8 && fabs(v.y) < 1e-8 && fabs(v.z) < 1e-8; }
static inline V vld(const double p[3]) { return v3(p[0], p[1], p[2]); }
static inline void vst(double p[3], V v) { p[0] = v.x; p[1] = v.y; p[2] = v.z; }

double rw_sin(double x) { return ro_sin(x); }
double rw_cos(double x) { return ro_cos(x); }
double rw_atan2(double y, double x) { return ro_atan2(y, x); }
double rw_acos(double x) { return ro_acos(x); }

/* ---------------------------------------------------- Zig std.Random -- */
static inline double rnd01(uint64_t s[4]) { return ro_random_f64(s); }
static inline double rnd_range(uint64_t s[4], double mn, double mx) { return mn + rnd01(s) * (mx - mn); }

/* Random.uintLessThan(u64) (Zig 0.14 std/Random.zig, Lemire's method with
 * the pcg-random "extra tweak") and intRangeLessThan for unsigned T
 * (= at_least + uintLessThan(less_than - at_least)); r.int(u64) is one
 * Xoshiro256.next() (fill of 8 bytes, little-endian).  rand.zig:8-10. */
uint64_t rw_int_range_less_than_u64(uint64_t rng[4], uint64_t at_least, uint64_t less_than) {
  const uint64_t lt = less_than - at_least;
  uint64_t x = ro_xoshiro256_next(rng);
  unsigned __int128 m = (unsigned __int128)x * lt;
  uint64_t l = (uint64_t)m;
  if (l < lt) {
    uint64_t t = (uint64_t)0 - lt;
    if (t >= lt) {
      t -= lt;
      if (t >= lt) t %= lt;
    }
    while (l < t) {
      x = ro_xoshiro256_next(rng);
      m = (unsigned __int128)x * lt;
      l = (uint64_t)m;
    }
  }
  return at_least + (uint64_t)(m >> 64);
}

/* ---------------------------------------------------------- perlin.zig -- */
/* Perlin.init, perlin.zig:18-40 */
static void perlin_init(rw_perlin *p, uint64_t rng[4]) {
  for (int i = 0; i < 256; ++i) {
    V r;
    r.x = rnd_range(rng, -1, 1);  /* Vec3.random, vec.zig:90-96 */
    r.y = rnd_range(rng, -1, 1);
    r.z = rnd_range(rng, -1, 1);
    vst(p->ranvec[i], vnormalized(r));
    p->perm[0][i] = p->perm[1][i] = p->perm[2][i] = (uint32_t)i;
  }
  for (int a = 0; a < 3; ++a) { /* permute, perlin.zig:93-102: target in [0, i) */
    uint32_t *q = p->perm[a];
    for (uint64_t i = 255; i > 0; --i) {
      const uint64_t target = rw_int_range_less_than_u64(rng, 0, i);
      const uint32_t tmp = q[i];
      q[i] = q[target];
      q[target] = tmp;
    }
  }
}

/* Perlin.noise, perlin.zig:49-79 (+ perlinInterp :104-124).  The reference
 * casts i + di to usize with @intCast; for negative cells that is illegal
 * behaviour in safe builds and a two's-complement wrap in ReleaseFast (the
 * `& 255` then picks the cell modulo 256) — the wrap is restated here. */
double rw_perlin_noise(const rw_perlin *p, const double pt[3]) {
  const double u = pt[0] - floor(pt[0]), v = pt[1] - floor(pt[1]), w = pt[2] - floor(pt[2]);
  const double uu = u * u * (3 - 2 * u), vv = v * v * (3 - 2 * v), ww = w * w * (3 - 2 * w);
  const int32_t i = (int32_t)floor(pt[0]), j = (int32_t)floor(pt[1]), k = (int32_t)floor(pt[2]);
  double accum = 0.0;
  for (int di = 0; di < 2; ++di)
    for (int dj = 0; dj < 2; ++dj)
      for (int dk = 0; dk < 2; ++dk) {
        const uint32_t ix = (uint32_t)(i + di) & 255u, iy = (uint32_t)(j + dj) & 255u, iz = (uint32_t)(k + dk) & 255u;
        const double *c = p->ranvec[p->perm[0][ix] ^ p->perm[1][iy] ^ p->perm[2][iz]];
        const double ti = (double)di, tj = (double)dj, tk = (double)dk;
        const V weight = v3(uu - ti, vv - tj, ww - tk);
        accum += (ti * uu + (1.0 - ti) * (1.0 - uu)) * (tj * vv + (1.0 - tj) * (1.0 - vv)) *
                 (tk * ww + (1.0 - tk) * (1.0 - ww)) * vdot(vld(c), weight);
      }
  return accum;
}

/* Perlin.turb, perlin.zig:81-91 */
double rw_perlin_turb(const rw_perlin *p, const double pt[3], uint32_t depth) {
  double accum = 0.0, weight = 1.0;
  double q[3] = {pt[0], pt[1], pt[2]};
  for (uint32_t i = 0; i < depth; ++i) {
    accum += weight * rw_perlin_noise(p, q);
    weight *= 0.5;
    q[0] = q[0] * 2.0;
    q[1] = q[1] * 2.0;
    q[2] = q[2] * 2.0;
  }
  return fabs(accum);
}

/* --------------------------------------------------------- texture.zig -- */
/* Texture.value, texture.zig:36-144. */
void rw_texture_value(const rw_world *w, uint32_t tex, double u, double v, const double p[3], double out[3]) {
  const rw_texture *t = &w->textures[tex];
  switch (t->kind) {
    case RW_TEX_CHECKER: { /* :79-82 */
      const double sines = ro_sin(10 * p[0]) * ro_sin(10 * p[1]) * ro_sin(10 * p[2]);
      const double *c = sines < 0 ? t->odd : t->even;
      out[0] = c[0], out[1] = c[1], out[2] = c[2];
      return;
    }
    case RW_TEX_NOISE: { /* :101-105 */
      const double k = 0.5 * (1.0 + ro_sin(t->scale * p[2] + 10.0 * rw_perlin_turb(&w->perlins[t->perlin], p, 7)));
      out[0] = 1 * k, out[1] = 1 * k, out[2] = 1 * k;
      return;
    }
    case RW_TEX_IMAGE: { /* :121-144 */
      const rw_image *im = &w->images[t->image];
      const double uc = fmax(0.0, fmin(u, 1.0));        /* std.math.clamp */
      const double vc = 1.0 - fmax(0.0, fmin(v, 1.0));
      const uint64_t i = (uint64_t)(uc * (double)im->width);
      const uint64_t j = (uint64_t)(vc * (double)im->height);
      const uint64_t i_ = i < im->width - 1 ? i : im->width - 1;
      /* :130 clamps j against width - 1 (a reference bug): j == height (only
       * at v == 0 exactly) would read past the pixels; clamped to the last
       * row here. */
      uint64_t j_ = j < im->width - 1 ? j : im->width - 1;
      if (j_ > im->height - 1) j_ = im->height - 1;
      const uint8_t *px = im->rgba + (j_ * im->width + i_) * 4;
      if ((double)px[3] == 0) { /* ocean */
        out[0] = 0, out[1] = 0, out[2] = 1.0;
      } else {
        const double s = 1.0 / 255.0;
        out[0] = s * (double)px[0], out[1] = s * (double)px[1], out[2] = s * (double)px[2];
      }
      return;
    }
    default: /* solid, :46-55 */
      out[0] = t->color[0], out[1] = t->color[1], out[2] = t->color[2];
      return;
  }
}

/* -------------------------------------------------------- hittable.zig -- */
/* Sphere.getSphereUv, hittable.zig:145-150 */
void rw_sphere_uv(const double p[3], double *u, double *v) {
  const double pi = 3.14159265358979323846;
  const double phi = ro_atan2(-p[2], p[0]) + pi;
  const double theta = ro_acos(-p[1]);
  *u = phi / (2.0 * pi);
  *v = theta / pi;
}

typedef struct { V o, d; double time; } Ray;
typedef struct { V p, normal; double t, u, v; int front; uint32_t mat; } Rec;

static inline V moving_center(const rw_prim *s, double time) { /* hittable.zig:219-221 */
  const V c0 = vld(s->a), c1 = vld(s->a + 3);
  return vadd(c0, vmul(vsub(c1, c0), (time - s->a[7]) / (s->a[8] - s->a[7])));
}

/* Object-space hit of one primitive (no wrappers). */
static int base_hit(const rw_prim *s, const Ray *r, double t_min, double t_max, Rec *rec) {
  if (s->kind == RW_SPHERE || s->kind == RW_MOVING) { /* :95-131, :165-201 */
    const V center = s->kind == RW_MOVING ? moving_center(s, r->time) : vld(s->a);
    const double radius = s->a[6];
    const V oc = vsub(r->o, center);
    const double a = vnorm2(r->d);
    const double half_b = vdot(oc, r->d);
    const double c = vnorm2(oc) - radius * radius;
    const double disc = half_b * half_b - a * c;
    if (disc < 0.0) return 0;
    const double sq = sqrt(disc);
    double root = (-half_b - sq) / a;
    if (root < t_min || t_max < root) {
      root = (-half_b + sq) / a;
      if (root < t_min || t_max < root) return 0;
    }
    rec->t = root;
    rec->p = vadd(r->o, vmul(r->d, root));
    const V outward = vdiv(vsub(rec->p, center), radius);
    rec->front = vdot(outward, r->d) < 0.0;
    rec->normal = rec->front ? outward : vmul(outward, -1.0);
    if (s->kind == RW_SPHERE) {
      double p[3];
      vst(p, outward);
      rw_sphere_uv(p, &rec->u, &rec->v);
    } else { /* MovingSphere.hit leaves u, v undefined; 0 here */
      rec->u = 0, rec->v = 0;
    }
    rec->mat = s->mat;
    return 1;
  }
  /* XyRect :278-302, XzRect :333-357, YzRect :388-412 */
  double ok, oa, ob, dk, da, db;
  V n;
  if (s->kind == RW_XY) {
    ok = r->o.z, oa = r->o.x, ob = r->o.y, dk = r->d.z, da = r->d.x, db = r->d.y, n = v3(0, 0, 1);
  } else if (s->kind == RW_XZ) {
    ok = r->o.y, oa = r->o.x, ob = r->o.z, dk = r->d.y, da = r->d.x, db = r->d.z, n = v3(0, 1, 0);
  } else {
    ok = r->o.x, oa = r->o.y, ob = r->o.z, dk = r->d.x, da = r->d.y, db = r->d.z, n = v3(1, 0, 0);
  }
  const double a0 = s->a[0], a1 = s->a[1], b0 = s->a[2], b1 = s->a[3], k = s->a[4];
  const double t = (k - ok) / dk;
  if (t < t_min || t > t_max) return 0;
  const double x = oa + t * da;
  const double y = ob + t * db;
  if (x < a0 || x > a1 || y < b0 || y > b1) return 0;
  rec->u = (x - a0) / (a1 - a0);
  rec->v = (y - b0) / (b1 - b0);
  rec->t = t;
  rec->mat = s->mat;
  rec->p = vadd(r->o, vmul(r->d, t));
  rec->front = vdot(n, r->d) < 0.0;
  rec->normal = rec->front ? n : vmul(n, -1.0);
  return 1;
}

/* Translate.hit (:478-491) / RotateY.hit (:561-600) wrappers, op 0 outermost. */
static int prim_hit(const rw_world *w, const rw_prim *s, const Ray *r, double t_min, double t_max, Rec *rec) {
  if (s->xform < 0) return base_hit(s, r, t_min, t_max, rec);
  const rw_xform *x = &w->xforms[s->xform];
  Ray rr = *r;
  for (uint32_t i = 0; i < x->n; ++i) { /* ray into object space, outermost first */
    if (x->op[i] == RW_XF_TRANSLATE) {
      rr.o = vsub(rr.o, vld(x->v[i]));
    } else {
      const double sn = x->v[i][0], cs = x->v[i][1];
      const V o = rr.o, d = rr.d;
      rr.o.x = cs * o.x - sn * o.z;
      rr.o.z = sn * o.x + cs * o.z;
      rr.d.x = cs * d.x - sn * d.z;
      rr.d.z = sn * d.x + cs * d.z;
    }
  }
  if (!base_hit(s, &rr, t_min, t_max, rec)) return 0;
  for (int i = (int)x->n - 1; i >= 0; --i) { /* record back to world space, innermost first */
    if (x->op[i] == RW_XF_TRANSLATE) {
      rec->p = vadd(rec->p, vld(x->v[i]));
    } else {
      const double sn = x->v[i][0], cs = x->v[i][1];
      const V p = rec->p, nn = rec->normal;
      rec->p.x = cs * p.x + sn * p.z;
      rec->p.z = -sn * p.x + cs * p.z;
      rec->normal.x = cs * nn.x + sn * nn.z;
      rec->normal.z = -sn * nn.x + cs * nn.z;
    }
  }
  return 1;
}

/* HittableList.hit, :231-244 over the flattened world. */
static int world_hit(const rw_world *w, const Ray *r, double t_min, double t_max, Rec *rec, ro_stats *st) {
  int hit = 0;
  double closest = t_max;
  if (st) st->segments++;
  for (uint32_t i = 0; i < w->n_prims; ++i) {
    Rec tmp;
    if (prim_hit(w, &w->prims[i], r, t_min, closest, &tmp)) {
      hit = 1;
      closest = tmp.t;
      *rec = tmp;
    }
  }
  return hit;
}

int rw_hit(const rw_world *w, const double o[3], const double d[3], double time, double t_min, double t_max,
           double *t_out, double p_out[3], double normal_out[3], double uv_out[2], int *front_out) {
  Ray r = {vld(o), vld(d), time};
  int best = -1;
  double closest = t_max;
  Rec rec, tmp;
  for (uint32_t i = 0; i < w->n_prims; ++i)
    if (prim_hit(w, &w->prims[i], &r, t_min, closest, &tmp)) {
      best = (int)i;
      closest = tmp.t;
      rec = tmp;
    }
  if (best >= 0) {
    *t_out = rec.t;
    vst(p_out, rec.p);
    vst(normal_out, rec.normal);
    uv_out[0] = rec.u, uv_out[1] = rec.v;
    *front_out = rec.front;
  }
  return best;
}

/* -------------------------------------------------------- material.zig -- */
static inline V reflect(V v, V n) { return vsub(v, vmul(n, 2 * vdot(v, n))); } /* :112-114 */
static inline V refract(V uv, V n, double eta) {                                 /* :116-121 */
  const double cos_theta = fmin(vdot(vmul(uv, -1.0), n), 1.0);
  const V perp = vmul(vadd(uv, vmul(n, cos_theta)), eta);
  const V par = vmul(n, -sqrt(fabs(1.0 - vnorm2(perp))));
  return vadd(perp, par);
}
static inline double reflectance(double cosine, double ref_idx) { /* :87-91, Zig pow(x, 5.0) */
  const double r0 = (1.0 - ref_idx) / (1.0 + ref_idx);
  const double r1 = r0 * r0;
  return r1 + (1.0 - r1) * ro_zig_pow(1.0 - cosine, 5.0);
}

static V tex_value(const rw_world *w, uint32_t tex, const Rec *rec) {
  double p[3], out[3];
  vst(p, rec->p);
  rw_texture_value(w, tex, rec->u, rec->v, p, out);
  return vld(out);
}

/* Draw source for scatter: the sequential stream (Tier A) or the Tier-B
 * counter stream. */
typedef struct {
  uint64_t *seq;  /* Tier A: Xoshiro256 state */
  uint64_t *ctr;  /* Tier B: SplitMix64 Weyl state */
} Rng;
static inline double rng01(Rng *g) { return g->seq ? ro_random_f64(g->seq) : ro_sm_f64(g->ctr); }
static inline double rng_range(Rng *g, double mn, double mx) { return mn + rng01(g) * (mx - mn); }
static V rng_in_unit_sphere(Rng *g, ro_stats *st) { /* rand.zig:22-28 */
  for (;;) {
    V p;
    p.x = rng_range(g, -1.0, 1.0);
    p.y = rng_range(g, -1.0, 1.0);
    p.z = rng_range(g, -1.0, 1.0);
    if (st) st->draws += 3;
    if (vnorm(p) >= 1) continue;
    return p;
  }
}
static V rng_in_unit_disk(Rng *g, ro_stats *st) { /* rand.zig:30-36 */
  for (;;) {
    V p;
    p.x = rng_range(g, -1.0, 1.0);
    p.y = rng_range(g, -1.0, 1.0);
    p.z = 0.0;
    if (st) st->draws += 2;
    if (vnorm(p) >= 1) continue;
    return p;
  }
}

/* Material.scatter, material.zig:22-29 (+ DiffuseLight :94-110: no scatter). */
static int scatter(const rw_world *w, const Ray *r_in, const Rec *rec, Rng *g, V *att, Ray *out, ro_stats *st) {
  const rw_material *m = &w->mats[rec->mat];
  switch (m->kind) {
    case RW_LAMBERT: { /* :44-52 */
      V dir = vadd(rec->normal, vnormalized(rng_in_unit_sphere(g, st)));
      if (vnear_zero(dir)) dir = rec->normal;
      out->o = rec->p, out->d = dir, out->time = r_in->time;
      *att = tex_value(w, m->tex, rec);
      return 1;
    }
    case RW_METAL: { /* :59-65 */
      const V refl = reflect(vnormalized(r_in->d), rec->normal);
      out->o = rec->p;
      out->d = vadd(refl, vmul(rng_in_unit_sphere(g, st), m->fuzz));
      out->time = r_in->time;
      *att = vld(m->albedo);
      return vdot(refl, rec->normal) > 0.0;
    }
    case RW_DIELECTRIC: { /* :72-85 */
      const double ratio = rec->front ? 1.0 / m->ir : m->ir;
      const V ud = vnormalized(r_in->d);
      const double cos_t = fmin(vdot(vmul(ud, -1.0), rec->normal), 1.0);
      const double sin_t = sqrt(1.0 - cos_t * cos_t);
      int refr = 0;
      if (ratio * sin_t <= 1.0) {
        if (st) st->draws++;
        refr = reflectance(cos_t, ratio) < rng01(g);
      }
      out->o = rec->p;
      out->d = refr ? refract(ud, rec->normal, ratio) : reflect(ud, rec->normal);
      out->time = r_in->time;
      *att = v3(1.0, 1.0, 1.0);
      return 1;
    }
    default:
      return 0; /* DiffuseLight */
  }
}

static V emitted(const rw_world *w, const Rec *rec) { /* Material.emitted, :31-38, :107-109 */
  const rw_material *m = &w->mats[rec->mat];
  if (m->kind != RW_LIGHT) return v3(0, 0, 0);
  return tex_value(w, m->tex, rec);
}

/* ------------------------------------------------------------- Tier A -- */
typedef struct {
  const rw_world *w;
  V bg;
  Rng g;
  ro_stats st;
} CtxA;

/* rayColor, main.zig:103-122 */
static V ray_color_a(CtxA *cx, const Ray *r, uint32_t depth) {
  if (depth == 0) return v3(0, 0, 0);
  Rec rec;
  if (!world_hit(cx->w, r, 0.001, INFINITY, &rec, &cx->st)) return cx->bg;
  Ray sc;
  V att;
  const V em = emitted(cx->w, &rec);
  if (scatter(cx->w, r, &rec, &cx->g, &att, &sc, &cx->st)) return vadd(em, vmulv(att, ray_color_a(cx, &sc, depth - 1)));
  return em;
}

/* Camera.getRay, main.zig:91-100 */
static Ray get_ray(const ro_camera *cam, Rng *g, double s, double t, ro_stats *st) {
  const V rd = vmul(rng_in_unit_disk(g, st), cam->lens_radius);
  const V offset = vadd(vmul(vld(cam->u), rd.x), vmul(vld(cam->v), rd.y));
  Ray r;
  r.d = vsub(vsub(vadd(vadd(vld(cam->lower_left_corner), vmul(vld(cam->horizontal), s)), vmul(vld(cam->vertical), t)),
                  vld(cam->origin)),
             offset);
  r.o = vadd(vld(cam->origin), offset);
  r.time = rng_range(g, cam->time0, cam->time1);
  if (st) st->draws++;
  return r;
}

/* Render loop, main.zig:378-402 */
void rw_render_tier_a(const rw_world *w, const ro_camera *cam, const double bg[3], uint32_t W, uint32_t H,
                      uint32_t spp, uint32_t depth, uint64_t rng[4], uint8_t *rgb, double *sum_out,
                      ro_stats *stats) {
  CtxA cx;
  memset(&cx, 0, sizeof(cx));
  cx.w = w;
  cx.bg = vld(bg);
  cx.g.seq = rng;
  for (uint32_t j = 0; j < H; ++j)
    for (uint32_t i = 0; i < W; ++i) {
      V pc = v3(0, 0, 0);
      for (uint32_t s = 0; s < spp; ++s) {
        const double u = ((double)i + rnd01(rng)) / ((double)W - 1.0);
        const double v = ((double)j + rnd01(rng)) / ((double)H - 1.0);
        cx.st.draws += 2;
        const Ray r = get_ray(cam, &cx.g, u, v, &cx.st);
        pc = vadd(pc, ray_color_a(&cx, &r, depth));
        cx.st.samples++;
      }
      const double scale = 1.0 / (double)spp;
      const size_t o = ((size_t)i + (size_t)(H - j - 1) * W) * 3;
      rgb[o] = ro_quantize(pc.x, scale);
      rgb[o + 1] = ro_quantize(pc.y, scale);
      rgb[o + 2] = ro_quantize(pc.z, scale);
      if (sum_out) sum_out[o] = pc.x, sum_out[o + 1] = pc.y, sum_out[o + 2] = pc.z;
    }
  if (stats) *stats = cx.st;
}

/* ------------------------------------------------------------- Tier B -- */
/* One sample of the world kernel's contract: the cover-scene Tier-B rules
 * (rtw_oracle.c tierb_state / ro_sm_f64, draw order of main.zig:390-392 and
 * :91-100) with rayColor evaluated forward:
 *   rad = 0, T = 1; per segment: closest hit (flat list in order, later wins
 *   ties); miss -> rad += T*background, stop; light -> rad += T*emitted,
 *   stop; scatter -> absorbed: stop, else T *= attenuation; after max_depth
 *   segments: stop.  (emitted == 0 of non-lights adds nothing.) */
static V sample_b(const rw_world *w, const ro_camera *cam, const ro_params *p, V bg, uint32_t i, uint32_t j,
                  uint64_t pixel, uint32_t s, ro_stats *st) {
  uint64_t state = ro_tierb_state(p->seed, pixel, s);
  Rng g = {NULL, &state};
  const double u = ((double)i + ro_sm_f64(&state)) / ((double)p->width - 1);
  const double v = ((double)j + ro_sm_f64(&state)) / ((double)p->height - 1);
  st->draws += 2;
  Ray r = get_ray(cam, &g, u, v, st);
  V T = v3(1, 1, 1), rad = v3(0, 0, 0);
  for (uint32_t depth = 0; depth < p->max_depth; ++depth) {
    Rec rec;
    if (!world_hit(w, &r, 0.001, INFINITY, &rec, st)) return vadd(rad, vmulv(T, bg));
    if (w->mats[rec.mat].kind == RW_LIGHT) return vadd(rad, vmulv(T, emitted(w, &rec)));
    Ray sc;
    V att;
    if (!scatter(w, &r, &rec, &g, &att, &sc, st)) return rad;
    T = vmulv(T, att);
    r = sc;
  }
  return rad;
}

void rw_render_tier_b(const rw_world *w, const ro_camera *cam, const ro_params *p, uint8_t *rgb,
                      float *mean_out, ro_stats *stats) {
  const uint32_t W = p->width, H = p->height;
  const uint32_t chunk = p->chunk ? p->chunk : RO_DEFAULT_CHUNK; /* the GPU contract's default (rtw_hip.h RTW_DEFAULT_CHUNK) */
  const double scale = 1.0 / (double)p->spp;
  const V bg = vld(p->background);
  ro_stats total;
  memset(&total, 0, sizeof(total));
#ifdef _OPENMP
  if (p->threads) omp_set_num_threads((int)p->threads);
#endif
#pragma omp parallel
  {
    ro_stats st;
    memset(&st, 0, sizeof(st));
    /* work item = (row, block of 32 pixels): a few rows of a large world
     * (configs[4]: 10k primitives tested per segment) still use every thread */
    const uint32_t nblk = (W + 31) / 32;
#pragma omp for schedule(dynamic, 1)
    for (int64_t qb = 0; qb < (int64_t)p->row_count * nblk; ++qb) {
      const int64_t q = qb / nblk;
      const uint32_t y = p->row_begin + (uint32_t)q * p->row_stride;
      const uint32_t j = H - 1 - y;
      const uint32_t i_end = (uint32_t)(qb % nblk) * 32 + 32 < W ? (uint32_t)(qb % nblk) * 32 + 32 : W;
      for (uint32_t i = (uint32_t)(qb % nblk) * 32; i < i_end; ++i) {
        const uint64_t pixel = (uint64_t)y * W + i;
        double tx = 0, ty = 0, tz = 0;
        for (uint32_t c0 = 0; c0 < p->spp; c0 += chunk) {
          const uint32_t c1 = (c0 + chunk < p->spp) ? c0 + chunk : p->spp;
          double sx = 0, sy = 0, sz = 0;
          for (uint32_t s = c0; s < c1; ++s) {
            const V col = sample_b(w, cam, p, bg, i, j, pixel, s, &st);
            sx += col.x, sy += col.y, sz += col.z;
            st.samples++;
          }
          tx += sx, ty += sy, tz += sz;
        }
        const size_t o = ((size_t)q * W + i) * 3;
        rgb[o] = ro_quantize(tx, scale);
        rgb[o + 1] = ro_quantize(ty, scale);
        rgb[o + 2] = ro_quantize(tz, scale);
        if (mean_out) {
          mean_out[o] = (float)(tx * scale);
          mean_out[o + 1] = (float)(ty * scale);
          mean_out[o + 2] = (float)(tz * scale);
        }
      }
    }
#pragma omp critical
    {
      total.samples += st.samples;
      total.segments += st.segments;
      total.draws += st.draws;
    }
  }
  if (stats) *stats = total;
}

/* ------------------------------------------------------------ scenes -- */

static rw_world *world_new(uint32_t np, uint32_t nx, uint32_t nt, uint32_t nm, uint32_t npl, uint32_t ni) {
  rw_world *w = (rw_world *)calloc(1, sizeof(rw_world));
  w->prims = (rw_prim *)calloc(np ? np : 1, sizeof(rw_prim));
  w->xforms = (rw_xform *)calloc(nx ? nx : 1, sizeof(rw_xform));
  w->textures = (rw_texture *)calloc(nt ? nt : 1, sizeof(rw_texture));
  w->mats = (rw_material *)calloc(nm ? nm : 1, sizeof(rw_material));
  w->perlins = (rw_perlin *)calloc(npl ? npl : 1, sizeof(rw_perlin));
  w->images = (rw_image *)calloc(ni ? ni : 1, sizeof(rw_image));
  return w;
}
void rw_world_free(rw_world *w) {
  if (!w) return;
  free(w->prims), free(w->xforms), free(w->textures), free(w->mats), free(w->perlins), free(w->images);
  free(w);
}
static uint32_t tex_solid(rw_world *w, V c) {
  rw_texture *t = &w->textures[w->n_textures];
  t->kind = RW_TEX_SOLID;
  vst(t->color, c);
  return w->n_textures++;
}
static uint32_t tex_checker(rw_world *w, V odd, V even) { /* Texture.makeChecker(odd, even), texture.zig:20-26 */
  rw_texture *t = &w->textures[w->n_textures];
  t->kind = RW_TEX_CHECKER;
  vst(t->odd, odd);
  vst(t->even, even);
  return w->n_textures++;
}
static uint32_t mat_new(rw_world *w, uint32_t kind, uint32_t tex, V albedo, double fuzz, double ir) {
  rw_material *m = &w->mats[w->n_mats];
  m->kind = kind, m->tex = tex, m->fuzz = fuzz, m->ir = ir;
  vst(m->albedo, albedo);
  return w->n_mats++;
}
static void sphere(rw_world *w, V c0, V c1, double r, int moving, double t0, double t1, uint32_t mat) {
  rw_prim *s = &w->prims[w->n_prims++];
  s->kind = moving ? RW_MOVING : RW_SPHERE, s->mat = mat, s->xform = -1;
  vst(s->a, c0);
  vst(s->a + 3, c1);
  s->a[6] = r, s->a[7] = t0, s->a[8] = t1;
}
static void rect(rw_world *w, uint32_t kind, double a0, double a1, double b0, double b1, double k, uint32_t mat,
                 int32_t xf) {
  rw_prim *s = &w->prims[w->n_prims++];
  s->kind = kind, s->mat = mat, s->xform = xf;
  s->a[0] = a0, s->a[1] = a1, s->a[2] = b0, s->a[3] = b1, s->a[4] = k;
}
/* Box.init, hittable.zig:434-452: six rects, this order. */
static void box(rw_world *w, V p0, V p1, uint32_t mat, int32_t xf) {
  rect(w, RW_XY, p0.x, p1.x, p0.y, p1.y, p1.z, mat, xf);
  rect(w, RW_XY, p0.x, p1.x, p0.y, p1.y, p0.z, mat, xf);
  rect(w, RW_XZ, p0.x, p1.x, p0.z, p1.z, p1.y, mat, xf);
  rect(w, RW_XZ, p0.x, p1.x, p0.z, p1.z, p0.y, mat, xf);
  rect(w, RW_YZ, p0.y, p1.y, p0.z, p1.z, p1.x, mat, xf);
  rect(w, RW_YZ, p0.y, p1.y, p0.z, p1.z, p0.x, mat, xf);
}
static void settings(rw_world *w, V lf, V la, double vfov, double aperture, V bg) {
  vst(w->look_from, lf);
  vst(w->look_at, la);
  w->vfov = vfov, w->aperture = aperture;
  vst(w->background, bg);
  w->aspect = 3.0 / 2.0, w->width = 600, w->spp = 50; /* main.zig:304-308 */
  w->height = ro_image_height(600, 3.0 / 2.0);
}
static uint32_t noise_tex(rw_world *w, double scale, uint64_t rng[4]) { /* Texture.makeNoise, texture.zig:28-30 */
  rw_texture *t = &w->textures[w->n_textures];
  t->kind = RW_TEX_NOISE, t->scale = scale, t->perlin = w->n_perlins;
  perlin_init(&w->perlins[w->n_perlins++], rng);
  return w->n_textures++;
}
/* Random spheres on the grid [lo, hi)^2, the loop body of main.zig:177-218
 * with the exclusion centre `ex` and radius `exr`. */
static void random_grid(rw_world *w, uint64_t rng[4], int lo, int hi, V ex, double exr) {
  for (int a = lo; a < hi; ++a)
    for (int b = lo; b < hi; ++b) {
      const double choose = rnd01(rng);
      V c;
      c.x = (double)a + 0.9 * rnd01(rng);
      c.y = 0.2;
      c.z = (double)b + 0.9 * rnd01(rng);
      if (vnorm(vsub(c, ex)) <= exr) continue;
      if (choose < 0.8) {
        V a1, a2;
        a1.x = rnd01(rng), a1.y = rnd01(rng), a1.z = rnd01(rng);
        a2.x = rnd01(rng), a2.y = rnd01(rng), a2.z = rnd01(rng);
        const uint32_t m = mat_new(w, RW_LAMBERT, tex_solid(w, vmulv(a1, a2)), v3(0, 0, 0), 0, 0);
        const V c1 = vadd(c, v3(0, rnd_range(rng, 0, 0.5), 0));
        sphere(w, c, c1, 0.2, 1, 0, 1, m);
      } else if (choose < 0.95) {
        V al;
        al.x = rnd_range(rng, 0.5, 1), al.y = rnd_range(rng, 0.5, 1), al.z = rnd_range(rng, 0.5, 1);
        const double fuzz = rnd_range(rng, 0, 0.5);
        sphere(w, c, c, 0.2, 0, 0, 0, mat_new(w, RW_METAL, 0, al, fuzz, 0));
      } else {
        sphere(w, c, c, 0.2, 0, 0, 0, mat_new(w, RW_DIELECTRIC, 0, v3(0, 0, 0), 0, 1.5));
      }
    }
}

rw_world *rw_scene(uint32_t id, uint64_t rng[4], const rw_image *image) {
  const V sky = v3(0.70, 0.80, 1.00), black = v3(0, 0, 0), o = v3(0, 0, 0);
  rw_world *w = NULL;
  switch (id) {
    case 1: { /* generateRandomScene, main.zig:157-221 */
      w = world_new(64, 0, 64, 64, 0, 0);
      const uint32_t ck = tex_checker(w, v3(0.2, 0.3, 0.1), v3(0.9, 0.9, 0.9));
      const uint32_t mg = mat_new(w, RW_LAMBERT, ck, o, 0, 0);
      const uint32_t m1 = mat_new(w, RW_DIELECTRIC, 0, o, 0, 1.5);
      const uint32_t m2 = mat_new(w, RW_LAMBERT, tex_solid(w, v3(0.4, 0.2, 0.1)), o, 0, 0);
      const uint32_t m3 = mat_new(w, RW_METAL, 0, v3(0.7, 0.6, 0.5), 0.0, 0);
      sphere(w, v3(0, -1000, 0), v3(0, -1000, 0), 1000, 0, 0, 0, mg);
      sphere(w, v3(0, 1, 0), v3(0, 1, 0), 1.0, 0, 0, 0, m1);
      sphere(w, v3(-4, 1, 0), v3(-4, 1, 0), 1.0, 0, 0, 0, m2);
      sphere(w, v3(4, 1, 0), v3(4, 1, 0), 1.0, 0, 0, 0, m3);
      random_grid(w, rng, -3, 3, v3(4, 0.2, 0), 0.9);
      settings(w, v3(13, 2, 3), o, 20.0, 0.1, sky);
      break;
    }
    case 2: { /* generateTwoSpheres, main.zig:123-138 */
      w = world_new(2, 0, 1, 2, 0, 0);
      const uint32_t ck = tex_checker(w, v3(0.2, 0.3, 0.1), v3(0.9, 0.9, 0.9));
      const uint32_t m1 = mat_new(w, RW_LAMBERT, ck, o, 0, 0), m2 = mat_new(w, RW_LAMBERT, ck, o, 0, 0);
      sphere(w, v3(0, -10, 0), v3(0, -10, 0), 10, 0, 0, 0, m1);
      sphere(w, v3(0, 10, 0), v3(0, 10, 0), 10, 0, 0, 0, m2);
      settings(w, v3(13, 2, 3), o, 20.0, 0, sky);
      break;
    }
    case 3:   /* generateTwoPerlinSpheres, main.zig:140-155 */
    case 5: { /* generateSimpleLightScene, main.zig:235-254 */
      w = world_new(3, 0, 2, 3, 1, 0);
      const uint32_t nt = noise_tex(w, 4.0, rng);
      const uint32_t m1 = mat_new(w, RW_LAMBERT, nt, o, 0, 0), m2 = mat_new(w, RW_LAMBERT, nt, o, 0, 0);
      sphere(w, v3(0, -1000, 0), v3(0, -1000, 0), 1000, 0, 0, 0, m1);
      sphere(w, v3(0, 2, 0), v3(0, 2, 0), 2, 0, 0, 0, m2);
      if (id == 3) {
        settings(w, v3(13, 2, 3), o, 20.0, 0, sky);
      } else {
        const uint32_t ml = mat_new(w, RW_LIGHT, tex_solid(w, v3(4, 4, 4)), o, 0, 0);
        rect(w, RW_XY, 3.0, 5.0, 1.0, 3.0, -2.0, ml, -1);
        settings(w, v3(26, 3, 6), v3(0, 2, 0), 20.0, 0, black);
        w->spp = 400; /* main.zig:358 */
      }
      break;
    }
    case 4: { /* generateEarthScene, main.zig:223-233 */
      w = world_new(1, 0, 1, 1, 0, 1);
      w->images[w->n_images++] = *image;
      rw_texture *t = &w->textures[w->n_textures];
      t->kind = RW_TEX_IMAGE, t->image = 0;
      const uint32_t m = mat_new(w, RW_LAMBERT, w->n_textures++, o, 0, 0);
      sphere(w, o, o, 2, 0, 0, 0, m);
      settings(w, v3(13, 2, 3), o, 20.0, 0, sky);
      break;
    }
    case 6: { /* generateCornellBox, main.zig:256-290 */
      w = world_new(18, 2, 4, 4, 0, 0);
      const uint32_t red = mat_new(w, RW_LAMBERT, tex_solid(w, v3(0.65, 0.05, 0.05)), o, 0, 0);
      const uint32_t white = mat_new(w, RW_LAMBERT, tex_solid(w, v3(0.73, 0.73, 0.73)), o, 0, 0);
      const uint32_t green = mat_new(w, RW_LAMBERT, tex_solid(w, v3(0.12, 0.45, 0.15)), o, 0, 0);
      const uint32_t light = mat_new(w, RW_LIGHT, tex_solid(w, v3(15, 15, 15)), o, 0, 0);
      rect(w, RW_YZ, 0, 555, 0, 555, 555, green, -1);
      rect(w, RW_YZ, 0, 555, 0, 555, 0, red, -1);
      rect(w, RW_XZ, 213, 343, 227, 332, 554, light, -1);
      rect(w, RW_XZ, 0, 555, 0, 555, 0, white, -1);
      rect(w, RW_XZ, 0, 555, 0, 555, 555, white, -1);
      rect(w, RW_XY, 0, 555, 0, 555, 555, white, -1);
      const double ang[2] = {15.0, -18.0}, h[2] = {330.0, 165.0};
      const V off[2] = {v3(265, 0, 295), v3(130, 0, 65)};
      for (int b = 0; b < 2; ++b) { /* Translate(RotateY(Box)), main.zig:277-287 */
        rw_xform *x = &w->xforms[w->n_xforms];
        const double t = ang[b] * 3.14159265358979323846 / 180.0; /* deg2rad, main.zig:36-38 */
        x->n = 2;
        x->op[0] = RW_XF_TRANSLATE;
        vst(x->v[0], off[b]);
        x->op[1] = RW_XF_ROTATE_Y;
        x->v[1][0] = ro_sin(t), x->v[1][1] = ro_cos(t), x->v[1][2] = t;
        box(w, o, v3(165, h[b], 165), white, (int32_t)w->n_xforms++);
      }
      settings(w, v3(278, 278, -800), v3(278, 278, 0), 40.0, 0, black);
      w->aspect = 1.0, w->width = 600, w->height = 600, w->spp = 200; /* main.zig:357-362 */
      break;
    }
    case 7: { /* configs[4]: globe + random spheres (not a reference scene) */
      w = world_new(2 + 10000, 0, 2 + 10000, 3 + 10000, 0, 1);
      w->images[w->n_images++] = *image;
      const uint32_t ck = tex_checker(w, v3(0.2, 0.3, 0.1), v3(0.9, 0.9, 0.9));
      const uint32_t mg = mat_new(w, RW_LAMBERT, ck, o, 0, 0);
      rw_texture *t = &w->textures[w->n_textures];
      t->kind = RW_TEX_IMAGE, t->image = 0;
      const uint32_t me = mat_new(w, RW_LAMBERT, w->n_textures++, o, 0, 0);
      sphere(w, v3(0, -1000, 0), v3(0, -1000, 0), 1000, 0, 0, 0, mg);
      sphere(w, v3(0, 2, 0), v3(0, 2, 0), 2, 0, 0, 0, me);
      random_grid(w, rng, -50, 50, v3(0, 0.2, 0), 2.5);
      settings(w, v3(13, 2, 3), v3(0, 1, 0), 20.0, 0.1, sky);
      w->aspect = 16.0 / 9.0, w->width = 1200, w->height = ro_image_height(1200, 16.0 / 9.0), w->spp = 100;
      break;
    }
    default:
      return NULL;
  }
  return w;
}
