/*
 * tierb_core.h — Tier-B oracle body, included twice by rtw_oracle.c with
 * TB_REAL = double (precision 0, "f64": the reference's arithmetic) and
 * TB_REAL = float (precision 1, "f32-hybrid").  TEST INFRASTRUCTURE ONLY.
 *
 * This file IS the written contract the HIP kernel implements:
 *  - per sample: the counter-based block of (seed, pixel, s) on SplitMix64's
 *    Weyl sequence (rtw_oracle.c tierb_state), each draw mixed by four Feistel
 *    half-rounds (ro_tb_mix; round 5, SplitMix64's output function before),
 *    pixel = image_row * W + column (image rows top-first), u64 -> real by
 *    Zig's Random.float;
 *  - draw order per sample (main.zig:390-392, main.zig:91-100): u jitter,
 *    v jitter, unit-disk rejection pairs, time; then per bounce the material's
 *    draws (rand.zig:22-40, material.zig:44-85);
 *  - rayColor (main.zig:103-122) evaluated forward: T <- T*att per bounce,
 *    colour = T*background on a miss, 0 on absorption or after max_depth hits;
 *  - closest hit over the list in order, later object wins ties
 *    (hittable.zig:231-244); the hit record is recomputed for the winner only;
 *  - per pixel: samples summed in f64 per chunk of `chunk` samples
 *    (0 + x0 + x1 + ...), chunk sums added in order to 0;
 *  - quantisation exactly main.zig:395-400.
 * f32-hybrid: everything in f32 except spheres with radius >= 100 ("wide"),
 * whose quadratic is solved in f64 from the f64 scene values (the radius-1000
 * ground sphere's c = |oc|^2 - r^2 cancels catastrophically in f32), its two
 * roots rounded to f32 before they are compared with anything; and a ray
 * that LEAVES a sphere outward (dot(new_dir, geometric outward normal) > 0)
 * does not test that sphere on its next segment (convex self-skip: exact in
 * real arithmetic, it stops f32 hit points that land a hair inside a sphere
 * at grazing incidence from re-hitting it and trapping the path).  f64 mode
 * has neither rule: it is the reference's arithmetic.
 */

#define TB_CAT_(a, b) a##b
#define TB_CAT(a, b) TB_CAT_(a, b)
#define TBF(name) TB_CAT(name, TB_SUFFIX)

typedef TB_REAL TBF(R);
typedef struct { TBF(R) x, y, z; } TBF(V);

#if TB_IS_F32
#define TB_SQRT sqrtf
#define TB_SIN sinf
#define TB_FABS fabsf
#define TB_FMIN fminf
#define TB_RAND01(s) ro_sm_f32(s)
#else
#define TB_SQRT sqrt
#define TB_SIN sin
#define TB_FABS fabs
#define TB_FMIN fmin
#define TB_RAND01(s) ro_sm_f64(s)
#endif

static inline TBF(V) TBF(mk)(TBF(R) x, TBF(R) y, TBF(R) z) { TBF(V) r = {x, y, z}; return r; }
static inline TBF(V) TBF(add)(TBF(V) a, TBF(V) b) { return TBF(mk)(a.x + b.x, a.y + b.y, a.z + b.z); }
static inline TBF(V) TBF(sub)(TBF(V) a, TBF(V) b) { return TBF(mk)(a.x - b.x, a.y - b.y, a.z - b.z); }
static inline TBF(V) TBF(mul)(TBF(V) a, TBF(R) t) { return TBF(mk)(a.x * t, a.y * t, a.z * t); }
static inline TBF(V) TBF(mulv)(TBF(V) a, TBF(V) b) { return TBF(mk)(a.x * b.x, a.y * b.y, a.z * b.z); }
static inline TBF(V) TBF(divs)(TBF(V) a, TBF(R) t) { return TBF(mk)(a.x / t, a.y / t, a.z / t); }
static inline TBF(R) TBF(dot)(TBF(V) a, TBF(V) b) { return a.x * b.x + a.y * b.y + a.z * b.z; }
static inline TBF(R) TBF(norm2)(TBF(V) a) { return a.x * a.x + a.y * a.y + a.z * a.z; }
static inline TBF(V) TBF(normalized)(TBF(V) v) {
  const TBF(R) n = TB_SQRT(TBF(norm2)(v));
  return (n == (TBF(R))0) ? v : TBF(divs)(v, n);
}
static inline TBF(V) TBF(ld)(const double p[3]) { return TBF(mk)((TBF(R))p[0], (TBF(R))p[1], (TBF(R))p[2]); }
static inline TBF(R) TBF(rrange)(uint64_t *s, TBF(R) mn, TBF(R) mx) { return mn + TB_RAND01(s) * (mx - mn); }

typedef struct {
  TBF(V) c0, dc;          /* centre at t0; c1 - c0 (computed in f64, rounded) */
  TBF(R) radius, r2, t0, t1;
  int moving, wide;
  uint32_t mat;
  const ro_sphere *src;   /* f64 originals for wide spheres */
} TBF(Sph);

typedef struct {
  uint32_t kind;
  TBF(V) albedo, odd;
  TBF(R) fuzz, ir;
} TBF(Mat);

typedef struct {
  TBF(Sph) sph[RO_MAX_SPHERES];
  TBF(Mat) mat[RO_MAX_SPHERES];
  uint32_t n;
  TBF(V) origin, horizontal, vertical, llc, u, v, bg;
  TBF(R) lens_radius, time0, time1;
} TBF(Scene);

static void TBF(prep)(TBF(Scene) *S, const ro_scene *sc, const ro_camera *cam, const double bg[3]) {
  S->n = sc->n_spheres;
  for (uint32_t i = 0; i < sc->n_spheres; ++i) {
    const ro_sphere *s = &sc->spheres[i];
    TBF(Sph) *d = &S->sph[i];
    d->c0 = TBF(ld)(s->c0);
    d->dc = TBF(mk)((TBF(R))(s->c1[0] - s->c0[0]), (TBF(R))(s->c1[1] - s->c0[1]), (TBF(R))(s->c1[2] - s->c0[2]));
    d->radius = (TBF(R))s->radius;
    d->r2 = d->radius * d->radius;
    d->t0 = (TBF(R))s->t0;
    d->t1 = (TBF(R))s->t1;
    d->moving = (int)s->moving;
    d->wide = TB_IS_F32 && (s->radius >= 100.0);
    d->mat = s->mat;
    d->src = s;
  }
  for (uint32_t i = 0; i < sc->n_mats; ++i) {
    const ro_material *m = &sc->mats[i];
    TBF(Mat) *d = &S->mat[i];
    d->kind = m->kind;
    d->albedo = TBF(ld)(m->albedo);
    d->odd = TBF(ld)(m->albedo_odd);
    d->fuzz = (TBF(R))m->fuzz;
    d->ir = (TBF(R))m->ir;
  }
  S->origin = TBF(ld)(cam->origin);
  S->horizontal = TBF(ld)(cam->horizontal);
  S->vertical = TBF(ld)(cam->vertical);
  S->llc = TBF(ld)(cam->lower_left_corner);
  S->u = TBF(ld)(cam->u);
  S->v = TBF(ld)(cam->v);
  S->lens_radius = (TBF(R))cam->lens_radius;
  S->time0 = (TBF(R))cam->time0;
  S->time1 = (TBF(R))cam->time1;
  S->bg = TBF(ld)(bg);
}

/* MovingSphere.center (hittable.zig:219-221) with c1 - c0 precomputed. */
static inline TBF(V) TBF(center)(const TBF(Sph) *s, TBF(R) time) {
  if (!s->moving) return s->c0;
  const TBF(R) frac = (time - s->t0) / (s->t1 - s->t0);
  return TBF(add)(s->c0, TBF(mul)(s->dc, frac));
}

/* rand.zig:22-28 (norm() >= 1 rejection) */
static inline TBF(V) TBF(in_unit_sphere)(uint64_t *s, ro_stats *st) {
  for (;;) {
    TBF(V) p;
    p.x = TBF(rrange)(s, -1, 1);
    p.y = TBF(rrange)(s, -1, 1);
    p.z = TBF(rrange)(s, -1, 1);
    st->draws += 3;
    if (TB_SQRT(TBF(norm2)(p)) >= 1) continue;
    return p;
  }
}

/* Sphere.hit's quadratic (hittable.zig:96-116) returning the accepted root. */
static inline int TBF(test)(const TBF(Sph) *s, TBF(V) o, TBF(V) d, TBF(R) time, TBF(R) a,
                            TBF(R) tmin, TBF(R) *tmax) {
#if TB_IS_F32
  if (s->wide) {
    const ro_sphere *q = s->src;
    double cx = q->c0[0], cy = q->c0[1], cz = q->c0[2];
    if (q->moving) {
      const double fr = ((double)time - q->t0) / (q->t1 - q->t0);
      cx = cx + (q->c1[0] - q->c0[0]) * fr;
      cy = cy + (q->c1[1] - q->c0[1]) * fr;
      cz = cz + (q->c1[2] - q->c0[2]) * fr;
    }
    const double ox = (double)o.x - cx, oy = (double)o.y - cy, oz = (double)o.z - cz;
    const double dx = d.x, dy = d.y, dz = d.z;
    const double ad = dx * dx + dy * dy + dz * dz;
    const double hb = ox * dx + oy * dy + oz * dz;
    const double c = (ox * ox + oy * oy + oz * oz) - q->radius * q->radius;
    const double disc = hb * hb - ad * c;
    if (disc < 0.0) return 0;
    const double sq = sqrt(disc);
    /* roots solved in f64, rounded to f32 before any comparison */
    float root = (float)((-hb - sq) / ad);
    if (root < tmin || *tmax < root) {
      root = (float)((-hb + sq) / ad);
      if (root < tmin || *tmax < root) return 0;
    }
    *tmax = root;
    return 1;
  }
#endif
  const TBF(V) oc = TBF(sub)(o, TBF(center)(s, time));
  const TBF(R) half_b = TBF(dot)(oc, d);
  const TBF(R) c = TBF(norm2)(oc) - s->r2;
  const TBF(R) disc = half_b * half_b - a * c;
  if (disc < 0) return 0;
  const TBF(R) sq = TB_SQRT(disc);
  TBF(R) root = (-half_b - sq) / a;
  if (root < tmin || *tmax < root) {
    root = (-half_b + sq) / a;
    if (root < tmin || *tmax < root) return 0;
  }
  *tmax = root;
  return 1;
}

static inline TBF(V) TBF(reflect)(TBF(V) v, TBF(V) n) { return TBF(sub)(v, TBF(mul)(n, 2 * TBF(dot)(v, n))); }
static inline TBF(V) TBF(refract)(TBF(V) uv, TBF(V) n, TBF(R) eta) {
  const TBF(R) cos_theta = TB_FMIN(TBF(dot)(TBF(mul)(uv, -1), n), 1);
  const TBF(V) perp = TBF(mul)(TBF(add)(uv, TBF(mul)(n, cos_theta)), eta);
  const TBF(V) par = TBF(mul)(n, -TB_SQRT(TB_FABS(1 - TBF(norm2)(perp))));
  return TBF(add)(perp, par);
}
/* reflectance with Zig's pow(x, 5.0) == x * ((x*x)*(x*x)) (see
 * zig_pow_posint; proven equal by tests/test_oracle_kat.py). */
static inline TBF(R) TBF(reflectance)(TBF(R) cosine, TBF(R) ref_idx) {
  const TBF(R) r0 = (1 - ref_idx) / (1 + ref_idx);
  const TBF(R) r1 = r0 * r0;
  const TBF(R) x = 1 - cosine;
  const TBF(R) x2 = x * x;
  return r1 + (1 - r1) * (x * (x2 * x2));
}

/* One sample: returns its colour (the forward restatement of rayColor). */
static TBF(V) TBF(sample)(const TBF(Scene) *S, const ro_params *p, uint32_t i, uint32_t j,
                          uint64_t pixel, uint32_t s_idx, ro_stats *st) {
  uint64_t rng_state = tierb_state(p->seed, pixel, s_idx);
  uint64_t *rng = &rng_state;
  /* main.zig:390-391 */
  const TBF(R) u = ((TBF(R))i + TB_RAND01(rng)) / ((TBF(R))p->width - 1);
  const TBF(R) v = ((TBF(R))j + TB_RAND01(rng)) / ((TBF(R))p->height - 1);
  st->draws += 2;
  /* Camera.getRay, main.zig:91-100 */
  TBF(V) disk;
  for (;;) {
    disk.x = TBF(rrange)(rng, -1, 1);
    disk.y = TBF(rrange)(rng, -1, 1);
    disk.z = 0;
    st->draws += 2;
    if (TB_SQRT(TBF(norm2)(disk)) >= 1) continue;
    break;
  }
  const TBF(V) rd = TBF(mul)(disk, S->lens_radius);
  const TBF(V) offset = TBF(add)(TBF(mul)(S->u, rd.x), TBF(mul)(S->v, rd.y));
  TBF(V) d = TBF(sub)(TBF(sub)(TBF(add)(TBF(add)(S->llc, TBF(mul)(S->horizontal, u)), TBF(mul)(S->vertical, v)), S->origin), offset);
  TBF(V) o = TBF(add)(S->origin, offset);
  const TBF(R) time = TBF(rrange)(rng, S->time0, S->time1);
  st->draws += 1;

  TBF(V) T = TBF(mk)(1, 1, 1);
  const TBF(R) tmin = (TBF(R))0.001;
  int skip = -1; /* f32 convex self-skip (never set in f64 mode) */
  for (uint32_t depth = 0; depth < p->max_depth; ++depth) {
    st->segments++;
    const TBF(R) a = TBF(norm2)(d);
    TBF(R) tmax = (TBF(R))INFINITY;
    int hit = -1;
    for (uint32_t k = 0; k < S->n; ++k) {
      if (S->sph[k].moving) st->moving_tests++; else st->static_tests++;
      if ((int)k == skip) continue;
      if (TBF(test)(&S->sph[k], o, d, time, a, tmin, &tmax)) hit = (int)k;
    }
    if (ro_tb_trace)
      fprintf(stderr, "[tierb] s %u depth %u o %.17g %.17g %.17g d %.17g %.17g %.17g t %.17g hit %d tmax %.17g\n",
              s_idx, depth, (double)o.x, (double)o.y, (double)o.z, (double)d.x, (double)d.y, (double)d.z,
              (double)time, hit, (double)tmax);
    if (hit < 0) return TBF(mulv)(T, S->bg); /* miss: background */
    /* hit record for the winner (hittable.zig:118-128 / :189-198) */
    const TBF(Sph) *sp = &S->sph[hit];
    const TBF(V) pnt = TBF(add)(o, TBF(mul)(d, tmax));
    const TBF(V) outward = TBF(divs)(TBF(sub)(pnt, TBF(center)(sp, time)), sp->radius);
    const int front = TBF(dot)(outward, d) < 0;
    const TBF(V) normal = front ? outward : TBF(mul)(outward, -1);
    const TBF(Mat) *m = &S->mat[sp->mat];
    TBF(V) att, ndir;
    switch (m->kind) {
      case RO_LAMBERT_SOLID:
      case RO_LAMBERT_CHECKER: {
        ndir = TBF(add)(normal, TBF(normalized)(TBF(in_unit_sphere)(rng, st)));
        if (TB_FABS(ndir.x) < (TBF(R))1e-8 && TB_FABS(ndir.y) < (TBF(R))1e-8 && TB_FABS(ndir.z) < (TBF(R))1e-8)
          ndir = normal;
        att = m->albedo;
        if (m->kind == RO_LAMBERT_CHECKER) {
          const TBF(R) sines = TB_SIN(10 * pnt.x) * TB_SIN(10 * pnt.y) * TB_SIN(10 * pnt.z);
          if (sines < 0) att = m->odd;
        }
        break;
      }
      case RO_METAL: {
        const TBF(V) refl = TBF(reflect)(TBF(normalized)(d), normal);
        ndir = TBF(add)(refl, TBF(mul)(TBF(in_unit_sphere)(rng, st), m->fuzz));
        att = m->albedo;
        if (!(TBF(dot)(refl, normal) > 0)) return TBF(mk)(0, 0, 0); /* absorbed */
        break;
      }
      default: { /* RO_DIELECTRIC */
        const TBF(R) ratio = front ? 1 / m->ir : m->ir;
        const TBF(V) ud = TBF(normalized)(d);
        const TBF(R) cos_theta = TB_FMIN(TBF(dot)(TBF(mul)(ud, -1), normal), 1);
        const TBF(R) sin_theta = TB_SQRT(1 - cos_theta * cos_theta);
        int refr = 0;
        if (ratio * sin_theta <= 1) {
          st->draws++;
          refr = TBF(reflectance)(cos_theta, ratio) < TB_RAND01(rng);
        }
        ndir = refr ? TBF(refract)(ud, normal, ratio) : TBF(reflect)(ud, normal);
        att = TBF(mk)(1, 1, 1);
        break;
      }
    }
    T = TBF(mulv)(T, att);
#if TB_IS_F32
    skip = (TBF(dot)(ndir, outward) > 0) ? hit : -1;
#endif
    o = pnt;
    d = ndir;
  }
  return TBF(mk)(0, 0, 0); /* depth exhausted: main.zig:105-108 */
}

/* Diagnostics (tests / tools only): the radiance of samples s0 .. s0+n-1 of
 * one pixel (image row y top-first, column x), n x 3 doubles. */
static void TBF(tierb_samples)(const ro_scene *sc, const ro_camera *cam, const ro_params *p, uint32_t y, uint32_t x,
                               uint32_t s0, uint32_t n, double *out) {
  TBF(Scene) *S = (TBF(Scene) *)malloc(sizeof(TBF(Scene)));
  TBF(prep)(S, sc, cam, p->background);
  ro_stats st;
  memset(&st, 0, sizeof(st));
  for (uint32_t k = 0; k < n; ++k) {
    const TBF(V) c = TBF(sample)(S, p, x, p->height - 1 - y, (uint64_t)y * p->width + x, s0 + k, &st);
    out[3 * k] = (double)c.x, out[3 * k + 1] = (double)c.y, out[3 * k + 2] = (double)c.z;
  }
  free(S);
}

static void TBF(tierb_render)(const ro_scene *sc, const ro_camera *cam, const ro_params *p,
                              uint8_t *rgb, float *mean_out, ro_stats *stats) {
  TBF(Scene) *S = (TBF(Scene) *)malloc(sizeof(TBF(Scene)));
  TBF(prep)(S, sc, cam, p->background);
  const uint32_t W = p->width, H = p->height;
  const uint32_t chunk = p->chunk ? p->chunk : RO_DEFAULT_CHUNK; /* the GPU contract's default (rtw_hip.h RTW_DEFAULT_CHUNK) */
  const double scale = 1.0 / (double)p->spp;
  ro_stats total;
  memset(&total, 0, sizeof(total));
#ifdef _OPENMP
  if (p->threads) omp_set_num_threads((int)p->threads);
#endif
#pragma omp parallel
  {
    ro_stats st;
    memset(&st, 0, sizeof(st));
#pragma omp for schedule(dynamic, 1)
    for (int64_t q = 0; q < (int64_t)p->row_count; ++q) {
      const uint32_t y = p->row_begin + (uint32_t)q * p->row_stride; /* image row, top-first */
      const uint32_t j = H - 1 - y;                                  /* reference row index */
      for (uint32_t i = 0; i < W; ++i) {
        const uint64_t pixel = (uint64_t)y * W + i;
        double tx = 0, ty = 0, tz = 0;
        for (uint32_t c0 = 0; c0 < p->spp; c0 += chunk) {
          const uint32_t c1 = (c0 + chunk < p->spp) ? c0 + chunk : p->spp;
          double sx = 0, sy = 0, sz = 0;
          for (uint32_t s = c0; s < c1; ++s) {
            const TBF(V) col = TBF(sample)(S, p, i, j, pixel, s, &st);
            sx += (double)col.x;
            sy += (double)col.y;
            sz += (double)col.z;
            st.samples++;
          }
          tx += sx;
          ty += sy;
          tz += sz;
        }
        const size_t o = ((size_t)q * W + i) * 3;
        rgb[o + 0] = ro_quantize(tx, scale);
        rgb[o + 1] = ro_quantize(ty, scale);
        rgb[o + 2] = ro_quantize(tz, scale);
        if (mean_out) {
          mean_out[o + 0] = (float)(tx * scale);
          mean_out[o + 1] = (float)(ty * scale);
          mean_out[o + 2] = (float)(tz * scale);
        }
      }
    }
#pragma omp critical
    {
      total.samples += st.samples;
      total.segments += st.segments;
      total.static_tests += st.static_tests;
      total.moving_tests += st.moving_tests;
      total.draws += st.draws;
    }
  }
  if (stats) *stats = total;
  free(S);
}

#undef TB_SQRT
#undef TB_SIN
#undef TB_FABS
#undef TB_FMIN
#undef TB_RAND01
