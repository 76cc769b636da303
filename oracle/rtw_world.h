/*
 * rtw_world.h — CPU ORACLE for the general-world renders (TEST
 * INFRASTRUCTURE ONLY; same rules as rtw_oracle.h: only tests/, smoke() and
 * bench.py's cpu_baseline leg may load it, only as the checker).
 *
 * Restates the reference's remaining scene vocabulary in plain C11:
 *   Hittable.{sphere, movingSphere, list, xyRect, xzRect, yzRect, box,
 *   translate, rotateY}            hittable.zig:22-608
 *   Material.{diffuse, metal, dielectric, diffuse_light} (+ emitted)
 *                                   material.zig:16-121
 *   Texture.{solid, checker, noise, image}   texture.zig:10-144
 *   Perlin (init/noise/turb, Lemire intRangeLessThan)  perlin.zig:10-124
 *   scenes 2-6 of main.zig:123-290 and the render loop main.zig:378-402
 *   with emission in rayColor (main.zig:103-122)
 * plus BASELINE.json configs[4]'s globe scene (defined here, documented in
 * the reference has no such scene).
 *
 * The world is FLATTENED: nested lists (Box = 6 rects) become consecutive
 * primitives, and each primitive carries its chain of Translate / RotateY
 * wrappers (outermost first).  The closest-hit search over the flat list in
 * order, later object winning ties, picks the same object as the
 * reference's nested HittableList.hit calls, and the wrapped hit applies the
 * same operations in the same order (hittable.zig:472-608).
 *
 * Tier A: the reference itself (one sequential DefaultPrng(42) stream shared
 *         by the scene build and the render, recursive rayColor).
 * Tier B: the GPU contract of the world kernel: counter RNG blocks per
 *         (pixel, sample) as in rtw_oracle.c, rayColor evaluated forward with
 *         emission (rad += T * emitted at a light, rad += T * background on a
 *         miss), per-chunk f64 sums, f64 arithmetic.  Transcendentals are the
 *         musl algorithms of ro_libm.h in BOTH tiers (Zig's std.math ports
 *         musl, so this is also the best restatement of the reference).
 */
#ifndef RTW_WORLD_H
#define RTW_WORLD_H
#include <stdint.h>

#include "rtw_oracle.h"

#ifdef __cplusplus
extern "C" {
#endif

enum { RW_SPHERE = 0, RW_MOVING = 1, RW_XY = 2, RW_XZ = 3, RW_YZ = 4 };
enum { RW_XF_TRANSLATE = 0, RW_XF_ROTATE_Y = 1 };
enum { RW_TEX_SOLID = 0, RW_TEX_CHECKER = 1, RW_TEX_NOISE = 2, RW_TEX_IMAGE = 3 };
enum { RW_LAMBERT = 0, RW_METAL = 1, RW_DIELECTRIC = 2, RW_LIGHT = 3 };

/* a[]: sphere / moving sphere: c0[3], c1[3], radius, t0, t1 (c1 = c0 static)
 *      xy rect: x0, x1, y0, y1, k;  xz: x0, x1, z0, z1, k;  yz: y0, y1, z0, z1, k */
typedef struct {
  uint32_t kind, mat;
  int32_t xform; /* index into xforms, -1 = none */
  uint32_t pad;
  double a[9];
} rw_prim;

#define RW_MAX_XF_OPS 4
/* op[0] is the OUTERMOST wrapper.  translate: v = offset;
 * rotateY: v = {sin_t, cos_t, angle} (RotateY.init, hittable.zig:514-517). */
typedef struct {
  uint32_t n;
  uint32_t op[RW_MAX_XF_OPS];
  double v[RW_MAX_XF_OPS][3];
} rw_xform;

typedef struct {
  uint32_t kind, perlin, image, pad;
  double color[3];         /* solid */
  double odd[3], even[3];  /* checker (texture.zig:79-82) */
  double scale;            /* noise (texture.zig:85-105) */
} rw_texture;

typedef struct {
  uint32_t kind, tex;      /* tex: diffuse albedo / light emit texture */
  double albedo[3];        /* metal */
  double fuzz, ir;
} rw_material;

typedef struct {           /* perlin.zig:10-40 */
  double ranvec[256][3];
  uint32_t perm[3][256];
} rw_perlin;

typedef struct {
  uint32_t width, height;
  const uint8_t *rgba;     /* width*height*4, row-major, top row first */
} rw_image;

typedef struct {
  uint32_t n_prims, n_xforms, n_textures, n_mats, n_perlins, n_images;
  rw_prim *prims;
  rw_xform *xforms;
  rw_texture *textures;
  rw_material *mats;
  rw_perlin *perlins;
  rw_image *images;
  /* main.zig:316-376 settings of the scene */
  double look_from[3], look_at[3], vfov, aperture, aspect, background[3];
  uint32_t width, height, spp;
} rw_world;

/* Scene ids: 1 cover (main.zig:157), 2 two spheres (:123), 3 two Perlin
 * spheres (:140), 4 earth (:223), 5 simple light (:235), 6 Cornell box
 * (:256), 7 globe + random spheres on a 100x100 grid (configs[4]).
 * rng: Xoshiro256 state, consumed as the reference's builders do.
 * image: the earth texture (scenes 4 and 7), pixels not copied. */
rw_world *rw_scene(uint32_t id, uint64_t rng[4], const rw_image *image);
void rw_world_free(rw_world *w);

/* Exposed pieces (tests/test_world_oracle.py). */
uint64_t rw_int_range_less_than_u64(uint64_t rng[4], uint64_t at_least, uint64_t less_than);
double rw_perlin_noise(const rw_perlin *p, const double pt[3]);
double rw_perlin_turb(const rw_perlin *p, const double pt[3], uint32_t depth);
void rw_texture_value(const rw_world *w, uint32_t tex, double u, double v, const double p[3], double out[3]);
void rw_sphere_uv(const double p[3], double *u, double *v);
double rw_sin(double x);
double rw_cos(double x);
double rw_atan2(double y, double x);
double rw_acos(double x);
/* Closest hit of one ray (Tier-A semantics): returns the primitive index or
 * -1; t_out, p_out[3], normal_out[3], uv_out[2], front_out. */
int rw_hit(const rw_world *w, const double o[3], const double d[3], double time, double t_min, double t_max,
           double *t_out, double p_out[3], double normal_out[3], double uv_out[2], int *front_out);

/* Tier A: the reference render loop over `w` (rng continues after the
 * build).  rgb: W*H*3 top row first.  sum_out optional (f64 pixel sums). */
void rw_render_tier_a(const rw_world *w, const ro_camera *cam, const double bg[3], uint32_t W, uint32_t H,
                      uint32_t spp, uint32_t depth, uint64_t rng[4], uint8_t *rgb, double *sum_out,
                      ro_stats *stats);
/* Tier B: the world kernel's contract (p->precision ignored: f64). */
void rw_render_tier_b(const rw_world *w, const ro_camera *cam, const ro_params *p, uint8_t *rgb,
                      float *mean_out, ro_stats *stats);

#ifdef __cplusplus
}
#endif
#endif
