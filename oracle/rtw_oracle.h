/*
 * rtw_oracle.h — CPU ORACLE for the RTIOW cover-scene render loop.
 *
 * TEST INFRASTRUCTURE ONLY.  Only tests/, __graft_entry__.smoke() and
 * bench.py's cpu_baseline leg may load this library, and only as the checker
 * (or the timed CPU baseline) — never as the product path.
 *
 * It restates nsfisis/RayTracingInOneWeekend.zig (reference @ /root/reference)
 * in plain C11:
 *
 *   Tier A  — the reference itself: f64 everywhere, ONE sequential Zig
 *             std.Random.DefaultPrng (Xoshiro256++) stream seeded 42 shared by
 *             the scene build and every sample in raster order, recursive
 *             rayColor.  (main.zig:295-402, hittable.zig, material.zig,
 *             texture.zig, rand.zig, vec.zig, ray.zig.)
 *   Tier B  — the GPU path's contract: identical per-sample semantics, but the
 *             RNG is counter-based: SplitMix64's Weyl counter split into
 *             disjoint 2^16-draw blocks per (seed, pixel, sample), each draw's
 *             state mixed by four Feistel half-rounds (ro_tb_mix, round 5),
 *             so every sample is independent and random-access; the bounce
 *             recursion is evaluated forward (throughput product); samples are
 *             summed per chunk, chunks summed in order.  Precision f64
 *             (reference arithmetic) or f32-hybrid (f32 + f64 for wide spheres).
 *
 * PARITY STATUS: the reference publishes no tests, goldens or KATs for this
 * path and cannot be built here (no Zig toolchain, un-vendored zigimg), so the
 * Tier-A restatement is pinned only by (1) the Zig std Xoshiro256 "sequence"
 * known-answer vector and the published SplitMix64 vector (tests/golden), and
 * (2) bit-identical agreement with an independent pure-Python restatement
 * (oracle/rtw_oracle_py.py).  Against the real Zig binary: parity unpinned.
 */
#ifndef RTW_ORACLE_H
#define RTW_ORACLE_H
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* Material kinds (material.zig:16-21, texture.zig:10-14 flattened). */
enum { RO_LAMBERT_SOLID = 0, RO_LAMBERT_CHECKER = 1, RO_METAL = 2, RO_DIELECTRIC = 3 };

/* Chunk of the GPU contract's per-pixel sum when params.chunk == 0 (rtw_hip.h
 * RTW_DEFAULT_CHUNK): chunks of 20 samples summed in order; spp <= 20 is the
 * reference's own sequential sum (main.zig:388-393). */
#define RO_DEFAULT_CHUNK 20u

typedef struct {
  double c0[3];     /* Sphere.center / MovingSphere.center0 */
  double c1[3];     /* MovingSphere.center1 (== c0 for static spheres) */
  double radius;
  double t0, t1;    /* MovingSphere.time0/time1 */
  uint32_t moving;  /* 0 = Sphere (hittable.zig:90), 1 = MovingSphere (:157) */
  uint32_t mat;     /* index into materials */
} ro_sphere;

typedef struct {
  uint32_t kind;
  double albedo[3];     /* solid colour / checker even / metal albedo */
  double albedo_odd[3]; /* checker odd */
  double fuzz;          /* metal */
  double ir;            /* dielectric */
} ro_material;

#define RO_MAX_SPHERES 1024
typedef struct {
  uint32_t n_spheres, n_mats;
  ro_sphere spheres[RO_MAX_SPHERES];
  ro_material mats[RO_MAX_SPHERES];
} ro_scene;

typedef struct { /* main.zig:40-50 */
  double origin[3], horizontal[3], vertical[3], lower_left_corner[3];
  double u[3], v[3], w[3];
  double lens_radius, time0, time1;
} ro_camera;

typedef struct {
  uint32_t width, height;     /* full image */
  uint32_t spp, max_depth;
  uint64_t seed;
  double background[3];
  uint32_t row_begin, row_stride, row_count; /* image rows (top-first) rendered */
  uint32_t chunk;             /* samples per accumulation chunk (0 = RO_DEFAULT_CHUNK, the GPU's default) */
  uint32_t precision;         /* 0 = f64, 1 = f32-hybrid */
  uint32_t threads;           /* OpenMP threads (0 = default) */
} ro_params;

typedef struct {
  uint64_t samples, segments, static_tests, moving_tests, draws;
} ro_stats;

/* ---- Zig std.Random restatement (Zig 0.14 std/Random/ *.zig) ---- */
uint64_t ro_splitmix64_next(uint64_t *state);
void ro_xoshiro256_seed(uint64_t s[4], uint64_t seed);
uint64_t ro_xoshiro256_next(uint64_t s[4]);
double ro_random_f64(uint64_t s[4]);
float ro_random_f32(uint64_t s[4]);

/* Tier-B counter-based stream (see rtw_oracle.c tierb_state). */
uint64_t ro_tierb_state(uint64_t seed, uint64_t pixel, uint64_t sample);
uint64_t ro_tb_mix(uint64_t weyl_state); /* the draw's u64 (Feistel mixer) */
double ro_sm_f64(uint64_t *state);
float ro_sm_f32(uint64_t *state);

/* std/math/pow.zig integer-exponent path (finite x >= 0, integral y > 0). */
double ro_zig_pow(double x, double y);

/* ---- host-side pieces ---- */
void ro_camera_init(ro_camera *cam, const double look_from[3], const double look_at[3],
                    const double vup[3], double vfov, double aspect, double aperture,
                    double focus_dist, double time0, double time1);
/* generateRandomScene (main.zig:157-221); consumes rng (state in/out). */
int ro_cover_scene(uint64_t rng[4], ro_scene *scene);
uint32_t ro_image_height(uint32_t width, double aspect); /* main.zig:306 */

/* ---- Tier A: the reference render loop (main.zig:378-402) ----
 * rng: state after the scene build.  rgb: W*H*3, top row first (main.zig:396).
 * sum_out (optional): W*H*3 f64 per-pixel sums, same layout. */
#define RO_BOOK1_SKY 1u
#define RO_BOOK1_NO_TIME 2u
/* Mutations of one hot-path rule, for the README pin's controls only
 * (tests/test_readme_image.py measures which of them the pin detects):
 * Metal absorbs on the scattered direction instead of `reflected`
 * (material.zig:64); Schlick with exponent 2 instead of 5 (:90); Lambertian
 * adds the unnormalised in-sphere point (:45); the dielectric draws even
 * when it cannot refract (no short circuit, :81). */
#define RO_MUT_METAL_SCATTERED 0x100u
#define RO_MUT_SCHLICK_EXP 0x200u
#define RO_MUT_LAMBERT_NONORM 0x400u
#define RO_MUT_DIEL_ALWAYS_DRAW 0x800u
void ro_render_tier_a_ex(const ro_scene *scene, const ro_camera *cam, const double bg[3],
                         uint32_t W, uint32_t H, uint32_t spp, uint32_t depth,
                         uint64_t rng[4], uint8_t *rgb, double *sum_out, ro_stats *stats,
                         uint32_t flags, uint32_t rows);
/* The README pin's renderer: Tier A arithmetic, one DefaultPrng stream per
 * pixel (seeded from seed + pixel), rows [row0, row1); f64 sums only. */
void ro_render_tier_a_pixel_streams(const ro_scene *scene, const ro_camera *cam, const double bg[3], uint32_t W,
                                    uint32_t H, uint32_t spp, uint32_t depth, uint64_t seed, double *sum_out,
                                    uint32_t flags, uint32_t row0, uint32_t row1);
void ro_render_tier_a(const ro_scene *scene, const ro_camera *cam, const double bg[3],
                      uint32_t W, uint32_t H, uint32_t spp, uint32_t depth,
                      uint64_t rng[4], uint8_t *rgb, double *sum_out, ro_stats *stats);

/* Whole reference main() for scene 1 with the given image parameters. */
void ro_main_cover(uint32_t W, double aspect, uint32_t spp, uint32_t depth, uint64_t seed,
                   uint8_t *rgb, ro_stats *stats);

/* ---- Tier B: the GPU contract ----
 * rgb: W*row_count*3 (local row q = image row row_begin + q*row_stride).
 * mean_out (optional): f32 W*row_count*3 = pixel sum * (1/spp).  */
void ro_render_tier_b(const ro_scene *scene, const ro_camera *cam, const ro_params *p,
                      uint8_t *rgb, float *mean_out, ro_stats *stats);

/* Quantise one channel exactly as main.zig:395-400. */
uint8_t ro_quantize(double c, double scale);
/* Diagnostics: Tier-B radiance of samples s0 .. s0+n-1 of pixel (row y
 * top-first, column x) -> out[n][3]; trace != 0 prints every segment. */
void ro_tierb_samples(const ro_scene *scene, const ro_camera *cam, const ro_params *p, uint32_t y, uint32_t x,
                      uint32_t s0, uint32_t n, double *out, int trace);

#ifdef __cplusplus
}
#endif
#endif
