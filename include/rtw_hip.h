/*
 * rtw_hip.h — C ABI of the MI355X (gfx950) path tracer for the RTIOW cover
 * scene.  Drop-in for the render loop of nsfisis/RayTracingInOneWeekend.zig.
 *
 * The reference has no plugin/FFI surface for this path: Camera, rayColor and
 * the render loop are private to src/main.zig (Camera: main.zig:40-101,
 * rayColor: main.zig:103-122, loop: main.zig:378-402).  This header defines
 * the boundary a Zig host would bind with `extern "rtw_hip" fn ...` (see
 * INTEGRATION.md): the host keeps building the world with the src/rtw API
 * (Hittable / Material / Texture) and flattens it into the plain arrays below.
 *
 * Conventions: plain C types only; 0 = success, negative = rtw_status;
 * the message of the last failure on the calling thread is rtw_last_error().
 * No pointer passed in is retained after a call returns (except device
 * buffers used by a still-running async render on the caller's stream).
 */
#ifndef RTW_HIP_H
#define RTW_HIP_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define RTW_ABI_VERSION 4

typedef enum {
  RTW_OK = 0,
  RTW_EINVAL = -1,      /* bad argument (null pointer, zero size, out of range) */
  RTW_UNSUPPORTED = -2, /* primitive / material / size the kernel does not implement */
  RTW_EHIP = -3,        /* HIP runtime error (message has the HIP error string) */
  RTW_ENOMEM = -4,      /* device allocation failed */
  RTW_ENODEV = -5       /* no GPU visible */
} rtw_status;

/* Material kinds: Material union (material.zig:16-21) x Texture union
 * (texture.zig:10-14) flattened.  DiffuseLight / noise / image textures are
 * not in the cover scene and return RTW_UNSUPPORTED. */
typedef enum {
  RTW_LAMBERT_SOLID = 0,   /* DiffuseMaterial{SolidTexture}   material.zig:41-53, texture.zig:46-55 */
  RTW_LAMBERT_CHECKER = 1, /* DiffuseMaterial{CheckerTexture} texture.zig:57-83 */
  RTW_METAL = 2,           /* MetalMaterial                   material.zig:55-66 */
  RTW_DIELECTRIC = 3,      /* DielectricMaterial              material.zig:68-92 */
  RTW_DIFFUSE_LIGHT = 4    /* DiffuseLightMaterial            material.zig:94-110 (unsupported) */
} rtw_material_kind;

typedef struct {
  uint32_t kind;          /* rtw_material_kind */
  uint32_t reserved;
  double albedo[3];       /* solid colour; checker EVEN colour; metal albedo */
  double albedo_odd[3];   /* checker ODD colour (texture.zig:79-82) */
  double fuzz;            /* metal fuzz (<= 1, material.zig:60) */
  double ir;              /* dielectric index of refraction */
} rtw_material;

/* Sphere (hittable.zig:90-94) or MovingSphere (hittable.zig:157-164). */
typedef struct {
  double c0[3];           /* center / center0 */
  double c1[3];           /* center1 (== c0 for a static sphere) */
  double radius;
  double t0, t1;          /* MovingSphere time0 / time1 (ignored when !moving) */
  uint32_t moving;        /* 0 = Sphere, 1 = MovingSphere */
  uint32_t mat;           /* index into the material array */
} rtw_sphere;

/* Camera fields (main.zig:40-50), computed on the host in f64 by
 * rtw_camera_init (= Camera.init, main.zig:52-89). */
typedef struct {
  double origin[3], horizontal[3], vertical[3], lower_left_corner[3];
  double u[3], v[3], w[3];
  double lens_radius, time0, time1;
} rtw_camera;

typedef enum {
  RTW_PRECISION_F64 = 0,      /* the reference's arithmetic (f64 everywhere) */
  RTW_PRECISION_F32 = 1       /* f32 + f64 for radius >= 100 spheres + convex self-skip */
} rtw_precision;

/* Render engine (both compute the same Tier-B image, bit for bit). */
typedef enum {
  RTW_ENGINE_MEGAKERNEL = 0,  /* one persistent trace kernel (BASELINE.json configs[1]) */
  RTW_ENGINE_WAVEFRONT = 1    /* per-bounce kernels over SoA path queues in HBM (configs[3]) */
} rtw_engine;

/* Wavefront engine, once the unit queue runs dry.  Every
 * choice renders the same image, bit for bit. */
typedef enum {
  RTW_WF_DRAIN_SAMPLES = 0,   /* wf_drain: a segment's remaining samples dealt to its free lanes (default) */
  RTW_WF_DRAIN_SLOTS = 1,     /* wf_finish: each lane runs its own slot's remaining samples */
  RTW_WF_DRAIN_NONE = 2       /* no in-register drain: the bounce kernels' queues run to the end */
} rtw_wf_drain;
typedef enum {
  RTW_WF_FUSED = 0,           /* one kernel per bounce: shade + the next closest hit (default) */
  RTW_WF_SPLIT = 1            /* separate extend (closest hit) and shade kernels per bounce */
} rtw_wf_form;

/* World kernel instantiation (rtw_world_*; every choice gives the same bits). */
typedef enum {
  RTW_WORLD_FEATURES_AUTO = 0, /* the smallest compiled feature set holding the world's features */
  RTW_WORLD_FEATURES_ALL = 1   /* the general kernel (every primitive, texture and transform) */
} rtw_world_features;
typedef enum {
  RTW_WORLD_TRAVERSAL_AUTO = 0,  /* per lane for sphere worlds of >= 256 BVH nodes, else the union */
  RTW_WORLD_TRAVERSAL_UNION = 1, /* the wave walks the union of its lanes' BVH paths (scalar node loads) */
  RTW_WORLD_TRAVERSAL_LANE = 2,  /* every lane walks its own path (sphere worlds with a BVH of depth <= 16 —
                                    rtw_world_create caps the depth of large sphere worlds' trees at 16 —
                                    other worlds take the union walk) */
  RTW_WORLD_TRAVERSAL_LINEAR = 3 /* (reported only, rtw_world_launch_info: a world without a BVH) */
} rtw_world_traversal;

typedef struct {
  uint32_t width, height;     /* full image (main.zig:305-306) */
  uint32_t spp;               /* samples_per_pixel (main.zig:308) */
  uint32_t max_depth;         /* max_depth (main.zig:307), 50 in the reference */
  uint64_t seed;              /* RNG seed (main.zig:300 uses 42) */
  double background[3];       /* main.zig:322 */
  uint32_t row_begin;         /* first IMAGE row rendered (top-first, main.zig:396) */
  uint32_t row_stride;        /* image-row stride (row sharding across GPUs) */
  uint32_t row_count;         /* rows rendered; output row q = image row row_begin+q*row_stride */
  uint32_t chunk;             /* samples per accumulation chunk, 0 = default (RTW_DEFAULT_CHUNK) */
  uint32_t precision;         /* rtw_precision */
  int32_t device;             /* HIP device for rtw_render (-1 = current) */
  uint32_t engine;            /* rtw_engine */
  uint32_t wf_paths;          /* wavefront: in-flight paths (queue capacity), 0 = RTW_DEFAULT_WF_PATHS */
  /* ABI v4: engine configuration, all 0 = default.  The library reads no
   * environment variable on the render path; rtw_workspace_bytes depends on
   * these fields only. */
  uint32_t wf_sets;           /* wavefront: independent queue sets (1-4), 0 = RTW_DEFAULT_WF_SETS */
  uint32_t wf_drain;          /* wavefront: rtw_wf_drain */
  uint32_t wf_form;           /* wavefront: rtw_wf_form */
  uint32_t world_waves;       /* world kernel: register budget in waves per SIMD: 3 or 4, or 1 = unconstrained
                                 (any other value fails with RTW_EINVAL); 0 = the feature set's default
                                 (4 sphere worlds, 3 rects / transforms, 1 noise textures) */
  uint32_t world_features;    /* world kernel: rtw_world_features */
  uint32_t world_traversal;   /* world kernel: rtw_world_traversal */
  uint32_t wf_bounces;        /* wavefront: bounce segments per path per wf_step launch (the path stays in
                                 registers between them), 0 = 1: one queue exchange per bounce (configs[3]) */
  uint32_t wf_passes;         /* wavefront, fused form: queue passes per wf_step launch (every pass moves each
                                 path through the queues), 0 = RTW_DEFAULT_WF_PASSES; at most 64.  (Round 5,
                                 in the place of v4's `reserved`: same layout, and 0 keeps the default.) */
} rtw_params;

/* Samples per accumulation chunk (a work unit = one pixel x one chunk; the
 * image's per-pixel sum adds each chunk's samples in order, then the chunks in
 * order: DESIGN.md §2).  Round 6: 20 (was 32) — every engine equal or faster,
 * the world kernel 3-10 % (profiles/r06/chunk_ab.txt); 20 divides every
 * configured spp (100, 200, 500, 2000). */
#define RTW_DEFAULT_CHUNK 20u
#define RTW_DEFAULT_WF_PATHS (5u << 17) /* 655,360 in-flight paths (with two sets; round 6) */
/* Wavefront queue sets: wf_paths is split over this many independent queue
 * sets, each driven on its own HIP stream (params.wf_sets overrides, 1-4). */
#define RTW_DEFAULT_WF_SETS 2u
#define RTW_MAX_WF_SETS 4u
/* Queue passes per wf_step launch (round 6: 16 with the paths above). */
#define RTW_DEFAULT_WF_PASSES 16u
#define RTW_MAX_SPHERES 4096u

/* ------------------------------------------------------------ queries -- */
int rtw_abi_version(void);
int rtw_device_count(void);
const char *rtw_last_error(void);

/* ------------------------------------------------- host-side helpers --- */
/* Camera.init (main.zig:52-89).  vfov in degrees. */
int rtw_camera_init(rtw_camera *cam, const double look_from[3], const double look_at[3],
                    const double vup[3], double vfov, double aspect_ratio, double aperture,
                    double focus_dist, double time0, double time1);
/* image_height = @intFromFloat(@divTrunc(@as(f64, width), aspect)) (main.zig:306). */
uint32_t rtw_image_height(uint32_t width, double aspect_ratio);
/* generateRandomScene (main.zig:157-221) on DefaultPrng.init(seed)
 * (main.zig:300).  Writes at most *n_spheres / *n_mats entries (in: capacity,
 * out: count).  rng_state_out (optional): the Xoshiro256 state after the
 * build, i.e. where the reference's render loop continues the stream. */
int rtw_cover_scene(uint64_t seed, rtw_sphere *spheres, uint32_t *n_spheres,
                    rtw_material *mats, uint32_t *n_mats, uint64_t rng_state_out[4]);

/* ------------------------------------------------------------ render --- */
/* Replaces the render loop main.zig:378-402.  Host buffers, synchronous.
 * rgb_out:  W * row_count * 3 bytes, rows in output order (see rtw_params).
 * mean_out: optional, W * row_count * 3 floats = pixel sum / spp (linear). */
int rtw_render(const rtw_camera *cam, const rtw_sphere *spheres, uint32_t n_spheres,
               const rtw_material *mats, uint32_t n_mats, const rtw_params *params,
               uint8_t *rgb_out, float *mean_out);

/* ---------------------------------------------- device-resident API --- */
typedef struct rtw_scene_s *rtw_scene;

/* Upload (validate + flatten) a scene to the CURRENT HIP device. */
int rtw_scene_create(const rtw_sphere *spheres, uint32_t n_spheres, const rtw_material *mats,
                     uint32_t n_mats, rtw_scene *out);
int rtw_scene_destroy(rtw_scene scene);

/* Device workspace needed by rtw_render_device for these params. */
size_t rtw_workspace_bytes(const rtw_params *params);

/* Optional kernel timer around the trace kernel (HIP events on the stream). */
typedef struct rtw_timer_s *rtw_timer;
int rtw_timer_create(rtw_timer *out);
int rtw_timer_destroy(rtw_timer t);
int rtw_timer_elapsed_ms(rtw_timer t, float *ms); /* waits for the stop event */

/* Shader-clock probe (diagnostic, for the bench line): one wave on `stream`
 * (launch it on a stream other than the render's) spins for `wall_ms` of wall
 * time and measures the SIMD clock over that window as
 * delta(s_memtime) / delta(s_memrealtime) x 100 MHz — the average SCLK while
 * the renders launched meanwhile run.  _end waits for the probe and frees it. */
typedef struct rtw_sclk_probe_s *rtw_sclk_probe;
int rtw_sclk_probe_begin(void *stream, double wall_ms, rtw_sclk_probe *out);
int rtw_sclk_probe_end(rtw_sclk_probe p, double *mhz);

/* Asynchronous render on `stream` (hipStream_t, NULL = default stream) into
 * DEVICE buffers d_rgb (W*row_count*3 bytes) and optional d_mean
 * (W*row_count*3 floats).  workspace: >= rtw_workspace_bytes(params) bytes
 * of device memory, 256-byte aligned.  timer (optional) brackets the trace
 * kernel.  Megakernel engine: graph-capturable (no allocation, no
 * synchronisation).  Wavefront engine: the host polls the queue length
 * between batches of bounce kernels, so the call returns after the last
 * bounce kernel was ENQUEUED (the finalize kernel is still asynchronous) and
 * it cannot be captured into a graph; the timer brackets all its kernels. */
int rtw_render_device(rtw_scene scene, const rtw_camera *cam, const rtw_params *params,
                      void *workspace, size_t workspace_bytes, uint8_t *d_rgb, float *d_mean,
                      void *stream, rtw_timer timer);

/* Statistics pass (diagnostic, not the product path's timing): counts the
 * bounce segments and sphere tests the same render performs.  counts_out[4] =
 * {samples, segments, static_tests, moving_tests}. Synchronous.  Both engines
 * count samples and segments (the wavefront engine in its shading step). */
int rtw_render_counts(rtw_scene scene, const rtw_camera *cam, const rtw_params *params,
                      void *workspace, size_t workspace_bytes, uint64_t counts_out[4]);
/* The same pass with counts_out[6]: the four above, then the segments traced
 * and the samples finished by the wavefront engine's in-register drain
 * (paths that no longer stream through the HBM queues; 0 for the megakernel
 * and with RTW_WF_DRAIN_NONE). */
int rtw_render_counts_ex(rtw_scene scene, const rtw_camera *cam, const rtw_params *params,
                         void *workspace, size_t workspace_bytes, uint64_t counts_out[6]);
/* The same pass with the kernels' raw statistics words (diagnostic):
 * stats_out[RTW_STATS_WORDS], indices RTW_STAT_*. */
#define RTW_STATS_WORDS 16
enum {
  RTW_STAT_SAMPLES = 0, RTW_STAT_SEGMENTS = 1, RTW_STAT_F32_SKIPS = 2,
  RTW_STAT_CAND_WAVE_ITERS = 3, RTW_STAT_CAND_LANES = 4, RTW_STAT_DISC_GE0_LANES = 5,
  RTW_STAT_SPHERE_LOOP_WAVE_ITERS = 6, RTW_STAT_CULL_SURVIVOR_LANES = 7, RTW_STAT_CULL_EXACT_WAVE_ITERS = 8,
  RTW_STAT_DRAIN_SEGMENTS = 9, RTW_STAT_DRAIN_SAMPLES = 10, RTW_STAT_CLUSTER_WAVE_TESTS = 11,
  RTW_STAT_CLUSTER_WAVE_SKIPS = 12, RTW_STAT_DRAIN_WAVE_ITERS = 13
};
int rtw_render_stats(rtw_scene scene, const rtw_camera *cam, const rtw_params *params,
                     void *workspace, size_t workspace_bytes, uint64_t stats_out[RTW_STATS_WORDS]);

/* =================================================== general worlds ===
 * Every other scene of the reference (main.zig:123-290) and BASELINE.json
 * configs[4] (globe + 10k spheres): the full Hittable / Material / Texture
 * vocabulary, flattened.  Nested lists (Box = 6 rects) become consecutive
 * primitives in list order; Translate / RotateY wrappers become a transform
 * chain per primitive.  Rendered by the world kernel (f64, BVH traversal),
 * whose per-sample contract is oracle/rtw_world.h Tier B. */

typedef enum {
  RTW_PRIM_SPHERE = 0,        /* Sphere        hittable.zig:90-155  a = c[3], c[3], r, 0, 0 */
  RTW_PRIM_MOVING_SPHERE = 1, /* MovingSphere  hittable.zig:157-226 a = c0[3], c1[3], r, t0, t1 */
  RTW_PRIM_XY_RECT = 2,       /* XyRect        hittable.zig:270-323 a = x0, x1, y0, y1, k */
  RTW_PRIM_XZ_RECT = 3,       /* XzRect        hittable.zig:325-378 a = x0, x1, z0, z1, k */
  RTW_PRIM_YZ_RECT = 4        /* YzRect        hittable.zig:380-427 a = y0, y1, z0, z1, k */
} rtw_prim_kind;

typedef struct {
  uint32_t kind, mat;
  int32_t xform;              /* index into xforms, -1 = none */
  uint32_t reserved;
  double a[9];
} rtw_prim;

#define RTW_MAX_XFORM_OPS 4
typedef enum {
  RTW_XF_TRANSLATE = 0,       /* Translate hittable.zig:472-503: v = offset */
  RTW_XF_ROTATE_Y = 1         /* RotateY   hittable.zig:505-608: v = {sin_t, cos_t, angle} */
} rtw_xform_op;
typedef struct {              /* op[0] is the OUTERMOST wrapper */
  uint32_t n;
  uint32_t op[RTW_MAX_XFORM_OPS];
  double v[RTW_MAX_XFORM_OPS][3];
} rtw_xform;

typedef enum {
  RTW_TEX_SOLID = 0,          /* texture.zig:46-55 */
  RTW_TEX_CHECKER = 1,        /* texture.zig:57-83 (solid odd / even) */
  RTW_TEX_NOISE = 2,          /* texture.zig:85-105 (perlin index, scale) */
  RTW_TEX_IMAGE = 3           /* texture.zig:107-144 (image index) */
} rtw_texture_kind;
typedef struct {
  uint32_t kind, perlin, image, reserved;
  double color[3], odd[3], even[3];
  double scale;
} rtw_texture;

typedef enum {
  RTW_WMAT_LAMBERT = 0,       /* DiffuseMaterial      material.zig:41-53 (albedo texture) */
  RTW_WMAT_METAL = 1,         /* MetalMaterial        material.zig:55-66 */
  RTW_WMAT_DIELECTRIC = 2,    /* DielectricMaterial   material.zig:68-92 */
  RTW_WMAT_LIGHT = 3          /* DiffuseLightMaterial material.zig:94-110 (emit texture) */
} rtw_wmaterial_kind;
typedef struct {
  uint32_t kind, tex;
  double albedo[3];
  double fuzz, ir;
} rtw_wmaterial;

typedef struct {              /* Perlin, perlin.zig:10-40 */
  double ranvec[256][3];
  uint32_t perm[3][256];
} rtw_perlin;

typedef struct {              /* decoded texture image: RGBA8, row-major, top row first */
  uint32_t width, height;
  const uint8_t *rgba;
} rtw_image;

typedef struct {
  const rtw_prim *prims;          uint32_t n_prims;
  const rtw_xform *xforms;        uint32_t n_xforms;
  const rtw_texture *textures;    uint32_t n_textures;
  const rtw_wmaterial *mats;      uint32_t n_mats;
  const rtw_perlin *perlins;      uint32_t n_perlins;
  const rtw_image *images;        uint32_t n_images;
} rtw_world_desc;

/* Camera / image settings a scene sets in main() (main.zig:303-376). */
typedef struct {
  double look_from[3], look_at[3], vfov, aperture, aspect;
  double background[3];
  uint32_t width, height, spp, reserved;
} rtw_scene_settings;

/* Scene builders of main.zig on DefaultPrng.init(seed): 1 cover (:157),
 * 2 two spheres (:123), 3 two Perlin spheres (:140), 4 earth (:223),
 * 5 simple light (:235), 6 Cornell box (:256), 7 globe + 10k random spheres
 * (configs[4]; not a reference scene).  `image` is the earth texture
 * (scenes 4, 7; pixels are copied).  The built scene owns its arrays;
 * rtw_built_scene_desc points into them until rtw_built_scene_free. */
typedef struct rtw_built_scene_s *rtw_built_scene;
int rtw_build_scene(uint32_t scene_id, uint64_t seed, const rtw_image *image, rtw_built_scene *out);
int rtw_built_scene_desc(rtw_built_scene b, rtw_world_desc *desc, rtw_scene_settings *settings,
                         uint64_t rng_state_after[4]);
int rtw_built_scene_free(rtw_built_scene b);

/* Upload a world to the CURRENT device: tables + a BVH over worlds of more
 * than 32 primitives (flags bit 0 = RTW_WORLD_LINEAR: no BVH, every segment
 * tests every primitive in a wave-uniform loop; bit 1 = RTW_WORLD_DEBUG_BVH). */
#define RTW_WORLD_LINEAR 1u
#define RTW_WORLD_DEBUG_BVH 2u /* diagnostic: the BVH root's two children (leaf / node, boxes) to stderr */
typedef struct rtw_world_s *rtw_world;
int rtw_world_create(const rtw_world_desc *desc, uint32_t flags, rtw_world *out);
int rtw_world_destroy(rtw_world world);
/* BVH statistics: nodes, leaves, max depth, max leaf size. */
int rtw_world_bvh_info(rtw_world world, uint32_t info_out[4]);

/* Device workspace of a world render on the CURRENT device (the world's):
 * rtw_workspace_bytes(params) + the tail dealing's per-lane sample rings
 * (one per lane of the persistent grid).  The rings live in the caller's
 * workspace, so renders on different streams, each with its own workspace,
 * are independent.  0 on error. */
size_t rtw_world_workspace_bytes(rtw_world world, const rtw_params *params);
/* Asynchronous render of a world (params.precision must be F64, engine
 * MEGAKERNEL); workspace sized by rtw_world_workspace_bytes(world, params).
 * A workspace of only rtw_workspace_bytes(params) bytes renders without tail
 * dealing (the same image, a few % slower on the large scenes). */
int rtw_world_render_device(rtw_world world, const rtw_camera *cam, const rtw_params *params,
                            void *workspace, size_t workspace_bytes, uint8_t *d_rgb, float *d_mean,
                            void *stream, rtw_timer timer);
/* Synchronous host-buffer render of a world description. */
int rtw_world_render(const rtw_camera *cam, const rtw_world_desc *desc, const rtw_params *params,
                     uint8_t *rgb_out, float *mean_out);
/* How a render of `world` with `params` would launch on the current device
 * (the world's): info_out[6] = {traversal (rtw_world_traversal: LANE, UNION
 * or LINEAR, after AUTO and the world's limits are applied), kernel feature
 * set, register budget (waves per SIMD: 4, 3, or 1 = unconstrained),
 * workgroups per CU, persistent grid (workgroups), dynamic LDS bytes per
 * workgroup}. */
int rtw_world_launch_info(rtw_world world, const rtw_params *params, uint32_t info_out[6]);
/* Statistics pass: counts_out[4] = {samples, segments, node_visits, prim_tests}. */
int rtw_world_render_counts(rtw_world world, const rtw_camera *cam, const rtw_params *params,
                            void *workspace, size_t workspace_bytes, uint64_t counts_out[4]);
/* The same pass with counts_out[8]: the four above (node visits and primitive
 * tests counted per lane: each lane's own under the per-lane traversal, the
 * wave's under the union walk), then the wave iterations of the persistent
 * kernel, whether tail dealing ran (1: the workspace held the per-lane rings,
 * 0: it did not — same image, slower end of launch), and the per-lane
 * traversal's interior-step and leaf-test wave iterations (0 for the union). */
int rtw_world_render_counts_ex(rtw_world world, const rtw_camera *cam, const rtw_params *params,
                               void *workspace, size_t workspace_bytes, uint64_t counts_out[8]);

#ifdef __cplusplus
}
#endif
#endif /* RTW_HIP_H */
