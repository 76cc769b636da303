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

#define RTW_ABI_VERSION 2

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
} rtw_params;

#define RTW_DEFAULT_CHUNK 32u
#define RTW_DEFAULT_WF_PATHS (1u << 20)
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
 * count samples and segments (the wavefront engine in its shade kernel). */
int rtw_render_counts(rtw_scene scene, const rtw_camera *cam, const rtw_params *params,
                      void *workspace, size_t workspace_bytes, uint64_t counts_out[4]);

#ifdef __cplusplus
}
#endif
#endif /* RTW_HIP_H */
