"""rtw_amd — Python binding of the MI355X path tracer's C ABI (include/rtw_hip.h).

The product path is lib/librtw_hip.so (HIP kernels for gfx950 + host helpers).
This module only marshals plain arrays through ctypes; there is NO CPU
fallback: if the library is missing or no GPU is visible, calls fail loudly.

Reference correspondence (nsfisis/RayTracingInOneWeekend.zig):
  camera_init   -> Camera.init          src/main.zig:52-89
  image_height  -> main.zig:306
  cover_scene   -> generateRandomScene  src/main.zig:157-221 (DefaultPrng.init(seed), main.zig:300)
  render        -> the render loop      src/main.zig:378-402 (+ rayColor :103-122)
"""
from __future__ import annotations

import ctypes as C
import os
import re

import numpy as np

PKG_DIR = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(PKG_DIR)                      # raytracinginoneweekend.zig_amd/
REPO = os.path.dirname(ROOT)
LIB_PATH = os.environ.get("RTW_LIB_PATH") or os.path.join(ROOT, "lib", "librtw_hip.so")  # (override: dev A/B)
HEADER_PATH = os.path.join(REPO, "include", "rtw_hip.h")

RTW_OK, RTW_EINVAL, RTW_UNSUPPORTED, RTW_EHIP, RTW_ENOMEM, RTW_ENODEV = 0, -1, -2, -3, -4, -5
LAMBERT_SOLID, LAMBERT_CHECKER, METAL, DIELECTRIC, DIFFUSE_LIGHT = 0, 1, 2, 3, 4
PRECISION = {"f64": 0, "f32": 1}
ENGINE = {"megakernel": 0, "wavefront": 1}
DEFAULT_WF_PATHS = 5 << 17  # rtw_hip.h RTW_DEFAULT_WF_PATHS
DEFAULT_WF_SETS = 2  # rtw_hip.h RTW_DEFAULT_WF_SETS (params.wf_sets overrides)
DEFAULT_WF_PASSES = 16  # rtw_hip.h RTW_DEFAULT_WF_PASSES (params.wf_passes overrides)
WF_DRAIN = {"samples": 0, "slots": 1, "none": 2}  # rtw_wf_drain
WF_FORM = {"fused": 0, "split": 1}  # rtw_wf_form
WORLD_FEATURES = {"auto": 0, "all": 1}  # rtw_world_features
WORLD_TRAVERSAL = {"auto": 0, "union": 1, "lane": 2}  # rtw_world_traversal
STATS_WORDS = 16  # rtw_hip.h RTW_STATS_WORDS
STAT_NAMES = ["samples", "segments", "f32_skips", "cand_wave_iters", "cand_lanes", "disc_ge0_lanes",
              "sphere_loop_wave_iters", "cull_survivor_lanes", "cull_exact_wave_iters", "drain_segments",
              "drain_samples", "cluster_wave_tests", "cluster_wave_skips", "drain_wave_iters"]  # RTW_STAT_*
DEFAULT_CHUNK = 20
COVER_BACKGROUND = (0.70, 0.80, 1.00)


class RtwError(RuntimeError):
    def __init__(self, status: int, msg: str):
        super().__init__(f"rtw status {status}: {msg}")
        self.status = status


class Material(C.Structure):
    _fields_ = [("kind", C.c_uint32), ("reserved", C.c_uint32), ("albedo", C.c_double * 3),
                ("albedo_odd", C.c_double * 3), ("fuzz", C.c_double), ("ir", C.c_double)]


class Sphere(C.Structure):
    _fields_ = [("c0", C.c_double * 3), ("c1", C.c_double * 3), ("radius", C.c_double),
                ("t0", C.c_double), ("t1", C.c_double), ("moving", C.c_uint32), ("mat", C.c_uint32)]


class Camera(C.Structure):
    _fields_ = [(n, C.c_double * 3) for n in
                ("origin", "horizontal", "vertical", "lower_left_corner", "u", "v", "w")] + \
               [("lens_radius", C.c_double), ("time0", C.c_double), ("time1", C.c_double)]


class Params(C.Structure):
    _fields_ = [("width", C.c_uint32), ("height", C.c_uint32), ("spp", C.c_uint32),
                ("max_depth", C.c_uint32), ("seed", C.c_uint64), ("background", C.c_double * 3),
                ("row_begin", C.c_uint32), ("row_stride", C.c_uint32), ("row_count", C.c_uint32),
                ("chunk", C.c_uint32), ("precision", C.c_uint32), ("device", C.c_int32),
                ("engine", C.c_uint32), ("wf_paths", C.c_uint32),
                ("wf_sets", C.c_uint32), ("wf_drain", C.c_uint32), ("wf_form", C.c_uint32),
                ("world_waves", C.c_uint32), ("world_features", C.c_uint32), ("world_traversal", C.c_uint32),
                ("wf_bounces", C.c_uint32), ("wf_passes", C.c_uint32)]


_lib = None


def lib() -> C.CDLL:
    """Load lib/librtw_hip.so (built by `make -C raytracinginoneweekend.zig_amd`)."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise RuntimeError(f"{LIB_PATH} is missing: run __graft_entry__.build() "
                           "(there is no CPU fallback for the render path)")
    # One HIP runtime per process: torch wheels bundle their own
    # libamdhip64.so.7 (same soname as /opt/rocm's).  Loading torch first makes
    # the dynamic loader bind this library to torch's copy, so torch's device
    # memory / streams and our kernels share one runtime.
    try:
        import torch  # noqa: F401
    except ImportError:
        pass
    L = C.CDLL(LIB_PATH)
    P = C.POINTER
    L.rtw_abi_version.restype = C.c_int
    L.rtw_device_count.restype = C.c_int
    L.rtw_last_error.restype = C.c_char_p
    L.rtw_camera_init.argtypes = [P(Camera)] + [C.c_double * 3] * 3 + [C.c_double] * 6
    L.rtw_image_height.restype = C.c_uint32
    L.rtw_image_height.argtypes = [C.c_uint32, C.c_double]
    L.rtw_cover_scene.argtypes = [C.c_uint64, C.c_void_p, P(C.c_uint32), C.c_void_p, P(C.c_uint32),
                                  C.c_uint64 * 4]
    L.rtw_render.argtypes = [P(Camera), C.c_void_p, C.c_uint32, C.c_void_p, C.c_uint32, P(Params),
                             C.c_void_p, C.c_void_p]
    L.rtw_scene_create.argtypes = [C.c_void_p, C.c_uint32, C.c_void_p, C.c_uint32, P(C.c_void_p)]
    L.rtw_scene_destroy.argtypes = [C.c_void_p]
    L.rtw_workspace_bytes.restype = C.c_size_t
    L.rtw_workspace_bytes.argtypes = [P(Params)]
    L.rtw_timer_create.argtypes = [P(C.c_void_p)]
    L.rtw_timer_destroy.argtypes = [C.c_void_p]
    L.rtw_timer_elapsed_ms.argtypes = [C.c_void_p, P(C.c_float)]
    L.rtw_sclk_probe_begin.argtypes = [C.c_void_p, C.c_double, P(C.c_void_p)]
    L.rtw_sclk_probe_end.argtypes = [C.c_void_p, P(C.c_double)]
    L.rtw_render_device.argtypes = [C.c_void_p, P(Camera), P(Params), C.c_void_p, C.c_size_t,
                                    C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p]
    L.rtw_render_counts.argtypes = [C.c_void_p, P(Camera), P(Params), C.c_void_p, C.c_size_t,
                                    C.c_uint64 * 4]
    L.rtw_render_counts_ex.argtypes = [C.c_void_p, P(Camera), P(Params), C.c_void_p, C.c_size_t,
                                       C.c_uint64 * 6]
    L.rtw_render_stats.argtypes = [C.c_void_p, P(Camera), P(Params), C.c_void_p, C.c_size_t,
                                   C.c_uint64 * STATS_WORDS]
    _lib = L
    return L


def header_symbols() -> list[str]:
    """Every function the C ABI header declares (for the export test)."""
    txt = open(HEADER_PATH).read()
    txt = re.sub(r"/\*.*?\*/", "", txt, flags=re.S)
    return sorted(set(re.findall(r"\b(rtw_[a-z0-9_]+)\s*\(", txt)))


def _check(status: int):
    if status != RTW_OK:
        raise RtwError(status, (lib().rtw_last_error() or b"").decode())


def abi_version() -> int:
    return lib().rtw_abi_version()


def device_count() -> int:
    return lib().rtw_device_count()


# ------------------------------------------------------ host helpers ----
def camera_init(look_from, look_at, vup, vfov, aspect, aperture, focus_dist, time0=0.0, time1=1.0) -> Camera:
    cam = Camera()
    arr = C.c_double * 3
    _check(lib().rtw_camera_init(C.byref(cam), arr(*look_from), arr(*look_at), arr(*vup), vfov, aspect,
                                 aperture, focus_dist, time0, time1))
    return cam


def cover_camera(aspect: float) -> Camera:
    """Scene-1 camera: main.zig:323-326 and :366-376."""
    return camera_init((13, 2, 3), (0, 0, 0), (0, 1, 0), 20.0, aspect, 0.1, 10.0, 0.0, 1.0)


def image_height(width: int, aspect: float) -> int:
    return int(lib().rtw_image_height(width, aspect))


def cover_scene(seed: int = 42):
    """generateRandomScene on DefaultPrng.init(seed) -> (spheres, materials, rng_state)."""
    ns, nm = C.c_uint32(0), C.c_uint32(0)
    st = (C.c_uint64 * 4)()
    _check(lib().rtw_cover_scene(seed, None, C.byref(ns), None, C.byref(nm), st))
    sph = (Sphere * ns.value)()
    mats = (Material * nm.value)()
    _check(lib().rtw_cover_scene(seed, sph, C.byref(ns), mats, C.byref(nm), st))
    return sph, mats, [int(x) for x in st]


def make_params(width, height, spp, max_depth=50, seed=42, background=COVER_BACKGROUND, row_begin=0,
                row_stride=1, row_count=None, chunk=0, precision="f64", device=-1, engine="megakernel",
                wf_paths=0, wf_sets=0, wf_drain="samples", wf_form="fused", world_waves=0,
                world_features="auto", world_traversal="auto", wf_bounces=0, wf_passes=0) -> Params:
    """rtw_params (ABI v4): every engine choice is a field (0 / the first
    name = the library default); nothing is read from the environment."""
    if row_count is None:
        row_count = (height - row_begin + row_stride - 1) // row_stride
    prec = PRECISION[precision] if isinstance(precision, str) else int(precision)
    eng = ENGINE[engine] if isinstance(engine, str) else int(engine)

    def enum(v, names):
        return names[v] if isinstance(v, str) else int(v)
    return Params(width, height, spp, max_depth, seed, (C.c_double * 3)(*background), row_begin, row_stride,
                  row_count, chunk, prec, device, eng, wf_paths, wf_sets, enum(wf_drain, WF_DRAIN),
                  enum(wf_form, WF_FORM), world_waves, enum(world_features, WORLD_FEATURES),
                  enum(world_traversal, WORLD_TRAVERSAL), wf_bounces, wf_passes)


def _arr(x, typ):
    if x is None or len(x) == 0:
        return None, 0
    return x, len(x)


def render(cam: Camera, spheres, mats, params: Params, want_mean=False):
    """Synchronous host-buffer render (rtw_render): rgb (rows, W, 3) uint8 [, mean f32]."""
    rgb = np.zeros((params.row_count, params.width, 3), np.uint8)
    mean = np.zeros((params.row_count, params.width, 3), np.float32) if want_mean else None
    s, n = _arr(spheres, Sphere)
    m, nm = _arr(mats, Material)
    _check(lib().rtw_render(C.byref(cam), s, n, m, nm, C.byref(params), rgb.ctypes.data,
                            mean.ctypes.data if want_mean else None))
    return (rgb, mean) if want_mean else rgb


def workspace_bytes(params: Params) -> int:
    n = lib().rtw_workspace_bytes(C.byref(params))
    if n == 0:
        _check(RTW_EINVAL)
    return int(n)


class SclkProbe:
    """Average shader clock (MHz) over a wall-time window (rtw_sclk_probe_*):
    start it on a side stream, run the renders, then read()."""

    def __init__(self, stream: int, wall_ms: float):
        self.h = C.c_void_p()
        _check(lib().rtw_sclk_probe_begin(C.c_void_p(stream), float(wall_ms), C.byref(self.h)))

    def read(self) -> float:
        mhz = C.c_double()
        h, self.h = self.h, C.c_void_p()
        _check(lib().rtw_sclk_probe_end(h, C.byref(mhz)))
        return float(mhz.value)


class Timer:
    """HIP events bracketing the trace kernel on the render stream."""

    def __init__(self):
        self.h = C.c_void_p()
        _check(lib().rtw_timer_create(C.byref(self.h)))

    def elapsed_ms(self) -> float:
        ms = C.c_float()
        _check(lib().rtw_timer_elapsed_ms(self.h, C.byref(ms)))
        return float(ms.value)

    def close(self):
        if self.h:
            lib().rtw_timer_destroy(self.h)
            self.h = C.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


class DeviceScene:
    """A scene resident in HBM of the current device (rtw_scene_create)."""

    def __init__(self, spheres, mats):
        self.h = C.c_void_p()
        s, n = _arr(spheres, Sphere)
        m, nm = _arr(mats, Material)
        _check(lib().rtw_scene_create(s, n, m, nm, C.byref(self.h)))
        self.n_spheres, self.n_materials = n, nm

    def render_async(self, cam: Camera, params: Params, workspace_ptr: int, workspace_bytes_: int,
                     rgb_ptr: int, mean_ptr: int | None = None, stream: int | None = None,
                     timer: Timer | None = None):
        """rtw_render_device on `stream` (a hipStream_t as int) into device buffers."""
        _check(lib().rtw_render_device(self.h, C.byref(cam), C.byref(params), C.c_void_p(workspace_ptr),
                                       workspace_bytes_, C.c_void_p(rgb_ptr),
                                       C.c_void_p(mean_ptr) if mean_ptr else None,
                                       C.c_void_p(stream) if stream else None,
                                       timer.h if timer is not None else None))

    def counts(self, cam: Camera, params: Params, workspace_ptr: int, workspace_bytes_: int) -> dict:
        out = (C.c_uint64 * 6)()
        _check(lib().rtw_render_counts_ex(self.h, C.byref(cam), C.byref(params), C.c_void_p(workspace_ptr),
                                          workspace_bytes_, out))
        return {"samples": int(out[0]), "segments": int(out[1]), "static_tests": int(out[2]),
                "moving_tests": int(out[3]), "drain_segments": int(out[4]), "drain_samples": int(out[5])}

    def stats(self, cam: Camera, params: Params, workspace_ptr: int, workspace_bytes_: int) -> dict:
        """The counting pass's raw statistics words (rtw_render_stats, RTW_STAT_*)."""
        out = (C.c_uint64 * STATS_WORDS)()
        _check(lib().rtw_render_stats(self.h, C.byref(cam), C.byref(params), C.c_void_p(workspace_ptr),
                                      workspace_bytes_, out))
        return {n: int(out[i]) for i, n in enumerate(STAT_NAMES)}

    def close(self):
        if self.h:
            lib().rtw_scene_destroy(self.h)
            self.h = C.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass
