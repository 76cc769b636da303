"""ctypes front-end of the CPU ORACLE (oracle/librtw_oracle.so).

TEST INFRASTRUCTURE ONLY: imported by tests/, __graft_entry__.smoke() and
bench.py's cpu_baseline leg — as the checker or the timed CPU baseline, never
as the product path.  See rtw_oracle.h for the Tier A / Tier B definitions and
the parity status ("parity unpinned" against the Zig binary; pinned by RNG
KATs and the independent Python restatement in rtw_oracle_py.py).
"""
from __future__ import annotations

import ctypes as C
import math
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(HERE, "librtw_oracle.so")

MAX_SPHERES = 1024
LAMBERT_SOLID, LAMBERT_CHECKER, METAL, DIELECTRIC = 0, 1, 2, 3


class Sphere(C.Structure):
    _fields_ = [("c0", C.c_double * 3), ("c1", C.c_double * 3), ("radius", C.c_double),
                ("t0", C.c_double), ("t1", C.c_double), ("moving", C.c_uint32), ("mat", C.c_uint32)]


class Material(C.Structure):
    _fields_ = [("kind", C.c_uint32), ("albedo", C.c_double * 3), ("albedo_odd", C.c_double * 3),
                ("fuzz", C.c_double), ("ir", C.c_double)]


class Scene(C.Structure):
    _fields_ = [("n_spheres", C.c_uint32), ("n_mats", C.c_uint32),
                ("spheres", Sphere * MAX_SPHERES), ("mats", Material * MAX_SPHERES)]


class Camera(C.Structure):
    _fields_ = [(n, C.c_double * 3) for n in
                ("origin", "horizontal", "vertical", "lower_left_corner", "u", "v", "w")] + \
               [("lens_radius", C.c_double), ("time0", C.c_double), ("time1", C.c_double)]


class Params(C.Structure):
    _fields_ = [("width", C.c_uint32), ("height", C.c_uint32), ("spp", C.c_uint32),
                ("max_depth", C.c_uint32), ("seed", C.c_uint64), ("background", C.c_double * 3),
                ("row_begin", C.c_uint32), ("row_stride", C.c_uint32), ("row_count", C.c_uint32),
                ("chunk", C.c_uint32), ("precision", C.c_uint32), ("threads", C.c_uint32)]


class Stats(C.Structure):
    _fields_ = [("samples", C.c_uint64), ("segments", C.c_uint64), ("static_tests", C.c_uint64),
                ("moving_tests", C.c_uint64), ("draws", C.c_uint64)]

    def as_dict(self):
        return {n: int(getattr(self, n)) for n, _ in self._fields_}


U64x4 = C.c_uint64 * 4
_lib = None


def build():
    """Compile the oracle with its own Makefile (gcc)."""
    subprocess.run(["make", "-s", "-C", HERE], check=True)


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            build()
        L = C.CDLL(LIB_PATH)
        L.ro_splitmix64_next.restype = C.c_uint64
        L.ro_splitmix64_next.argtypes = [C.POINTER(C.c_uint64)]
        L.ro_xoshiro256_seed.argtypes = [U64x4, C.c_uint64]
        L.ro_xoshiro256_next.restype = C.c_uint64
        L.ro_xoshiro256_next.argtypes = [U64x4]
        L.ro_random_f64.restype = C.c_double
        L.ro_random_f64.argtypes = [U64x4]
        L.ro_random_f32.restype = C.c_float
        L.ro_random_f32.argtypes = [U64x4]
        L.ro_tierb_state.restype = C.c_uint64
        L.ro_tierb_state.argtypes = [C.c_uint64, C.c_uint64, C.c_uint64]
        L.ro_tb_mix.restype = C.c_uint64
        L.ro_tb_mix.argtypes = [C.c_uint64]
        L.ro_sm_f64.restype = C.c_double
        L.ro_sm_f64.argtypes = [C.POINTER(C.c_uint64)]
        L.ro_sm_f32.restype = C.c_float
        L.ro_sm_f32.argtypes = [C.POINTER(C.c_uint64)]
        L.ro_zig_pow.restype = C.c_double
        L.ro_zig_pow.argtypes = [C.c_double, C.c_double]
        L.ro_camera_init.argtypes = [C.POINTER(Camera)] + [C.c_double * 3] * 3 + [C.c_double] * 6
        L.ro_cover_scene.restype = C.c_int
        L.ro_cover_scene.argtypes = [U64x4, C.POINTER(Scene)]
        L.ro_image_height.restype = C.c_uint32
        L.ro_image_height.argtypes = [C.c_uint32, C.c_double]
        L.ro_render_tier_a.argtypes = [C.POINTER(Scene), C.POINTER(Camera), C.c_double * 3,
                                       C.c_uint32, C.c_uint32, C.c_uint32, C.c_uint32, U64x4,
                                       C.c_void_p, C.c_void_p, C.POINTER(Stats)]
        L.ro_main_cover.argtypes = [C.c_uint32, C.c_double, C.c_uint32, C.c_uint32, C.c_uint64,
                                    C.c_void_p, C.POINTER(Stats)]
        L.ro_render_tier_b.argtypes = [C.POINTER(Scene), C.POINTER(Camera), C.POINTER(Params),
                                       C.c_void_p, C.c_void_p, C.POINTER(Stats)]
        L.ro_render_tier_a_ex.argtypes = [C.POINTER(Scene), C.POINTER(Camera), C.c_double * 3, C.c_uint32,
                                          C.c_uint32, C.c_uint32, C.c_uint32, U64x4, C.c_void_p, C.c_void_p,
                                          C.POINTER(Stats), C.c_uint32, C.c_uint32]
        L.ro_render_tier_a_pixel_streams.argtypes = [C.POINTER(Scene), C.POINTER(Camera), C.c_double * 3,
                                                     C.c_uint32, C.c_uint32, C.c_uint32, C.c_uint32, C.c_uint64,
                                                     C.c_void_p, C.c_uint32, C.c_uint32, C.c_uint32]
        L.ro_tierb_samples.argtypes = [C.POINTER(Scene), C.POINTER(Camera), C.POINTER(Params), C.c_uint32,
                                       C.c_uint32, C.c_uint32, C.c_uint32, C.c_void_p, C.c_int]
        L.ro_quantize.restype = C.c_uint8
        L.ro_quantize.argtypes = [C.c_double, C.c_double]
        _lib = L
    return _lib


# ---------------------------------------------------------------- RNG ----
class ZigRandom:
    """DefaultPrng (Xoshiro256++) stream, as main.zig:300 uses it."""

    def __init__(self, seed: int | None = None, state=None):
        self.s = U64x4()
        if state is not None:
            for i in range(4):
                self.s[i] = state[i]
        else:
            lib().ro_xoshiro256_seed(self.s, seed)

    def next(self) -> int:
        return lib().ro_xoshiro256_next(self.s)

    def f64(self) -> float:
        return lib().ro_random_f64(self.s)

    def f32(self) -> float:
        return lib().ro_random_f32(self.s)

    def state(self):
        return [int(self.s[i]) for i in range(4)]


def splitmix64_seq(seed: int, n: int):
    st = C.c_uint64(seed)
    return [lib().ro_splitmix64_next(C.byref(st)) for _ in range(n)]


# -------------------------------------------------------------- scene ----
COVER_BG = (0.70, 0.80, 1.00)


def image_height(width: int, aspect: float) -> int:
    return int(lib().ro_image_height(width, aspect))


def cover_scene(seed: int = 42):
    """generateRandomScene on a fresh DefaultPrng.init(seed); returns
    (Scene, ZigRandom positioned after the build)."""
    rng = ZigRandom(seed)
    sc = Scene()
    lib().ro_cover_scene(rng.s, C.byref(sc))
    return sc, rng


def cover_camera(aspect: float) -> Camera:
    """Scene-1 camera (main.zig:320-326, :366-376)."""
    cam = Camera()
    arr = C.c_double * 3
    lib().ro_camera_init(C.byref(cam), arr(13, 2, 3), arr(0, 0, 0), arr(0, 1, 0),
                         20.0, aspect, 0.1, 10.0, 0.0, 1.0)
    return cam


def scene_table(sc: Scene) -> dict:
    """Plain-python dump of the flattened scene (for golden fixtures)."""
    sph = []
    for i in range(sc.n_spheres):
        s = sc.spheres[i]
        sph.append({"c0": list(s.c0), "c1": list(s.c1), "radius": s.radius, "t0": s.t0, "t1": s.t1,
                    "moving": int(s.moving), "mat": int(s.mat)})
    mats = []
    for i in range(sc.n_mats):
        m = sc.mats[i]
        mats.append({"kind": int(m.kind), "albedo": list(m.albedo), "albedo_odd": list(m.albedo_odd),
                     "fuzz": m.fuzz, "ir": m.ir})
    return {"spheres": sph, "materials": mats}


def scene_from_table(t: dict) -> Scene:
    sc = Scene()
    sc.n_spheres = len(t["spheres"])
    sc.n_mats = len(t["materials"])
    for i, s in enumerate(t["spheres"]):
        d = sc.spheres[i]
        d.c0[:] = s["c0"]
        d.c1[:] = s["c1"]
        d.radius, d.t0, d.t1 = s["radius"], s["t0"], s["t1"]
        d.moving, d.mat = s["moving"], s["mat"]
    for i, m in enumerate(t["materials"]):
        d = sc.mats[i]
        d.kind = m["kind"]
        d.albedo[:] = m["albedo"]
        d.albedo_odd[:] = m["albedo_odd"]
        d.fuzz, d.ir = m["fuzz"], m["ir"]
    return sc


# ------------------------------------------------------------- render ----
def main_cover(width: int, aspect: float, spp: int, depth: int = 50, seed: int = 42):
    """Tier A: the whole reference main() for scene 1 -> (H, W, 3) uint8."""
    H = image_height(width, aspect)
    out = np.zeros((H, width, 3), np.uint8)
    st = Stats()
    lib().ro_main_cover(width, aspect, spp, depth, seed, out.ctypes.data, C.byref(st))
    return out, st.as_dict()


def render_tier_a(scene: Scene, cam: Camera, rng: ZigRandom, width: int, height: int, spp: int,
                  depth: int = 50, bg=COVER_BG, want_sum=False):
    out = np.zeros((height, width, 3), np.uint8)
    sums = np.zeros((height, width, 3), np.float64) if want_sum else None
    st = Stats()
    lib().ro_render_tier_a(C.byref(scene), C.byref(cam), (C.c_double * 3)(*bg), width, height, spp,
                           depth, rng.s, out.ctypes.data, sums.ctypes.data if want_sum else None,
                           C.byref(st))
    return out, sums, st.as_dict()


# ------------------------------------------ CPU baseline port (bench) ----
PORT_SRC = os.path.join(HERE, "ro_cpu_port.c")
PORT_LIB = os.path.join(HERE, "librtw_cpu_port.so")  # portable x86-64-v3 build (oracle/Makefile)
PORT_FLAGS = ["-O3", "-march=native", "-std=gnu11", "-fPIC", "-ffp-contract=off", "-fno-fast-math"]


def build_cpu_port(out_path: str, flags=None) -> str:
    """Compile ro_cpu_port.c on THIS host (bench.py: -O3 -march=native, so the
    timed port is tuned for the timing CPU); returns the gcc command line."""
    cmd = ["gcc"] + list(flags or PORT_FLAGS) + ["-shared", "-o", out_path, PORT_SRC, "-lm"]
    subprocess.run(cmd, check=True)
    return " ".join(cmd[:-4] + ["ro_cpu_port.c"])


def cpu_port_lib(path: str | None = None):
    L = C.CDLL(path or PORT_LIB)
    L.rp_render.argtypes = [C.POINTER(Scene), C.POINTER(Camera), C.c_double * 3, C.c_uint32, C.c_uint32,
                            C.c_uint32, C.c_uint32, U64x4, C.c_void_p, C.c_uint32]
    return L


def render_cpu_port(L, scene: Scene, cam: Camera, rng: ZigRandom, width: int, height: int, spp: int,
                    depth: int = 50, bg=COVER_BG, rows: int | None = None) -> np.ndarray:
    """The CPU baseline's performance port of Tier A (ro_cpu_port.c): the same
    image as render_tier_a, bit for bit (rows: only the first `rows` image rows
    of the loop, main.zig:385 — a prefix of the same stream)."""
    out = np.zeros((height, width, 3), np.uint8)
    L.rp_render(C.byref(scene), C.byref(cam), (C.c_double * 3)(*bg), width, height, spp, depth, rng.s,
                out.ctypes.data, height if rows is None else rows)
    return out


# ----------------------------------------------- README image (pin) ----
# The reference's committed README image (RayTracingInOneWeekend.png, 600x400)
# is a render of an EARLIER revision of generateRandomScene: the scene of the
# book's first volume.  These restate that revision with the same Zig RNG
# restatement, so the image pins the restated DefaultPrng stream (Xoshiro256++
# seeded by SplitMix64, Random.float(f64)), the scene builder's draw order and
# Tier A's camera / sphere / material arithmetic (tests/test_readme_image.py).
BOOK1_SKY, BOOK1_NO_TIME = 1, 2  # rtw_oracle.h RO_BOOK1_*
# rtw_oracle.h RO_MUT_*: one hot-path rule mutated (the pin's controls only)
MUT_METAL_SCATTERED, MUT_SCHLICK_EXP, MUT_LAMBERT_NONORM, MUT_DIEL_ALWAYS_DRAW = 0x100, 0x200, 0x400, 0x800


def readme_scene(seed: int = 42, f64=None):
    """generateRandomScene (main.zig:157-221) as the README image has it: the
    draw order of main.zig:177-218 (choose_mat, center.x, center.z, then
    random01 * random01 albedo / metal albedo + fuzz) on a 22x22 grid
    (a, b in [-11, 11)), static spheres (no center1 draw), a grey Lambertian
    ground (0.5) and the three big spheres after the grid.  Returns the scene
    and the DefaultPrng stream positioned after the build (main.zig:300-301:
    the render continues the same stream)."""
    rng = ZigRandom(seed)
    draw = (lambda: f64(rng)) if f64 else rng.f64  # f64: an alternative float conversion (tests' control)
    sph, mats = [], []

    def add(c, r, kind, albedo=(0.0, 0.0, 0.0), fuzz=0.0, ir=0.0):
        mats.append((kind, albedo, fuzz, ir))
        sph.append((c, r, len(mats) - 1))

    add((0.0, -1000.0, 0.0), 1000.0, LAMBERT_SOLID, (0.5, 0.5, 0.5))
    for a in range(-11, 11):
        for b in range(-11, 11):
            choose = draw()
            c = (a + 0.9 * draw(), 0.2, b + 0.9 * draw())
            dx, dy, dz = c[0] - 4.0, c[1] - 0.2, c[2] - 0.0  # center.sub(4, 0.2, 0).norm() (vec.zig:12-18)
            if math.sqrt(dx * dx + dy * dy + dz * dz) <= 0.9:
                continue
            if choose < 0.8:
                a1 = [draw() for _ in range(3)]
                a2 = [draw() for _ in range(3)]
                add(c, 0.2, LAMBERT_SOLID, tuple(x * y for x, y in zip(a1, a2)))
            elif choose < 0.95:
                albedo = tuple(0.5 + draw() * 0.5 for _ in range(3))
                add(c, 0.2, METAL, albedo, 0.0 + draw() * 0.5)
            else:
                add(c, 0.2, DIELECTRIC, ir=1.5)
    add((0.0, 1.0, 0.0), 1.0, DIELECTRIC, ir=1.5)
    add((-4.0, 1.0, 0.0), 1.0, LAMBERT_SOLID, (0.4, 0.2, 0.1))
    add((4.0, 1.0, 0.0), 1.0, METAL, (0.7, 0.6, 0.5), 0.0)
    sc = Scene()
    sc.n_spheres, sc.n_mats = len(sph), len(mats)
    for i, (c, r, m) in enumerate(sph):
        q = sc.spheres[i]
        q.c0[:], q.c1[:], q.radius, q.t0, q.t1, q.moving, q.mat = c, c, r, 0.0, 1.0, 0, m
    for i, (k, albedo, fuzz, ir) in enumerate(mats):
        q = sc.mats[i]
        q.kind, q.fuzz, q.ir = k, fuzz, ir
        q.albedo[:], q.albedo_odd[:] = albedo, albedo
    return sc, rng


def readme_camera(look_from=(12, 2, 3)) -> Camera:
    """Camera.init (main.zig:52-89) of the README image: 3:2, vfov 20,
    aperture 0.1, focus 10, looking at the origin from (12, 2, 3) — fitted
    to the image (the current scene 1 looks from (13, 2, 3))."""
    cam = Camera()
    arr = C.c_double * 3
    lib().ro_camera_init(C.byref(cam), arr(*look_from), arr(0, 0, 0), arr(0, 1, 0), 20.0, 1.5, 0.1, 10.0, 0.0, 1.0)
    return cam


def render_tier_a_ex(scene: Scene, cam: Camera, rng: ZigRandom, width: int, height: int, spp: int,
                     depth: int = 50, flags: int = BOOK1_SKY | BOOK1_NO_TIME, rows: int | None = None, bg=COVER_BG):
    """Tier A with the README revision's differences (flags: gradient sky of the
    book's first volume, no shutter-time draw); `rows` renders only the first
    rows of the loop (j = 0.. : the bottom image rows)."""
    out = np.zeros((height, width, 3), np.uint8)
    st = Stats()
    lib().ro_render_tier_a_ex(C.byref(scene), C.byref(cam), (C.c_double * 3)(*bg), width, height, spp, depth,
                              rng.s, out.ctypes.data, None, C.byref(st), flags, height if rows is None else rows)
    return out, st.as_dict()


def render_pixel_streams(scene: Scene, cam: Camera, width: int, height: int, spp: int, seed: int,
                         flags: int = BOOK1_SKY | BOOK1_NO_TIME, depth: int = 50, bg=COVER_BG,
                         threads: int = 8) -> np.ndarray:
    """The README pin's renderer (ro_render_tier_a_pixel_streams): Tier A's
    arithmetic with one DefaultPrng stream per pixel, so renders with and
    without a mutated rule share their random numbers (common random numbers);
    row bands on `threads` threads.  Returns the linear per-pixel mean (H, W, 3)."""
    from concurrent.futures import ThreadPoolExecutor
    out = np.zeros((height, width, 3), np.float64)
    L = lib()
    bands = [(b * height // threads, (b + 1) * height // threads) for b in range(threads)]

    def run(band):
        L.ro_render_tier_a_pixel_streams(C.byref(scene), C.byref(cam), (C.c_double * 3)(*bg), width, height, spp,
                                         depth, seed, out.ctypes.data, flags, band[0], band[1])
    with ThreadPoolExecutor(threads) as ex:  # (ctypes releases the GIL)
        list(ex.map(run, bands))
    return out / spp


def render_tier_b(scene: Scene, cam: Camera, width: int, height: int, spp: int, depth: int = 50,
                  seed: int = 42, bg=COVER_BG, row_begin: int = 0, row_stride: int = 1,
                  row_count: int | None = None, chunk: int = 0, precision: int = 0,
                  threads: int = 0, want_mean=False):
    """Tier B (the GPU contract) -> (rows, W, 3) uint8 [, mean f32]."""
    if row_count is None:
        row_count = (height - row_begin + row_stride - 1) // row_stride
    p = Params(width, height, spp, depth, seed, (C.c_double * 3)(*bg), row_begin, row_stride,
               row_count, chunk, precision, threads)
    out = np.zeros((row_count, width, 3), np.uint8)
    mean = np.zeros((row_count, width, 3), np.float32) if want_mean else None
    st = Stats()
    lib().ro_render_tier_b(C.byref(scene), C.byref(cam), C.byref(p), out.ctypes.data,
                           mean.ctypes.data if want_mean else None, C.byref(st))
    if want_mean:
        return out, mean, st.as_dict()
    return out, st.as_dict()


def tierb_samples(scene: Scene, cam: Camera, width: int, height: int, y: int, x: int, s0: int, n: int,
                  depth: int = 50, seed: int = 42, bg=COVER_BG, precision: int = 0, trace: bool = False) -> np.ndarray:
    """Diagnostics: Tier-B radiance of samples s0 .. s0+n-1 of pixel (row y,
    top-first; column x) -> (n, 3) f64; trace prints every segment on stderr."""
    p = Params(width, height, max(1, s0 + n), depth, seed, (C.c_double * 3)(*bg), y, 1, 1, 0, precision, 1)
    out = np.zeros((n, 3), np.float64)
    lib().ro_tierb_samples(C.byref(scene), C.byref(cam), C.byref(p), y, x, s0, n, out.ctypes.data, int(trace))
    return out


def write_ppm(path: str, img: np.ndarray):
    h, w, _ = img.shape
    with open(path, "wb") as f:
        f.write(b"P6\n%d %d\n255\n" % (w, h))
        f.write(np.ascontiguousarray(img, np.uint8).tobytes())


# ------------------------------------------------------ general worlds ----
# rtw_world.h: flattened Hittable/Material/Texture/Perlin worlds (scenes 1-7).
RW_SPHERE, RW_MOVING, RW_XY, RW_XZ, RW_YZ = 0, 1, 2, 3, 4
RW_XF_TRANSLATE, RW_XF_ROTATE_Y = 0, 1
RW_TEX_SOLID, RW_TEX_CHECKER, RW_TEX_NOISE, RW_TEX_IMAGE = 0, 1, 2, 3
RW_LAMBERT, RW_METAL, RW_DIELECTRIC, RW_LIGHT = 0, 1, 2, 3


class WPrim(C.Structure):
    _fields_ = [("kind", C.c_uint32), ("mat", C.c_uint32), ("xform", C.c_int32), ("pad", C.c_uint32),
                ("a", C.c_double * 9)]


class WXform(C.Structure):
    _fields_ = [("n", C.c_uint32), ("op", C.c_uint32 * 4), ("v", (C.c_double * 3) * 4)]


class WTexture(C.Structure):
    _fields_ = [("kind", C.c_uint32), ("perlin", C.c_uint32), ("image", C.c_uint32), ("pad", C.c_uint32),
                ("color", C.c_double * 3), ("odd", C.c_double * 3), ("even", C.c_double * 3),
                ("scale", C.c_double)]


class WMaterial(C.Structure):
    _fields_ = [("kind", C.c_uint32), ("tex", C.c_uint32), ("albedo", C.c_double * 3), ("fuzz", C.c_double),
                ("ir", C.c_double)]


class WPerlin(C.Structure):
    _fields_ = [("ranvec", (C.c_double * 3) * 256), ("perm", (C.c_uint32 * 256) * 3)]


class WImage(C.Structure):
    _fields_ = [("width", C.c_uint32), ("height", C.c_uint32), ("rgba", C.c_void_p)]


class World(C.Structure):
    _fields_ = [("n_prims", C.c_uint32), ("n_xforms", C.c_uint32), ("n_textures", C.c_uint32),
                ("n_mats", C.c_uint32), ("n_perlins", C.c_uint32), ("n_images", C.c_uint32),
                ("prims", C.POINTER(WPrim)), ("xforms", C.POINTER(WXform)), ("textures", C.POINTER(WTexture)),
                ("mats", C.POINTER(WMaterial)), ("perlins", C.POINTER(WPerlin)), ("images", C.POINTER(WImage)),
                ("look_from", C.c_double * 3), ("look_at", C.c_double * 3), ("vfov", C.c_double),
                ("aperture", C.c_double), ("aspect", C.c_double), ("background", C.c_double * 3),
                ("width", C.c_uint32), ("height", C.c_uint32), ("spp", C.c_uint32)]


def _world_lib():
    L = lib()
    if getattr(L, "_world_ready", False):
        return L
    P = C.POINTER
    L.rw_scene.restype = P(World)
    L.rw_scene.argtypes = [C.c_uint32, U64x4, P(WImage)]
    L.rw_world_free.argtypes = [P(World)]
    L.rw_int_range_less_than_u64.restype = C.c_uint64
    L.rw_int_range_less_than_u64.argtypes = [U64x4, C.c_uint64, C.c_uint64]
    L.rw_perlin_noise.restype = C.c_double
    L.rw_perlin_noise.argtypes = [P(WPerlin), C.c_double * 3]
    L.rw_perlin_turb.restype = C.c_double
    L.rw_perlin_turb.argtypes = [P(WPerlin), C.c_double * 3, C.c_uint32]
    L.rw_texture_value.argtypes = [P(World), C.c_uint32, C.c_double, C.c_double, C.c_double * 3, C.c_double * 3]
    L.rw_sphere_uv.argtypes = [C.c_double * 3, P(C.c_double), P(C.c_double)]
    for n in ("rw_sin", "rw_cos", "rw_acos"):
        getattr(L, n).restype = C.c_double
        getattr(L, n).argtypes = [C.c_double]
    L.rw_atan2.restype = C.c_double
    L.rw_atan2.argtypes = [C.c_double, C.c_double]
    L.rw_hit.restype = C.c_int
    L.rw_hit.argtypes = [P(World), C.c_double * 3, C.c_double * 3, C.c_double, C.c_double, C.c_double,
                         P(C.c_double), C.c_double * 3, C.c_double * 3, C.c_double * 2, P(C.c_int)]
    L.rw_render_tier_a.argtypes = [P(World), P(Camera), C.c_double * 3, C.c_uint32, C.c_uint32, C.c_uint32,
                                   C.c_uint32, U64x4, C.c_void_p, C.c_void_p, P(Stats)]
    L.rw_render_tier_b.argtypes = [P(World), P(Camera), P(Params), C.c_void_p, C.c_void_p, P(Stats)]
    L._world_ready = True
    return L


class OracleWorld:
    """A world built by the oracle's scene builders (rw_scene).  Keeps the
    image buffer alive; frees the C world on close/GC."""

    def __init__(self, scene_id: int, seed: int = 42, image: np.ndarray | None = None,
                 rng: "ZigRandom | None" = None):
        L = _world_lib()
        self.rng = rng if rng is not None else ZigRandom(seed)
        self._img = None
        wi = None
        if image is not None:
            self._img = np.ascontiguousarray(image, np.uint8)
            h, w, _ = self._img.shape
            wi = WImage(w, h, self._img.ctypes.data)
        self.ptr = L.rw_scene(scene_id, self.rng.s, C.byref(wi) if wi is not None else None)
        if not self.ptr:
            raise ValueError(f"unknown scene {scene_id}")
        self.w = self.ptr.contents
        self.scene_id = scene_id

    def close(self):
        if getattr(self, "ptr", None):
            _world_lib().rw_world_free(self.ptr)
            self.ptr = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def camera(self, aspect: float | None = None) -> Camera:
        """Camera.init with the scene's settings (main.zig:316-376)."""
        cam = Camera()
        arr = C.c_double * 3
        w = self.w
        lib().ro_camera_init(C.byref(cam), arr(*w.look_from), arr(*w.look_at), arr(0, 1, 0), w.vfov,
                             aspect if aspect is not None else w.aspect, w.aperture, 10.0, 0.0, 1.0)
        return cam

    @property
    def background(self):
        return tuple(self.w.background)

    def table(self) -> dict:
        """Plain-python dump (compared with the product's scene builders)."""
        w = self.w
        prims = [{"kind": p.kind, "mat": p.mat, "xform": p.xform, "a": list(p.a)}
                 for p in (w.prims[i] for i in range(w.n_prims))]
        xfs = [{"n": x.n, "op": list(x.op)[:x.n], "v": [list(x.v[k]) for k in range(x.n)]}
               for x in (w.xforms[i] for i in range(w.n_xforms))]
        texs = [{"kind": t.kind, "perlin": t.perlin, "image": t.image, "color": list(t.color), "odd": list(t.odd),
                 "even": list(t.even), "scale": t.scale} for t in (w.textures[i] for i in range(w.n_textures))]
        mats = [{"kind": m.kind, "tex": m.tex, "albedo": list(m.albedo), "fuzz": m.fuzz, "ir": m.ir}
                for m in (w.mats[i] for i in range(w.n_mats))]
        perl = [{"ranvec": [list(p.ranvec[k]) for k in range(256)], "perm": [list(p.perm[a]) for a in range(3)]}
                for p in (w.perlins[i] for i in range(w.n_perlins))]
        return {"prims": prims, "xforms": xfs, "textures": texs, "materials": mats, "perlins": perl,
                "settings": {"look_from": list(w.look_from), "look_at": list(w.look_at), "vfov": w.vfov,
                             "aperture": w.aperture, "aspect": w.aspect, "background": list(w.background),
                             "width": w.width, "height": w.height, "spp": w.spp}}

    def render_tier_a(self, cam: Camera, width: int, height: int, spp: int, depth: int = 50, bg=None):
        """Tier A over this world, continuing self.rng (the reference's stream)."""
        out = np.zeros((height, width, 3), np.uint8)
        st = Stats()
        _world_lib().rw_render_tier_a(self.ptr, C.byref(cam), (C.c_double * 3)(*(bg or self.background)), width,
                                      height, spp, depth, self.rng.s, out.ctypes.data, None, C.byref(st))
        return out, st.as_dict()

    def render_tier_b(self, cam: Camera, width: int, height: int, spp: int, depth: int = 50, seed: int = 42,
                      bg=None, row_begin: int = 0, row_stride: int = 1, row_count: int | None = None,
                      chunk: int = 0, threads: int = 0, want_mean=False):
        if row_count is None:
            row_count = (height - row_begin + row_stride - 1) // row_stride
        p = Params(width, height, spp, depth, seed, (C.c_double * 3)(*(bg or self.background)), row_begin,
                   row_stride, row_count, chunk, 0, threads)
        out = np.zeros((row_count, width, 3), np.uint8)
        mean = np.zeros((row_count, width, 3), np.float32) if want_mean else None
        st = Stats()
        _world_lib().rw_render_tier_b(self.ptr, C.byref(cam), C.byref(p), out.ctypes.data,
                                      mean.ctypes.data if want_mean else None, C.byref(st))
        return (out, mean, st.as_dict()) if want_mean else (out, st.as_dict())

    def hit(self, o, d, time=0.0, t_min=0.001, t_max=float("inf")):
        arr = C.c_double * 3
        t = C.c_double()
        p, n, uv, fr = arr(), arr(), (C.c_double * 2)(), C.c_int()
        k = _world_lib().rw_hit(self.ptr, arr(*o), arr(*d), time, t_min, t_max, C.byref(t), p, n, uv, C.byref(fr))
        if k < 0:
            return None
        return {"prim": k, "t": t.value, "p": list(p), "normal": list(n), "uv": list(uv), "front": bool(fr.value)}


def libm(name: str):
    """The Tier-B transcendental (ro_libm.h) as a Python callable."""
    return getattr(_world_lib(), "rw_" + name)


class TableWorld(OracleWorld):
    """An oracle world built from plain tables (e.g. a product rtw_world_desc
    read back through ctypes) instead of rw_scene: prims / xforms / textures /
    materials / perlins as lists of the WPrim/WXform/... field dicts, images
    as (H, W, 4) uint8 arrays."""

    def __init__(self, prims, xforms=(), textures=(), materials=(), perlins=(), images=(), background=(0, 0, 0)):
        _world_lib()
        self.rng = ZigRandom(0)
        self.ptr = None
        self.scene_id = 0
        self._keep = []

        def arr(typ, items, fill):
            a = (typ * max(1, len(items)))()
            for i, it in enumerate(items):
                fill(a[i], it)
            self._keep.append(a)
            return C.cast(a, C.POINTER(typ))

        def f_prim(d, p):
            d.kind, d.mat, d.xform = p["kind"], p["mat"], p["xform"]
            d.a[:] = list(p["a"]) + [0.0] * (9 - len(p["a"]))

        def f_xf(d, x):
            d.n = x["n"]
            for k in range(x["n"]):
                d.op[k] = x["op"][k]
                d.v[k][:] = x["v"][k]

        def f_tex(d, t):
            d.kind, d.perlin, d.image = t["kind"], t.get("perlin", 0), t.get("image", 0)
            d.color[:], d.odd[:], d.even[:] = t.get("color", (0, 0, 0)), t.get("odd", (0, 0, 0)), t.get("even", (0, 0, 0))
            d.scale = t.get("scale", 0.0)

        def f_mat(d, m):
            d.kind, d.tex = m["kind"], m.get("tex", 0)
            d.albedo[:] = m.get("albedo", (0, 0, 0))
            d.fuzz, d.ir = m.get("fuzz", 0.0), m.get("ir", 0.0)

        def f_perlin(d, p):
            for k in range(256):
                d.ranvec[k][:] = p["ranvec"][k]
            for a in range(3):
                d.perm[a][:] = p["perm"][a]

        imgs = [np.ascontiguousarray(im, np.uint8) for im in images]
        self._keep.extend(imgs)

        def f_img(d, im):
            d.width, d.height, d.rgba = im.shape[1], im.shape[0], im.ctypes.data

        w = World()
        w.n_prims, w.n_xforms, w.n_textures = len(prims), len(xforms), len(textures)
        w.n_mats, w.n_perlins, w.n_images = len(materials), len(perlins), len(imgs)
        w.prims = arr(WPrim, prims, f_prim)
        w.xforms = arr(WXform, xforms, f_xf)
        w.textures = arr(WTexture, textures, f_tex)
        w.mats = arr(WMaterial, materials, f_mat)
        w.perlins = arr(WPerlin, perlins, f_perlin)
        w.images = arr(WImage, imgs, f_img)
        w.background[:] = background
        self.w = w
        self.ptr = C.pointer(w)

    def close(self):
        self.ptr = None
