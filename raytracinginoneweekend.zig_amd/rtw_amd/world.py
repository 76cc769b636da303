"""General worlds through the C ABI (include/rtw_hip.h "general worlds"):
every scene of the reference's main.zig (1 cover, 2 two spheres, 3 two Perlin
spheres, 4 earth, 5 simple light, 6 Cornell box) and BASELINE.json
configs[4] (7: globe + 10k random spheres), rendered by the world kernel
(csrc/rtw_world.hip).  Plain ctypes marshalling; no CPU fallback.

Reference correspondence:
  build_scene     -> generate* scene builders   src/main.zig:123-290 (+ DefaultPrng, :300)
  scene_camera    -> Camera.init with the scene's settings  main.zig:316-376
  load_png        -> Image.fromFilePath (zigimg) of texture.zig:111 (RGBA8, non-interlaced PNG)
  DeviceWorld     -> the world upload + the render loop     main.zig:378-402
"""
from __future__ import annotations

import ctypes as C
import os
import struct
import zlib

import numpy as np

from . import RTW_EINVAL, Camera, Params, RtwError, Timer, _check, camera_init, lib

PRIM_SPHERE, PRIM_MOVING_SPHERE, PRIM_XY_RECT, PRIM_XZ_RECT, PRIM_YZ_RECT = 0, 1, 2, 3, 4
XF_TRANSLATE, XF_ROTATE_Y = 0, 1
TEX_SOLID, TEX_CHECKER, TEX_NOISE, TEX_IMAGE = 0, 1, 2, 3
WMAT_LAMBERT, WMAT_METAL, WMAT_DIELECTRIC, WMAT_LIGHT = 0, 1, 2, 3
WORLD_LINEAR = 1
WORLD_DEBUG_BVH = 2  # rtw_hip.h RTW_WORLD_DEBUG_BVH: the BVH root's children to stderr (diagnostic)
SCENES = {1: "cover", 2: "two_spheres", 3: "two_perlin_spheres", 4: "earth", 5: "simple_light",
          6: "cornell_box", 7: "globe_10k"}


class Prim(C.Structure):
    _fields_ = [("kind", C.c_uint32), ("mat", C.c_uint32), ("xform", C.c_int32), ("reserved", C.c_uint32),
                ("a", C.c_double * 9)]


class Xform(C.Structure):
    _fields_ = [("n", C.c_uint32), ("op", C.c_uint32 * 4), ("v", (C.c_double * 3) * 4)]


class Texture(C.Structure):
    _fields_ = [("kind", C.c_uint32), ("perlin", C.c_uint32), ("image", C.c_uint32), ("reserved", C.c_uint32),
                ("color", C.c_double * 3), ("odd", C.c_double * 3), ("even", C.c_double * 3),
                ("scale", C.c_double)]


class WMaterial(C.Structure):
    _fields_ = [("kind", C.c_uint32), ("tex", C.c_uint32), ("albedo", C.c_double * 3), ("fuzz", C.c_double),
                ("ir", C.c_double)]


class Perlin(C.Structure):
    _fields_ = [("ranvec", (C.c_double * 3) * 256), ("perm", (C.c_uint32 * 256) * 3)]


class Image(C.Structure):
    _fields_ = [("width", C.c_uint32), ("height", C.c_uint32), ("rgba", C.c_void_p)]


class WorldDesc(C.Structure):
    _fields_ = [("prims", C.POINTER(Prim)), ("n_prims", C.c_uint32),
                ("xforms", C.POINTER(Xform)), ("n_xforms", C.c_uint32),
                ("textures", C.POINTER(Texture)), ("n_textures", C.c_uint32),
                ("mats", C.POINTER(WMaterial)), ("n_mats", C.c_uint32),
                ("perlins", C.POINTER(Perlin)), ("n_perlins", C.c_uint32),
                ("images", C.POINTER(Image)), ("n_images", C.c_uint32)]


class SceneSettings(C.Structure):
    _fields_ = [("look_from", C.c_double * 3), ("look_at", C.c_double * 3), ("vfov", C.c_double),
                ("aperture", C.c_double), ("aspect", C.c_double), ("background", C.c_double * 3),
                ("width", C.c_uint32), ("height", C.c_uint32), ("spp", C.c_uint32), ("reserved", C.c_uint32)]


def _wlib():
    L = lib()
    if getattr(L, "_world_ready", False):
        return L
    P = C.POINTER
    L.rtw_build_scene.argtypes = [C.c_uint32, C.c_uint64, P(Image), P(C.c_void_p)]
    L.rtw_built_scene_desc.argtypes = [C.c_void_p, P(WorldDesc), P(SceneSettings), C.c_uint64 * 4]
    L.rtw_built_scene_free.argtypes = [C.c_void_p]
    L.rtw_world_create.argtypes = [P(WorldDesc), C.c_uint32, P(C.c_void_p)]
    L.rtw_world_destroy.argtypes = [C.c_void_p]
    L.rtw_world_bvh_info.argtypes = [C.c_void_p, C.c_uint32 * 4]
    L.rtw_world_workspace_bytes.restype = C.c_size_t
    L.rtw_world_workspace_bytes.argtypes = [C.c_void_p, P(Params)]
    L.rtw_world_render_device.argtypes = [C.c_void_p, P(Camera), P(Params), C.c_void_p, C.c_size_t, C.c_void_p,
                                          C.c_void_p, C.c_void_p, C.c_void_p]
    L.rtw_world_render.argtypes = [P(Camera), P(WorldDesc), P(Params), C.c_void_p, C.c_void_p]
    L.rtw_world_render_counts.argtypes = [C.c_void_p, P(Camera), P(Params), C.c_void_p, C.c_size_t,
                                          C.c_uint64 * 4]
    L.rtw_world_render_counts_ex.argtypes = [C.c_void_p, P(Camera), P(Params), C.c_void_p, C.c_size_t,
                                             C.c_uint64 * 8]
    if hasattr(L, "rtw_world_launch_info"):  # (A/B timing may load an older build without it)
        L.rtw_world_launch_info.argtypes = [C.c_void_p, P(Params), C.c_uint32 * 6]
    L._world_ready = True
    return L


# ------------------------------------------------------------ images ----
def load_png(path: str) -> np.ndarray:
    """Decode an 8-bit, non-interlaced PNG to (H, W, 4) uint8 RGBA (grey,
    grey+alpha, RGB, palette are expanded; RGBA is taken as is, which is the
    only layout texture.zig:133-140's 4-byte stride reads correctly)."""
    data = open(path, "rb").read()
    if data[:8] != b"\x89PNG\r\n\x1a\n":
        raise ValueError(f"{path}: not a PNG")
    i, idat, plte, trns, hdr = 8, [], None, None, None
    while i < len(data):
        n = struct.unpack(">I", data[i:i + 4])[0]
        typ, body = data[i + 4:i + 8], data[i + 8:i + 8 + n]
        if typ == b"IHDR":
            hdr = struct.unpack(">IIBBBBB", body)
        elif typ == b"PLTE":
            plte = np.frombuffer(body, np.uint8).reshape(-1, 3)
        elif typ == b"tRNS":
            trns = np.frombuffer(body, np.uint8)
        elif typ == b"IDAT":
            idat.append(body)
        elif typ == b"IEND":
            break
        i += 12 + n
    w, h, depth, ctype, _, _, interlace = hdr
    if depth != 8 or interlace != 0:
        raise ValueError(f"{path}: only 8-bit non-interlaced PNGs are supported")
    ch = {0: 1, 2: 3, 3: 1, 4: 2, 6: 4}[ctype]
    raw = np.frombuffer(zlib.decompress(b"".join(idat)), np.uint8)
    stride = w * ch
    out = np.zeros((h, stride), np.int32)
    prev = np.zeros(stride, np.int32)
    for y in range(h):
        f = raw[y * (stride + 1)]
        line = raw[y * (stride + 1) + 1:(y + 1) * (stride + 1)].astype(np.int32)
        if f == 0:
            cur = line
        elif f == 2:
            cur = (line + prev) & 255
        else:  # Sub / Average / Paeth need the running left neighbour
            cur = np.zeros(stride, np.int32)
            for x in range(stride):
                a = cur[x - ch] if x >= ch else 0
                b = prev[x]
                c = prev[x - ch] if x >= ch else 0
                if f == 1:
                    pred = a
                elif f == 3:
                    pred = (a + b) >> 1
                else:
                    p = a + b - c
                    pa, pb, pc = abs(p - a), abs(p - b), abs(p - c)
                    pred = a if pa <= pb and pa <= pc else (b if pb <= pc else c)
                cur[x] = (line[x] + pred) & 255
        out[y] = cur
        prev = cur
    px = out.astype(np.uint8).reshape(h, w, ch)
    if ctype == 6:
        return np.ascontiguousarray(px)
    rgba = np.full((h, w, 4), 255, np.uint8)
    if ctype == 2:
        rgba[..., :3] = px
    elif ctype == 0:
        rgba[..., :3] = px[..., :1]
    elif ctype == 4:
        rgba[..., :3] = px[..., :1]
        rgba[..., 3] = px[..., 1]
    else:
        rgba[..., :3] = plte[px[..., 0]]
        if trns is not None:
            a = np.full(len(plte), 255, np.uint8)
            a[:len(trns)] = trns
            rgba[..., 3] = a[px[..., 0]]
    return rgba


EARTH_PNG = os.path.join(os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))),
                         "assets", "sekaichizu.png")


def earth_map(path: str | None = None) -> np.ndarray:
    """The reference's globe texture (assets/sekaichizu.png, 500 x 282 RGBA8,
    ocean = alpha 0; loaded by ImageTexture.init, texture.zig:107-119, for
    main.zig:226 and BASELINE configs[4]).  The repo carries the reference's
    asset file unchanged, with the reference's own note (assets/LICENSE), so
    the GPU box renders the real texture; RTW_EARTH_MAP names another PNG.
    Decoded by the library's PNG reader."""
    return load_png(path or os.environ.get("RTW_EARTH_MAP") or EARTH_PNG)


def synthetic_world_map(width: int = 500, height: int = 282) -> np.ndarray:
    """A deterministic map of the globe asset's size and format (500 x 282
    RGBA8, ocean = alpha 0): smooth 'continents' from a few sinusoids.  Used
    only by tests that want a texture independent of the asset file."""
    y, x = np.mgrid[0:height, 0:width].astype(np.float64)
    u, v = x / width * 2 * np.pi, y / height * np.pi
    f = np.sin(3 * u) * np.sin(2 * v) + 0.6 * np.sin(5 * u + 1.3) * np.cos(3 * v) + 0.4 * np.cos(7 * u - 2 * v)
    land = f > 0.35
    img = np.zeros((height, width, 4), np.uint8)
    img[..., 0] = np.clip(80 + 120 * np.sin(u + v) ** 2, 0, 255).astype(np.uint8)
    img[..., 1] = np.clip(150 + 80 * np.cos(2 * u) * np.sin(v), 0, 255).astype(np.uint8)
    img[..., 2] = np.clip(60 + 40 * np.sin(3 * v), 0, 255).astype(np.uint8)
    img[..., 3] = np.where(land, 255, 0).astype(np.uint8)
    return img


# ------------------------------------------------------------ scenes ----
class BuiltScene:
    """A scene built by the library's builders (rtw_build_scene): desc points
    into library-owned arrays until close()."""

    def __init__(self, scene_id: int, seed: int = 42, image: np.ndarray | None = None):
        L = _wlib()
        self._img = None
        img = None
        if image is not None:
            self._img = np.ascontiguousarray(image, np.uint8)
            img = Image(self._img.shape[1], self._img.shape[0], self._img.ctypes.data)
        self.h = C.c_void_p()
        _check(L.rtw_build_scene(scene_id, seed, C.byref(img) if img is not None else None, C.byref(self.h)))
        self.desc = WorldDesc()
        self.settings = SceneSettings()
        st = (C.c_uint64 * 4)()
        _check(L.rtw_built_scene_desc(self.h, C.byref(self.desc), C.byref(self.settings), st))
        self.rng_state = [int(x) for x in st]
        self.scene_id = scene_id

    def camera(self, aspect: float | None = None) -> Camera:
        s = self.settings
        return camera_init(tuple(s.look_from), tuple(s.look_at), (0, 1, 0), s.vfov,
                           aspect if aspect is not None else s.aspect, s.aperture, 10.0, 0.0, 1.0)

    @property
    def background(self):
        return tuple(self.settings.background)

    def table(self) -> dict:
        """Resolved plain-python dump (materials with their texture values
        inlined), comparable with oracle.OracleWorld.table()."""
        d = self.desc
        prims = [{"kind": p.kind, "mat": p.mat, "xform": p.xform, "a": list(p.a)}
                 for p in (d.prims[i] for i in range(d.n_prims))]
        xfs = [{"n": x.n, "op": list(x.op)[:x.n], "v": [list(x.v[k]) for k in range(x.n)]}
               for x in (d.xforms[i] for i in range(d.n_xforms))]
        texs = [{"kind": t.kind, "perlin": t.perlin, "image": t.image, "color": list(t.color), "odd": list(t.odd),
                 "even": list(t.even), "scale": t.scale} for t in (d.textures[i] for i in range(d.n_textures))]
        mats = [{"kind": m.kind, "tex": m.tex, "albedo": list(m.albedo), "fuzz": m.fuzz, "ir": m.ir}
                for m in (d.mats[i] for i in range(d.n_mats))]
        perl = [{"ranvec": [list(p.ranvec[k]) for k in range(256)], "perm": [list(p.perm[a]) for a in range(3)]}
                for p in (d.perlins[i] for i in range(d.n_perlins))]
        return {"prims": prims, "xforms": xfs, "textures": texs, "materials": mats, "perlins": perl}

    def close(self):
        if self.h:
            _wlib().rtw_built_scene_free(self.h)
            self.h = C.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def render_world(cam: Camera, desc: WorldDesc, params: Params, want_mean=False):
    """Synchronous host-buffer render of a world (rtw_world_render)."""
    rgb = np.zeros((params.row_count, params.width, 3), np.uint8)
    mean = np.zeros((params.row_count, params.width, 3), np.float32) if want_mean else None
    _check(_wlib().rtw_world_render(C.byref(cam), C.byref(desc), C.byref(params), rgb.ctypes.data,
                                    mean.ctypes.data if want_mean else None))
    return (rgb, mean) if want_mean else rgb


TRAVERSAL_NAMES = {1: "union", 2: "lane", 3: "linear"}  # rtw_world_traversal (rtw_hip.h)


class DeviceWorld:
    """A world resident in HBM of the current device (rtw_world_create)."""

    def __init__(self, desc: WorldDesc, linear: bool = False, debug_bvh: bool = False):
        self.h = C.c_void_p()
        flags = (WORLD_LINEAR if linear else 0) | (WORLD_DEBUG_BVH if debug_bvh else 0)
        _check(_wlib().rtw_world_create(C.byref(desc), flags, C.byref(self.h)))

    def bvh_info(self) -> dict:
        info = (C.c_uint32 * 4)()
        _check(_wlib().rtw_world_bvh_info(self.h, info))
        return {"nodes": info[0], "leaves": info[1], "max_depth": info[2], "max_leaf": info[3]}

    def workspace_bytes(self, params: Params) -> int:
        """Device workspace of a render of this world (rtw_world_workspace_bytes:
        the common region + the tail dealing's per-lane rings)."""
        n = _wlib().rtw_world_workspace_bytes(self.h, C.byref(params))
        if n == 0:
            raise RtwError(RTW_EINVAL, lib().rtw_last_error().decode())
        return n

    def render_async(self, cam: Camera, params: Params, workspace_ptr: int, workspace_bytes_: int, rgb_ptr: int,
                     mean_ptr: int | None = None, stream: int | None = None, timer: Timer | None = None):
        _check(_wlib().rtw_world_render_device(self.h, C.byref(cam), C.byref(params), C.c_void_p(workspace_ptr),
                                               workspace_bytes_, C.c_void_p(rgb_ptr),
                                               C.c_void_p(mean_ptr) if mean_ptr else None,
                                               C.c_void_p(stream) if stream else None,
                                               timer.h if timer is not None else None))

    def launch_info(self, params: Params) -> dict:
        """rtw_world_launch_info: how a render with these params launches on the
        current device — the traversal that runs (after AUTO and the world's
        limits), kernel feature set, register budget, workgroups per CU, grid, LDS."""
        out = (C.c_uint32 * 6)()
        _check(_wlib().rtw_world_launch_info(self.h, C.byref(params), out))
        return {"traversal": TRAVERSAL_NAMES.get(int(out[0]), str(out[0])), "feature_set": int(out[1]),
                "waves": int(out[2]), "blocks_per_cu": int(out[3]), "grid": int(out[4]), "lds_bytes": int(out[5])}

    def counts(self, cam: Camera, params: Params, workspace_ptr: int, workspace_bytes_: int) -> dict:
        """rtw_world_render_counts_ex: the counts, the persistent kernel's wave
        iterations and whether tail dealing ran (the workspace held the rings),
        plus the traversal that ran (rtw_world_launch_info)."""
        out = (C.c_uint64 * 8)()
        _check(_wlib().rtw_world_render_counts_ex(self.h, C.byref(cam), C.byref(params),
                                                  C.c_void_p(workspace_ptr), workspace_bytes_, out))
        return {"samples": int(out[0]), "segments": int(out[1]), "node_visits": int(out[2]),
                "prim_tests": int(out[3]), "wave_iters": int(out[4]), "tail_dealing": bool(out[5]),
                "lane_interior_iters": int(out[6]), "lane_leaf_iters": int(out[7]),
                "traversal": self.launch_info(params)["traversal"] if hasattr(_wlib(), "rtw_world_launch_info")
                else None}

    def close(self):
        if self.h:
            _wlib().rtw_world_destroy(self.h)
            self.h = C.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


__all__ = ["BuiltScene", "DeviceWorld", "render_world", "load_png", "earth_map", "synthetic_world_map", "RtwError", "SCENES"]
