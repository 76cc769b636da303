"""Independent pure-Python restatement of the reference (Tier A) — ORACLE,
test infrastructure only, for SMALL images (it is ~10^4x slower than C).

Written directly from the Zig sources (not from rtw_oracle.c) so that the two
restatements cross-check each other bit for bit (tests/test_oracle_tier_a.py).
Python floats are IEEE f64 and every expression below is evaluated in the
same order as the Zig expression it cites, so results are exact restatements.
Transcendentals (tan, sin, atan2, acos) come from the platform libm, as in
the C oracle; Zig links its own musl-derived versions — a <=1-ulp source of
unpinned difference, documented in DESIGN.md.
"""
from __future__ import annotations

import math

M64 = (1 << 64) - 1


# ---------------------------------------------- Zig std.Random (0.14) ----
class SplitMix64:  # std/Random/SplitMix64.zig
    def __init__(self, seed):
        self.s = seed & M64

    def next(self):
        self.s = (self.s + 0x9E3779B97F4A7C15) & M64
        z = self.s
        z = ((z ^ (z >> 30)) * 0xBF58476D1CE4E5B9) & M64
        z = ((z ^ (z >> 27)) * 0x94D049BB133111EB) & M64
        return z ^ (z >> 31)


def tb_mix(z):
    """Tier-B draw word of a Weyl state (the GPU contract, not the reference:
    oracle/rtw_oracle.c ro_tb_mix): four Feistel half-rounds on the 32-bit
    words, each a 32x32 -> 64-bit product and one xor."""
    hi, lo = (z >> 32) & 0xFFFFFFFF, z & 0xFFFFFFFF
    for i, m in enumerate((0xD2511F53, 0xCD9E8D57, 0x9E3779B1, 0x85EBCA6B)):
        if i % 2 == 0:
            t = hi * m
            lo ^= t >> 32
            hi = t & 0xFFFFFFFF
        else:
            t = lo * m
            hi ^= t >> 32
            lo = t & 0xFFFFFFFF
    return (hi << 32) | lo


def _rotl(x, k):
    return ((x << k) | (x >> (64 - k))) & M64


class Xoshiro256:  # std/Random/Xoshiro256.zig
    def __init__(self, seed):
        g = SplitMix64(seed)
        self.s = [g.next(), g.next(), g.next(), g.next()]

    def next(self):
        s = self.s
        r = (_rotl((s[0] + s[3]) & M64, 23) + s[0]) & M64
        t = (s[1] << 17) & M64
        s[2] ^= s[0]
        s[3] ^= s[1]
        s[1] ^= s[2]
        s[0] ^= s[3]
        s[2] ^= t
        s[3] = _rotl(s[3], 45)
        return r

    def float64(self):  # std/Random.zig float(f64)
        rnd = self.next()
        lz = 64 - rnd.bit_length()
        if lz >= 12:
            lz = 12
            while True:
                addl = 64 - self.next().bit_length()
                lz += addl
                if addl != 64:
                    break
                if lz >= 1022:
                    lz = 1022
                    break
        bits = ((1022 - lz) << 52) | (rnd & ((1 << 52) - 1))
        return _bits_to_f64(bits)


def _bits_to_f64(bits):
    import struct
    return struct.unpack("<d", struct.pack("<Q", bits))[0]


def zig_pow(x, y):
    """std/math/pow.zig for finite x >= 0 and a positive integral y."""
    if y == 0 or x == 1:
        return 1.0
    if y == 1:
        return x
    if x == 0:
        return x if (y % 2 == 1) else 0.0
    yi = math.floor(abs(y))
    a1, ae = 1.0, 0
    x1, xe = math.frexp(x)
    i = int(yi)
    while i != 0:
        if xe < -(1 << 12) or (1 << 12) < xe:
            ae += xe
            break
        if i & 1 == 1:
            a1 *= x1
            ae += xe
        x1 *= x1
        xe <<= 1
        if x1 < 0.5:
            x1 += x1
            xe -= 1
        i >>= 1
    return math.ldexp(a1, ae)


# ------------------------------------------------------------- vec.zig ----
def add(u, v): return (u[0] + v[0], u[1] + v[1], u[2] + v[2])
def sub(u, v): return (u[0] - v[0], u[1] - v[1], u[2] - v[2])
def mul(v, t): return (v[0] * t, v[1] * t, v[2] * t)
def mulv(u, v): return (u[0] * v[0], u[1] * v[1], u[2] * v[2])
def div(v, t): return (v[0] / t, v[1] / t, v[2] / t)
def dot(u, v): return u[0] * v[0] + u[1] * v[1] + u[2] * v[2]
def norm2(v): return v[0] * v[0] + v[1] * v[1] + v[2] * v[2]
def norm(v): return math.sqrt(norm2(v))
def cross(u, v): return (u[1] * v[2] - u[2] * v[1], u[2] * v[0] - u[0] * v[2], u[0] * v[1] - u[1] * v[0])


def normalized(v):
    n = norm(v)
    return v if n == 0.0 else div(v, n)


def near_zero(v):
    e = 1e-8
    return abs(v[0]) < e and abs(v[1]) < e and abs(v[2]) < e


# ------------------------------------------------------------ rand.zig ----
def real(rng, lo, hi): return lo + rng.float64() * (hi - lo)


def in_unit_sphere(rng):
    while True:
        p = (real(rng, -1.0, 1.0), real(rng, -1.0, 1.0), real(rng, -1.0, 1.0))
        if norm(p) >= 1:
            continue
        return p


def in_unit_disk(rng):
    while True:
        p = (real(rng, -1.0, 1.0), real(rng, -1.0, 1.0), 0.0)
        if norm(p) >= 1:
            continue
        return p


# ---------------------------------------------------- scene (main.zig) ----
# materials: ("lambert", albedo) | ("checker", odd, even) | ("metal", albedo, fuzz) | ("glass", ir)
# objects: ("sphere", center, radius, mat) | ("moving", c0, c1, t0, t1, radius, mat)
def generate_random_scene(rng):  # main.zig:157-221
    objs = [("sphere", (0.0, -1000.0, 0.0), 1000.0, ("checker", (0.2, 0.3, 0.1), (0.9, 0.9, 0.9))),
            ("sphere", (0.0, 1.0, 0.0), 1.0, ("glass", 1.5)),
            ("sphere", (-4.0, 1.0, 0.0), 1.0, ("lambert", (0.4, 0.2, 0.1))),
            ("sphere", (4.0, 1.0, 0.0), 1.0, ("metal", (0.7, 0.6, 0.5), 0.0))]
    for a in range(-3, 3):
        for b in range(-3, 3):
            choose = rng.float64()
            cx = float(a) + 0.9 * rng.float64()
            cz = float(b) + 0.9 * rng.float64()
            center = (cx, 0.2, cz)
            if norm(sub(center, (4.0, 0.2, 0.0))) <= 0.9:
                continue
            if choose < 0.8:
                r1 = (rng.float64(), rng.float64(), rng.float64())
                r2 = (rng.float64(), rng.float64(), rng.float64())
                albedo = mulv(r1, r2)
                c1 = add(center, (0.0, real(rng, 0.0, 0.5), 0.0))
                objs.append(("moving", center, c1, 0.0, 1.0, 0.2, ("lambert", albedo)))
            elif choose < 0.95:
                albedo = (real(rng, 0.5, 1.0), real(rng, 0.5, 1.0), real(rng, 0.5, 1.0))
                fuzz = real(rng, 0.0, 0.5)
                objs.append(("sphere", center, 0.2, ("metal", albedo, fuzz)))
            else:
                objs.append(("sphere", center, 0.2, ("glass", 1.5)))
    return objs


class Camera:  # main.zig:40-101
    def __init__(self, look_from, look_at, vup, vfov, aspect, aperture, focus, t0, t1):
        theta = vfov * math.pi / 180.0
        h = math.tan(theta / 2)
        vh = 2.0 * h
        vw = aspect * vh
        w = normalized(sub(look_from, look_at))
        u = normalized(cross(vup, w))
        v = cross(w, u)
        self.origin = look_from
        self.horizontal = mul(u, vw * focus)
        self.vertical = mul(v, vh * focus)
        self.llc = sub(sub(sub(self.origin, div(self.horizontal, 2.0)), div(self.vertical, 2.0)), mul(w, focus))
        self.u, self.v, self.w = u, v, w
        self.lens_radius = aperture / 2.0
        self.t0, self.t1 = t0, t1

    def get_ray(self, rng, s, t):
        rd = mul(in_unit_disk(rng), self.lens_radius)
        offset = add(mul(self.u, rd[0]), mul(self.v, rd[1]))
        d = sub(sub(add(add(self.llc, mul(self.horizontal, s)), mul(self.vertical, t)), self.origin), offset)
        return (add(self.origin, offset), d, real(rng, self.t0, self.t1))


# ------------------------------------------------------ hittable.zig ----
def hit_object(obj, ray, t_min, t_max):
    o, d, time = ray
    if obj[0] == "sphere":
        center, radius, mat = obj[1], obj[2], obj[3]
    else:
        c0, c1, t0, t1, radius, mat = obj[1:]
        center = add(c0, mul(sub(c1, c0), (time - t0) / (t1 - t0)))
    oc = sub(o, center)
    a = norm2(d)
    hb = dot(oc, d)
    c = norm2(oc) - radius * radius
    disc = hb * hb - a * c
    if disc < 0.0:
        return None
    sq = math.sqrt(disc)
    root = (-hb - sq) / a
    if root < t_min or t_max < root:
        root = (-hb + sq) / a
        if root < t_min or t_max < root:
            return None
    p = add(o, mul(d, root))
    outward = div(sub(p, center), radius)
    front = dot(outward, d) < 0.0
    normal = outward if front else mul(outward, -1.0)
    return (root, p, normal, front, mat)


def world_hit(objs, ray, t_min, t_max):
    rec = None
    closest = t_max
    for obj in objs:
        r = hit_object(obj, ray, t_min, closest)
        if r is not None:
            closest = r[0]
            rec = r
    return rec


# ------------------------------------------------------ material.zig ----
def reflect(v, n): return sub(v, mul(n, 2 * dot(v, n)))


def refract(uv, n, eta):
    cos_t = min(dot(mul(uv, -1.0), n), 1.0)
    perp = mul(add(uv, mul(n, cos_t)), eta)
    par = mul(n, -math.sqrt(abs(1.0 - norm2(perp))))
    return add(perp, par)


def reflectance(cosine, ref_idx):
    r0 = (1.0 - ref_idx) / (1.0 + ref_idx)
    r1 = r0 * r0
    return r1 + (1.0 - r1) * zig_pow(1.0 - cosine, 5.0)


def scatter(mat, ray, rec, rng):
    o, d, time = ray
    _, p, normal, front, _ = rec
    kind = mat[0]
    if kind in ("lambert", "checker"):
        sd = add(normal, normalized(in_unit_sphere(rng)))
        if near_zero(sd):
            sd = normal
        if kind == "lambert":
            att = mat[1]
        else:
            sines = math.sin(10 * p[0]) * math.sin(10 * p[1]) * math.sin(10 * p[2])
            att = mat[1] if sines < 0 else mat[2]
        return True, att, (p, sd, time)
    if kind == "metal":
        refl = reflect(normalized(d), normal)
        sd = add(refl, mul(in_unit_sphere(rng), mat[2]))
        return dot(refl, normal) > 0.0, mat[1], (p, sd, time)
    ir = mat[1]
    ratio = 1.0 / ir if front else ir
    ud = normalized(d)
    cos_t = min(dot(mul(ud, -1.0), normal), 1.0)
    sin_t = math.sqrt(1.0 - cos_t * cos_t)
    can = ratio * sin_t <= 1.0
    if can and reflectance(cos_t, ratio) < rng.float64():
        nd = refract(ud, normal, ratio)
    else:
        nd = reflect(ud, normal)
    return True, (1.0, 1.0, 1.0), (p, nd, time)


def ray_color(ray, bg, objs, rng, depth):  # main.zig:103-122
    if depth == 0:
        return (0.0, 0.0, 0.0)
    rec = world_hit(objs, ray, 0.001, math.inf)
    if rec is None:
        return bg
    emitted = (0.0, 0.0, 0.0)
    ok, att, scattered = scatter(rec[4], ray, rec, rng)
    if ok:
        return add(emitted, mulv(att, ray_color(scattered, bg, objs, rng, depth - 1)))
    return emitted


def quantize(c, scale):  # main.zig:395-400
    g = math.sqrt(c * scale)
    return int(256.0 * max(0.0, min(g, 0.999)))


def main_cover(width, aspect, spp, depth=50, seed=42):
    """main.zig:295-402 for scene 1; returns rows (top-first) of (r, g, b)."""
    rng = Xoshiro256(seed)
    objs = generate_random_scene(rng)
    bg = (0.70, 0.80, 1.00)
    height = int(math.trunc(float(width) / aspect))
    cam = Camera((13.0, 2.0, 3.0), (0.0, 0.0, 0.0), (0.0, 1.0, 0.0), 20.0, aspect, 0.1, 10.0, 0.0, 1.0)
    img = [[None] * width for _ in range(height)]
    for j in range(height):
        for i in range(width):
            pc = (0.0, 0.0, 0.0)
            for _ in range(spp):
                u = (float(i) + rng.float64()) / (float(width) - 1.0)
                v = (float(j) + rng.float64()) / (float(height) - 1.0)
                pc = add(pc, ray_color(cam.get_ray(rng, u, v), bg, objs, rng, depth))
            scale = 1.0 / float(spp)
            img[height - j - 1][i] = (quantize(pc[0], scale), quantize(pc[1], scale), quantize(pc[2], scale))
    return img, objs
