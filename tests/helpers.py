"""Shared test helpers: product scene -> oracle scene, image diff summaries."""
import numpy as np


def to_oracle_scene(oracle, spheres, mats):
    t = {"spheres": [], "materials": []}
    for s in spheres:
        t["spheres"].append({"c0": list(s.c0), "c1": list(s.c1), "radius": s.radius, "t0": s.t0, "t1": s.t1,
                             "moving": int(s.moving), "mat": int(s.mat)})
    for m in mats:
        t["materials"].append({"kind": int(m.kind), "albedo": list(m.albedo), "albedo_odd": list(m.albedo_odd),
                               "fuzz": m.fuzz, "ir": m.ir})
    return oracle.scene_from_table(t)


def to_oracle_camera(oracle, cam):
    oc = oracle.Camera()
    for n in ("origin", "horizontal", "vertical", "lower_left_corner", "u", "v", "w"):
        getattr(oc, n)[:] = list(getattr(cam, n))
    oc.lens_radius, oc.time0, oc.time1 = cam.lens_radius, cam.time0, cam.time1
    return oc


def diff_stats(a, b):
    d = a.astype(np.int32) - b.astype(np.int32)
    return {
        "max": int(np.abs(d).max()) if d.size else 0,
        "frac_exact": float((d == 0).mean()) if d.size else 1.0,
        "mean": [float(x) for x in d.reshape(-1, 3).mean(axis=0)],
        "rms": float(np.sqrt((d.astype(np.float64) ** 2).mean())) if d.size else 0.0,
    }


def deep_cluster_world(W, n=12000, seed=1):
    """A sphere world whose unconstrained SAH tree is deeper than the per-lane
    walk's 16-entry stack: nested clusters, each holding half
    of the remaining spheres at a third of the previous one's scale (binned SAH
    peels the levels off one by one: depth 24).  Lambertian and metal spheres
    on a thin slab y ~ 0, one solid texture.  Returns (prims, mats, textures)."""
    rng = np.random.default_rng(seed)
    prims, k, scale, c = [], 0, 100.0, np.zeros(3)
    while k < n:
        for _ in range(max(1, (n - k) // 2)):
            p = c + rng.uniform(-scale, scale, 3) * np.array([1.0, 0.02, 1.0])
            r = scale * 0.01
            y = abs(p[1]) + r
            prims.append(dict(kind=W.PRIM_SPHERE, mat=k % 2, xform=-1, a=[p[0], y, p[2], p[0], y, p[2], r, 0, 0]))
            k += 1
        scale /= 3
    tex = [dict(kind=W.TEX_SOLID, color=(0.6, 0.5, 0.4))]
    mats = [dict(kind=W.WMAT_LAMBERT, tex=0), dict(kind=W.WMAT_METAL, albedo=(0.8, 0.8, 0.9), fuzz=0.2)]
    return prims, mats, tex
