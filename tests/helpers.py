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
