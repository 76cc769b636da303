"""Tier A (the reference restated) — C oracle vs independent Python restatement,
and the committed fixtures.  Against the Zig binary itself: parity unpinned
(no toolchain; the reference ships no goldens), see DESIGN.md."""
import json
import os

import numpy as np
import pytest

from conftest import GOLDEN


def read_ppm(path):
    with open(path, "rb") as f:
        data = f.read()
    parts = data.split(b"\n", 3)
    assert parts[0] == b"P6"
    w, h = map(int, parts[1].split())
    return np.frombuffer(parts[3], np.uint8).reshape(h, w, 3)


def test_cover_scene_golden(oracle):
    with open(os.path.join(GOLDEN, "cover_scene_seed42.json")) as f:
        g = json.load(f)
    sc, rng = oracle.cover_scene(42)
    t = oracle.scene_table(sc)
    assert t["spheres"] == g["spheres"]
    assert t["materials"] == g["materials"]
    assert rng.state() == g["rng_state_after"]
    # always 40 spheres; seed 42 -> 26 moving, 8+1 metal, 2+1 glass.
    kinds = [g["materials"][s["mat"]]["kind"] for s in g["spheres"]]
    assert len(g["spheres"]) == 40
    assert sum(s["moving"] for s in g["spheres"]) == 26
    assert kinds.count(oracle.METAL) == 9 and kinds.count(oracle.DIELECTRIC) == 3


def test_python_scene_matches_c(oracle):
    import rtw_oracle_py as P
    sc, _ = oracle.cover_scene(42)
    objs = P.generate_random_scene(P.Xoshiro256(42))
    assert len(objs) == sc.n_spheres
    for i, o in enumerate(objs):
        s = sc.spheres[i]
        assert tuple(s.c0) == (o[1] if o[0] == "sphere" else o[1])
        r = o[2] if o[0] == "sphere" else o[5]
        assert s.radius == r


@pytest.mark.parametrize("w,aspect,spp", [(60, 1.5, 4), (32, 16 / 9, 3)])
def test_tier_a_c_equals_python(oracle, w, aspect, spp):
    import rtw_oracle_py as P
    c, _ = oracle.main_cover(w, aspect, spp)
    p, _ = P.main_cover(w, aspect, spp)
    assert (np.array(p, np.uint8) == c).all()


@pytest.mark.parametrize("name,w,aspect,spp", [("tier_a_60x40_4spp.ppm", 60, 1.5, 4),
                                               ("tier_a_40x22_8spp.ppm", 40, 16 / 9, 8)])
def test_tier_a_fixtures(oracle, name, w, aspect, spp):
    c, _ = oracle.main_cover(w, aspect, spp)
    assert (read_ppm(os.path.join(GOLDEN, name)) == c).all()


def test_tier_a_workload_profile(oracle):
    """SURVEY.md §3.2 probe: ~2.27 segments, ~93 tests, ~12.1 draws per sample (16:9)."""
    _, st = oracle.main_cover(160, 16 / 9, 8)
    seg = st["segments"] / st["samples"]
    assert 2.1 < seg < 2.45
    assert 11.0 < st["draws"] / st["samples"] < 13.5


def test_config0_artifact(oracle):
    """BASELINE configs[0] (400x225x100, the Zig CPU reference to PPM) as the
    oracle's Tier A restatement of the whole main(): the committed digest
    (tests/golden/make_config0.py) is reproduced bit for bit (~3-10 s, 1 core)."""
    import hashlib
    import json
    import os

    from conftest import GOLDEN
    rec = json.load(open(os.path.join(GOLDEN, "config0_tier_a_400x225x100.json")))
    img, st = oracle.main_cover(400, 16 / 9, 100, 50, 42)
    assert img.shape == (225, 400, 3) and st["samples"] == 400 * 225 * 100 == rec["samples"]
    ppm = b"P6\n400 225\n255\n" + img.tobytes()
    assert hashlib.sha256(ppm).hexdigest() == rec["ppm_sha256"]
    assert [round(float(x), 4) for x in img.reshape(-1, 3).mean(0)] == rec["mean_rgb"]


@pytest.mark.parametrize("w,spp,native", [(120, 6, False), (64, 16, True)])
def test_cpu_port_equals_tier_a(oracle, tmp_path, w, spp, native):
    """bench.py's CPU baseline is the performance port ro_cpu_port.c (SIMD
    two-pass closest hit, hoisted invariants, record for the winner only): its
    image is Tier A's bit for bit, on the same stream — the prebuilt portable
    copy and the -O3 -march=native build bench.py makes on the timing host."""
    path = None
    if native:
        path = str(tmp_path / "port.so")
        oracle.build_cpu_port(path)
    L = oracle.cpu_port_lib(path)
    sc, rng = oracle.cover_scene(42)
    cam = oracle.cover_camera(16 / 9)
    h = oracle.lib().ro_image_height(w, 16 / 9)
    rng2 = oracle.ZigRandom(state=list(rng.s))
    a, _, _ = oracle.render_tier_a(sc, cam, rng, w, h, spp)
    b = oracle.render_cpu_port(L, sc, cam, rng2, w, h, spp)
    assert (a == b).all()
    assert list(rng.s) == list(rng2.s)  # the same number of draws


def test_cpu_port_equals_config0_artifact(oracle):
    """... and the committed configs[0] digest (400x225x100) through the port."""
    import hashlib
    import json

    rec = json.load(open(os.path.join(GOLDEN, "config0_tier_a_400x225x100.json")))
    L = oracle.cpu_port_lib()
    sc, rng = oracle.cover_scene(42)
    img = oracle.render_cpu_port(L, sc, oracle.cover_camera(16 / 9), rng, 400, 225, 100)
    assert hashlib.sha256(b"P6\n400 225\n255\n" + img.tobytes()).hexdigest() == rec["ppm_sha256"]
