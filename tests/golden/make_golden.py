"""Regenerates the committed fixtures in tests/golden/.

PROVENANCE: the reference (Zig) cannot be built or run in this pipeline (no
Zig toolchain, un-vendored zigimg dependency) and ships no tests or golden
outputs for this path, so every fixture here is produced by the ORACLE
restatements, not by the reference binary:
  * rng_kat.json — the two published vectors (Zig std Xoshiro256 "sequence"
    test: state {1,2,3,4}; SplitMix64 seed 1234567) are external pins; the
    DefaultPrng(42) stream / float(f64) values are restatement outputs, agreed
    by the C and the independent Python restatement.
  * cover_scene_seed42.json — generateRandomScene(DefaultPrng.init(42)).
  * tier_a_*.ppm — the reference main() restated (Tier A), C == Python.
  * tier_b_*.ppm — the GPU contract (Tier B) from the C oracle.
Run: python tests/golden/make_golden.py
"""
import json
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, os.path.join(REPO, "oracle"))

import numpy as np  # noqa: E402

import rtw_oracle as O  # noqa: E402
import rtw_oracle_py as P  # noqa: E402


def first_long_lz(seed, limit=200000):
    r = P.Xoshiro256(seed)
    for i in range(limit):
        v = r.next()
        if v >> 52 == 0:
            return i
    return None


def main():
    kat = {}
    r = O.ZigRandom(state=[1, 2, 3, 4])
    kat["xoshiro256_state_1234"] = [r.next() for _ in range(6)]
    kat["splitmix64_1234567"] = O.splitmix64_seq(1234567, 5)
    r = O.ZigRandom(42)
    kat["defaultprng42_u64"] = [r.next() for _ in range(8)]
    r = O.ZigRandom(42)
    kat["defaultprng42_f64_hex"] = [float.hex(r.f64()) for _ in range(8)]
    idx = first_long_lz(42)
    kat["defaultprng42_first_lz12_draw"] = idx
    r = O.ZigRandom(42)
    for _ in range(idx):
        r.next()
    kat["defaultprng42_f64_at_lz12_hex"] = float.hex(r.f64())
    kat["defaultprng42_u64_after_lz12_float"] = r.next()
    r = O.ZigRandom(7)
    kat["defaultprng7_f32_hex"] = [float.hex(r.f32()) for _ in range(8)]
    # Tier-B counter-based stream: Weyl blocks of (seed 42, pixel, sample),
    # draws = ro_tb_mix of the states (round 5; C == the Python tb_mix)
    import ctypes as C
    L = O.lib()
    kat["tierb_state_42_p0_s0"] = L.ro_tierb_state(42, 0, 0)
    kat["tierb_state_42_p1234_s77"] = L.ro_tierb_state(42, 1234, 77)
    st = C.c_uint64(L.ro_tierb_state(42, 1234, 77))
    kat["tierb_42_p1234_s77_f64_hex"] = [float.hex(L.ro_sm_f64(C.byref(st))) for _ in range(6)]
    kat["tb_mix_in"] = [0, 1, 1 << 32, 0x9E3779B97F4A7C15, (1 << 64) - 1, kat["tierb_state_42_p1234_s77"]]
    kat["tb_mix_out"] = [L.ro_tb_mix(x) for x in kat["tb_mix_in"]]
    assert kat["tb_mix_out"] == [P.tb_mix(x) for x in kat["tb_mix_in"]], "C and Python tb_mix disagree"
    with open(os.path.join(HERE, "rng_kat.json"), "w") as f:
        json.dump(kat, f, indent=1)

    sc, rng = O.cover_scene(42)
    t = O.scene_table(sc)
    t["rng_state_after"] = rng.state()
    with open(os.path.join(HERE, "cover_scene_seed42.json"), "w") as f:
        json.dump(t, f, indent=1)

    for (w, asp, spp, name) in [(60, 1.5, 4, "tier_a_60x40_4spp.ppm"), (40, 16 / 9, 8, "tier_a_40x22_8spp.ppm")]:
        img, _ = O.main_cover(w, asp, spp)
        pimg, _ = P.main_cover(w, asp, spp)
        assert (np.array(pimg, np.uint8) == img).all(), "C and Python Tier A disagree"
        O.write_ppm(os.path.join(HERE, name), img)

    cam = O.cover_camera(16 / 9)
    for prec, name in [(0, "tier_b_f64_48x27_8spp.ppm"), (1, "tier_b_f32_48x27_8spp.ppm")]:
        img, _ = O.render_tier_b(sc, cam, 48, 27, 8, precision=prec, chunk=3)
        O.write_ppm(os.path.join(HERE, name), img)
    print("fixtures written to", HERE)


if __name__ == "__main__":
    main()
