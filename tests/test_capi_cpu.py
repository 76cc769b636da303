"""The C-ABI library on the CPU: it loads, exports every symbol include/rtw_hip.h
declares, and its host-side helpers (Camera.init, generateRandomScene, image
height, argument validation) agree with the oracle.  No compute call here."""
import ctypes as C
import json
import os

import pytest

from conftest import GOLDEN, REPO
from helpers import to_oracle_camera


def test_library_exports_every_header_symbol(rtw):
    syms = rtw.header_symbols()
    assert len(syms) >= 15
    for s in syms:
        assert hasattr(rtw.lib(), s), s


def test_abi_version(rtw):
    assert rtw.abi_version() == 4


def test_struct_layouts_match_header(rtw):
    # sizes of the C structs (x86-64 / gfx950 host ABI)
    assert C.sizeof(rtw.Material) == 8 + 3 * 8 * 2 + 16
    assert C.sizeof(rtw.Sphere) == 6 * 8 + 3 * 8 + 8
    assert C.sizeof(rtw.Camera) == 7 * 24 + 24
    assert C.sizeof(rtw.Params) == 16 + 8 + 24 + 12 + 12 + 8 + 8 * 4  # + ABI v4 engine fields


def test_cover_scene_equals_oracle_golden(rtw):
    with open(os.path.join(GOLDEN, "cover_scene_seed42.json")) as f:
        g = json.load(f)
    sph, mats, st = rtw.cover_scene(42)
    assert st == g["rng_state_after"]
    assert len(sph) == len(g["spheres"]) and len(mats) == len(g["materials"])
    for s, gs in zip(sph, g["spheres"]):
        assert list(s.c0) == gs["c0"] and list(s.c1) == gs["c1"]
        assert s.radius == gs["radius"] and s.moving == gs["moving"] and s.mat == gs["mat"]
        if s.moving:
            assert (s.t0, s.t1) == (gs["t0"], gs["t1"])
    for m, gm in zip(mats, g["materials"]):
        assert m.kind == gm["kind"] and list(m.albedo) == gm["albedo"]
        assert list(m.albedo_odd) == gm["albedo_odd"] and m.fuzz == gm["fuzz"] and m.ir == gm["ir"]


@pytest.mark.parametrize("aspect", [16 / 9, 1.5, 1.0])
def test_camera_init_equals_oracle(rtw, oracle, aspect):
    a = rtw.cover_camera(aspect)
    b = oracle.cover_camera(aspect)
    for n in ("origin", "horizontal", "vertical", "lower_left_corner", "u", "v", "w"):
        assert list(getattr(a, n)) == list(getattr(b, n)), n
    assert (a.lens_radius, a.time0, a.time1) == (b.lens_radius, b.time0, b.time1)
    c = to_oracle_camera(oracle, a)
    assert list(c.lower_left_corner) == list(b.lower_left_corner)


@pytest.mark.parametrize("w,aspect", [(400, 16 / 9), (1200, 16 / 9), (3840, 16 / 9), (600, 1.5), (600, 1.0)])
def test_image_height(rtw, oracle, w, aspect):
    assert rtw.image_height(w, aspect) == oracle.image_height(w, aspect)


def test_configs_heights(rtw):
    assert [rtw.image_height(w, 16 / 9) for w in (400, 1200, 3840)] == [225, 675, 2160]


@pytest.mark.parametrize("kw,status", [
    (dict(width=1, height=10, spp=1), -1),
    (dict(width=10, height=10, spp=0), -1),
    (dict(width=10, height=10, spp=1, row_stride=0, row_count=1), -1),
    (dict(width=10, height=10, spp=1, row_begin=9, row_stride=2, row_count=2), -1),
    (dict(width=5000, height=5000, spp=1), -2),
    (dict(width=10, height=10, spp=1, precision=7), -1),
    (dict(width=10, height=10, spp=1, engine=2), -1),
    (dict(width=10, height=10, spp=1, engine="wavefront", wf_paths=8), -1),
    (dict(width=10, height=10, spp=1, engine="wavefront", max_depth=70000), -2),
])
def test_render_rejects_bad_params_before_touching_the_gpu(rtw, kw, status):
    sph, mats, _ = rtw.cover_scene(42)
    with pytest.raises(rtw.RtwError) as e:
        rtw.render(rtw.cover_camera(16 / 9), sph, mats, rtw.make_params(**kw))
    assert e.value.status == status
    assert rtw.lib().rtw_last_error()


def test_scene_rejects_unsupported_material(rtw):
    sph, mats, _ = rtw.cover_scene(42)
    mats[0].kind = rtw.DIFFUSE_LIGHT
    with pytest.raises(rtw.RtwError) as e:
        rtw.DeviceScene(sph, mats)
    assert e.value.status == rtw.RTW_UNSUPPORTED


def test_scene_rejects_bad_material_index(rtw):
    sph, mats, _ = rtw.cover_scene(42)
    sph[3].mat = 999
    with pytest.raises(rtw.RtwError) as e:
        rtw.DeviceScene(sph, mats)
    assert e.value.status == rtw.RTW_EINVAL


def test_workspace_bytes(rtw):
    p = rtw.make_params(1200, 675, 500)
    n = rtw.workspace_bytes(p)
    chunks = -(-500 // rtw.DEFAULT_CHUNK)  # (rtw_hip.h RTW_DEFAULT_CHUNK)
    assert n >= chunks * 1200 * 675 * 3 * 8
    assert n < chunks * 1200 * 675 * 3 * 8 + 4096


@pytest.mark.parametrize("sets", [1, 2, 3])
@pytest.mark.parametrize("ring", [True, False])
def test_workspace_bytes_wavefront(rtw, monkeypatch, sets, ring):
    """Wavefront engine: + two SoA path queues (each with the fused engine's
    hit winner per path; its hit point rides in the path's origin since round 6),
    the split engine's hit arrays, the home
    slots and (wf_drain only: params.wf_drain RTW_WF_DRAIN_SAMPLES) its ring of 32 R x3 sample
    radiances (rtw_capi.hip ws_layout) per in-flight path, + per-segment
    words; wf_paths is split over params.wf_sets queue sets, so the bytes per
    path do not grow with the sets (exact bounds: an upper bound per path,
    ADVICE r3)."""
    base = rtw.workspace_bytes(rtw.make_params(1200, 675, 500))
    for prec, r in (("f64", 8), ("f32", 4)):
        for n in (1 << 16, 1 << 20, 3 << 18):
            p = rtw.make_params(1200, 675, 500, precision=prec, engine="wavefront", wf_paths=n, wf_sets=sets,
                                wf_drain="samples" if ring else "slots")
            per_path = 2 * (10 * r + 8 + 4 + 4 + 4) + (r + 4) + 32 + (32 * 3 * r if ring else 0)
            segs = -(-n // (64 * sets))  # per set: one 64-path queue segment = 2 counts + a unit reservoir
            paths = segs * 64
            extra = rtw.workspace_bytes(p) - base
            lo = sets * (paths * per_path + segs * 16)
            assert lo <= extra <= lo + sets * 64 * 256, (prec, n, extra, lo)
            assert extra <= n * (per_path + 1) + sets * (64 * per_path + 64 * 256)  # per-path upper bound
    d = rtw.make_params(64, 36, 1, engine="wavefront")
    assert rtw.workspace_bytes(d) > rtw.DEFAULT_WF_PATHS * 100


ENV_KNOBS = {  # every environment variable a development (-DRTW_MEASURE) build reads
    "RTW_WF_SETS": "1", "RTW_WF_DRAIN": "0", "RTW_WF_FINISH": "0", "RTW_WF_FUSED": "0", "RTW_WF_BATCH": "8",
    "RTW_WF_GRID": "2", "RTW_WF_SET_GRID": "2", "RTW_WF_TIMEOUT_S": "1", "RTW_UNIT_ORDER": "rev",
    "RTW_VARIANT": "516", "RTW_WORLD_OCC": "1", "RTW_WORLD_FEAT": "all", "RTW_WORLD_TAIL": "0",
    "RTW_PHASE_PROFILE": "1", "RTW_COUNTS_VERBOSE": "1"}


def test_workspace_bytes_ignore_the_environment(rtw):
    """ABI v4: the product library reads no environment
    variable on the render path, so rtw_workspace_bytes is a function of the
    params alone — checked in a fresh process with every knob set."""
    import json
    import subprocess
    import sys
    code = (
        "import json, sys; sys.path.insert(0, %r); import rtw_amd as R\n"
        "out = []\n"
        "for eng in ('megakernel', 'wavefront'):\n"
        "    for prec in ('f64', 'f32'):\n"
        "        for kw in ({}, {'wf_sets': 1}, {'wf_sets': 3, 'wf_drain': 'slots'}, {'wf_drain': 'none'}):\n"
        "            p = R.make_params(1200, 675, 500, precision=prec, engine=eng, **kw)\n"
        "            out.append(R.workspace_bytes(p))\n"
        "print(json.dumps(out))\n") % os.path.join(REPO, "raytracinginoneweekend.zig_amd")
    env0 = {k: v for k, v in os.environ.items() if not k.startswith("RTW_")}
    a = json.loads(subprocess.run([sys.executable, "-c", code], env=env0, capture_output=True, text=True,
                                  check=True).stdout)
    b = json.loads(subprocess.run([sys.executable, "-c", code], env={**env0, **ENV_KNOBS}, capture_output=True,
                                  text=True, check=True).stdout)
    assert a == b
    # and the params fields do change it (wavefront f64: without the drain ring
    # for wf_finish / no drain; the megakernel ignores the wavefront fields)
    assert a[8] != a[10] and a[8] != a[11] and len(set(a[0:4])) == 1


def test_product_library_reads_no_environment():
    """The only getenv of the product sources is the development-knob helper,
    compiled in the -DRTW_MEASURE build alone."""
    import glob
    import re
    src = os.path.join(REPO, "raytracinginoneweekend.zig_amd", "csrc")
    hits = []
    for f in glob.glob(os.path.join(src, "*.hip")) + glob.glob(os.path.join(src, "*.cpp")) + \
            glob.glob(os.path.join(src, "*.hpp")):
        for i, line in enumerate(open(f), 1):
            if re.search(r"\bgetenv\s*\(", line):
                hits.append((os.path.basename(f), i, line.strip()))
    assert [h[:2] for h in hits] == [("rtw_capi.hip", hits[0][1])], hits
    txt = open(os.path.join(src, "rtw_capi.hip")).read()
    i = txt.find("const char* dev_knob(const char* name) {")
    body = txt[i:txt.find("}", txt.find("#endif", i))]
    assert "#ifdef RTW_MEASURE" in body and "return getenv(name);" in body and "return nullptr;" in body


@pytest.mark.parametrize("field,value", [("wf_sets", 5), ("wf_drain", 3), ("wf_form", 2), ("world_waves", 5),
                                         ("world_waves", 2), ("world_features", 2), ("world_traversal", 3), ("wf_bounces", 17),
                                         ("wf_passes", 65)])
def test_params_v4_fields_validated(rtw, field, value):
    p = rtw.make_params(64, 36, 1, engine="wavefront")
    setattr(p, field, value)
    with pytest.raises(rtw.RtwError) as e:
        rtw.workspace_bytes(p)
    assert e.value.status == rtw.RTW_EINVAL


def test_no_cpu_fallback_without_gpu(rtw):
    """The product path must fail loudly (RTW_ENODEV) when no GPU is visible."""
    import torch
    if torch.cuda.is_available():
        pytest.skip("GPU visible")
    sph, mats, _ = rtw.cover_scene(42)
    with pytest.raises(rtw.RtwError) as e:
        rtw.render(rtw.cover_camera(16 / 9), sph, mats, rtw.make_params(16, 9, 1))
    assert e.value.status == rtw.RTW_ENODEV


def test_python_engine_defaults_are_the_headers(rtw):
    """rtw_amd's DEFAULT_WF_* / DEFAULT_CHUNK (what bench.py reports and
    matches PMC evidence against) are the C header's RTW_DEFAULT_* values, so a
    default changed on one side only cannot label a line with the wrong
    configuration (round 6 changed the wavefront's paths and passes)."""
    import re
    hdr = open(os.path.join(REPO, "include", "rtw_hip.h")).read()

    def define(name):
        m = re.search(rf"#define {name} \(?(\d+)u(?: << (\d+))?\)?", hdr)
        assert m, name
        return int(m.group(1)) << int(m.group(2) or 0)

    assert rtw.DEFAULT_WF_PATHS == define("RTW_DEFAULT_WF_PATHS")
    assert rtw.DEFAULT_WF_SETS == define("RTW_DEFAULT_WF_SETS")
    assert rtw.DEFAULT_WF_PASSES == define("RTW_DEFAULT_WF_PASSES")
    assert rtw.DEFAULT_CHUNK == define("RTW_DEFAULT_CHUNK")
