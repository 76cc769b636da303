"""GPU parity of the wavefront engine (BASELINE.json configs[3]: SoA path
queues in HBM, per-bounce kernels — fused shade + closest hit, or separate
extend / shade — persistent grids, and an in-register drain once slots
retire: wf_drain, the remaining samples dealt to the wave's free lanes and
folded in sample order, or wf_finish, a lane per slot).

It computes the same Tier-B image as the megakernel: every sample runs the
same device functions in the same order and a home slot adds its unit's
samples in sample order, so the bar is bit-identical output — against the
oracle (same bar as test_gpu_parity.py) and against the megakernel (every
byte of rgb and every float of the linear mean).  Queue capacities from 64
paths (heavy slot recycling, long drain) to more paths than work units.
"""
import numpy as np
import pytest

from helpers import diff_stats, to_oracle_camera, to_oracle_scene
from test_gpu_parity import ASPECT, assert_parity, clustered_scene, custom_scene, oracle_render

pytestmark = pytest.mark.gpu


@pytest.fixture(params=["samples", "finish", "queues"])
def drain(request):
    """Every test runs with the three drains (params.wf_drain): in registers
    once slots retire, by wf_drain (samples dealt to free lanes, the default)
    or wf_finish (RTW_WF_DRAIN_SLOTS), and the bounce kernels' queues to the
    end (RTW_WF_DRAIN_NONE)."""
    return request.param


@pytest.fixture(params=["fused", "fused1", "split"])
def engine_form(request):
    """... and both forms of the engine (params.wf_form): one fused kernel per
    bounce (shade + the next closest hit, the default) and separate extend /
    shade kernels; the fused form with the default queue passes per launch
    (params.wf_passes: a wave moves its segments through the queues pass after
    pass inside one launch) and with one pass per launch ("fused1")."""
    return request.param


@pytest.fixture(params=["sets1", "sets2"])
def queue_sets(request):
    """... and one or two queue sets (params.wf_sets): the in-flight paths
    split over independent sets on their own HIP streams, sharing the device
    unit queue (a unit still belongs to one slot, so the bits cannot change)."""
    return int(request.param[-1])


@pytest.fixture(autouse=True)
def wf_config(rtw, monkeypatch, drain, engine_form, queue_sets):
    """The engine configuration travels in rtw_params (ABI v4): every params
    the test makes carries this case's wf_drain / wf_form / wf_sets."""
    orig = rtw.make_params
    cfg = dict(wf_drain={"samples": "samples", "finish": "slots", "queues": "none"}[drain],
               wf_form="split" if engine_form == "split" else "fused", wf_sets=queue_sets,
               wf_passes=1 if engine_form == "fused1" else 0)

    def make_params(*a, **kw):
        for k, v in cfg.items():
            kw.setdefault(k, v)
        return orig(*a, **kw)
    monkeypatch.setattr(rtw, "make_params", make_params)


@pytest.fixture(scope="module")
def cover(rtw, oracle):
    sph, mats, _ = rtw.cover_scene(42)
    cam = rtw.cover_camera(ASPECT)
    return sph, mats, cam, to_oracle_scene(oracle, sph, mats), to_oracle_camera(oracle, cam)


def both(rtw, cam, sph, mats, **kw):
    """(megakernel rgb, mean), (wavefront rgb, mean) for the same params."""
    wf = {k: kw.pop(k) for k in ("wf_paths", "wf_passes") if k in kw}
    a = rtw.render(cam, sph, mats, rtw.make_params(**kw), want_mean=True)
    b = rtw.render(cam, sph, mats, rtw.make_params(engine="wavefront", **wf, **kw), want_mean=True)
    return a, b


def assert_identical(a, b, what):
    (ra, ma), (rb, mb) = a, b
    assert (ra == rb).all(), (what, diff_stats(ra, rb))
    assert np.array_equal(ma.view(np.uint32), mb.view(np.uint32)), what


@pytest.mark.parametrize("precision", ["f64", "f32"])
@pytest.mark.parametrize("w,spp,chunk,paths", [(400, 16, 0, 0), (160, 40, 7, 4096), (96, 3, 0, 64),
                                              (64, 9, 4, 1 << 16)])
def test_wavefront_cover_parity(rtw, oracle, cover, precision, w, spp, chunk, paths):
    sph, mats, cam, osc, ocam = cover
    h = rtw.image_height(w, ASPECT)
    kw = dict(width=w, height=h, spp=spp, chunk=chunk, precision=precision)
    mk, wf = both(rtw, cam, sph, mats, wf_paths=paths, **kw)
    assert_identical(mk, wf, f"wavefront vs megakernel {precision} {w}x{h}x{spp} paths {paths}")
    o = oracle_render(oracle, osc, ocam, **kw)
    assert_parity(wf[0], o, f"wavefront {precision} {w}x{h}x{spp} chunk {chunk} paths {paths}")


@pytest.mark.parametrize("passes", [2, 3, 8, 64])
def test_wavefront_queue_passes_per_launch(rtw, cover, passes):
    """params.wf_passes other than the default (16) and 1: an even count
    returns each launch's output to its input queue, an odd count alternates
    the queues per launch as one pass does; 64 (the maximum) lets a batch run
    past the drain trigger.  Same image as the megakernel."""
    sph, mats, cam, _, _ = cover
    kw = dict(width=400, height=rtw.image_height(400, ASPECT), spp=16)
    mk, wf = both(rtw, cam, sph, mats, wf_paths=4096, wf_passes=passes, **kw)
    assert_identical(mk, wf, f"wf_passes {passes}")


@pytest.mark.parametrize("depth", [0, 1, 2, 5])
def test_wavefront_depth_edges(rtw, oracle, cover, depth):
    sph, mats, cam, osc, ocam = cover
    kw = dict(width=64, height=36, spp=4, max_depth=depth)
    mk, wf = both(rtw, cam, sph, mats, wf_paths=256, **kw)
    assert_identical(mk, wf, f"depth {depth}")
    assert_parity(wf[0], oracle_render(oracle, osc, ocam, **kw), f"wavefront depth {depth}")
    if depth == 0:
        assert (wf[0] == 0).all()


def test_wavefront_empty_scene(rtw, cover):
    _, _, cam, _, _ = cover
    a = rtw.render(cam, None, None, rtw.make_params(32, 18, 3))
    b = rtw.render(cam, None, None, rtw.make_params(32, 18, 3, engine="wavefront", wf_paths=64))
    assert (a == b).all()


@pytest.mark.parametrize("precision", ["f64", "f32"])
def test_wavefront_custom_scene(rtw, oracle, precision):
    sph, mats = custom_scene(rtw)
    cam = rtw.camera_init((13, 2, 3), (0, 0.5, 0), (0, 1, 0), 30.0, ASPECT, 0.2, 10.0, 0.0, 1.0)
    kw = dict(width=128, height=72, spp=16, precision=precision, chunk=5)
    mk, wf = both(rtw, cam, sph, mats, wf_paths=2048, **kw)
    assert_identical(mk, wf, f"custom {precision}")
    o = oracle_render(oracle, to_oracle_scene(oracle, sph, mats), to_oracle_camera(oracle, cam), **kw)
    assert_parity(wf[0], o, f"wavefront custom {precision}")


@pytest.mark.parametrize("time1", [1.0, 1.2])
def test_wavefront_clustered_pretest(rtw, oracle, time1):
    """The bounce kernels run the megakernel's clustered pretest since round 6
    (rtw_internal.hpp RTW_WF_VAR_EXTRA): three time groups mixed in clusters,
    odd cluster sizes, with a shutter inside every group (clusters on) and one
    outside a group (clusters off, the flat pretest) — the megakernel's image
    bit for bit and the oracle's."""
    sph, mats = clustered_scene(rtw)
    cam = rtw.camera_init((13, 2, 3), (0, 0.3, 0), (0, 1, 0), 30.0, ASPECT, 0.1, 10.0, 0.0, time1)
    kw = dict(width=192, height=108, spp=12, chunk=5)
    mk, wf = both(rtw, cam, sph, mats, wf_paths=4096, **kw)
    assert_identical(mk, wf, f"clustered scene, shutter [0, {time1}]")
    o = oracle_render(oracle, to_oracle_scene(oracle, sph, mats), to_oracle_camera(oracle, cam), **kw)
    assert_parity(wf[0], o, f"wavefront clustered scene, shutter [0, {time1}]")


def test_wavefront_row_shards(rtw, cover):
    sph, mats, cam, _, _ = cover
    W, H = 120, 68
    full = rtw.render(cam, sph, mats, rtw.make_params(W, H, 8))
    for world in (2, 8):
        for r in (0, world - 1):
            part = rtw.render(cam, sph, mats, rtw.make_params(W, H, 8, row_begin=r, row_stride=world,
                                                              engine="wavefront", wf_paths=1000))
            assert (part == full[r::world]).all(), (world, r)


@pytest.mark.parametrize("bounces", [1, 3])
@pytest.mark.parametrize("precision", ["f64", "f32"])
def test_wavefront_config2_full_frame_identical(rtw, cover, precision, bounces):
    """configs[1] at full size (1200x675x500): the wavefront frame equals the
    megakernel frame byte for byte (the megakernel's rows are oracle-checked
    in test_gpu_parity.py) — with one bounce segment per wf_step launch and
    with three (params.wf_bounces: the path kept in registers between them)."""
    import torch
    from rtw_amd.device import TorchRenderer

    sph, mats, cam, _, _ = cover
    R = TorchRenderer(sph, mats, 0)
    outs = []
    for eng in ("megakernel", "wavefront"):
        p = rtw.make_params(1200, 675, 500, precision=precision, engine=eng, wf_bounces=bounces)
        rgb = torch.empty((675, 1200, 3), dtype=torch.uint8, device="cuda:0")
        mean = torch.empty((675, 1200, 3), dtype=torch.float32, device="cuda:0")
        R.render(cam, p, out=rgb, mean=mean)
        torch.cuda.synchronize()
        outs.append((rgb.cpu().numpy(), mean.cpu().numpy()))
    assert_identical(outs[0], outs[1], f"config2 {precision}")


@pytest.mark.parametrize("w,spp,paths,chunk", [(400, 128, 360_000, 0), (1200, 64, 0, 0), (160, 40, 64, 0),
                                               (160, 40, 256, 32)])
def test_wavefront_traces_every_sample_exactly_once(rtw, cover, w, spp, paths, chunk, drain, queue_sets):
    """Statistics pass: the wavefront shades exactly W*H*spp samples and the
    megakernel's number of bounce segments.  Duplicated or lost units would
    leave the image bits unchanged (a unit's samples are deterministic) but
    change these counts.  (400x225x128 at 360k paths: more segments than
    resident waves, so waves own several segments.)"""
    import torch
    from rtw_amd.device import TorchRenderer

    sph, mats, cam, _, _ = cover
    h = rtw.image_height(w, ASPECT)
    R = TorchRenderer(sph, mats, 0)
    mk = R.counts(cam, rtw.make_params(w, h, spp, chunk=chunk))
    wf = R.counts(cam, rtw.make_params(w, h, spp, chunk=chunk, engine="wavefront", wf_paths=paths))
    torch.cuda.synchronize()
    assert mk["samples"] == w * h * spp
    assert (wf["samples"], wf["segments"]) == (mk["samples"], mk["segments"])
    # the in-register drain's share (rtw_render_counts_ex): part of the same totals
    assert mk["drain_segments"] == mk["drain_samples"] == 0
    if drain == "queues":
        assert wf["drain_segments"] == wf["drain_samples"] == 0
    else:
        assert wf["drain_segments"] < wf["segments"] and wf["drain_samples"] < wf["samples"]
        # (one 64-path segment on the sky units the queue deals last: every
        # slot's last unit ends in the same bounce, so no poll sees slots
        # retiring and the drain may not run at all; 256 paths, split over
        # at most 2 sets, is the small case whose drain must run — with units
        # of 32 samples: the default 20's shorter units can all end inside one
        # polled batch of 32 bounces, so that no poll sees slots retiring)
        if (paths or rtw.DEFAULT_WF_PATHS) // queue_sets > 64:
            assert wf["drain_segments"] > 0 and wf["drain_samples"] > 0
