"""The shader-clock probe the bench line reads (rtw_sclk_probe_*, VERDICT r3
W7: every timing beside the clock it ran at): one wave on a side stream,
delta(s_memtime) / delta(s_memrealtime) x 100 MHz over a wall-time window,
while a render runs on the main stream."""
import pytest

pytestmark = pytest.mark.gpu


def test_sclk_probe_reads_a_plausible_clock(rtw):
    import torch
    from rtw_amd.device import TorchRenderer

    sph, mats, _ = rtw.cover_scene(42)
    rend = TorchRenderer(sph, mats, 0)
    cam = rtw.cover_camera(16 / 9)
    p = rtw.make_params(1200, 675, 64)
    rend.render(cam, p)
    torch.cuda.synchronize()
    side = torch.cuda.Stream()
    probe = rtw.SclkProbe(side.cuda_stream, 20.0)
    for _ in range(4):
        rend.render(cam, p)
    torch.cuda.synchronize()
    mhz = probe.read()
    print(f"SCLK over the window: {mhz:.1f} MHz")
    assert 500.0 < mhz < 3500.0
    with pytest.raises(rtw.RtwError):
        rtw.SclkProbe(side.cuda_stream, 0.0)
