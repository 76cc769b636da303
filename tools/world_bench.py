"""World-kernel timing on the GPU box: the reference's scenes at their own
main.zig settings (scene 6 Cornell 600x600x200 is the reference's default
scene) and configs[4] (scene 7, globe + 10k spheres, 1200x675x100), plus
scene 1 through the world kernel vs the cover megakernel.  HIP-event timed;
counts pass for BVH statistics."""
import json
import os
import sys
import time

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                                "raytracinginoneweekend.zig_amd"))
import torch  # noqa: E402

import rtw_amd as R  # noqa: E402
from rtw_amd import world as Wd  # noqa: E402


def run(scene, reps=3, spp=None, width=None, linear=False, **pkw):
    """pkw: rtw_params fields (world_traversal="lane", world_waves=3, ...)."""
    earth = Wd.earth_map()
    b = Wd.BuiltScene(scene, 42, image=earth if scene in (4, 7) else None)
    s = b.settings
    W = width or s.width
    H = R.image_height(W, s.aspect) if width else s.height
    spp = spp or s.spp
    cam = b.camera()
    p = R.make_params(W, H, spp, 50, 42, background=b.background, **pkw)
    dw = Wd.DeviceWorld(b.desc, linear=linear)
    need = dw.workspace_bytes(p)  # + the tail dealing's rings (rtw_world_workspace_bytes)
    ws = torch.empty(need + 256, dtype=torch.uint8, device="cuda:0")
    ptr = (ws.data_ptr() + 255) & ~255
    rgb = torch.empty((H, W, 3), dtype=torch.uint8, device="cuda:0")
    st = torch.cuda.current_stream().cuda_stream
    dw.render_async(cam, p, ptr, need, rgb.data_ptr(), None, st)
    torch.cuda.synchronize()
    best = 1e9
    for _ in range(reps):
        t = R.Timer()
        dw.render_async(cam, p, ptr, need, rgb.data_ptr(), None, st, t)
        ms = t.elapsed_ms()
        t.close()
        best = min(best, ms)
    c = dw.counts(cam, p, ptr, need)
    out = {"scene": scene, "name": Wd.SCENES[scene], "W": W, "H": H, "spp": spp, "linear": linear,
           "ms": round(best, 3), "msamples_s": round(W * H * spp / best / 1e3, 1), "bvh": dw.bvh_info(),
           "segments_per_sample": round(c["segments"] / c["samples"], 3),
           "node_visits_per_segment": round(c["node_visits"] / max(1, c["segments"]), 2),
           "prim_tests_per_segment": round(c["prim_tests"] / max(1, c["segments"]), 2),
           "wave_iters_per_segment": round(64 * c["wave_iters"] / max(1, c["segments"]), 3),
           # per-lane traversal: wave-level interior / leaf iterations per wave-iteration's segments
           "lane_interior_iters_per_seg": round(64 * c["lane_interior_iters"] / max(1, c["segments"]), 2),
           "lane_leaf_iters_per_seg": round(64 * c["lane_leaf_iters"] / max(1, c["segments"]), 2), **pkw}
    dw.close()
    return out


if __name__ == "__main__":
    # python tools/world_bench.py [scenes] [cfg ...]; cfg = "-" (defaults) or
    # comma-separated rtw_params fields, e.g. "world_traversal=lane,world_waves=3"; WORLD_REPS renders (best of)
    which = [int(x) for x in sys.argv[1].split(",")] if len(sys.argv) > 1 else [6, 7, 1, 5, 3, 2, 4]
    cfgs = sys.argv[2:] or ["-"]
    for sc in which:
        for cfg in cfgs:
            kw = {}
            for kv in ([] if cfg == "-" else cfg.split(",")):
                k, v = kv.split("=")
                kw[k] = int(v) if v.isdigit() else v
            print(json.dumps(run(sc, reps=int(os.environ.get("WORLD_REPS", "3")), **kw)), flush=True)
