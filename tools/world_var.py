"""Where does the globe's run-to-run spread come from?  python tools/world_var.py [instances] [reps]
Creates the configs[4] world N times in one process (each a new device allocation, the earlier
ones kept alive so the addresses differ) with a new workspace each, renders each `reps` times,
and prints every time: a spread between instances with stable times inside each instance points
at memory placement, a spread inside an instance at the device."""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                                "raytracinginoneweekend.zig_amd"))
import torch  # noqa: E402

import rtw_amd as R  # noqa: E402
from rtw_amd import world as Wd  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 6
reps = int(sys.argv[2]) if len(sys.argv) > 2 else 4
earth = Wd.earth_map()
b = Wd.BuiltScene(7, 42, image=earth)
s = b.settings
cam = b.camera()
p = R.make_params(s.width, s.height, s.spp, 50, 42, background=b.background)
keep = []
st = torch.cuda.current_stream().cuda_stream
rgb = torch.empty((s.height, s.width, 3), dtype=torch.uint8, device="cuda:0")
for i in range(n):
    dw = Wd.DeviceWorld(b.desc)
    need = dw.workspace_bytes(p)
    ws = torch.empty(need + 256, dtype=torch.uint8, device="cuda:0")
    ptr = (ws.data_ptr() + 255) & ~255
    dw.render_async(cam, p, ptr, need, rgb.data_ptr(), None, st)
    torch.cuda.synchronize()
    ts = []
    for _ in range(reps):
        t = R.Timer()
        dw.render_async(cam, p, ptr, need, rgb.data_ptr(), None, st, t)
        ts.append(t.elapsed_ms())
        t.close()
    # the same world with the first instance's workspace (placement of the world vs of the workspace)
    if keep:
        w0, ptr0, need0 = keep[0][0], keep[0][2], keep[0][3]
        t = R.Timer()
        dw.render_async(cam, p, ptr0, need0, rgb.data_ptr(), None, st, t)
        tx = t.elapsed_ms()
        t.close()
    else:
        tx = float("nan")
    print(f"instance {i}: world buf {dw.buf_ptr() if hasattr(dw, 'buf_ptr') else '?'} ws {ptr:#x}: "
          + " ".join(f"{x:.2f}" for x in ts) + f" ms; with workspace 0: {tx:.2f} ms", flush=True)
    keep.append((dw, ws, ptr, need))
