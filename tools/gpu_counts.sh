set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
RTW_COUNTS_VERBOSE=1 timeout -k 10 300 python -c "
import sys; sys.path.insert(0,'raytracinginoneweekend.zig_amd')
import rtw_amd as R
from rtw_amd.device import TorchRenderer
sph, mats, _ = R.cover_scene(42); cam = R.cover_camera(16/9)
rend = TorchRenderer(sph, mats, 0)
for prec in ('f64','f32'):
    print(prec, rend.counts(cam, R.make_params(1200, 675, 500, precision=prec)), flush=True)
" > gpurun_out/counts.log 2>&1
