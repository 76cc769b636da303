"""Device check of the kernel's exact arithmetic shortcuts (csrc/rtw_math.hpp):
sqrt_rn is the compiler's f64 sqrt sequence without its input scaling, so it
can only be checked where v_rsq_f64 runs.  bin/gpu_math_check (built in-tree
by build()) compares sqrt_rn with __builtin_sqrt and div_rn with IEEE
division bit for bit on 2^28 device-generated inputs."""
import os
import re
import subprocess

import pytest

from conftest import PKG_ROOT

pytestmark = pytest.mark.gpu


def test_sqrt_rn_and_div_rn_bit_exact_on_device():
    exe = os.path.join(PKG_ROOT, "bin", "gpu_math_check")
    assert os.path.exists(exe), "bin/gpu_math_check missing: run build() first"
    r = subprocess.run([exe, str(1 << 28)], capture_output=True, text=True, timeout=120)
    print(r.stdout)
    m = re.search(r"tested (\d+) sqrt_rn mismatches (\d+) div_rn mismatches (\d+)", r.stdout)
    assert m, r.stdout + r.stderr
    assert int(m.group(1)) == 1 << 28 and int(m.group(2)) == 0 and int(m.group(3)) == 0
    assert r.returncode == 0
