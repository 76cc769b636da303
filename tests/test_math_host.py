"""CPU check of the kernel's exactness-preserving shortcuts (csrc/rtw_math.hpp):
sin_sign == sign(libm sin) and div_rn == IEEE division, bit for bit."""
import os
import subprocess

import pytest

from conftest import PKG_ROOT, REPO


@pytest.fixture(scope="module")
def checker(tmp_path_factory):
    out = tmp_path_factory.mktemp("math") / "math_check"
    src = os.path.join(REPO, "tests", "native", "math_check.cpp")
    cmd = ["g++", "-O2", "-std=c++17", "-ffp-contract=off", "-mfma", "-I", os.path.join(PKG_ROOT, "csrc"),
           src, "-o", str(out)]
    subprocess.run(cmd, check=True)
    return str(out)


def test_sin_sign_and_div_rn_exact(checker):
    r = subprocess.run([checker, "2000000"], capture_output=True, text=True)
    print(r.stdout)
    assert r.returncode == 0, r.stdout + r.stderr
    assert " 0/" in r.stdout
