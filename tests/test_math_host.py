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


def test_udiv_magic_exact(tmp_path):
    """The work-unit decode's division by a per-render constant (rtwm::udiv,
    magic multiplier) equals integer division for every checked divisor."""
    out = tmp_path / "udiv_check"
    src = os.path.join(REPO, "tests", "native", "udiv_check.cpp")
    subprocess.run(["g++", "-O2", "-std=c++17", "-I", os.path.join(PKG_ROOT, "csrc"), src, "-o", str(out)], check=True)
    r = subprocess.run([str(out)], capture_output=True, text=True)
    print(r.stdout)
    assert r.returncode == 0 and "bad 0/" in r.stdout, r.stdout + r.stderr
