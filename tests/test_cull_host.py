"""The packed-f32 closest-hit pretest (csrc/rtw_cull.hpp) is conservative:
on adversarial near-grazing (ray, sphere) pairs, x < 0 always implies the
exact discriminant of hittable.zig:96-101 (f64, and the f32 precision-1
variant) is negative, so skipping the exact test never changes a result.
Also checks that the check has teeth: with the margin scaled by 0.01 it
finds violations."""
import os
import re
import shutil
import subprocess

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC = os.path.join(REPO, "raytracinginoneweekend.zig_amd", "csrc")
SRC = os.path.join(REPO, "tests", "cull_bound_check.cpp")


def _build(tmp_path, header_dir):
    exe = str(tmp_path / "cullchk")
    subprocess.run(["g++", "-O2", "-ffp-contract=off", "-std=c++17", "-I", header_dir, SRC, "-o", exe], check=True)
    return exe


def _run(exe, n, seed):
    p = subprocess.run([exe, str(n), str(seed)], capture_output=True, text=True)
    m = re.search(r"cases (\d+) skipped (\d+) violations (\d+)", p.stdout)
    assert m, p.stdout + p.stderr
    return p.returncode, int(m.group(1)), int(m.group(2)), int(m.group(3))


@pytest.mark.skipif(shutil.which("g++") is None, reason="g++ not available")
def test_pretest_never_skips_a_nonnegative_discriminant(tmp_path):
    exe = _build(tmp_path, CSRC)
    for seed in (1, 2, 3):
        rc, cases, skipped, viol = _run(exe, 1_000_000, seed)
        assert viol == 0 and rc == 0
        assert cases > 900_000 and skipped > cases // 20  # the pretest does skip


@pytest.mark.skipif(shutil.which("g++") is None, reason="g++ not available")
def test_check_detects_a_too_small_margin(tmp_path):
    weak = tmp_path / "weak"
    weak.mkdir()
    src = open(os.path.join(CSRC, "rtw_cull.hpp")).read()
    needle = "return {a * std::fma(16.0f, e, 100.0f * kU), ok};"
    assert needle in src
    (weak / "rtw_cull.hpp").write_text(src.replace(needle, needle.replace("), ok}", ") * 0.01f, ok}")))
    exe = _build(tmp_path, str(weak))
    rc, _, _, viol = _run(exe, 2_000_000, 1)
    assert viol > 0 and rc == 1


CLSRC = os.path.join(REPO, "tests", "cluster_bound_check.cpp")


@pytest.mark.skipif(shutil.which("g++") is None, reason="g++ not available")
def test_cluster_pretest_never_skips_a_member_that_can_be_hit(tmp_path):
    """Clustered pretest (trace VAR kVarCluster, rtw_cull.hpp cluster_sphere):
    a cluster proven missed has every member's exact f64 discriminant negative
    (at every shutter time); with the bound radius shrunk by 2 % the check
    finds violations (it has teeth)."""
    exe = str(tmp_path / "clchk")
    subprocess.run(["g++", "-O2", "-ffp-contract=off", "-std=c++17", "-I", CSRC, CLSRC, "-o", exe], check=True)

    def run(n, seed, shrink="0"):
        p = subprocess.run([exe, str(n), str(seed), shrink], capture_output=True, text=True)
        m = re.search(r"cases (\d+) skipped (\d+) violations (\d+)", p.stdout)
        assert m, p.stdout + p.stderr
        return p.returncode, int(m.group(1)), int(m.group(2)), int(m.group(3))
    for seed in (1, 2):
        rc, cases, skipped, viol = run(400_000, seed)
        assert viol == 0 and rc == 0
        assert skipped > cases // 10  # the cluster pretest does skip
    rc, cases, skipped, viol = run(400_000, 3, "0.02")
    assert viol > 0
