import os
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG_ROOT = os.path.join(REPO, "raytracinginoneweekend.zig_amd")
ORACLE = os.path.join(REPO, "oracle")
for p in (REPO, PKG_ROOT, ORACLE):
    if p not in sys.path:
        sys.path.insert(0, p)

GOLDEN = os.path.join(REPO, "tests", "golden")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a real MI355X (runs on the GPU box)")
    config.addinivalue_line("markers", "slow: long CPU oracle runs")


@pytest.fixture(scope="session")
def oracle():
    import rtw_oracle
    rtw_oracle.lib()
    return rtw_oracle


@pytest.fixture(scope="session")
def rtw():
    import rtw_amd
    rtw_amd.lib()
    return rtw_amd
