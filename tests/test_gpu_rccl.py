"""RCCL on the card: the multi-GPU exchange's collectives (dist.gather of the
rendered row tiles, all_reduce of the sample counts) in a world-size-1 "nccl"
group, in a child process so the process group never leaks into the other GPU
tests.  N > 1 RCCL ranks need the driver's 8-GPU node; the N-rank logic itself
is covered by tests/test_shard_gloo.py and tests/test_bench_launch.py."""
import json
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu

HERE = os.path.dirname(os.path.abspath(__file__))


def test_rccl_gather_of_rendered_row_tiles():
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    p = subprocess.run([sys.executable, os.path.join(HERE, "rccl_gather_check.py")], env=env,
                       capture_output=True, text=True, timeout=110)
    print(p.stdout, p.stderr[-2000:])
    assert p.returncode == 0, p.stderr[-2000:]
    res = json.loads(p.stdout.strip().splitlines()[-1])
    assert res["backend"] == "nccl" and res["world_size"] == 1
    assert res["gather_bit_exact"] and res["assembled_equals_full"]
