"""bench.py's multi-GPU entry point as the driver invokes it: plain
`python bench.py --gpus N` (no torchrun wrapper, no WORLD_SIZE) must start N
rank processes itself before anything touches the GPU, and rank 0 must print
one JSON line that names the backend and world size.

CPU-only: RTW_BENCH_DRYRUN=1 runs the launcher, the rendezvous (gloo), the
row split, the gather to rank 0 and the all-reduce of the sample counts, with
no rendering (the GPU path of the same ranks is bench.py main())."""
import json
import os
import subprocess
import sys

import pytest

from conftest import REPO

sys.path.insert(0, REPO)


def run_bench(*argv, timeout=240):
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR",
                                                            "MASTER_PORT")}
    env["RTW_BENCH_DRYRUN"] = "1"
    p = subprocess.run([sys.executable, os.path.join(REPO, "bench.py"), *argv], env=env, capture_output=True,
                       text=True, timeout=timeout, cwd=REPO)
    assert p.returncode == 0, p.stderr[-4000:]
    lines = [l for l in p.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, p.stdout  # rank 0 only
    return json.loads(lines[0])


@pytest.mark.parametrize("n", [2, 3])
def test_plain_invocation_spawns_n_ranks(n):
    r = run_bench("--gpus", str(n), "--steps", "2", "--warmup", "0")
    d = r["dist"]
    assert (d["backend"], d["world_size"]) == ("gloo", n)
    # per-rank timings and the trace imbalance (max / mean) of the GPU line
    assert len(d["rank_step_ms"]) == len(d["rank_trace_ms"]) == n
    assert d["imbalance"] >= 1.0 and abs(d["imbalance"] - max(d["rank_trace_ms"]) * n / sum(d["rank_trace_ms"])) < 0.05
    assert r["rows_interleaved_ok"]
    # configs[1] weak scaling: the 1200x675 frame at n x 500 spp
    assert (r["width"], r["height"], r["spp_frame"]) == (1200, 675, 500 * n)
    assert r["samples_all"] == 1200 * 675 * 500 * n
    # the full key set of the line, and no silent null evidence: every rank
    # renders the N=1 frame's samples within 1 %, so the N=1 launch's PMC
    # evidence applies and is named
    assert set(r) == {"dry_run", "dist", "width", "height", "spp_frame", "samples_all", "rows_interleaved_ok",
                      "evidence", "trace_ms_per_launch"}
    # the roofline's launch time is the slowest rank's (bench.roofline_launch_ms; VERDICT r5 ask 6), not
    # rank 0's: the dry run's rank r takes 1 + r/4 of the step
    assert r["trace_ms_per_launch"] == max(d["rank_trace_ms"]) > d["rank_trace_ms"][0]
    assert set(d) == {"backend", "world_size", "rank_step_ms", "rank_trace_ms", "imbalance"}
    ev = r["evidence"]
    assert ev["traffic"] and ev["valu_issue"]["valu_per_wave_iteration"] > 0 and ev["wf_traffic"], ev
    assert f"rows r::{n}" in ev["evidence_scope"]


def test_config2_is_strong_scaling_over_the_ranks():
    r = run_bench("--gpus", "2", "--config", "2")
    assert r["dist"]["world_size"] == 2 and r["rows_interleaved_ok"]
    assert (r["width"], r["height"], r["spp_frame"]) == (3840, 2160, 2000)
    assert r["samples_all"] == 3840 * 2160 * 2000


def test_single_gpu_does_not_spawn():
    import bench
    args = bench.parse_args(["--gpus", "1"])
    assert bench.maybe_launch(args, []) is None


def test_launch_command_shape():
    import bench
    cmd = bench.launch_command(["--gpus", "8", "--steps", "3"], 8, 29517)
    assert cmd[:3] == [sys.executable, "-m", "torch.distributed.run"]
    assert "--nproc-per-node=8" in cmd and "--master-addr=127.0.0.1" in cmd and "--master-port=29517" in cmd
    assert cmd[-3:] == ["--gpus", "8", "--steps", "3"][-3:]
    assert cmd[cmd.index("--master-port=29517") + 1].endswith("bench.py")
