"""bench.py's rank launcher: `python3 bench.py --gpus N` starts N ranks itself
(one torch.distributed.run child, before any GPU call in the parent) unless it
already is a rank (WORLD_SIZE set)."""
import json
import os
import subprocess
import sys

import pytest

from conftest import ROOT

sys.path.insert(0, ROOT)
import bench  # noqa: E402


def test_launcher_decision():
    assert bench.launcher_command(["--gpus", "1"], 1, {}) is None
    assert bench.launcher_command(["--gpus", "8"], 8, {"WORLD_SIZE": "8"}) is None
    cmd = bench.launcher_command(["--gpus", "8", "--steps", "3"], 8, {"RNVP_BENCH_PORT": "29777"})
    assert cmd[:3] == [sys.executable, "-m", "torch.distributed.run"]
    assert cmd[cmd.index("--nproc-per-node") + 1] == "8"
    assert cmd[cmd.index("--master-addr") + 1] == "127.0.0.1"
    assert cmd[cmd.index("--master-port") + 1] == "29777"
    assert cmd[-4:] == ["--gpus", "8", "--steps", "3"]
    assert os.path.samefile(cmd[-5], os.path.join(ROOT, "bench.py"))
    # a free port is picked when none is given
    cmd = bench.launcher_command(["--gpus", "2"], 2, {})
    assert int(cmd[cmd.index("--master-port") + 1]) > 0


def test_launcher_spawns_ranks_on_cpu():
    """the real launcher path, stopped in each rank before the GPU"""
    env = dict(os.environ)
    env.pop("WORLD_SIZE", None)
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--launch-check"],
                       capture_output=True, text=True, timeout=300, env=env, cwd=ROOT)
    assert r.returncode == 0, r.stderr[-2000:]
    lines = [json.loads(x) for x in r.stdout.splitlines() if x.startswith("{")]
    assert sorted(d["rank"] for d in lines) == [0, 1]
    assert all(d["world_size"] == 2 and d["master"] == "127.0.0.1" for d in lines)


def test_rank_refuses_mismatched_world():
    env = dict(os.environ, WORLD_SIZE="2", RANK="0", LOCAL_RANK="0")
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "4", "--launch-check"],
                       capture_output=True, text=True, timeout=300, env=env, cwd=ROOT)
    assert r.returncode != 0 and "WORLD_SIZE=2" in r.stderr


@pytest.mark.gpu
def test_two_rank_line_is_complete():
    """`bench.py --gpus 2` (ranks sharing the box's GPU over gloo, a small
    custom model): rank 0's single JSON line carries the whole-job value, the
    roofline, the data-parallel diagnostics AND the CPU baseline -- what the
    driver's multi-GPU runs record."""
    env = dict(os.environ, RNVP_BENCH_BACKEND="gloo")
    env.pop("WORLD_SIZE", None)
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--steps", "1", "--warmup", "1",
                        "--size", "32", "--res-blocks", "1", "--base-dim", "8", "--batch", "4", "--no-secondary",
                        "--cpu-steps", "1", "--cpu-batch", "2"],
                       capture_output=True, text=True, timeout=900, env=env, cwd=ROOT)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [json.loads(x) for x in r.stdout.splitlines() if x.startswith("{")]
    assert len(lines) == 1, r.stdout[-2000:]
    d = lines[0]
    assert d["n_gpus"] == 2 and d["value"] > 0 and d["config"]["global_batch"] == 8
    assert d["roofline"]["bound"] in ("hbm", "mfma") and d["roofline"]["peak"] > 0
    assert d["dp"]["world_size_rccl"] == 2 and len(d["dp"]["rank_ms_per_step"]) == 2
    cb = d["cpu_baseline"]
    assert cb and cb["value"] > 0 and cb["cores"] >= 1 and cb["kind"] == "port"
