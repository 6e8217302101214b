"""bench.py's rank launcher: `python3 bench.py --gpus N` starts N ranks itself
(one torch.distributed.run child, before any GPU call in the parent) unless it
already is a rank (WORLD_SIZE set)."""
import json
import os
import subprocess
import sys

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
