"""bench.py --gpus N starts and checks its ranks itself, on the CPU:
the launcher, the WORLD_SIZE / --gpus consistency check, and the world size the process group
reports, through --dry-run (process group only, no GPU work)."""
import json
import os
import subprocess
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
import bench  # noqa: E402


def _env(**kw):
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR",
                                                            "MASTER_PORT", "LOCAL_WORLD_SIZE")}
    env.update(kw)
    return env


def test_resolve_world():
    a = bench.parse(["--gpus", "4"])
    assert bench.resolve_world(a, {}) == (4, True)
    assert bench.resolve_world(a, {"WORLD_SIZE": "4"}) == (4, False)
    with pytest.raises(SystemExit):
        bench.resolve_world(a, {"WORLD_SIZE": "2"})
    assert bench.resolve_world(bench.parse([]), {}) == (1, False)
    assert bench.resolve_world(bench.parse([]), {"WORLD_SIZE": "8"}) == (8, False)
    assert bench.resolve_world(bench.parse(["--gpus", "1"]), {}) == (1, False)


def test_rank_launch_cmd_is_the_drivers_form():
    cmd = bench.rank_launch_cmd(8, ["--gpus", "8", "--steps", "3"], 29555)
    assert cmd[1:3] == ["-m", "torch.distributed.run"]
    assert "--nproc-per-node=8" in cmd and "--master-addr=127.0.0.1" in cmd and "--master-port=29555" in cmd
    assert cmd[-4:] == ["--gpus", "8", "--steps", "3"] and cmd[-5].endswith("bench.py")


def test_gpus_mismatch_with_launcher_exits_nonzero():
    r = subprocess.run([sys.executable, os.path.join(REPO, "bench.py"), "--gpus", "4", "--dry-run"],
                       env=_env(WORLD_SIZE="2", RANK="0", LOCAL_RANK="0"), capture_output=True, text=True, timeout=300)
    assert r.returncode != 0
    assert "WORLD_SIZE=2" in r.stderr


def test_gpus_2_starts_two_ranks_without_a_launcher():
    r = subprocess.run([sys.executable, os.path.join(REPO, "bench.py"), "--gpus", "2", "--dry-run"],
                       env=_env(MMU_BENCH_BACKEND="gloo"), capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-2000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout
    out = json.loads(lines[0])
    assert out["n_gpus"] == 2 and out["world_size_reported"] == 2 and sorted(out["ranks_seen"]) == [0, 1]
