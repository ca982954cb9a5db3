"""CPU: bench.py's multi-GPU launcher and workload selection (no GPU call is made).

`python bench.py --gpus N` outside torch.distributed.run must start N ranks itself through a
torch.distributed.run child process, fail fast when fewer than N GPUs are visible, and the N > 1
workload must be BASELINE's cfg4 (S_total = 65536 split over the ranks) or cfg5."""
import json
import os
import subprocess
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)


def _run(*argv, env=None):
    e = dict(os.environ)
    e.pop("WORLD_SIZE", None)
    e.update(env or {})
    return subprocess.run([sys.executable, os.path.join(REPO, "bench.py"), *argv], capture_output=True, text=True,
                          env=e, timeout=300)


def test_dry_run_prints_the_torchrun_child_command():
    r = _run("--gpus", "8", "--steps", "4", "--warmup", "2", "--launch-dry-run")
    assert r.returncode == 0, r.stderr
    doc = json.loads(r.stdout.strip().splitlines()[-1])
    cmd = doc["launch"]
    assert cmd[:3] == [sys.executable, "-m", "torch.distributed.run"]
    assert "--nnodes=1" in cmd and "--nproc-per-node=8" in cmd
    assert cmd[cmd.index("--master-addr") + 1] == "127.0.0.1"
    assert int(cmd[cmd.index("--master-port") + 1]) > 0
    i = cmd.index(os.path.join(REPO, "bench.py"))
    assert cmd[i + 1:] == ["--gpus", "8", "--steps", "4", "--warmup", "2"]  # the flag itself is not forwarded
    assert isinstance(doc["visible_gpus"], int)


def test_too_few_gpus_fails_fast_and_nonzero():
    # this container sees no GPU: a --gpus 2 run must not fall back to one device
    r = _run("--gpus", "2", env={"HIP_VISIBLE_DEVICES": ""})
    assert r.returncode == 2
    assert "needs 2 visible GPUs" in r.stderr
    assert r.stdout.strip() == ""


def test_world_size_mismatch_is_refused():
    r = _run("--gpus", "4", env={"WORLD_SIZE": "2", "RANK": "0", "LOCAL_RANK": "0"})
    assert r.returncode == 2
    assert "WORLD_SIZE 2" in r.stderr


@pytest.mark.parametrize("world,config,want", [
    (1, None, ("cfg3", 32, 32, 128, 16384)),
    (2, None, ("cfg4", 32, 32, 128, 32768)),
    (8, None, ("cfg4", 32, 32, 128, 8192)),
    (8, "cfg5", ("cfg5", 40, 40, 128, 4096)),
    (1, "cfg5", ("cfg5", 40, 40, 128, 32768)),
    (1, "cfg4", ("cfg4", 32, 32, 128, 65536)),
])
def test_config_resolution(world, config, want):
    import argparse
    import bench
    a = argparse.Namespace(config=config, layers=None, heads=None, head_dim=None, seq=None)
    bench.resolve_config(a, world)
    assert (a.config, a.layers, a.heads, a.head_dim, a.seq) == want
    assert a.seq * world == bench.CONFIGS[a.config]["seq_total"]


def test_config_that_does_not_split_is_refused():
    import argparse
    import bench
    with pytest.raises(SystemExit):
        bench.resolve_config(argparse.Namespace(config="cfg4", layers=None, heads=None, head_dim=None, seq=None), 3)
