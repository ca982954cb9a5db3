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


def test_visible_gpu_count_without_hip(tmp_path):
    """The launcher's GPU count opens render nodes and applies the visibility masks; it never calls HIP."""
    import bench
    assert bench.visible_gpu_count(str(tmp_path / "absent"), env={}) == 0
    dri = tmp_path / "dri"
    dri.mkdir()
    for i in range(4):
        (dri / f"renderD{128 + i}").write_bytes(b"")
    (dri / "card0").write_bytes(b"")
    assert bench.visible_gpu_count(str(dri), env={}) == 4
    assert bench.visible_gpu_count(str(dri), env={"HIP_VISIBLE_DEVICES": "0,2"}) == 2
    assert bench.visible_gpu_count(str(dri), env={"HIP_VISIBLE_DEVICES": ""}) == 0
    assert bench.visible_gpu_count(str(dri), env={"ROCR_VISIBLE_DEVICES": "1", "HIP_VISIBLE_DEVICES": "0,1"}) == 1
    assert bench.visible_gpu_count(str(dri), env={"CUDA_VISIBLE_DEVICES": "0,7,1"}) == 1  # stops at ordinal 7
    with pytest.raises(RuntimeError):
        bench.visible_gpu_count(str(dri), env={"HIP_VISIBLE_DEVICES": "GPU-1234"})
    assert "torch.cuda" not in "".join(__import__("inspect").getsource(bench.visible_gpu_count).split('"""')[2:])


def test_metric_label_and_scaling_fields():
    """The N > 1 line is labelled by its own config and N, and carries a same-workload single-GPU time."""
    import argparse
    import bench
    a = argparse.Namespace(config=None, layers=None, heads=None, head_dim=None, seq=None)
    bench.resolve_config(a, 1)
    assert bench.metric_label(a, 1) == json.load(open(os.path.join(REPO, "BASELINE.json")))["metric"]
    a = argparse.Namespace(config=None, layers=None, heads=None, head_dim=None, seq=None)
    bench.resolve_config(a, 8)
    assert bench.metric_label(a, 8) == "prefill KV-compress GB/s + TTFT, Llama-2-7B S=64k, 8 GPUs"
    a = argparse.Namespace(config="cfg5", layers=None, heads=None, head_dim=None, seq=None)
    bench.resolve_config(a, 4)
    assert bench.metric_label(a, 4) == "prefill KV-compress GB/s + TTFT, Llama-2-13B S=32k, 4 GPUs"
    f = bench.scaling_fields(10.0, 27.0, 8, "x")
    assert f == {"single_gpu_ms_same_workload": 27.0, "speedup": 2.7, "strong_scaling_efficiency": 0.3375, "how": "x"}


def test_union_inputs_are_the_ranks_chunks():
    """The single-GPU reference of an N-rank line reads exactly the bytes the ranks hold."""
    import argparse
    import torch
    import bench
    a = argparse.Namespace(seq=40, heads=2, head_dim=4, layers=3)
    U = bench.union_inputs(a, "cpu", 3, torch.float32)
    P = max(1, min(120 // 5, 128))
    for j in range(3):
        g = torch.Generator(device="cpu")
        g.manual_seed(1234 + 7919 * j)
        for l in range(3):
            K, V, W = bench.synth_layer(l, 40, 2, 4, P, torch.float32, "cpu", g, row0=40 * j)
            sl = slice(40 * j, 40 * (j + 1))
            assert torch.equal(U[l][0][:, sl], K) and torch.equal(U[l][1][:, sl], V)
            assert torch.equal(U[l][2][:, :, sl], W)
    assert U[0][0].shape == (1, 120, 8) and U[0][2].shape == (1, 2, 120, P)


def test_param_sets_match_the_published_runs():
    import bench
    cov, pub = bench.PARAM_SETS["coverage"], bench.PARAM_SETS["pub16"]
    assert (pub["high_precision_bits"], pub["medium_precision_bits"], pub["low_precision_bits"]) == (16, 8, 4)
    assert (pub["alpha"], pub["beta"], pub["gamma"], pub["theta_h"], pub["theta_m"]) == (0.6, 0.2, 0.2, 0.6, 0.2)
    assert (cov["high_precision_bits"], cov["medium_precision_bits"], cov["low_precision_bits"]) == (8, 4, 2)
