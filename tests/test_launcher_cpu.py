"""bench.py's own N-rank launcher (bin/pool.py:61-91: one replica per GPU), on CPU.

`python bench.py --gpus N` must start N ranks itself (the driver's BENCH/SCALE command has no outer launcher),
refuse to oversubscribe a GPU, and agree with an outer torch.distributed.run when there is one."""
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import bench  # noqa: E402


def _env(**kw):
    return {k: str(v) for k, v in kw.items()}


def test_plan_single_gpu_runs_in_process():
    assert bench.launch_plan(1, _env(), 1, [], "bench.py", 1234) == ("rank", None)
    assert bench.launch_plan(1, _env(), 8, [], "bench.py", 1234) == ("rank", None)


def test_plan_spawns_n_ranks_with_the_same_arguments():
    kind, cmd = bench.launch_plan(8, _env(), 8, ["--gpus", "8", "--steps", "3"], "/x/bench.py", 29555)
    assert kind == "spawn"
    assert cmd[:3] == [sys.executable, "-m", "torch.distributed.run"]
    assert "--nproc-per-node=8" in cmd and "--nnodes=1" in cmd and "--master-port=29555" in cmd
    assert cmd[cmd.index("--master-addr") + 1] == "127.0.0.1"
    assert cmd[-5:] == ["/x/bench.py", "--gpus", "8", "--steps", "3"]


def test_plan_refuses_more_ranks_than_gpus():
    kind, msg = bench.launch_plan(2, _env(), 1, [], "bench.py", 1)
    assert kind == "error" and "exceeds" in msg
    kind, msg = bench.launch_plan(8, _env(), 0, [], "bench.py", 1)
    assert kind == "error"


def test_plan_rehearsal_runs_n_ranks_on_one_gpu():
    kind, cmd = bench.launch_plan(2, _env(FO_DIST_REHEARSAL=1), 1, [], "bench.py", 1)
    assert kind == "spawn" and "--nproc-per-node=2" in cmd


def test_plan_under_an_outer_launcher():
    # a rank of torch.distributed.run: runs in process when --gpus agrees with WORLD_SIZE
    assert bench.launch_plan(4, _env(WORLD_SIZE=4, LOCAL_RANK=3), 8, [], "b", 1) == ("rank", None)
    kind, msg = bench.launch_plan(2, _env(WORLD_SIZE=4, LOCAL_RANK=0), 8, [], "b", 1)
    assert kind == "error" and "WORLD_SIZE=4" in msg
    # the default --gpus 1 under a 2-rank launcher is a disagreement too (never two ranks reporting n_gpus 1)
    assert bench.launch_plan(1, _env(WORLD_SIZE=2, LOCAL_RANK=0), 8, [], "b", 1)[0] == "error"
    # a local rank beyond the visible devices
    kind, msg = bench.launch_plan(2, _env(WORLD_SIZE=2, LOCAL_RANK=1), 1, [], "b", 1)
    assert kind == "error" and "LOCAL_RANK=1" in msg
    assert bench.launch_plan(2, _env(WORLD_SIZE=2, LOCAL_RANK=1, FO_DIST_REHEARSAL=1), 1, [], "b", 1) == ("rank", None)


def test_topology_labels_a_rehearsal_as_one_gpu(monkeypatch):
    monkeypatch.delenv("FO_DIST_REHEARSAL", raising=False)
    t = bench.topology(4)
    assert t["n_gpus"] == 4 and t["physical_gpus"] == 4 and t["ranks"] == 4 and t["rehearsal"] is None
    monkeypatch.setenv("FO_DIST_REHEARSAL", "1")
    t = bench.topology(2)
    assert t["n_gpus"] == 1 and t["physical_gpus"] == 1 and t["ranks"] == 2 and t["rehearsal"]


def _clean_env():
    env = dict(os.environ)
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT", "FO_DIST_REHEARSAL"):
        env.pop(k, None)
    return env


def test_spawned_ranks_see_their_rank_and_device():
    """The real spawn path (torch.distributed.run child ranks, gloo), stopped before any GPU call."""
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--launch-selftest"],
                       env=_clean_env(), capture_output=True, text=True, timeout=180)
    assert r.returncode == 0, r.stderr[-2000:]
    lines = [json.loads(x) for x in r.stdout.splitlines() if x.startswith("{")]
    assert len(lines) == 1, r.stdout   # rank 0 alone prints
    got = lines[0]["launch_selftest"]
    assert [g["rank"] for g in got] == [0, 1]
    assert [g["local_rank"] for g in got] == [0, 1]
    assert {g["world"] for g in got} == {2}
    assert [g["device"] for g in got] == ["cuda:0", "cuda:1"]
    assert {g["master"].split(":")[0] for g in got} == {"127.0.0.1"}


@pytest.mark.skipif(__import__("torch").cuda.device_count() >= 2, reason="needs a host with fewer than 2 GPUs")
def test_two_gpus_on_a_smaller_host_fail_fast():
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--steps", "1"],
                       env=_clean_env(), capture_output=True, text=True, timeout=120)
    assert r.returncode == 2
    assert "refusing" in r.stderr and r.stdout.strip() == ""
