"""bench.py's launch decision (VERDICT r05 "do this" #1): `--gpus N` either runs as
one rank of an N-rank job, starts the N ranks itself (torch.distributed.run as a child
process), or refuses; a 1-GPU line is never printed for an N-GPU request. CPU only:
the decision is made before any GPU call."""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import bench  # noqa: E402


def test_single_gpu_runs_in_process():
    assert bench.launch_decision(1, {}, 0, []) == ("run", 1)


def test_rank_of_driver_job_runs_with_its_world():
    env = {"WORLD_SIZE": "8", "RANK": "3", "LOCAL_RANK": "3"}
    assert bench.launch_decision(8, env, 8, ["--gpus", "8"]) == ("run", 8)


def test_world_size_disagreeing_with_gpus_is_refused():
    kind, why = bench.launch_decision(2, {"WORLD_SIZE": "4"}, 8, ["--gpus", "2"])
    assert kind == "error" and "WORLD_SIZE=4" in why
    kind, _ = bench.launch_decision(1, {"WORLD_SIZE": "2"}, 8, [])
    assert kind == "error"


def test_more_gpus_than_visible_is_refused():
    kind, why = bench.launch_decision(2, {}, 1, ["--gpus", "2"])
    assert kind == "error" and "1 GPU(s) visible" in why


def test_n_gpus_spawns_torchrun_child_with_same_arguments():
    argv = ["--gpus", "4", "--steps", "7", "--warmup", "2"]
    kind, cmd = bench.launch_decision(4, {}, 8, argv, master_port=29555)
    assert kind == "spawn"
    assert cmd[:3] == [sys.executable, "-m", "torch.distributed.run"]
    assert "--nproc-per-node=4" in cmd and "--master-addr=127.0.0.1" in cmd and "--master-port=29555" in cmd
    script = cmd.index(os.path.abspath(bench.__file__))
    assert cmd[script + 1:] == argv  # each rank sees WORLD_SIZE = 4 = --gpus: ("run", 4)


def _dry(*args, env=None):
    e = dict(os.environ)
    e.pop("WORLD_SIZE", None)
    e.update(env or {})
    p = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), *args, "--dry-run"], capture_output=True, text=True, env=e, timeout=300)
    return p.returncode, json.loads(p.stdout.strip().splitlines()[-1])


def test_dry_run_reports_world_size():
    rc, d = _dry()
    assert rc == 0 and d["decision"] == "run" and d["world_size"] == 1
    rc, d = _dry("--gpus", "2", env={"WORLD_SIZE": "2", "RANK": "0", "LOCAL_RANK": "0"})
    assert rc == 0 and d["decision"] == "run" and d["world_size"] == 2


def test_dry_run_without_gpus_fails_nonzero():
    # this container has no GPU: a 2-GPU request must fail, not print a 1-GPU line
    rc, d = _dry("--gpus", "2", env={"HIP_VISIBLE_DEVICES": ""})
    assert rc != 0 and d["decision"] == "error" and d["world_size"] is None
