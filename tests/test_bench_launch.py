"""bench.py launch paths on the CPU: the dispatch decision, and `--gpus N` from a plain
``python`` call starting N rank processes itself (the reference's default entry spawns its
ranks, multi_proc_single_gpu.py:284-285, :359), exercised with --dry-run (gloo rendezvous,
no GPU)."""
import importlib.util
import json
import os
import subprocess
import sys

import pytest

from conftest import REPO, free_port


def _bench():
    spec = importlib.util.spec_from_file_location("bench_mod", os.path.join(REPO, "bench.py"))
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    return mod


def test_launch_mode_decision():
    b = _bench()
    assert b.launch_mode(1, {}) == "single"
    assert b.launch_mode(8, {}) == "spawn"
    assert b.launch_mode(4, {"WORLD_SIZE": "4", "RANK": "1"}) == "worker"
    assert b.launch_mode(1, {"WORLD_SIZE": "1"}) == "single"
    with pytest.raises(SystemExit):
        b.launch_mode(8, {"WORLD_SIZE": "4"})


def _run(args, env=None):
    e = dict(os.environ)
    for k in ("RANK", "WORLD_SIZE", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT"):
        e.pop(k, None)
    e.update(env or {})
    return subprocess.run([sys.executable, os.path.join(REPO, "bench.py"), *args], cwd=REPO,
                          env=e, capture_output=True, text=True, timeout=300)


@pytest.mark.parametrize("n", [2, 4])
def test_self_spawn_emits_one_line(n):
    r = _run(["--gpus", str(n), "--dry-run"])
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-2000:]
    lines = [l for l in r.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, r.stdout
    d = json.loads(lines[0])
    assert d["n_gpus"] == n and d["launch"] == "spawned"
    assert d["rank_sum"] == n * (n - 1) / 2          # every rank joined the one group


def test_launcher_route_still_works():
    r = subprocess.run([sys.executable, "-m", "torch.distributed.run", "--nnodes=1",
                        "--nproc-per-node", "2", "--master-addr", "127.0.0.1", "--master-port",
                        str(free_port()), os.path.join(REPO, "bench.py"), "--gpus", "2",
                        "--dry-run"], cwd=REPO, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-2000:]
    lines = [l for l in r.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1
    d = json.loads(lines[0])
    assert d["n_gpus"] == 2 and d["launch"] == "launcher" and d["rank_sum"] == 1


def test_failing_rank_fails_the_job(tmp_path):
    """A rank that dies takes the job down with a non-zero status (the others are stopped,
    no hang): WORLD_SIZE mismatch makes every rank exit at once."""
    r = _run(["--gpus", "2", "--dry-run"], env={"PDM_BENCH_FAIL_RANK": "1"})
    assert r.returncode != 0
    assert "rank 1 exited" in r.stderr
