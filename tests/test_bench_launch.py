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


def _line(r):
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-2000:]
    lines = [l for l in r.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, r.stdout
    return json.loads(lines[0])


def test_calibration_without_faults_picks_fastest():
    d = _line(_run(["--gpus", "2", "--dry-run"]))
    assert d["config"]["grad_transport"] == "rccl-early"       # the cheapest stand-in
    assert len(d["config"]["transport_calibration_ms_per_step"]) == 5
    assert d["comm"]["fallback"] == []


def test_calibration_drops_candidates_failing_on_one_rank():
    """Each kind of failure on ONE rank (an exception in setup / timed steps, a device sync
    that hits its deadline, replicas that drift apart) drops that candidate on EVERY rank,
    with the reason recorded; the fastest survivor is chosen and one JSON line printed."""
    faults = "1:rccl-early:timed,0:rccl:diverge,1:xgmi:hang,0:xgmi-noxchg:setup"
    d = _line(_run(["--gpus", "2", "--dry-run"], env={"PDM_CALIB_FAULT": faults}))
    assert d["config"]["grad_transport"] == "rccl-nocarry"
    assert list(d["config"]["transport_calibration_ms_per_step"]) == ["rccl-nocarry"]
    notes = " | ".join(d["comm"]["fallback"])
    for what in ("rccl-early failed calibration: timed on rank 1",
                 "rccl failed calibration: replicas diverged",
                 "xgmi failed calibration: warm on rank 1",
                 "xgmi-noxchg failed calibration: setup on rank 0"):
        assert what in notes, notes


def test_calibration_failure_in_check_phase_four_ranks():
    d = _line(_run(["--gpus", "4", "--dry-run"], env={"PDM_CALIB_FAULT": "3:rccl-early:check"}))
    assert d["config"]["grad_transport"] == "rccl"
    assert "rccl-early failed calibration: check on rank 3" in d["comm"]["fallback"][0]


def test_calibration_with_no_survivor_is_fatal():
    faults = ",".join(f"1:{n}:setup" for n in ("xgmi", "xgmi-noxchg", "rccl", "rccl-nocarry",
                                                 "rccl-early"))
    r = _run(["--gpus", "2", "--dry-run"], env={"PDM_CALIB_FAULT": faults})
    assert r.returncode != 0
    assert "no step structure survived" in r.stderr


class _Red:
    """A stand-in reducer for step_candidates (xgmi: whether the conv bucket is one-shot)."""
    def __init__(self, one_shot=True):
        self.one_shot = one_shot

    def exchange_ok(self, bucket):
        return self.one_shot


def test_candidates_at_most_four_per_batch(monkeypatch):
    """The automatic calibration list: at most four structures per batch, each with its N>1
    argument (bench.step_candidates); 'side' and 'zero' only when forced."""
    b = _bench()
    monkeypatch.delenv("PDM_RCCL_MODE", raising=False)
    reds = {"xgmi": _Red(), "rccl": _Red()}
    big = [c[0] for c in b.step_candidates(reds, "cnn", 256, lambda r: True)]
    small = [c[0] for c in b.step_candidates(reds, "cnn", 32, lambda r: True)]
    assert big == ["xgmi", "xgmi-noxchg", "rccl-nocarry", "rccl"]
    assert small == ["xgmi", "xgmi-noxchg", "rccl-nocarry", "rccl-early"]
    # the xgmi fallback without the in-launch exchange is a distinct structure only when the
    # exchange is possible (one-shot conv channel) and on (StepStructure.xgmi_exchange)
    reds2 = {"xgmi": _Red(one_shot=False), "rccl": _Red()}
    assert [c[0] for c in b.step_candidates(reds2, "cnn", 256, lambda r: True)] == \
        ["xgmi", "rccl-nocarry", "rccl"]
    assert [c[0] for c in b.step_candidates(reds, "cnn", 256, lambda r: True,
                                            exchange_step=False)] == \
        ["xgmi", "rccl-nocarry", "rccl"]
    flags = {c[0]: c[3] for c in b.step_candidates(reds, "cnn", 256, lambda r: True)}
    assert flags["xgmi"] is True and flags["xgmi-noxchg"] is False
    # the gloo rehearsal's reducer is a candidate of its own
    assert [c[0] for c in b.step_candidates({"xgmi": _Red(), "torch": _Red()}, "cnn", 256,
                                            lambda r: True)] == ["xgmi", "xgmi-noxchg", "torch"]


def test_zero_and_side_are_never_automatic_candidates(monkeypatch):
    b = _bench()
    reds = {"xgmi": _Red(), "rccl": _Red()}
    monkeypatch.delenv("PDM_RCCL_MODE", raising=False)
    names = [c[0] for c in b.step_candidates(reds, "cnn", 256, lambda r: True)]
    assert "rccl-zero" not in names and "rccl-side" not in names
    monkeypatch.setenv("PDM_RCCL_MODE", "zero")
    assert [c[0] for c in b.step_candidates(reds, "cnn", 256, lambda r: True)] == \
        ["xgmi", "xgmi-noxchg", "rccl-zero"]
    assert [c[0] for c in b.step_candidates(reds, "cnn", 256, lambda r: False)] == \
        ["xgmi", "xgmi-noxchg"]
    monkeypatch.setenv("PDM_RCCL_MODE", "side")
    assert [c[0] for c in b.step_candidates(reds, "cnn", 32, lambda r: True)] == \
        ["xgmi", "xgmi-noxchg", "rccl-side"]
