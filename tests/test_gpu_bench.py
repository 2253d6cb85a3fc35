"""bench.py driver contract on one MI355X: one JSON line with the BASELINE metric/config."""
import json
import os
import subprocess
import sys

import pytest

from conftest import REPO

pytestmark = pytest.mark.gpu


def test_bench_json_contract(gpu):
    r = subprocess.run([sys.executable, os.path.join(REPO, "bench.py"), "--steps", "20",
                        "--warmup", "3"], cwd=REPO, capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-2000:]
    lines = [l for l in r.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, r.stdout
    d = json.loads(lines[0])
    assert d["metric"] == json.load(open(os.path.join(REPO, "BASELINE.json")))["metric"]
    assert d["n_gpus"] == 1 and d["steps"] == 20 and d["warmup"] == 3
    assert d["unit"] == "images/sec" and d["higher_is_better"] is True
    assert d["scaling"] == "weak" and d["dtype"] == "bf16" and d["data"].startswith("synthetic")
    assert d["config"]["model"] == "mnist_cnn" and d["config"]["parallelism"] == "dp1"
    assert d["value"] > 0 and d["ms_per_step"] > 0
    # value is the whole-job images/sec of the timed steps: the reference's epoch sequence
    # (full batches, then the 96-image ragged tail of 60000 / 256) with a boundary inside
    c = d["config"]
    assert c["epoch_steps"] == 235 and c["tail_batch_per_rank"] == 96
    assert c["images_timed"] == 19 * 256 + 96
    el = d["ms_per_step"] * d["steps"] / 1e3
    assert abs(d["value"] - c["images_timed"] / el) / d["value"] < 0.01
    assert d["launch"] == "single" and isinstance(d["knobs"], dict)
    assert d["vs_baseline"] > 1.0
    # an epoch boundary (next epoch's sampler order: upload + gather) falls in the window
    assert d["config"]["epoch_boundaries_timed"] >= 1
    assert d["comm"]["world_size"] == 1
    # N = 1: the strong-scaling (reference DDP) configuration is the same 256-image step
    assert d["strong"]["global_batch"] == 256 and d["strong"]["batch_per_rank"] == 256


def test_bench_transport_calibration(gpu):
    """PDM_FORCE_COMM=1 at N=1 runs the multi-GPU step structure, so both gradient
    transports (direct xGMI, RCCL) are built, calibrated on the real step, and the faster
    one is timed."""
    env = dict(os.environ, PDM_FORCE_COMM="1")
    r = subprocess.run([sys.executable, os.path.join(REPO, "bench.py"), "--steps", "20",
                        "--warmup", "3"], cwd=REPO, env=env, capture_output=True, text=True,
                       timeout=600)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-2000:]
    d = json.loads([l for l in r.stdout.splitlines() if l.startswith("{")][-1])
    cal = d["config"]["transport_calibration_ms_per_step"]
    # at most four structures per batch ('zero' and 'side' only when PDM_RCCL_MODE forces them)
    assert set(cal) == {"xgmi", "xgmi-noxchg", "rccl-nocarry", "rccl"}, cal
    assert d["comm"].get("fallback", []) == []
    assert d["config"]["grad_transport"] == min(cal, key=cal.get)
    # what the data plane saw: a 1-rank RCCL communicator, no xGMI peer to map
    assert d["comm"]["rccl_comm_count"] == 1
    assert d["comm"]["xgmi_peers_mapped"] == 0


def test_bench_two_rank_flow_rehearsal(gpu):
    """The N>1 driver path (torch.distributed.run, env rendezvous, barrier + max over ranks,
    rank-0 JSON) rehearsed with 2 ranks on one GPU over a gloo data plane."""
    from conftest import free_port
    env = dict(os.environ, PDM_SHARE_DEVICE="1", PDM_BENCH_BACKEND="gloo")
    r = subprocess.run([sys.executable, "-m", "torch.distributed.run", "--nnodes=1",
                        "--nproc-per-node", "2", "--master-addr", "127.0.0.1", "--master-port",
                        str(free_port()), os.path.join(REPO, "bench.py"), "--gpus", "2",
                        "--steps", "10", "--warmup", "2"], cwd=REPO, env=env,
                       capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-2000:]
    lines = [l for l in r.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, r.stdout
    d = json.loads(lines[0])
    assert d["n_gpus"] == 2 and d["config"]["parallelism"] == "dp2"
    assert d["config"]["global_batch"] == 2 * d["config"]["batch_per_rank"]
    # strong scaling = the reference's split of the node batch (S:174): 128 per rank
    assert d["strong"]["batch_per_rank"] == 128 and d["strong"]["global_batch"] == 256
    assert d["strong"]["value"] > 0


def test_bench_two_rank_xgmi_rehearsal(gpu):
    """The N>1 bench with the direct xGMI gradient transport: 2 ranks on one GPU (hipIpc
    between the two processes, gloo control plane)."""
    from conftest import free_port
    env = dict(os.environ, PDM_SHARE_DEVICE="1", PDM_BENCH_BACKEND="gloo", PDM_COMM="xgmi")
    r = subprocess.run([sys.executable, "-m", "torch.distributed.run", "--nnodes=1",
                        "--nproc-per-node", "2", "--master-addr", "127.0.0.1", "--master-port",
                        str(free_port()), os.path.join(REPO, "bench.py"), "--gpus", "2",
                        "--steps", "24", "--warmup", "4"], cwd=REPO, env=env,
                       capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-2000:]
    lines = [l for l in r.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, r.stdout
    d = json.loads(lines[0])
    assert d["n_gpus"] == 2 and d["config"]["grad_transport"] == "xgmi"


def test_bench_self_spawn_rehearsal(gpu):
    """`python bench.py --gpus 2` with no launcher starts its two ranks itself (before any GPU
    call) and forwards rank 0's one JSON line; rehearsed on one GPU over gloo."""
    env = dict(os.environ, PDM_SHARE_DEVICE="1", PDM_BENCH_BACKEND="gloo")
    for k in ("RANK", "WORLD_SIZE", "LOCAL_RANK"):
        env.pop(k, None)
    r = subprocess.run([sys.executable, os.path.join(REPO, "bench.py"), "--gpus", "2",
                        "--steps", "20", "--warmup", "5"], cwd=REPO, env=env,
                       capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-2000:]
    lines = [l for l in r.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, r.stdout
    d = json.loads(lines[0])
    assert d["n_gpus"] == 2 and d["launch"] == "spawned"
    assert d["config"]["parallelism"] == "dp2" and d["strong"]["batch_per_rank"] == 128
    knobs = {k: v for k, v in d["knobs"].items() if k != "PDM_EXT_PATH"}   # (debug-build runs)
    assert knobs == {"PDM_BENCH_BACKEND": "gloo", "PDM_SHARE_DEVICE": "1"}


def test_bench_calibration_survives_failing_candidates(gpu):
    """Calibration on the real step with injected faults (an exception while the xgmi step
    is captured, one in xgmi-noxchg's check): those candidates are dropped and recorded, the
    replicas restored from rank 0 (1-rank RCCL broadcast, bf16 copies re-derived), and the
    fastest survivor timed."""
    env = dict(os.environ, PDM_FORCE_COMM="1",
               PDM_CALIB_FAULT="0:xgmi:setup,0:xgmi-noxchg:check")
    r = subprocess.run([sys.executable, os.path.join(REPO, "bench.py"), "--steps", "20",
                        "--warmup", "3", "--scaling", "weak"], cwd=REPO, env=env,
                       capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-2000:]
    d = json.loads([l for l in r.stdout.splitlines() if l.startswith("{")][-1])
    cal = d["config"]["transport_calibration_ms_per_step"]
    assert set(cal) == {"rccl", "rccl-nocarry"}, cal
    assert d["config"]["grad_transport"] in cal
    notes = " | ".join(d["comm"]["fallback"])
    for name in ("xgmi", "xgmi-noxchg"):
        assert f"{name} failed calibration" in notes, notes
    assert d["value"] > 0


def test_bench_calibration_survives_rccl_abort(gpu):
    """A device stall past a candidate's host deadline on the RCCL data plane (a bounded spin
    kernel queued behind rccl's steps): the deadline aborts the RCCL communicator, the
    candidate is dropped, every rank drains its device and joins a fresh communicator
    (RcclComm.revive), the RCCL reducer is rebuilt on it, and calibration and the timed run
    continue over the new one."""
    env = dict(os.environ, PDM_FORCE_COMM="1", PDM_XGMI_TIMEOUT="2", PDM_CALIB_TIMEOUT_S="2",
               PDM_CALIB_FAULT="0:rccl:spin")
    r = subprocess.run([sys.executable, os.path.join(REPO, "bench.py"), "--steps", "20",
                        "--warmup", "3", "--scaling", "weak"], cwd=REPO, env=env,
                       capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-2000:]
    d = json.loads([l for l in r.stdout.splitlines() if l.startswith("{")][-1])
    cal = d["config"]["transport_calibration_ms_per_step"]
    assert set(cal) == {"xgmi", "xgmi-noxchg", "rccl-nocarry"}, cal
    notes = " | ".join(d["comm"]["fallback"])
    assert "rccl failed calibration" in notes and "did not finish within" in notes, notes
    assert "re-created after an abort" in r.stderr
    assert d["comm"]["rccl_comm_count"] == 1        # the revived communicator answers
    assert d["value"] > 0


def test_bench_calibration_survives_xgmi_device_hang(gpu):
    """A real device hang in one candidate on one rank: in the two-rank rehearsal (ranks
    sharing the GPU, gloo data plane, xgmi calibrated against it) rank 1 never launches its
    persistent xGMI collective, so rank 0's collective waits for rank 1's buckets and rank 1's
    optimizer for its reduced buckets.  Those device waits give up at PDM_XGMI_TIMEOUT (error
    words, fail-fast), before the host deadline (timeout + PDM_CALIB_TIMEOUT_S), so nothing
    is aborted: the candidate is dropped on both ranks from its error word, the replicas are
    restored from rank 0, the run goes on with the gloo reducer and ends with one JSON line
    naming xgmi in comm.fallback and bit-equal replicas (bench.py checks the fingerprints)."""
    from conftest import free_port
    env = dict(os.environ, PDM_SHARE_DEVICE="1", PDM_BENCH_BACKEND="gloo",
               PDM_XGMI_TIMEOUT="3", PDM_CALIB_TIMEOUT_S="20",
               PDM_CALIB_FAULT="1:xgmi:devhang")
    r = subprocess.run([sys.executable, "-m", "torch.distributed.run", "--nnodes=1",
                        "--nproc-per-node", "2", "--master-addr", "127.0.0.1", "--master-port",
                        str(free_port()), os.path.join(REPO, "bench.py"), "--gpus", "2",
                        "--steps", "10", "--warmup", "2", "--scaling", "weak"], cwd=REPO,
                       env=env, capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-2000:]
    lines = [l for l in r.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, r.stdout
    d = json.loads(lines[0])
    notes = " | ".join(d["comm"]["fallback"])
    assert "xgmi failed calibration" in notes and "timed out" in notes, notes
    assert "did not finish within" not in notes            # no host deadline fired
    assert d["config"]["grad_transport"] == "torch"
    assert list(d["config"]["transport_calibration_ms_per_step"]) == ["torch"]
    assert d["value"] > 0


def test_bench_emulated_rank_pricing(gpu):
    """PDM_EMULATE_WS=8 with a forced 1-rank communicator: the per-rank chain of an 8-rank job
    at the reference's per-rank batch (256 / 8 = 32), the fc1 update sharded over 16 rows."""
    env = dict(os.environ, PDM_FORCE_COMM="1", PDM_EMULATE_WS="8", PDM_RCCL_MODE="zero",
               PDM_COMM="rccl")
    r = subprocess.run([sys.executable, os.path.join(REPO, "bench.py"), "--steps", "20",
                        "--warmup", "3", "--scaling", "weak", "--batch-per-rank", "32"],
                       cwd=REPO, env=env, capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-2000:]
    d = json.loads([l for l in r.stdout.splitlines() if l.startswith("{")][-1])
    c = d["config"]
    assert c["emulated_world_size"] == 8 and c["fc1_update_sharded"] is True
    assert c["grad_transport"] == "rccl-zero" and c["batch_per_rank"] == 32
    assert d["value"] > 0
