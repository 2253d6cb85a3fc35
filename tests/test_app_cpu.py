"""End-to-end CLI runs on CPU/gloo: stdout contract, checkpoints, resume, evaluate, spawn,
world-size invariance (BASELINE config 1)."""
import os
import re
import subprocess
import sys

import pytest
import torch

from conftest import REPO, free_port

EPOCH_RE = re.compile(r"^Epoch: (\d+)/(\d+), train loss: (\d+\.\d{6}), train acc: (\d+\.\d{2})%, "
                      r"test loss: (\d+\.\d{6}), test acc: (\d+\.\d{2})%\.$")


def run_cli(args, cwd, timeout=300):
    env = dict(os.environ)
    env["PYTHONPATH"] = REPO + os.pathsep + env.get("PYTHONPATH", "")
    cmd = [sys.executable, os.path.join(REPO, "multi_proc_single_gpu.py"), "--device", "cpu",
           "--backend", "gloo", "-i", f"tcp://127.0.0.1:{free_port()}", "--synthetic"] + args
    r = subprocess.run(cmd, cwd=cwd, env=env, capture_output=True, text=True, timeout=timeout)
    assert r.returncode == 0, r.stdout + r.stderr
    return r.stdout


def test_train_checkpoint_resume_evaluate(tmp_path):
    out = run_cli(["--epochs", "2", "--synthetic-size", "2048", "--seed", "3"], tmp_path)
    lines = out.splitlines()
    assert any(l.startswith("Namespace(") for l in lines)
    assert "rank: 0, device count: 1, workers:4" in lines
    epochs = [l for l in lines if l.startswith("Epoch:")]
    assert len(epochs) == 2 and all(EPOCH_RE.match(l) for l in epochs), epochs
    ck = tmp_path / "checkpoints"
    assert (ck / "checkpoint_0.pth.tar").exists() and (ck / "checkpoint_1.pth.tar").exists()
    assert (ck / "model_best.pth.tar").exists()
    sd = torch.load(ck / "checkpoint_1.pth.tar", weights_only=True)
    assert sd["epoch"] == 2 and 0 <= sd["best_acc"] <= 1
    assert list(sd["state_dict"]) == ["module.fc.weight", "module.fc.bias"]
    st = sd["optimizer"]["state"]
    assert float(st[0]["step"]) == 16.0      # 2 epochs x 8 steps of 256

    # resume -> continues at epoch 2
    out = run_cli(["--epochs", "3", "--synthetic-size", "2048", "--resume",
                   str(ck / "checkpoint_1.pth.tar")], tmp_path)
    assert f"=> loading checkpoint '{ck / 'checkpoint_1.pth.tar'}'" in out
    assert "(epoch 2)" in out
    ep = [l for l in out.splitlines() if l.startswith("Epoch:")]
    assert len(ep) == 1 and ep[0].startswith("Epoch: 2/3,")

    # evaluate best -> same test line as the epoch that produced it
    out = run_cli(["--evaluate", "--resume", str(ck / "checkpoint_1.pth.tar")], tmp_path)
    test_line = [l for l in out.splitlines() if l.startswith("test loss:")]
    assert len(test_line) == 1
    ep1 = [l for l in epochs if l.startswith("Epoch: 1/2")][0]
    assert test_line[0].split("test loss: ")[1] == ep1.split("test loss: ")[1]


def test_missing_checkpoint_message(tmp_path):
    out = run_cli(["--evaluate", "--resume", "nope.pth.tar"], tmp_path)
    assert "=> no checkpoint found at 'nope.pth.tar'" in out
    assert re.search(r"^test loss: \d+\.\d{6}, test acc: \d+\.\d{2}%\.$", out, re.M)


@pytest.mark.slow
def test_spawn_two_ranks_and_world_size_invariance(tmp_path):
    d1, d2 = tmp_path / "ws1", tmp_path / "ws2"
    d1.mkdir()
    d2.mkdir()
    common = ["--epochs", "1", "--synthetic-size", "2048", "--seed", "11", "--arch", "linear"]
    run_cli(common + ["--world-size", "1"], d1)
    out = run_cli(common + ["--world-size", "2", "--perf"], d2)
    # --perf: one node img/s line (rank 0) over the slowest rank's train time
    perf = [l for l in out.splitlines() if l.startswith("perf:")]
    assert len(perf) == 1 and "on the slowest rank" in perf[0], perf
    assert "rank: 0, device count: 2, workers:2" in out
    assert "rank: 1, device count: 2, workers:2" in out
    ep = [l for l in out.splitlines() if l.startswith("Epoch:")]
    assert len(ep) == 2
    # test metrics are identical across ranks (unsharded eval)
    assert ep[0].split("test loss")[1] == ep[1].split("test loss")[1]
    a = torch.load(d1 / "checkpoints" / "checkpoint_0.pth.tar", weights_only=True)["state_dict"]
    b = torch.load(d2 / "checkpoints" / "checkpoint_0.pth.tar", weights_only=True)["state_dict"]
    for k in a:
        assert torch.allclose(a[k], b[k], atol=1e-6, rtol=0), (k, (a[k] - b[k]).abs().max())


@pytest.mark.slow
def test_cnn_sgd_cpu_two_ranks(tmp_path):
    out = run_cli(["--epochs", "1", "--synthetic-size", "512", "--world-size", "2", "--arch", "cnn",
                   "--optimizer", "sgd", "--lr", "0.05", "--batch-size", "128"], tmp_path)
    assert len([l for l in out.splitlines() if EPOCH_RE.match(l)]) == 2
    sd = torch.load(tmp_path / "checkpoints" / "checkpoint_0.pth.tar", weights_only=True)
    assert list(sd["state_dict"])[0] == "module.conv1.weight"
    assert set(sd["optimizer"]["state"][0]) == {"momentum_buffer"}


def run_torchrun(args, cwd, nproc=2, timeout=300):
    env = dict(os.environ)
    env["PYTHONPATH"] = REPO + os.pathsep + env.get("PYTHONPATH", "")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={nproc}",
           "--master-addr", "127.0.0.1", "--master-port", str(free_port()),
           os.path.join(REPO, "multi_proc_single_gpu.py"), "--device", "cpu", "--backend", "gloo",
           "--synthetic"] + args
    r = subprocess.run(cmd, cwd=cwd, env=env, capture_output=True, text=True, timeout=timeout)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
    return r.stdout


@pytest.mark.slow
@pytest.mark.parametrize("explicit_init", [False, True])
def test_launch_mode_matches_spawn(tmp_path, explicit_init):
    """torchrun (launch mode, reference S:278-281 / RM:8-35) gives the same run as spawn."""
    d1, d2 = tmp_path / "spawn", tmp_path / "launch"
    d1.mkdir()
    d2.mkdir()
    common = ["--epochs", "1", "--synthetic-size", "2048", "--seed", "4", "--world-size", "2"]
    a = run_cli(common, d1)
    extra = ["-i", f"tcp://127.0.0.1:{free_port()}"] if explicit_init else []
    b = run_torchrun(common + extra, d2)
    ea = sorted(l for l in a.splitlines() if l.startswith(("Epoch:", "rank:")))
    eb = sorted(l for l in b.splitlines() if l.startswith(("Epoch:", "rank:")))
    assert len(ea) == 4 and ea == eb, (ea, eb)
    sa = torch.load(d1 / "checkpoints" / "checkpoint_0.pth.tar", weights_only=True)["state_dict"]
    sb = torch.load(d2 / "checkpoints" / "checkpoint_0.pth.tar", weights_only=True)["state_dict"]
    for k in sa:   # torchrun sets OMP_NUM_THREADS=1: CPU GEMM sums may differ in the last ulp
        assert torch.allclose(sa[k], sb[k], atol=1e-6, rtol=0), k


@pytest.mark.slow
def test_cnn_sharded_fc1_update_matches_replicated_cpu(tmp_path):
    """--shard-fc on the gloo CPU path (world size 2): each rank updates its 64 rows of fc1
    and the rows are all-gathered; the full state is gathered before rank 0 saves.  The
    checkpoint (parameters and momentum) is bit-identical to the replicated run's, and it
    resumes at world size 1."""
    d1, d2 = tmp_path / "rep", tmp_path / "shard"
    d1.mkdir()
    d2.mkdir()
    common = ["--epochs", "1", "--synthetic-size", "512", "--world-size", "2", "--arch", "cnn",
              "--optimizer", "sgd", "--lr", "0.05", "--batch-size", "128", "--seed", "4"]
    run_cli(common, d1)
    out = run_cli(common + ["--shard-fc"], d2)
    assert len([l for l in out.splitlines() if EPOCH_RE.match(l)]) == 2
    a = torch.load(d1 / "checkpoints" / "checkpoint_0.pth.tar", weights_only=True)
    b = torch.load(d2 / "checkpoints" / "checkpoint_0.pth.tar", weights_only=True)
    for k in a["state_dict"]:
        assert torch.equal(a["state_dict"][k], b["state_dict"][k]), k
    for i, st in a["optimizer"]["state"].items():
        assert torch.equal(st["momentum_buffer"], b["optimizer"]["state"][i]["momentum_buffer"]), i
    out = run_cli(["--arch", "cnn", "--optimizer", "sgd", "--evaluate", "--resume",
                   str(d2 / "checkpoints" / "checkpoint_0.pth.tar")], d2)
    assert re.search(r"^test loss: \d+\.\d{6}, test acc: \d+\.\d{2}%\.$", out, re.M)


def test_structure_check_falls_back_with_identical_epoch_lines(tmp_path):
    """The start-up structure check on CPU/gloo, two ranks (parallel/startup.py): the first
    structure fails on rank 1 (an injected fault in its check phase), every rank drops it and
    keeps the fallback, with a warning on stderr; the training state the check changed is
    restored, so the epoch lines equal those of a run without the check."""
    d1, d2 = tmp_path / "off", tmp_path / "on"
    d1.mkdir()
    d2.mkdir()
    common = ["--epochs", "2", "--synthetic-size", "2048", "--seed", "5", "--arch", "cnn",
              "--optimizer", "sgd", "--lr", "0.05", "--world-size", "2"]
    ref = run_cli(common + ["--structure-check", "off"], d1)
    env = dict(os.environ, PYTHONPATH=REPO + os.pathsep + os.environ.get("PYTHONPATH", ""),
               PDM_CALIB_FAULT="1:torch:check")
    cmd = [sys.executable, os.path.join(REPO, "multi_proc_single_gpu.py"), "--device", "cpu",
           "--backend", "gloo", "-i", f"tcp://127.0.0.1:{free_port()}", "--synthetic"] + \
        common + ["--structure-check", "on"]
    r = subprocess.run(cmd, cwd=d2, env=env, capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "torch failed calibration: check on rank 1" in r.stderr, r.stderr
    assert "using step structure 'torch-rebuilt' instead of 'torch'" in r.stderr, r.stderr
    # (each rank prints its own epoch lines, in either order)
    ep = lambda out: sorted(l for l in out.splitlines() if l.startswith("Epoch:"))
    assert len(ep(ref)) == 4 and ep(r.stdout) == ep(ref)
    a = torch.load(d1 / "checkpoints" / "checkpoint_1.pth.tar", weights_only=True)
    b = torch.load(d2 / "checkpoints" / "checkpoint_1.pth.tar", weights_only=True)
    for k, v in a["state_dict"].items():
        assert torch.equal(v, b["state_dict"][k]), k
