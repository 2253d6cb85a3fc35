"""Parity against the reference itself (SURVEY.md §4.3 "Reference parity").

The unmodified reference script (/root/reference/multi_proc_single_gpu.py, read-only) is run
on CPU/gloo with the torchvision stand-in in tests/refshim, and this
framework's CLI is run on the same IDX files from the same initial checkpoint.  Both resume
from that checkpoint (reference S:196-214), train and evaluate, and print the reference's
stdout contract (S:183, S:199-214, S:238-242); the printed lines must be identical and the
written checkpoints must agree.
"""
import os
import shutil
import subprocess
import sys

import numpy as np
import pytest
import torch

from conftest import REPO, free_port

REF_SCRIPT = "/root/reference/multi_proc_single_gpu.py"
SHIM = os.path.join(os.path.dirname(os.path.abspath(__file__)), "refshim")

pytestmark = pytest.mark.skipif(not os.path.exists(REF_SCRIPT), reason="reference not mounted")


def _write_data(root, n_train, n_test):
    from pytorch_distributed_mnist_amd.data.mnist import synthetic_split, write_idx
    raw = os.path.join(root, "MNIST", "raw")
    for train, n, pre in ((True, n_train, "train"), (False, n_test, "t10k")):
        s = synthetic_split(n, train)
        write_idx(os.path.join(raw, f"{pre}-images-idx3-ubyte"), s.images.view(n, 28, 28).numpy())
        write_idx(os.path.join(raw, f"{pre}-labels-idx1-ubyte"), s.labels.numpy().astype(np.uint8))


def _init_checkpoint(path, seed=5):
    """A reference-format checkpoint (S:249-255) of a fresh Linear(784,10) + Adam, epoch 0."""
    torch.manual_seed(seed)
    fc = torch.nn.Linear(784, 10)
    opt = torch.optim.Adam(fc.parameters(), lr=1e-3)
    sd = {"module.fc.weight": fc.weight.detach().clone(), "module.fc.bias": fc.bias.detach().clone()}
    torch.save({"epoch": 0, "state_dict": sd, "best_acc": 0.0, "optimizer": opt.state_dict()}, path)


def _run(cmd, cwd, env_extra, timeout=600):
    env = dict(os.environ)
    env.update(env_extra)
    r = subprocess.run(cmd, cwd=cwd, env=env, capture_output=True, text=True, timeout=timeout)
    assert r.returncode == 0, r.stdout[-4000:] + r.stderr[-4000:]
    return [l for l in r.stdout.splitlines() if not l.startswith("Namespace(")]


def _compare(tmp_path, ws, epochs):
    data = tmp_path / "data"
    _write_data(str(data), 2048, 512)
    ck = tmp_path / "init.pth.tar"
    _init_checkpoint(str(ck))
    ref_dir, new_dir = tmp_path / "ref", tmp_path / "new"
    ref_dir.mkdir()
    new_dir.mkdir()
    common = ["--world-size", str(ws), "--backend", "gloo", "--epochs", str(epochs),
              "--root", str(data), "-j", "0", "--resume", str(ck)]
    ref = _run([sys.executable, REF_SCRIPT] + common + ["-i", f"tcp://127.0.0.1:{free_port()}"],
               ref_dir, {"PYTHONPATH": SHIM, "FAKE_NGPU": str(ws)})
    new = _run([sys.executable, os.path.join(REPO, "multi_proc_single_gpu.py"), "--device", "cpu"]
               + common + ["-i", f"tcp://127.0.0.1:{free_port()}"],
               new_dir, {"PYTHONPATH": REPO})
    # same lines (ranks interleave, so compare as multisets)
    assert sorted(ref) == sorted(new), "\n".join(["reference:"] + ref + ["new:"] + new)
    assert sum(l.startswith("Epoch:") for l in new) == ws * epochs
    for e in range(epochs):
        a = torch.load(ref_dir / "checkpoints" / f"checkpoint_{e}.pth.tar", weights_only=True)
        b = torch.load(new_dir / "checkpoints" / f"checkpoint_{e}.pth.tar", weights_only=True)
        assert a["epoch"] == b["epoch"] and a["best_acc"] == b["best_acc"]
        for k in a["state_dict"]:
            assert torch.allclose(a["state_dict"][k], b["state_dict"][k], atol=1e-6, rtol=0), k
        sa, sb = a["optimizer"]["state"], b["optimizer"]["state"]
        assert sa.keys() == sb.keys()
        for i in sa:
            assert float(sa[i]["step"]) == float(sb[i]["step"])
            for name in ("exp_avg", "exp_avg_sq"):
                assert torch.allclose(sa[i][name], sb[i][name], atol=1e-7, rtol=1e-5), (i, name)
        pa = {k: v for k, v in a["optimizer"]["param_groups"][0].items()}
        pb = {k: v for k, v in b["optimizer"]["param_groups"][0].items()}
        assert pa == pb
    # --evaluate on the final checkpoint prints the same line in both
    last = f"checkpoints/checkpoint_{epochs - 1}.pth.tar"
    ev_ref = _run([sys.executable, REF_SCRIPT, "--world-size", "1", "--backend", "gloo", "--root",
                   str(data), "-j", "0", "--evaluate", "--resume", last,
                   "-i", f"tcp://127.0.0.1:{free_port()}"], ref_dir,
                  {"PYTHONPATH": SHIM, "FAKE_NGPU": "1"})
    ev_new = _run([sys.executable, os.path.join(REPO, "multi_proc_single_gpu.py"), "--device", "cpu",
                   "--world-size", "1", "--backend", "gloo", "--root", str(data), "-j", "0",
                   "--evaluate", "--resume", os.path.join(str(ref_dir), last),
                   "-i", f"tcp://127.0.0.1:{free_port()}"], new_dir, {"PYTHONPATH": REPO})
    t_ref = [l for l in ev_ref if l.startswith("test loss:")]
    t_new = [l for l in ev_new if l.startswith("test loss:")]
    assert len(t_ref) == 1 and t_ref == t_new, (ev_ref, ev_new)


def test_reference_parity_ws1(tmp_path):
    _compare(tmp_path, ws=1, epochs=2)


@pytest.mark.slow
def test_reference_parity_ws2(tmp_path):
    _compare(tmp_path, ws=2, epochs=1)
